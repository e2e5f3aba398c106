#!/bin/bash
# round 6, step i: bench.py's N > 1 launch path with 4 gloo ranks sharing the
# GPU (self-check, weak-scaled C3 headline, strong-scaled C5 leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BSLS_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 4 --steps 20 --warmup 5 --windows 2 \
  > gpurun_out/r6i_gloo4.json 2> gpurun_out/r6i_gloo4.err || exit 1
