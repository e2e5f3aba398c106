#!/bin/bash
# round 5, step l: bench.py's N = 2 launch path end to end (torchrun, env
# rendezvous, the native sharded driver over gloo callbacks, max-over-ranks
# windows, the JSON line with its (workload, world) traffic keys) -- both
# ranks on the one GPU, so the timing means nothing; the contract does
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BSLS_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/r5l_n2.json 2> gpurun_out/r5l_n2.err || exit 1
