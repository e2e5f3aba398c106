#!/bin/bash
# round 6, step a: the N > 1 self-check rehearsed (2 gloo ranks sharing the
# GPU through bench.py's launch path), then the sharded-driver tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
BSLS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 20 --warmup 5 --windows 2 \
  --no-extras > gpurun_out/r6a_gloo2.json 2> gpurun_out/r6a_gloo2.err || exit 1
timeout -k 10 1100 $T tests/test_gpu_shard_native.py > gpurun_out/r6a_shard.log 2>&1 || exit 1
