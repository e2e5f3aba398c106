#!/bin/bash
# Per-rank kernel trace of an 8-way C5 partition's rank 0 through the sharded
# (RCCL) driver on one GPU: bench.py --rehearse-shard 8 under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/reh8 -o run \
    -- python3 bench.py --rehearse-shard 8 --steps 200 --warmup 20 --no-extras > gpurun_out/reh8.log 2>&1
echo "rehearse rc=$?"
