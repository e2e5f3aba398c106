#!/bin/bash
# round 5: per-dispatch kernel trace of the driver's bench arguments (C3
# main leg), to see which kernel is slower in the early iterations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run \
  -- python3 bench.py --legs main --steps 20 --warmup 5 --profile-iters 0 > gpurun_out/kt.log 2>&1
