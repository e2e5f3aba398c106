#!/bin/bash
# round 5, step s: K2 with its z indices staged into LDS by DMA under the walk
# (BSLS_K2_XZL, default on where the tile fits) -- the BB tests, then C3
# with it and without, twice each on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py \
  tests/test_gpu_fullsize.py > gpurun_out/r5s_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for x in 1 0; do
    BSLS_K2_XZL=$x timeout -k 10 300 python -u bench.py --legs main --steps 200 --windows 5 > gpurun_out/r5s_x$x.$rep.json 2> gpurun_out/r5s_x$x.$rep.err || exit 1
  done
done
