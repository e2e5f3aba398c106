#!/bin/bash
# round 5, step f: the lane-maxima lower bound (one Michelot pass less at
# C2), direct and LDS-staged, parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lds in 0 1; do
  BSLS_PROJ_PIPE_LDS=$lds timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5f_tests_lds$lds.log 2>&1 || exit 1
done
for rep in 1 2; do
  for lds in 0 1; do
    BSLS_PROJ_PIPE_LDS=$lds timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5f_lds$lds.$rep.json 2> gpurun_out/r5f_lds$lds.$rep.err || exit 1
  done
done
