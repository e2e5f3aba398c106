#!/bin/bash
# round 5, step k: the lean Michelot pass (int counts, reciprocal tau, fmax
# relu: BSLS_PIPE_LEAN=1 variant build) against the default, parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
BSLS_LIB=$L/libbsls_hip_lean.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5k_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5k_def.$rep.json 2> gpurun_out/r5k_def.$rep.err || exit 1
  BSLS_LIB=$L/libbsls_hip_lean.so timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5k_lean.$rep.json 2> gpurun_out/r5k_lean.$rep.err || exit 1
done
