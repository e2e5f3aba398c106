#!/bin/bash
# round 5, step j: two groups per wave through LDS (BSLS_PROJ_PIPE_LDS=2,
# built for 6 waves per SIMD, and the _w8 variant at 8 with spills) against
# the one-group default; parity of the fast projection tests first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
BSLS_PROJ_PIPE_LDS=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5j_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5j_lds1.$rep.json 2> gpurun_out/r5j_lds1.$rep.err || exit 1
  BSLS_PROJ_PIPE_LDS=2 timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5j_lds2.$rep.json 2> gpurun_out/r5j_lds2.$rep.err || exit 1
  BSLS_PROJ_PIPE_LDS=2 BSLS_LIB=$L/libbsls_hip_w8.so timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5j_lds2w8.$rep.json 2> gpurun_out/r5j_lds2w8.$rep.err || exit 1
done
