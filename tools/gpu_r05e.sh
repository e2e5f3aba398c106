#!/bin/bash
# round 5, step e: the LDS-staged projection (BSLS_PROJ_PIPE_LDS=1) against
# the direct pipe kernel, its load trim and its knock-out, beside the
# same-size scale floor the bench leg now reports
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
BSLS_PROJ_PIPE_LDS=1 BSLS_LIB=$L/libbsls_hip_ptrim.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5e_trim_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5e_direct.$rep.json 2> gpurun_out/r5e_direct.$rep.err || exit 1
  for v in "" _ptrim _pko; do
    BSLS_PROJ_PIPE_LDS=1 BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5e_lds$v.$rep.json 2> gpurun_out/r5e_lds$v.$rep.err || exit 1
  done
done
