#!/bin/bash
# round 5, step d: the pipelined projection's store policy (write-through sc1
# default vs plain), its knock-out (no passes) with write-through, and the
# LDS-staged coalesced variant (BSLS_PROJ_PIPE_LDS=1) -- first its parity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
BSLS_PROJ_PIPE_LDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5d_lds_tests.log 2>&1 || exit 1
for rep in 1 2; do
for v in "" _pplain _pko lds; do
  if [ "$v" = lds ]; then
    BSLS_PROJ_PIPE_LDS=1 timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5d_proj_lds.$rep.json 2> gpurun_out/r5d_proj_lds.$rep.err || exit 1
  else
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5d_proj$v.$rep.json 2> gpurun_out/r5d_proj$v.$rep.err || exit 1
  fi
done
done
