#!/bin/bash
# round 5, step g: LDS-staged projection by default (trimmed clamps, one
# division up front): parity of every projection test, then the C2 leg twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_batch.py > gpurun_out/r5g_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5g_proj.$rep.json 2> gpurun_out/r5g_proj.$rep.err || exit 1
done
# standalone PAVA: the product build and the no-pass knock-out, beside the floor
L=block-simplex-least-squares_amd/lib
for v in "" _iko; do
  BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 240 python -u bench.py --legs iso > gpurun_out/r5g_iso$v.json 2> gpurun_out/r5g_iso$v.err || exit 1
done
