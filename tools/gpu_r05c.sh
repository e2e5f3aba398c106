#!/bin/bash
# round 5, step c: PMC width calibration (tools/fetch_calib.hip), the
# projection's lanes-per-block / knock-out variants, PMC bytes of the
# projection kernels, and the tests the last step's first failure skipped.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
L=block-simplex-least-squares_amd/lib
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r5c_calib_$c -o calib -- ./tools/fetch_calib > gpurun_out/r5c_calib_$c.log 2>&1 || exit 1
done
for v in "" _lpb4 _lpb16 _pko; do
  BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5c_proj$v.json 2> gpurun_out/r5c_proj$v.err || exit 1
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r5c_pmcproj_$c -o pmc -- python3 bench.py --legs proj > gpurun_out/r5c_pmcproj_$c.log 2>&1 || exit 1
done
timeout -k 10 600 $T tests/test_gpu_lsq.py tests/test_gpu_bb.py -k "fixed_point or fixed_iterations" > gpurun_out/r5c_lsq_bb.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_batch.py -k "fast_projection" > gpurun_out/r5c_batch_fast.log 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_deep.py -k c3 > gpurun_out/r5c_deep_c3.log 2>&1 || exit 1
