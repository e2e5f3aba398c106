#!/bin/bash
# K3 / wave-PAVA change check: the bit-exact tests that run the wave PAVA, then
# per-stage timing on C3 and C5 (tools/stage_time.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_bb.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py \
    -k "k3 or isotonic or pava or trajectory or oracle_at_scale" > gpurun_out/k3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k3_tests.log; [ $rc -eq 0 ] || exit $rc
for S in C3 C5; do
    timeout -k 10 200 python -u tools/stage_time.py --shape $S --iters 200 --reps 30 > gpurun_out/k3_time_$S.log 2>&1
    rc=$?; echo "$S rc=$rc"; grep -E "iteration|K1|K2|K3" gpurun_out/k3_time_$S.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u tools/iso_time.py > gpurun_out/k3_iso.log 2>&1; echo "iso rc=$?"; tail -4 gpurun_out/k3_iso.log
