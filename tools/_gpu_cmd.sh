set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py -k k3 > gpurun_out/cap_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for V in "" _nocap; do
BSLS_LIB=block-simplex-least-squares_amd/lib/libbsls_hip$V.so timeout -k 10 250 python tools/stage_time.py --iters 50 --reps 10 --shape C5 > gpurun_out/cap_C5$V.log 2>&1
rc=$?; echo "C5 $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
for M in 1 0; do
BSLS_K3_MERGE=$M BSLS_LIB=block-simplex-least-squares_amd/lib/libbsls_hip$V.so timeout -k 10 250 python tools/stage_time.py --iters 100 --reps 10 --shape C3 > gpurun_out/cap_C3_m$M$V.log 2>&1
rc=$?; echo "C3 m$M $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
