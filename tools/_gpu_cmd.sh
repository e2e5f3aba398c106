set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py tests/test_gpu_kernels.py > gpurun_out/mrg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for M in 1 0; do
for S in C3 C5; do
BSLS_K3_MERGE=$M timeout -k 10 200 python tools/stage_time.py --iters 100 --reps 10 --shape $S > gpurun_out/mrg_${S}_$M.log 2>&1
rc=$?; echo "stage $S $M rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
