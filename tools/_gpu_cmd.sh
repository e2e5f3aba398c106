set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py > gpurun_out/k2e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for S in C3 C5; do
timeout -k 10 200 python tools/stage_time.py --iters 100 --reps 10 --shape $S > gpurun_out/k2e_${S}.log 2>&1
rc=$?; echo "stage $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
