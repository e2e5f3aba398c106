set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_lsq.py > gpurun_out/isop_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/iso_time.py > gpurun_out/isop_time.log 2>&1
echo "iso rc=$?"
