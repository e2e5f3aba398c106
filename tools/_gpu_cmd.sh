set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/t20.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python tools/stress_time.py --what proj,multi > gpurun_out/stress3.log 2>&1
echo "stress rc=$?"
