set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/t11.log 2>&1
echo "tests rc=$?"
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/b11.log 2>&1
echo "bench rc=$?"
