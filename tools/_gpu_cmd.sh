set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bb.py -k "k3 or long_blocks" > gpurun_out/t14.log 2>&1
echo "tests rc=$?"
timeout -k 10 700 python bench.py > gpurun_out/b14.log 2>&1
echo "bench rc=$?"
