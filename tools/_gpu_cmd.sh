mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_fullsize.py > gpurun_out/full.log 2>&1 ; echo "rc=$?" >> gpurun_out/full.log
