mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/batch_tests.log 2>&1
