mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/kt.log 2>&1 && \
timeout -k 10 300 python -u tools/proj_time.py > gpurun_out/projtime.log 2>&1
