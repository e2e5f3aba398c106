mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stage_time.py > gpurun_out/st_new.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py > gpurun_out/tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/tests.log
