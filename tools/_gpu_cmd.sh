mkdir -p gpurun_out
BSLS_LIB=$PWD/build/libbsls_hip_wm.so timeout -k 10 300 python -u tools/stage_time.py > gpurun_out/st_wm.log 2>&1 && \
BSLS_LIB=$PWD/build/libbsls_hip_wm.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bb.py > gpurun_out/tests_wm.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/tests_wm.log
