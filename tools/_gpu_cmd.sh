mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py > gpurun_out/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/stage_time.py --iters 100 > gpurun_out/ko.log 2>&1 && timeout -k 10 200 python3 tools/stage_time.py --iters 100 >> gpurun_out/ko.log 2>&1
