mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_lsq.py tests/test_gpu_batch.py > gpurun_out/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/stage_time.py --iters 100 > gpurun_out/ko.log 2>&1 && timeout -k 10 300 python3 tools/bxs.py > gpurun_out/bxs.log 2>&1
