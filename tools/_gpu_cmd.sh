mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xprof -o run -- python3 tools/bxs.py > gpurun_out/bxs.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_lsq.py > gpurun_out/tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/tests.log
