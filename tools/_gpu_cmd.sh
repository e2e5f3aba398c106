mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lsq.py tests/test_gpu_batch.py > gpurun_out/lsq.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mdprof -o run -- python3 tools/bmd.py > gpurun_out/bmd.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xprof -o run -- python3 tools/xspace_probe.py --rounds 3 > gpurun_out/xprobe.log 2>&1
