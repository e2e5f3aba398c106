mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lsq.py > gpurun_out/lsq.log 2>&1 && \
timeout -k 10 200 python -u tools/xspace_probe.py --panels 1 > gpurun_out/probe1.log 2>&1 && \
timeout -k 10 200 python -u tools/xspace_probe.py --panels 0 --rounds 30 > gpurun_out/probe0.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/batch.log 2>&1
