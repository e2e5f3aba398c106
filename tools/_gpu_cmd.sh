mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bb.py -k "k3 or deterministic" > gpurun_out/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/iso_time.py > gpurun_out/iso.log 2>&1
