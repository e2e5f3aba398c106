set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "isotonic or dense_row" tests/test_gpu_bb.py::test_dense_row_network_falls_back_to_tiles > gpurun_out/t3.log 2>&1 || exit 1
timeout -k 10 200 python tools/iso_time.py > gpurun_out/iso.log 2>&1
