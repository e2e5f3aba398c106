mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_batch.py > gpurun_out/tests.log 2>&1 || exit 1
for v in _1g "" _1g ""; do
  echo "== lib$v" >> gpurun_out/ko.log
  BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$v.so timeout -k 10 200 python3 tools/bproj.py >> gpurun_out/ko.log 2>&1 || exit 1
done
