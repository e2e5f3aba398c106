mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py > gpurun_out/tests.log 2>&1 || exit 1
for v in _c0 "" _c0 ""; do
  echo "== lib$v" >> gpurun_out/ko.log
  BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$v.so timeout -k 10 200 python3 tools/stage_time.py --iters 100 >> gpurun_out/ko.log 2>&1 || exit 1
done
