set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "dore or DORE" > gpurun_out/dore_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/dore_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/dore_time.py > gpurun_out/dore_time.log 2>&1; echo "time rc=$?"; tail -1 gpurun_out/dore_time.log | cut -c1-400
