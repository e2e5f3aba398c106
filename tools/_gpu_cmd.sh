set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pk3_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 250 python tools/stage_time.py --iters 100 --reps 10 --shape C5 --world 8 > gpurun_out/pk3_sh8.log 2>&1
echo "sh8 rc=$?"
