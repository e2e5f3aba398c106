set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; echo "suite rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for S in C3 C5; do
timeout -k 10 200 python tools/stage_time.py --iters 100 --reps 10 --shape $S > gpurun_out/def_$S.log 2>&1
rc=$?; echo "stage $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
