#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step runs under its own timeout; a crash / timeout / abort ends the
# script (no further GPU work), an ordinary test failure (pytest rc 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"

fatal() {  # rc -> 0 if the next GPU step may run
    case "$1" in
        0|1) return 0 ;;
        *) echo "step failed with rc=$1: stopping GPU work" | tee -a $OUT/status.txt; exit "$1" ;;
    esac
}

for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    alltests)
      timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=600 > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "alltests rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
          -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/prof.log 2>&1
      rc=$?; echo "prof rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
  esac
done
echo done | tee -a $OUT/status.txt
