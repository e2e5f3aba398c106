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

fatal() {  # timeouts (124/137), aborts (134), faults (139) and other signals end the session
    if [ "$1" -eq 124 ] || [ "$1" -ge 128 ]; then
        echo "step failed with rc=$1: stopping GPU work" | tee -a $OUT/status.txt; exit "$1"
    fi
    return 0
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
    list)
      timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
      rc=$?; echo "list rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    pmc)
      # one rocprofv3 pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass),
      # over tools/kprof.py on each workload; traffic -> profiles/traffic_r02.json
      for cfg in C3 C5; do
        i=0
        for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
          i=$((i+1))
          timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${cfg}_$i -o pmc \
              -- python3 tools/kprof.py --config $cfg --iters 10 --proj 10 > $OUT/pmc_${cfg}_$i.log 2>&1
          rc=$?; echo "pmc $cfg $i rc=$rc" | tee -a $OUT/status.txt; fatal $rc
        done
        python3 tools/traffic.py $cfg $OUT/traffic.json $OUT/pmc_${cfg}_1 $OUT/pmc_${cfg}_2 > /dev/null 2> $OUT/traffic_$cfg.err
        python3 tools/pmc_summary.py $OUT/pmc_${cfg}_* > $OUT/pmc_summary_$cfg.txt 2>&1
      done ;;
  esac
done
echo done | tee -a $OUT/status.txt
