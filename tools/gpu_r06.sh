#!/bin/bash
# One GPU-box session (round 6): parity tests, smoke, bench, and one rocprofv3
# kernel-trace run per workload (profiles/r06_<key>_kernel_stats.csv), so a
# kernel name's rows never mix workloads.  Every GPU step runs under its own
# timeout; a crash / timeout / abort ends the script (no further GPU work), an
# ordinary test failure (pytest rc 1) does not.
#   STEPS="tests smoke bench prof pmc pmcx sq" tools/gpu_r06.sh
#   PROF="C5 C3 C2 C4iso md_xs C5x8" (the prof step's workloads)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
PROF="${PROF:-C3 C5 C2 C4iso md_xs gdlbfgs C5x8}"
TESTS="${TESTS:-tests}"

fatal() {  # timeouts (124/137), aborts (134), faults (139) and other signals end the session
    if [ "$1" -eq 124 ] || [ "$1" -ge 128 ]; then
        echo "step failed with rc=$1: stopping GPU work" | tee -a $OUT/status.txt; exit "$1"
    fi
    return 0
}

prof() {  # prof <key> <bench args...>
    local key=$1; shift
    rm -rf $OUT/prof_$key
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$key -o run \
        -- python3 bench.py "$@" > $OUT/prof_$key.log 2>&1
    local rc=$?
    echo "prof $key rc=$rc" | tee -a $OUT/status.txt; fatal $rc
    local f
    f=$(find $OUT/prof_$key -name '*kernel_stats.csv' | head -n 1)
    [ -n "$f" ] && cp "$f" $OUT/r06_${key}_kernel_stats.csv
    return 0
}

for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
          > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    alltests)
      timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread \
          > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "alltests rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    driverlike)
      # the driver's own arguments (BENCH_rNN: --steps 20 --warmup 5)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_driverlike.log 2>&1
      rc=$?; echo "driverlike rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    legs)
      timeout -k 10 600 python bench.py --legs "${LEGS:-lbfgs}" > $OUT/bench_legs.log 2>&1
      rc=$?; echo "legs rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    exit)
      timeout -k 10 300 python tools/exit_iters.py > $OUT/exit_iters.log 2>&1
      rc=$?; echo "exit rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    rehearse)
      timeout -k 10 400 python bench.py --rehearse-shard 8 --steps 200 --warmup 20 \
          > $OUT/rehearse8.log 2>&1
      rc=$?; echo "rehearse rc=$rc" | tee -a $OUT/status.txt; fatal $rc ;;
    pmc)
      # one rocprofv3 pass per counter group (FETCH_SIZE and WRITE_SIZE cannot
      # share a pass) over tools/kprof.py; traffic -> gpurun_out/traffic.json
      for cfg in ${PMC_CFG:-C3 C5}; do
        extra=""
        [ "$cfg" = C3 ] && extra="--proj 10 --iso 10"
        i=0
        for grp in "FETCH_SIZE" "WRITE_SIZE"; do
          i=$((i+1))
          rm -rf $OUT/pmc_${cfg}_$i
          timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${cfg}_$i -o pmc \
              -- python3 tools/kprof.py --config $cfg --iters 10 $extra > $OUT/pmc_${cfg}_$i.log 2>&1
          rc=$?; echo "pmc $cfg $i rc=$rc" | tee -a $OUT/status.txt; fatal $rc
        done
        python3 tools/traffic.py $cfg $OUT/traffic_r06.json $OUT/pmc_${cfg}_1 $OUT/pmc_${cfg}_2 \
            > /dev/null 2> $OUT/traffic_$cfg.err
      done
      # rank 0 of the 8-way C5 split (the rehearsal bench.py --rehearse-shard 8
      # runs): its kernels keyed C5_x8, as bench.py reads them at N > 1
      if [ -n "${PMC_X8:-1}" ]; then
        i=0
        for grp in "FETCH_SIZE" "WRITE_SIZE"; do
          i=$((i+1))
          rm -rf $OUT/pmc_C5x8_$i
          timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_C5x8_$i -o pmc \
              -- python3 bench.py --rehearse-shard 8 --steps 30 --warmup 5 --windows 1 > $OUT/pmc_C5x8_$i.log 2>&1
          rc=$?; echo "pmc C5x8 $i rc=$rc" | tee -a $OUT/status.txt; fatal $rc
        done
        python3 tools/traffic.py C5_x8 $OUT/traffic_r06.json $OUT/pmc_C5x8_1 $OUT/pmc_C5x8_2 \
            > /dev/null 2> $OUT/traffic_C5x8.err
      fi ;;
    pmcx)
      # rank 0's kernels for every N-GPU line the driver can print (C3 weak
      # shards, C5 strong shards; N = 2, 4, 8) over the one-GPU rehearsal of
      # that rank, merged into traffic_r06.json as '<workload>_x<N>'
      for wl in C3 C5; do
        for n in 2 4 8; do
          [ "$wl$n" = C58 ] && continue      # (C5_x8: the pmc step's)
          i=0
          for grp in FETCH_SIZE WRITE_SIZE; do
            i=$((i+1))
            d=$OUT/pmcx_${wl}_${n}_$i
            rm -rf $d
            timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $d -o pmc \
                -- python3 bench.py --rehearse-shard $n --rehearse-workload $wl --steps 30 --warmup 5 --windows 1 \
                > $d.log 2>&1
            rc=$?; echo "pmcx $wl $n $i rc=$rc" | tee -a $OUT/status.txt; fatal $rc
          done
          python3 tools/traffic.py ${wl}_x$n $OUT/traffic_r06.json $OUT/pmcx_${wl}_${n}_1 $OUT/pmcx_${wl}_${n}_2 \
              > /dev/null 2> $OUT/traffic_${wl}x$n.err
        done
      done ;;
    sq)
      # SQ occupancy / issue / wait counters over the C3 kernels, the C2
      # projection and the planned standalone PAVA (two passes, 8 SQ each)
      i=0
      for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
                 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
        i=$((i+1))
        rm -rf $OUT/sq_$i
        timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq_$i -o pmc \
            -- python3 tools/kprof.py --config C3 --iters 5 --proj 5 --iso 10 > $OUT/sq_$i.log 2>&1
        rc=$?; echo "sq $i rc=$rc" | tee -a $OUT/status.txt; fatal $rc
      done
      python3 tools/pmc_summary.py $OUT/sq_1 $OUT/sq_2 > $OUT/r06_sq_summary_C3.txt 2>&1 ;;
    prof)
      for k in $PROF; do
        case "$k" in
          C3)    prof C3 --legs main --steps 200 --warmup 10 ;;
          C5)    prof C5 --legs c5 --steps 100 --warmup 10 ;;
          gdlbfgs) prof gdlbfgs --legs gdlbfgs ;;
          C2)    prof C2 --legs proj ;;
          C4iso) prof C4iso --legs iso ;;
          md_xs) prof md_xs --legs xspace,md,dore,lbfgs ;;
          C5x8)  prof C5_x8 --rehearse-shard 8 --steps 100 --warmup 10 ;;
        esac
      done ;;
  esac
done
echo done | tee -a $OUT/status.txt
