#!/bin/bash
# round 5, step i: PMC traffic of the fused kernels with dz . dg as
# ||r - r_prev||^2 (BSLS_SY_DR=1: K3 writes no dz, K2 reads none), C3 and C5,
# -> gpurun_out/traffic_r05_sydr.json; and the C3 / C5 kernel traces with it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp BSLS_SY_DR=1
for cfg in C3 C5; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    rm -rf $OUT/pmcs_${cfg}_$i
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmcs_${cfg}_$i -o pmc \
        -- python3 tools/kprof.py --config $cfg --iters 10 --proj 0 > $OUT/pmcs_${cfg}_$i.log 2>&1 || exit 1
  done
  python3 tools/traffic.py $cfg $OUT/traffic_r05_sydr.json $OUT/pmcs_${cfg}_1 $OUT/pmcs_${cfg}_2 > /dev/null || exit 1
done
for k in C3:main C5:c5; do
  key=${k%%:*}; leg=${k##*:}
  rm -rf $OUT/profs_$key
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profs_$key -o run \
      -- python3 bench.py --legs $leg --steps 100 --warmup 10 --windows 2 > $OUT/profs_$key.log 2>&1 || exit 1
  cp "$(find $OUT/profs_$key -name '*kernel_stats.csv' | head -n 1)" $OUT/r05_${key}_sydr_kernel_stats.csv
done
