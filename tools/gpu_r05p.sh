#!/bin/bash
# round 5, step p: PMC traffic of rank 0's kernels for every N-GPU line the
# driver can print (C3 weak shards, C5 strong shards; N = 2, 4, 8) over the
# one-GPU rehearsal of that rank, merged into traffic_r05.json as
# '<workload>_x<N>' -- bench.py's lookup keys at N GPUs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cp profiles/traffic_r05.json $OUT/traffic_r05.json || exit 1
for wl in C3 C5; do
  for n in 2 4 8; do
    i=0
    for grp in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      d=$OUT/pmcx_${wl}_${n}_$i
      rm -rf $d
      timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $d -o pmc \
          -- python3 bench.py --rehearse-shard $n --rehearse-workload $wl --steps 30 --warmup 5 --windows 1 \
          > $d.log 2>&1 || exit 1
    done
    python3 tools/traffic.py ${wl}_x$n $OUT/traffic_r05.json $OUT/pmcx_${wl}_${n}_1 $OUT/pmcx_${wl}_${n}_2 > /dev/null || exit 1
  done
done
