#!/bin/bash
# Round-3 A/B session: the sharded schedule (ShardedBB fuse, BSLS_SHARD_FUSE
# 1 = stage 8 with the previous iteration's stop test folded into K2, 0 =
# stage 3 + a stage-9 launch after every exchange), rehearsed on one GPU as
# rank 0 of the 8-way C5 split.  (Also used this round for the lane-pair /
# quad projection variants and a fused ||r||^2 schedule on one GPU, both
# measured slower and removed)  Every GPU step has its own
# timeout; a crash / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -eq 124 ] || [ "$1" -ge 128 ]; then echo "rc=$1: stop" | tee -a $OUT/ab.txt; exit "$1"; fi; }
for v in 0 1; do
  BSLS_SHARD_FUSE=$v timeout -k 10 400 python bench.py --rehearse-shard 8 --steps 200 --warmup 20 \
      > $OUT/ab_shard_fuse$v.log 2>&1
  rc=$?; echo "shard fuse=$v rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
done
rm -rf $OUT/prof_shard0
BSLS_SHARD_FUSE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard0 -o run \
    -- python3 bench.py --rehearse-shard 8 --steps 100 --warmup 10 > $OUT/prof_shard0.log 2>&1
rc=$?; echo "prof shard fuse=0 rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
echo done | tee -a $OUT/ab.txt
