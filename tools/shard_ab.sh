#!/bin/bash
# 8-way C5 shard rehearsal A/B over BSLS_SHARD_FUSE (1: K2 folds the previous
# iteration's ||r||^2 / f / stop test, stage 8; 0: stage 3 + a stage-9 launch
# per iteration), then the C2 projection kernel trace on the current default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in ${FUSE:-1 0}; do
  BSLS_SHARD_FUSE=$f timeout -k 10 400 python bench.py --rehearse-shard 8 --steps 200 --warmup 20 \
      > gpurun_out/rehearse8_fuse$f.log 2>&1
  rc=$?; echo "rehearse fuse=$f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/rehearse8_fuse$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('fuse', $f, 'value', d['value'], 'ms', d['ms_per_step'])"
done
if [ -n "${PROF_C2:-1}" ]; then
  rm -rf gpurun_out/prof_C2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_C2 -o run \
      -- python3 bench.py --legs proj > gpurun_out/prof_C2.log 2>&1
  rc=$?; echo "prof C2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_C2 -name '*kernel_stats.csv' | head -n 1)
  [ -n "$f" ] && cp "$f" gpurun_out/r03_C2_kernel_stats.csv
fi
