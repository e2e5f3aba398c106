#!/bin/bash
# DORE device loop A/B: the reused Ax (default) against BSLS_DORE_RECOMPUTE=1
# (the reference's linop(x) at the top of every iteration), 200 iterations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1 0 1; do
  BSLS_DORE_RECOMPUTE=$v timeout -k 10 300 python -u tools/dore_time.py 200 > gpurun_out/dore_ab_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  echo "recompute=$v $(grep '^{' gpurun_out/dore_ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_iter"], d["extrapolation_taken"])')"
done
