#!/bin/bash
# round 5: the driver's arguments against a long warmup, with K3's repair
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 5 400; do
    timeout -k 10 300 python -u bench.py --legs main --steps 20 --warmup $w --profile-iters 0 \
      > gpurun_out/r5ws_w$w.$rep.json 2> gpurun_out/r5ws_w$w.$rep.err || exit 1
  done
done
