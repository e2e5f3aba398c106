#!/bin/bash
# round 5: K3's pack form at C5 once the warm start repairs failed partitions
# -- two packs per wave (the default from 64k packs) vs one (BSLS_K3_MERGE=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for m in 1 0; do
    BSLS_K3_MERGE=$m timeout -k 10 300 python -u bench.py --legs main --workload C5 --steps 50 --warmup 20 --windows 5 --profile-iters 0 \
      > gpurun_out/r5mg_m$m.$rep.json 2> gpurun_out/r5mg_m$m.$rep.err || exit 1
  done
done
