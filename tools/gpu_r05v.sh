#!/bin/bash
# round 5, step v: K3's pack form at C3 now that the warm start skips most
# passes -- two packs per wave (BSLS_K3_MERGE=1) against the default one
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for m in 1 0; do
    BSLS_K3_MERGE=$m timeout -k 10 300 python -u bench.py --legs main --steps 200 --windows 5 > gpurun_out/r5v_m$m.$rep.json 2> gpurun_out/r5v_m$m.$rep.err || exit 1
  done
done
