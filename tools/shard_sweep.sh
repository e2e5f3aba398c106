#!/bin/bash
# Tile-plan sweep on one C5 shard (rank 0 of W): tools/stage_time.py per plan,
# BSLS_TILE_PLAN_A / BSLS_TILE_PLAN_AT = "H,groups" ("-" = the default plan).
#   W=8 bash tools/shard_sweep.sh "A_plan AT_plan" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
W=${W:-8}
for pr in "$@"; do
    set -- $pr
    a=$1; at=$2
    envs=""
    [ "$a" != "-" ] && envs="BSLS_TILE_PLAN_A=$a"
    [ "$at" != "-" ] && envs="$envs BSLS_TILE_PLAN_AT=$at"
    log=gpurun_out/sweep_w${W}_${a//,/x}_${at//,/x}.log
    echo "== W=$W A=$a AT=$at" | tee -a gpurun_out/sweep.txt
    env $envs timeout -k 10 200 python -u tools/stage_time.py --shape C5 --world $W --iters 200 --reps 30 > $log 2>&1
    rc=$?
    grep -E "tiles|iteration|K1|K2|K3" $log | tee -a gpurun_out/sweep.txt
    if [ $rc -ne 0 ]; then echo "rc=$rc: stop" | tee -a gpurun_out/sweep.txt; exit $rc; fi
done
