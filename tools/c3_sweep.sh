#!/bin/bash
# C3 variants through environment switches only (no rebuild): K3 merged packs,
# K1 / K2 tile plans.  tools/stage_time.py per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "X=0" "BSLS_K3_MERGE=1" "BSLS_TILE_PLAN_A=3125,8 BSLS_TILE_PLAN_AT=7813,1" "BSLS_TILE_PLAN_A=6250,4" "BSLS_TILE_PLAN_AT=3907,2"; do
    echo "== $v" | tee -a gpurun_out/c3_sweep.txt
    env $v timeout -k 10 200 python -u tools/stage_time.py --shape C3 --iters 300 --reps 50 > gpurun_out/c3_sweep_tmp.log 2>&1
    rc=$?
    grep -E "tiles|iteration|K1|K2|K3" gpurun_out/c3_sweep_tmp.log | tee -a gpurun_out/c3_sweep.txt
    [ $rc -eq 0 ] || { echo "rc=$rc: stop" | tee -a gpurun_out/c3_sweep.txt; exit $rc; }
done
# bench.py's N > 1 launch path (torchrun, env rendezvous, sharded driver), two
# ranks on this one GPU over gloo
BSLS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/gloo2.log 2>&1
echo "gloo2 rc=$?" | tee -a gpurun_out/c3_sweep.txt
