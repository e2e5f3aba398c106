set -u
mkdir -p gpurun_out
S="python tools/stage_time.py --shape C5 --world 8 --iters 100 --reps 20"
{
timeout -k 10 200 $S || exit 1
BSLS_TILE_PLAN_AT=9766,2 timeout -k 10 200 $S 2>&1 | grep -E "K2|iteration" || exit 1
BSLS_TILE_PLAN_AT=18000,4 timeout -k 10 200 $S 2>&1 | grep -E "K2|iteration" || exit 1
BSLS_TILE_PLAN_AT=4883,1 timeout -k 10 200 $S 2>&1 | grep -E "K2|iteration" || exit 1
BSLS_TILE_PLAN_AT=18000,8 timeout -k 10 200 $S 2>&1 | grep -E "K2|iteration" || exit 1
BSLS_TILE_PLAN_A=15625,8 timeout -k 10 200 $S 2>&1 | grep -E "K1|iteration" || exit 1
BSLS_TILE_PLAN_A=7813,4 timeout -k 10 200 $S 2>&1 | grep -E "K1|iteration" || exit 1
BSLS_TILE_PLAN_A=7813,8 timeout -k 10 200 $S 2>&1 | grep -E "K1|iteration" || exit 1
timeout -k 10 500 python tools/stage_time.py --shape C5 --iters 20 --reps 5 || exit 1
} > gpurun_out/st_c5b.log 2>&1
