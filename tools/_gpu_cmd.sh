set -u
mkdir -p gpurun_out
{
for PT in 9766,2 19532,4 6510,1; do
echo "== shard K2 $PT"; BSLS_TILE_PLAN_AT=$PT timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 8 | grep -E "K2|iteration" || exit 1
done
for PT in 19532,2 9766,1; do
echo "== shard/4 K2 $PT"; BSLS_TILE_PLAN_AT=$PT timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 4 | grep -E "K2|iteration" || exit 1
done
} > gpurun_out/st24.log 2>&1
echo "stage rc=$?"
timeout -k 10 700 python bench.py --no-cpu-baseline > gpurun_out/b24.log 2>&1
echo "bench rc=$?"
