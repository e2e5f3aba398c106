set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_distributed.py > gpurun_out/t22.log 2>&1
echo "tests rc=$?"
{
echo "== C5"; timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 | grep -E "K1|K2|K3|iteration" || exit 1
echo "== shard"; timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 8 | grep -E "K1|K2|K3|iteration" || exit 1
echo "== shard/2"; timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 2 | grep -E "K1|K2|K3|iteration" || exit 1
echo "== shard/4"; timeout -k 10 200 python tools/stage_time.py --iters 50 --reps 10 --shape C5 --world 4 | grep -E "K1|K2|K3|iteration" || exit 1
} > gpurun_out/st22.log 2>&1
echo "stage rc=$?"
