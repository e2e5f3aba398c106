set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_bb.py > gpurun_out/k2s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 250 python tools/stage_time.py --iters 100 --reps 10 --shape C5 --world 8 > gpurun_out/k2s_sh8.log 2>&1
echo "sh8 rc=$?"
timeout -k 10 300 python bench.py --rehearse-shard 8 --steps 200 --warmup 20 > gpurun_out/k2s_reh8.log 2>&1
echo "reh8 rc=$?"
