mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lsq.py > gpurun_out/lsq.log 2>&1 && \
timeout -k 10 400 python -u -c "
import bench, json
from synthetic import make_shard, add_noise, SEED
sh = make_shard(1_000_000, 50_000, 100_000, 16, seed=SEED)
b = add_noise(sh['Ax'], 0.02, seed=SEED)
print(json.dumps(bench.bench_md(sh, b)), flush=True)
print(json.dumps(bench.bench_xspace(sh, b)), flush=True)
" > gpurun_out/bmd.log 2>&1
