#!/bin/bash
# Round-4 session e: plugin / batch / distributed tests, then the rehearsed
# 8-way shard A/B (tools/shard_ab_r04.sh, one repetition), the x-space legs
# and the LBFGS.solve timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
    tests/test_gpu_plugins.py tests/test_gpu_batch.py tests/test_gpu_distributed.py tests/test_gpu_lsq.py \
    "tests/test_gpu_deep.py::test_two_rank_c5_density_shards_vs_oracle" > gpurun_out/e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/e_tests.log; [ $rc -eq 0 ] || exit 1
REPS=1 bash tools/shard_ab_r04.sh || exit 1
timeout -k 10 300 python -u bench.py --legs xspace --steps 200 --warmup 20 > gpurun_out/e_xspace.json \
    2> gpurun_out/e_xspace.err || exit 1
python - <<'PY'
import json
t = open('gpurun_out/e_xspace.json').read()
d = json.loads(t[t.index('{'):])
for k in ('xspace_bb', 'xspace_bb_panels', 'xspace_bb_tiles'):
    print(k, round(d[k]['us_per_round'], 1), 'us/round')
PY
ITERS=20 timeout -k 10 300 python -u tools/lbfgs_ls_time.py > gpurun_out/e_lbfgs.log 2>&1 || exit 1
head -3 gpurun_out/e_lbfgs.log
