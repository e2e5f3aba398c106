#!/bin/bash
# Per-ITERATION plan sweep of the rehearsed 8-way C5 rank-0 shard (VERDICT r03:
# the plans were swept per kernel, not inside the iteration).  Each line: the
# K1 / K2 tile plans ("H,groups") and the rehearsed rank-0 iterations/s through
# the native sharded driver (bsls_bb_shard_iterate).  A variant library built
# with -DBSLS_K1_SPLIT=0 (K1's group sum in the walk launch's last arriver)
# rides along via BSLS_LIB.
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 \
      > gpurun_out/sweep_$label.json 2> gpurun_out/sweep_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/sweep_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k), flush=True)
PY
}
run default || exit 1
run k1_2x128 BSLS_TILE_PLAN_A=7813,2 || exit 1
run k1_4x128 BSLS_TILE_PLAN_A=7813,4 || exit 1
run k1_8x50 BSLS_TILE_PLAN_A=20000,8 || exit 1
run k2_1x256 BSLS_TILE_PLAN_AT=4883,1 || exit 1
run k2_2x64 BSLS_TILE_PLAN_AT=19532,2 || exit 1
run k2_1x128 BSLS_TILE_PLAN_AT=9766,1 || exit 1
run k2_4x64 BSLS_TILE_PLAN_AT=19532,4 || exit 1
if [ -f block-simplex-least-squares_amd/lib/libbsls_hip_nosplit.so ]; then
  run k1_nosplit BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip_nosplit.so || exit 1
fi
run python_loop BSLS_SHARD_NATIVE=0 || exit 1
