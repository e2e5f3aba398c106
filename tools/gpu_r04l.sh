#!/bin/bash
# Rehearsed 8-way shard: taller K1 tiles (the LDS's 20k row sums) with 4 / 5
# column groups (atomic sums), against the default 4 x 64 of 15.6k rows.
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 \
      > gpurun_out/l_$label.json 2> gpurun_out/l_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/l_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k),
      flush=True)
PY
}
run default || exit 1
run k1_4x50 BSLS_TILE_PLAN_A=20000,4 || exit 1
run k1_5x50 BSLS_TILE_PLAN_A=20000,5 || exit 1
run k1_3x85 BSLS_TILE_PLAN_A=11765,3 || exit 1
STEPS=prof PROF="C3 md_xs gdlbfgs" bash tools/gpu_r04.sh || exit 1
