#!/bin/bash
# Rehearsed 8-way shard: K2 tile heights with one group; then the C3 / C5
# kernel traces refreshed with the final bench (K3 timed inside iterations).
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 \
      > gpurun_out/j_$label.json 2> gpurun_out/j_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/j_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k),
      flush=True)
PY
}
run default || exit 1
run k2_1x128 BSLS_TILE_PLAN_AT=9766,1 || exit 1
run k2_1x384 BSLS_TILE_PLAN_AT=3256,1 || exit 1
STEPS=prof PROF="C3 C5" bash tools/gpu_r04.sh || exit 1
