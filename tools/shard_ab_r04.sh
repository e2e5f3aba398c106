#!/bin/bash
# Repeated A/B of the rehearsed 8-way C5 rank-0 iteration (bench.py
# --rehearse-shard 8, native driver): the defaults against K2 with one column
# group (BSLS_TILE_PLAN_AT=4883,1), K3 without the warm start
# (BSLS_K3_WARM=0) and K1 with the group sums (BSLS_K1_ATOMIC=0).
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 \
      > gpurun_out/sab_$label.json 2> gpurun_out/sab_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/sab_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k),
      flush=True)
PY
}
for rep in $(seq 1 ${REPS:-2}); do
  run default_$rep || exit 1
  run k2one_$rep BSLS_TILE_PLAN_AT=4883,1 || exit 1
  run nowarm_$rep BSLS_K3_WARM=0 || exit 1
  run k1sum_$rep BSLS_K1_ATOMIC=0 || exit 1
done
