#!/bin/bash
# C5 on one GPU: K1 with more column groups (an XCD's resident workgroups on
# one narrower x slice) once the group sums are atomics (BSLS_K1_ATOMIC=1:
# no partials), against the default plan (4 groups, partials + bb_k1_sum).
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --legs main --workload C5 --steps 100 --warmup 10 \
      > gpurun_out/i_$label.json 2> gpurun_out/i_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/i_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-12s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k),
      flush=True)
PY
}
run default || exit 1
run atom_g4 BSLS_K1_ATOMIC=1 || exit 1
run atom_g8 BSLS_K1_ATOMIC=1 BSLS_TILE_PLAN_A=15625,8 || exit 1
run atom_g16 BSLS_K1_ATOMIC=1 BSLS_TILE_PLAN_A=15625,16 || exit 1
timeout -k 10 300 python -u bench.py --legs main --steps 200 --warmup 20 > gpurun_out/i_c3.json 2> gpurun_out/i_c3.err || exit 1
python - <<'PY'
import json
t = open('gpurun_out/i_c3.json').read()
d = json.loads(t[t.index('{'):])
print('C3', round(d['value'], 1), 'it/s', {k: round(v['avg_us'], 1) for k, v in d['kernels'].items() if k != 'formats'})
PY
