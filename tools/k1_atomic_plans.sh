#!/bin/bash
# The atomic K1 (the default on a column shard since this commit): the
# distributed / BB / two-rank deep tests first, then the rehearsed 8-way C5
# rank-0 iteration against the split finish and over K1 / K2 tile plans.
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 \
      > gpurun_out/k1p_$label.json 2> gpurun_out/k1p_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/k1p_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k), flush=True)
PY
}
leg() {   # label, workload, then env
  local label=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --legs main --workload $wl --steps 200 --warmup 20 \
      > gpurun_out/k1p_$label.json 2> gpurun_out/k1p_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/k1p_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
def walk(d, p=''):
    for k, v in d.items():
        if isinstance(v, dict) and 'avg_us' in v: print('  %s%s %.1f us' % (p, k, v['avg_us']))
        elif isinstance(v, dict): walk(v, p + k + '.')
print(sys.argv[1], 'value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'] * 1e3, 1), flush=True)
walk(d.get('kernels', {}))
PY
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py tests/test_gpu_bb.py "tests/test_gpu_deep.py::test_two_rank_c5_density_shards_vs_oracle" \
    > gpurun_out/k1p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k1p_tests.log; [ $rc -eq 0 ] || exit 1
run default || exit 1
run split BSLS_K1_ATOMIC=0 || exit 1
run a_8x64 BSLS_TILE_PLAN_A=15625,8 || exit 1
run a_4x128 BSLS_TILE_PLAN_A=7813,4 || exit 1
run a_2x128 BSLS_TILE_PLAN_A=7813,2 || exit 1
run a_k2_1x256 BSLS_TILE_PLAN_AT=4883,1 || exit 1
