#!/bin/bash
# The LSQ / BATCH / plugin tests (x-space max pass, line-search finish), then
# repeated A/B of the rehearsed 8-way C5 rank-0 iteration (alternating runs:
# the default = atomic K1 on a shard, BSLS_K1_ATOMIC=1 = atomic everywhere,
# BSLS_K1_ATOMIC=0 = group partials + bb_k1_sum), then the x-space legs.
set -o pipefail
mkdir -p gpurun_out
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 \
      > gpurun_out/k1r_$label.json 2> gpurun_out/k1r_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/k1r_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
e = [l.strip() for l in open('gpurun_out/k1r_%s.err' % sys.argv[1]) if 'iterations in' in l]
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3,
                                            e[-1][-60:] if e else ''), flush=True)
PY
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_lsq.py tests/test_gpu_batch.py tests/test_gpu_plugins.py > gpurun_out/k1r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/k1r_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  run default_$rep || exit 1
  run env1_$rep BSLS_K1_ATOMIC=1 || exit 1
  run env0_$rep BSLS_K1_ATOMIC=0 || exit 1
done
timeout -k 10 300 python -u bench.py --legs xspace --steps 200 --warmup 20 > gpurun_out/k1r_xspace.json \
    2> gpurun_out/k1r_xspace.err || exit 1
python - <<'PY'
import json
t = open('gpurun_out/k1r_xspace.json').read()
d = json.loads(t[t.index('{'):])
for k in ('xspace_bb', 'xspace_bb_panels', 'xspace_bb_tiles'):
    print(k, round(d[k]['us_per_round'], 1), 'us/round')
PY
ITERS=20 timeout -k 10 300 python -u tools/lbfgs_ls_time.py > gpurun_out/k1r_lbfgs.log 2>&1 || exit 1
head -3 gpurun_out/k1r_lbfgs.log
