#!/bin/bash
# Round-4 session f: the x-space max in 64 slots, one K2 group on sparse
# shards -- LSQ / batch / distributed tests, the x-space and LBFGS.solve legs,
# then the rehearsed 8-way shard: atomic K1 (default) against the group sums.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
    tests/test_gpu_lsq.py tests/test_gpu_batch.py tests/test_gpu_distributed.py \
    "tests/test_gpu_deep.py::test_two_rank_c5_density_shards_vs_oracle" > gpurun_out/f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/f_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --legs xspace,gdlbfgs --steps 200 --warmup 20 > gpurun_out/f_legs.json \
    2> gpurun_out/f_legs.err || exit 1
python - <<'PY'
import json
t = open('gpurun_out/f_legs.json').read()
d = json.loads(t[t.index('{'):])
for k in ('xspace_bb', 'xspace_bb_panels', 'xspace_bb_tiles'):
    print(k, round(d[k]['us_per_round'], 1), 'us/round')
print('lbfgs_solve', round(d['lbfgs_solve']['ms_per_iteration'], 3), 'ms/iteration')
PY
run() {   # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 \
      > gpurun_out/f_$label.json 2> gpurun_out/f_$label.err || { echo "$label FAILED"; return 1; }
  python - "$label" <<'PY'
import json, sys
t = open('gpurun_out/f_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
k = {n: round(v['avg_us'], 1) for n, v in d['kernels'].items() if n != 'formats'}
print('%-14s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3, k),
      flush=True)
PY
}
for rep in 1 2; do
  run default_$rep || exit 1
  run k1sum_$rep BSLS_K1_ATOMIC=0 || exit 1
done
