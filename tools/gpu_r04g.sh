#!/bin/bash
# LBFGS.solve per-iteration time: the bench leg alone, with and without K3's
# warm start, and the timing tool (device / host line search).
set -o pipefail
mkdir -p gpurun_out
for w in 1 0; do
  BSLS_K3_WARM=$w timeout -k 10 300 python -u bench.py --legs gdlbfgs --steps 200 --warmup 20 \
      > gpurun_out/g_gd_$w.json 2> gpurun_out/g_gd_$w.err || exit 1
  python - $w <<'PY'
import json, sys
t = open('gpurun_out/g_gd_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
print('warm', sys.argv[1], 'lbfgs_solve', round(d['lbfgs_solve']['ms_per_iteration'], 3), 'ms/iteration',
      'direction', round(d['lbfgs_solve']['direction']['us'], 1), 'us', flush=True)
PY
done
ITERS=20 timeout -k 10 300 python -u tools/lbfgs_ls_time.py > gpurun_out/g_lbfgs.log 2>&1 || exit 1
head -4 gpurun_out/g_lbfgs.log
