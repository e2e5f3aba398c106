#!/bin/bash
# LBFGS.solve: trials enqueued per state read (device.LineSearch.CHUNK).
set -o pipefail
mkdir -p gpurun_out
for c in 4 2 3 6 4; do
  BSLS_LS_CHUNK=$c timeout -k 10 300 python -u bench.py --legs gdlbfgs --steps 100 --warmup 10 \
      > gpurun_out/o_$c.json 2> gpurun_out/o_$c.err || exit 1
  python3 - $c <<'PY'
import json, sys
t = open('gpurun_out/o_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])['lbfgs_solve']
print('chunk', sys.argv[1], round(d['ms_per_iteration'], 3), 'ms/it (20-it run)', round(d['ms_per_iteration_marginal'], 3), 'marginal', flush=True)
PY
done
