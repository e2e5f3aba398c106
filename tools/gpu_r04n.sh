#!/bin/bash
# DORE on the device with and without K3's warm start.
set -o pipefail
mkdir -p gpurun_out
for w in 1 0 1 0; do
  BSLS_K3_WARM=$w timeout -k 10 300 python -u bench.py --legs dore --steps 200 --warmup 20 \
      > gpurun_out/n_dore_$w.json 2> gpurun_out/n_dore_$w.err || exit 1
  python3 - $w <<'PY'
import json, sys
t = open('gpurun_out/n_dore_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
print('warm', sys.argv[1], 'dore', round(d['dore']['us_per_iter'], 1), flush=True)
PY
done
