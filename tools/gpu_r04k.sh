#!/bin/bash
# C3 tile-walk knock-outs (BSLS_TILE_KO=1: plain LDS add instead of ds_add_f64,
# 2: no LDS accumulation; variant builds through BSLS_LIB, timing only -- the
# results are wrong by construction) against the product build.
set -o pipefail
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
for v in "" _ko1 _ko2; do
  lib=$PWD/$L/libbsls_hip$v.so
  BSLS_LIB=$lib timeout -k 10 300 python -u bench.py --legs main --steps 200 --warmup 20 \
      > gpurun_out/k_c3$v.json 2> gpurun_out/k_c3$v.err || exit 1
  python - "c3$v" <<'PY'
import json, sys
t = open('gpurun_out/k_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
print('%-8s %8.1f it/s  %6.1f us/it  %s' % (sys.argv[1], d['value'], d['ms_per_step'] * 1e3,
      {k: round(v['avg_us'], 1) for k, v in d['kernels'].items() if k != 'formats'}), flush=True)
PY
done
