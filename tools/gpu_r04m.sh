#!/bin/bash
# K3 masks per projection slot (DORE's second projection, the line search's
# trials): plugin / BB tests, then the DORE and LBFGS.solve legs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_plugins.py tests/test_gpu_bb.py > gpurun_out/m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --legs dore,gdlbfgs --steps 200 --warmup 20 \
    > gpurun_out/m_legs.json 2> gpurun_out/m_legs.err || exit 1
python3 - <<'PY'
import json
t = open('gpurun_out/m_legs.json').read()
d = json.loads(t[t.index('{'):])
print('dore', round(d['dore']['us_per_iter'], 1), 'lbfgs_solve', round(d['lbfgs_solve']['ms_per_iteration'], 3),
      round(d['lbfgs_solve']['ms_per_iteration_marginal'], 3))
PY
