#!/bin/bash
# Kernel trace of the x-space legs (fixed-point residual: max pass in slots)
# and the LBFGS.solve leg timed after two warm runs.
set -o pipefail
mkdir -p gpurun_out/h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h/xs -o xs -- \
    python3 bench.py --legs xspace,gdlbfgs --steps 100 --warmup 10 > gpurun_out/h/legs.json 2> gpurun_out/h/legs.err || exit 1
python3 - <<'PY'
import json, glob, csv
t = open('gpurun_out/h/legs.json').read()
d = json.loads(t[t.index('{'):])
for k in ('xspace_bb', 'xspace_bb_panels', 'xspace_bb_tiles'):
    print(k, round(d[k]['us_per_round'], 1), 'us/round')
print('lbfgs_solve', round(d['lbfgs_solve']['ms_per_iteration'], 3), 'ms/iteration')
f = sorted(glob.glob('gpurun_out/h/xs/**/*kernel_stats.csv', recursive=True))
for r in csv.DictReader(open(f[0])):
    if any(s in r['Name'] for s in ('lsq', 'xbb', 'proj_lds', 'xlb')):
        print('%8.1f us %6s %s' % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:80]))
PY
