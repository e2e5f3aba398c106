#!/bin/bash
# K3 warm start + LBFGS line-search finish: the LBFGS trace (device vs host
# line search), the K3 / BB / plugin tests, then C3 and C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lbfgs_debug.py > gpurun_out/d_lbfgs_debug.log 2>&1
rc=$?; echo "lbfgs_debug rc=$rc"; grep -v "^ *search" gpurun_out/d_lbfgs_debug.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
    tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py > gpurun_out/d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/d_tests.log; [ $rc -eq 0 ] || exit 1
for wl in C3 C5; do
  timeout -k 10 300 python -u bench.py --legs main --workload $wl --steps 200 --warmup 20 \
      > gpurun_out/d_bench_$wl.json 2> gpurun_out/d_bench_$wl.err || exit 1
  python - $wl <<'PY'
import json, sys
t = open('gpurun_out/d_bench_%s.json' % sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
print(sys.argv[1], round(d['value'], 1), 'it/s', round(d['ms_per_step'] * 1e3, 1), 'us/it',
      {k: round(v['avg_us'], 1) for k, v in d['kernels'].items() if k != 'formats'}, flush=True)
PY
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
    > gpurun_out/d_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/d_kernels.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --legs proj --steps 200 --warmup 20 > gpurun_out/d_proj.json \
    2> gpurun_out/d_proj.err || exit 1
python - <<'PY'
import json
t = open('gpurun_out/d_proj.json').read()
d = json.loads(t[t.index('{'):])
for k in ('proj_simplex', 'proj_simplex_fast'):
    v = d[k]
    print(k, round(v['avg_us'], 2), 'us', round(v['frac_hbm_peak'], 3), 'isolated', round(v['isolated_median_us'], 2),
          'maxrel', v['max_rel_diff_vs_oracle'])
PY
