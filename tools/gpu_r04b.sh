#!/bin/bash
# fast projection A/B (lanes per block x min waves), then the r04a remainder
set -o pipefail
mkdir -p gpurun_out
for l in 4; do
  echo "LPB=$l MINW=8"; BSLS_PROJ_LPB=$l timeout -k 10 120 python -u tools/proj_fast_time.py || exit 1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py tests/test_gpu_lsq.py -x -q \
  -k "proj or native or rccl or lsq" --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1
rc=$?; tail -5 gpurun_out/t_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --legs main,proj --steps 200 --warmup 20 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || exit 1
python - <<'PY'
import json
d=json.load(open('gpurun_out/bench_b.json'))
print('headline', d['value'], d['unit'], d['ms_per_step'], d['roofline']['kernel'], round(d['roofline']['frac'],3))
print('kernels', {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='formats'})
print('c5', d.get('c5',{}).get('value'), d.get('c5',{}).get('ms_per_step'))
for k in ('proj_simplex','proj_simplex_exact'):
    p=d[k]; print(k, round(p['avg_us'],2), round(p['frac_hbm_peak'],3), p['max_rel_diff_vs_oracle'])
PY
timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 > gpurun_out/reh_native.json 2> gpurun_out/reh_native.err || exit 1
BSLS_SHARD_NATIVE=0 timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 > gpurun_out/reh_py.json 2> gpurun_out/reh_py.err || exit 1
python - <<'PY'
import json
for f in ('gpurun_out/reh_native.json','gpurun_out/reh_py.json'):
    d=json.load(open(f)); print(f, round(d['value'],1), round(d['ms_per_step']*1e3,1), {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='formats'})
PY
