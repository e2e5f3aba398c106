#!/bin/bash
# sliced sharded schedule + native driver + LBFGS device line search: tests, rehearsal, trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_plugins.py tests/test_gpu_lsq.py -x -q \
  -k "native or rccl or sharded or lbfgs or lsq" --timeout 300 --timeout-method thread > gpurun_out/t_c.log 2>&1
rc=$?; tail -4 gpurun_out/t_c.log; [ $rc -eq 0 ] || exit $rc
for mode in 2 1; do
  BSLS_SHARD_FUSE=$mode timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 400 --warmup 20 > gpurun_out/reh_f$mode.json 2> gpurun_out/reh_f$mode.err || exit 1
  python - $mode <<'PY'
import json, sys
t=open('gpurun_out/reh_f%s.json'%sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
print('fuse', sys.argv[1], round(d['value'],1), 'it/s', round(d['ms_per_step']*1e3,1), 'us/it', {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='formats'})
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_reh2 -o reh -- python3 bench.py --rehearse-shard 8 --steps 200 --warmup 20 --profile-iters 0 > gpurun_out/prof_reh2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --legs gdlbfgs --steps 50 > gpurun_out/gdlbfgs.json 2> gpurun_out/gdlbfgs.err || exit 1
python - <<'PY'
import json
t=open('gpurun_out/gdlbfgs.json').read(); d=json.loads(t[t.index('{'):])
print('lbfgs_solve', json.dumps(d.get('lbfgs_solve'))[:400])
PY
