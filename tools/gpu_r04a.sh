#!/bin/bash
# round-4 first GPU check: fast projection timing (LPB variants), projection +
# distributed GPU tests, the bench headline and the 8-way rehearsal (native driver)
set -o pipefail
mkdir -p gpurun_out
for l in 4 2 8; do
  echo "LPB=$l"
  BSLS_PROJ_LPB=$l timeout -k 10 180 python -u tools/proj_fast_time.py || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -x -q \
  -k "proj or native or rccl" --timeout 300 --timeout-method thread > gpurun_out/t_a.log 2>&1
rc=$?; tail -5 gpurun_out/t_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --legs main,proj --steps 200 --warmup 20 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || exit 1
tail -c 1500 gpurun_out/bench_a.json
timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 100 --warmup 10 > gpurun_out/reh_native.json 2> gpurun_out/reh_native.err || exit 1
BSLS_SHARD_NATIVE=0 timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 100 --warmup 10 > gpurun_out/reh_py.json 2> gpurun_out/reh_py.err || exit 1
python - <<'PY'
import json
for f in ('gpurun_out/reh_native.json','gpurun_out/reh_py.json'):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='formats'})
PY
