#!/bin/bash
# round 6: wave_pass without the integer fold -- PAVA parity tests, the probe,
# the iso and main bench legs
OUT=gpurun_out/r06p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py \
  -k "isotonic or pava or k3 or iterates" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $OUT/status.txt; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "0 100 1 256" "0 100 1 256"; do timeout -k 10 60 tools/iso_ubench $a >> $OUT/probe.txt 2>&1 || exit 1; done
cat $OUT/probe.txt
timeout -k 10 300 python bench.py --legs iso > $OUT/iso.log 2>&1; rc=$?; echo "iso rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?; echo "bench rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import json
i=json.loads(open('gpurun_out/r06p/iso.log').read().strip().splitlines()[-1])['isotonic']
print('iso', i['avg_us'], i['frac_hbm_peak'], i['bit_exact_vs_oracle'])
b=json.loads(open('gpurun_out/r06p/bench.log').read().strip().splitlines()[-1])
print('bench', b['value'], b['ms_per_step'], b.get('roofline',{}).get('frac'))
PY
