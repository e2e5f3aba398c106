#!/bin/bash
# round 6: standalone PAVA A/B -- two packs per wave with shared passes
# (BSLS_K3_MERGE=1) against one pack per wave (=0) at the C3/C4 z layout
OUT=gpurun_out/r06m; mkdir -p $OUT
for mg in 0 1 0 1; do
  BSLS_K3_MERGE=$mg timeout -k 10 300 python bench.py --legs iso > $OUT/iso_merge$mg.log 2>&1
  rc=$?; echo "merge=$mg rc=$rc" | tee -a $OUT/status.txt
  [ $rc -ne 0 ] && exit $rc
  python3 -c "import json,sys; d=json.loads(open('$OUT/iso_merge$mg.log').read().strip().splitlines()[-1]); i=d['isotonic']; print('merge=$mg', i['avg_us'], i['frac_hbm_peak'], i['bit_exact_vs_oracle'])" | tee -a $OUT/status.txt
done
