#!/bin/bash
# round 6: iso_ubench sweep -- passes knocked out, packs per wave, grid
# fraction, and the four-pack workgroup merge (mode 3)
OUT=gpurun_out/r06n; mkdir -p $OUT
B=tools/iso_ubench
for a in ${ARGS:-"0 100 1 256|3 100 1 256|0 100 1 256|3 100 1 256|3 100 0.5 256"}; do :; done
IFS='|' read -ra LIST <<< "${ARGS:-0 100 1 256|3 100 1 256|0 100 1 256|3 100 1 256|3 100 0.5 256}"
for a in "${LIST[@]}"; do
  timeout -k 10 60 $B $a >> $OUT/sweep.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc at $a" >> $OUT/sweep.txt; cat $OUT/sweep.txt; exit $rc; }
done
cat $OUT/sweep.txt
