#!/bin/bash
# round 6, step r: link parts with full-width K1 parts -- the 8-way C5 rank-0
# rehearsal at parts 1 / 2, with and without the modelled exchange, K1's tile
# plan default (H 15625 x 4 groups: a part is 128 workgroups) against 8 groups
# (a part is 256 workgroups, each half the columns; the fixed-point atomic K1
# is order-free, so the groups do not change the bits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06r; mkdir -p $OUT
: > $OUT/summary.txt
for spec in ${SPECS:-"1 none def|2 none def|2 none g8|1 11.25,10 def|2 11.25,10 def|2 11.25,10 g8|4 11.25,10 g16|4 none g16"}; do :; done
IFS='|' read -ra LIST <<< "${SPECS:-1 none def|2 none def|2 none g8|1 11.25,10 def|2 11.25,10 def|2 11.25,10 g8|4 11.25,10 g16|4 none g16}"
for spec in "${LIST[@]}"; do
  set -- $spec
  M=""; [ "$2" != none ] && M="--model-exchange $2"
  E=""; [ "$3" = g8 ] && E="15625,8"; [ "$3" = g16 ] && E="15625,16"; [ "$3" = h2 ] && E="7813,4"; [ "$3" = h4 ] && E="3907,4"
  BSLS_TILE_PLAN_A=$E timeout -k 10 400 python -u bench.py --rehearse-shard 8 --parts $1 $M --steps 100 --windows 5 > $OUT/reh_p$1_$2_$3.json 2> $OUT/reh_p$1_$2_$3.err || { echo "fail $spec" >> $OUT/summary.txt; cat $OUT/summary.txt; exit 1; }
  python -c "
import json; d = json.loads(open('$OUT/reh_p$1_$2_$3.json').read().strip().splitlines()[-1])
k = d.get('kernels', {})
print('parts $1 model $2 plan $3: %.1f us/it  K1 %s K2 %s' % (d['ms_per_step'] * 1e3, k.get('K1_spmv_A', {}).get('avg_us'), k.get('K2_spmvT_Nt_dots', {}).get('avg_us')))
" >> $OUT/summary.txt
done
cat $OUT/summary.txt
