#!/bin/bash
# round 6, step x: the dealt walks' gathers as buffer loads with a cache-policy
# word (BSLS_TILE_GAUX = 0 plain, 1 sc0, 2 nt: lib/libbsls_hip_g<a>.so) against
# the shipped global loads -- parity tests on each variant, then C3 + C5 bench
# lines and the 8-way C5 rank-0 rehearsal, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06x; mkdir -p $OUT
L=$PWD/block-simplex-least-squares_amd/lib
for v in _g0 _g1 _g2; do
  BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_c5.py -x -q --timeout 250 --timeout-method thread > $OUT/tests$v.log 2>&1 || { echo "tests failed $v"; tail -30 $OUT/tests$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/tests$v.log)"
done
for rep in 1 2; do
  for v in "" _g0 _g1 _g2; do
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 200 python -u bench.py --legs main,c5 --steps 200 --warmup 20 > $OUT/main$v.$rep.json 2> $OUT/main$v.$rep.err || { echo "bench failed $v"; tail -5 $OUT/main$v.$rep.err; exit 1; }
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 200 python -u bench.py --rehearse-shard 8 --steps 100 --windows 5 > $OUT/reh$v.$rep.json 2> $OUT/reh$v.$rep.err || { echo "rehearsal failed $v"; tail -5 $OUT/reh$v.$rep.err; exit 1; }
    python -c "
import json
d = json.loads(open('$OUT/main$v.$rep.json').read().strip().splitlines()[-1])
r = json.loads(open('$OUT/reh$v.$rep.json').read().strip().splitlines()[-1])
k = lambda x, n='K2_spmvT_Nt_dots': x['kernels'][n]['avg_us']
print('lib%s rep $rep: C3 %.0f it/s (K2 %.2f K1 %.2f us)  C5 %.1f it/s (K2 %.1f K1 %.1f us)  C5/8 rank0 %.1f us/it (K2 %.1f K1 %.1f us)' % ('$v' or '(shipped)', d['value'], k(d), k(d, 'K1_spmv_A'), d['c5']['value'], k(d['c5']), k(d['c5'], 'K1_spmv_A'), r['ms_per_step'] * 1e3, k(r), k(r, 'K1_spmv_A')))
" | tee -a $OUT/summary.txt
  done
done
