#!/bin/bash
# round 6, step q: single-GPU iteration with K1's ||r||^2 / stop test folded
# into the next K2 (BSLS_BB_FUSE1, lib _fz) against the default: the BB parity
# tests on the variant, then C3 + C5 whole iterations alternating builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06q; mkdir -p $OUT
LV=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip_fz.so
BSLS_LIB=$LV timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py tests/test_gpu_deep.py > $OUT/tests_fz.log 2>&1
rc=$?; echo "tests_fz rc=$rc" | tee -a $OUT/status.txt; tail -3 $OUT/tests_fz.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/summary.txt
for rep in 1 2; do
for V in "" _fz; do
  L=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$V.so
  BSLS_LIB=$L timeout -k 10 300 python -u bench.py --legs main,c5 --steps 200 --warmup 20 --windows 5 > $OUT/b$V.json 2> $OUT/b$V.err || exit 1
  python -c "
import json; d = json.loads(open('$OUT/b$V.json').read().strip().splitlines()[-1])
k = d['kernels']; c = d['c5']['kernels']
print('lib=$V C3 it/s %.0f K2 %.2f K1 %.2f K3 %.2f | C5 it/s %.1f K2 %.2f K1 %.2f' % (d['value'], k['K2_spmvT_Nt_dots']['avg_us'], k['K1_spmv_A']['avg_us'], k['K3_pava_clip_z2x']['avg_us'], d['c5']['value'], c['K2_spmvT_Nt_dots']['avg_us'], c['K1_spmv_A']['avg_us']))
" >> $OUT/summary.txt
done
done
cat $OUT/summary.txt
