#!/bin/bash
# round 6, step j: K2's epilogue batch (K2E 8 shipped / 4) at C3 and C5:
# stage timing and whole iterations, alternating builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6j_summary.txt
for rep in 1 2; do
for V in "" _k2e4; do
  L=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$V.so
  BSLS_LIB=$L timeout -k 10 300 python -u bench.py --legs main,c5 --steps 200 --warmup 20 --windows 5 > gpurun_out/r6j_b$V.json 2> gpurun_out/r6j_b$V.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r6j_b$V.json').read().strip().splitlines()[-1])
k = d['kernels']; c = d['c5']['kernels']
print('lib=$V C3 it/s %.0f K2 %.2f K1 %.2f K3 %.2f | C5 it/s %.1f K2 %.2f' % (d['value'], k['K2_spmvT_Nt_dots']['avg_us'], k['K1_spmv_A']['avg_us'], k['K3_pava_clip_z2x']['avg_us'], d['c5']['value'], c['K2_spmvT_Nt_dots']['avg_us']))
" >> gpurun_out/r6j_summary.txt
done
done
