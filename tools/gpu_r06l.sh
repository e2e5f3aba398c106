#!/bin/bash
# round 6, step l: the walks' lookahead (BSLS_TILE_P entry steps ahead,
# BSLS_TILE_D gather steps ahead; shipped 4 / 1) -- C3 + C5 whole iterations
# and the 8-way C5 rank-0 rehearsal, alternating builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6l_summary.txt
for rep in 1 2; do
for V in "" _p6d1 _p4d2 _p8d2; do
  L=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$V.so
  BSLS_LIB=$L timeout -k 10 300 python -u bench.py --legs main,c5 --steps 200 --warmup 20 --windows 5 > gpurun_out/r6l_b$V.json 2> gpurun_out/r6l_b$V.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r6l_b$V.json').read().strip().splitlines()[-1])
k = d['kernels']; c = d['c5']['kernels']
print('lib=$V C3 it/s %.0f K2 %.2f K1 %.2f K3 %.2f | C5 it/s %.1f K2 %.2f' % (d['value'], k['K2_spmvT_Nt_dots']['avg_us'], k['K1_spmv_A']['avg_us'], k['K3_pava_clip_z2x']['avg_us'], d['c5']['value'], c['K2_spmvT_Nt_dots']['avg_us']))
" >> gpurun_out/r6l_summary.txt
  BSLS_LIB=$L timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 --windows 5 > gpurun_out/r6l_r8$V.json 2> gpurun_out/r6l_r8$V.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r6l_r8$V.json').read().strip().splitlines()[-1])
k = d['kernels']
print('lib=$V C5/8 rank0 us/it %.1f K2 %.2f K1 %.2f' % (d['ms_per_step'] * 1e3, k['K2_spmvT_Nt_dots']['avg_us'], k['K1_spmv_A']['avg_us']))
" >> gpurun_out/r6l_summary.txt
done
done
