#!/bin/bash
# round 6, step g: the exact pipelined projection vs launch bounds (VGPR cap:
# 8 WGs/CU = 64 VGPRs with spills, 5, 2 = 95 VGPRs), C2 leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6g_summary.txt
for V in "" _mb5 _mb2; do
  L=block-simplex-least-squares_amd/lib/libbsls_hip$V.so
  BSLS_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r6g_proj$V.json 2> gpurun_out/r6g_proj$V.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r6g_proj$V.json').read().strip().splitlines()[-1])
for k in ('proj_simplex', 'proj_simplex_fast'):
    v = d[k]; print('lib=$V', k, round(v['avg_us'], 2), round(v['frac_hbm_peak'], 3), v['bit_exact_vs_oracle'])
" >> gpurun_out/r6g_summary.txt
done
