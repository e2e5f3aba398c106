#!/bin/bash
# round 6, step f: the exact projection on the pipelined layout -- the exact
# projection tests (bit-identity vs the oracle), then the C2 leg A/B:
# BSLS_PROJ_EXACT_PIPE=1 (new default) / 0 (the lane-per-block sorting kernel)
# (the knob went with the kernel when it was reverted: commit 31d8bb5 holds both)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py -k "proj" > gpurun_out/r6f_proj_tests.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_shard_native.py -k uneven > gpurun_out/r6f_uneven.log 2>&1 || exit 1
for ep in 1 0 1 0; do
  BSLS_PROJ_EXACT_PIPE=$ep timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r6f_proj_ep$ep.json 2> gpurun_out/r6f_proj_ep$ep.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r6f_proj_ep$ep.json').read().strip().splitlines()[-1])
for k in ('proj_simplex', 'proj_simplex_fast'):
    v = d[k]; print('ep=$ep', k, round(v['avg_us'], 2), round(v['frac_hbm_peak'], 3), v['bit_exact_vs_oracle'], v['same_size_scale_floor_us'])
" >> gpurun_out/r6f_summary.txt
done
