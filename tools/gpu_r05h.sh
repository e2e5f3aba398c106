#!/bin/bash
# round 5, step h: dz . dg as ||r - r_prev||^2 (bsls_bb_problem.sy_dr): the BB
# tests on it, then the C3 headline and C5 with it and without (BSLS_SY_DR=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_bb.py -k "sy_dr or k3_wave" \
  > gpurun_out/r5h_tests.log 2>&1 || exit 1
for sy in 1 0; do
  BSLS_SY_DR=$sy timeout -k 10 300 python -u bench.py --legs main,c5 > gpurun_out/r5h_bench_sy$sy.json 2> gpurun_out/r5h_bench_sy$sy.err || exit 1
done
