#!/bin/bash
# round 5, step t: the one-GPU loop with ||r||^2 / f / the stop test moved
# into K2 (BSLS_BB_FUSE1=1: stage 8 per iteration, K1 ends at r, stage 9
# after the call) -- the BB / deep / plugin suites on it, then C3 / C5 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BSLS_BB_FUSE1=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bb.py \
  tests/test_gpu_deep.py tests/test_gpu_plugins.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py > gpurun_out/r5t_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5t_tests.log
for rep in 1 2; do
  for f in 1 0; do
    BSLS_BB_FUSE1=$f timeout -k 10 300 python -u bench.py --legs main,c5 --steps 200 --windows 5 > gpurun_out/r5t_f$f.$rep.json 2> gpurun_out/r5t_f$f.$rep.err || exit 1
  done
done
