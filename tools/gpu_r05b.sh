#!/bin/bash
# round 5, step b: the native sharded driver at world 2 with the fixed-point r
# (runs to the reference's exit), link parts (native + Python loops), the
# upfront-load projection A/B, and the 8-way C5 rank-0 rehearsal with link
# parts under a modelled exchange.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_shard_native.py > gpurun_out/r5b_shard_native.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_distributed.py > gpurun_out/r5b_distributed.log 2>&1 || exit 1
for g in 1 2 4; do
  BSLS_PROJ_PIPE=$g timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5b_proj_g$g.json 2> gpurun_out/r5b_proj_g$g.err || exit 1
done
for spec in "1 none" "2 none" "4 none" "1 11.25,10" "2 11.25,10" "4 11.25,10"; do
  set -- $spec
  M=""; [ "$2" != none ] && M="--model-exchange $2"
  timeout -k 10 400 python -u bench.py --rehearse-shard 8 --parts $1 $M --steps 100 --windows 5 > gpurun_out/r5b_reh_p$1_$2.json 2> gpurun_out/r5b_reh_p$1_$2.err || exit 1
done
timeout -k 10 600 $T tests/test_gpu_lsq.py tests/test_gpu_bb.py -k "fixed_point or fixed_iterations" > gpurun_out/r5b_lsq_bb.log 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_deep.py -k c3 > gpurun_out/r5b_deep_c3.log 2>&1 || exit 1
