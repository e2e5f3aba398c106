#!/bin/bash
# round 5, step a: the pipelined sort-free projection (tests, then an A/B of
# groups per wave: BSLS_PROJ_PIPE 4 / 2 / 8 / 1, 0 = round 4's lane-per-block
# Michelot), then the native sharded driver at world 2 (CallbackComm) and the
# Python loop on stages 15 / 14.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_kernels.py -k "fast_proj" > gpurun_out/r5a_fastproj.log 2>&1 || exit 1
for g in 4 2 8 1 0; do
  BSLS_PROJ_PIPE=$g timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5a_proj_g$g.json 2> gpurun_out/r5a_proj_g$g.err || exit 1
done
timeout -k 10 1000 $T tests/test_gpu_shard_native.py tests/test_gpu_distributed.py > gpurun_out/r5a_shard.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_lsq.py tests/test_gpu_bb.py -k "fixed_point or fixed_iterations" > gpurun_out/r5a_lsq_bb.log 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_deep.py -k c3 > gpurun_out/r5a_deep_c3.log 2>&1 || exit 1
