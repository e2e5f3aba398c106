#!/bin/bash
# round 5, step z: K3's warm start with repair (pava_warm_repair, the default
# build) -- the warm / K3 / BB tests, then the driver's bench arguments and
# 200-step windows against the build without it (lib/libbsls_hip_norep.so:
# make VAR=_norep DEFS=-DBSLS_K3_REPAIR=0), C3 and C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_shard_native.py -m gpu \
  > gpurun_out/r5z_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in "" _norep; do
    BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$v.so timeout -k 10 300 \
      python -u bench.py --legs main --steps 20 --warmup 5 --profile-iters 0 \
      > gpurun_out/r5z_w5$v.$rep.json 2> gpurun_out/r5z_w5$v.$rep.err || exit 1
    BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$v.so timeout -k 10 300 \
      python -u bench.py --legs main --steps 200 --warmup 20 --windows 5 --profile-iters 0 \
      > gpurun_out/r5z_s200$v.$rep.json 2> gpurun_out/r5z_s200$v.$rep.err || exit 1
  done
done
for v in "" _norep; do
  BSLS_LIB=$PWD/block-simplex-least-squares_amd/lib/libbsls_hip$v.so timeout -k 10 300 \
    python -u bench.py --legs main --workload C5 --steps 20 --warmup 5 --windows 5 --profile-iters 0 \
    > gpurun_out/r5z_c5$v.json 2> gpurun_out/r5z_c5$v.err || exit 1
done
