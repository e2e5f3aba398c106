#!/bin/bash
# Round-3 A/B session: the lane-pair projection (BSLS_PROJ_LANES=2) and the
# fused ||r||^2 schedule on one GPU (BSLS_BB_FUSE_RR=1) -- parity tests under
# each variant, then timings.  Every GPU step has its own timeout; a crash /
# timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -eq 124 ] || [ "$1" -ge 128 ]; then echo "rc=$1: stop" | tee -a $OUT/ab.txt; exit "$1"; fi; }
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
BSLS_PROJ_LANES=2 timeout -k 10 300 $T tests/test_gpu_kernels.py -k "proj" > $OUT/ab_pair_tests.log 2>&1
rc=$?; echo "pair tests rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
BSLS_BB_FUSE_RR=1 timeout -k 10 600 $T tests/test_gpu_plugins.py tests/test_gpu_bb.py > $OUT/ab_fuse_tests.log 2>&1
rc=$?; echo "fuse tests rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
for v in "BSLS_PROJ_LANES=2" "BSLS_PROJ_LANES=1"; do
  env $v timeout -k 10 200 python bench.py --legs proj > $OUT/ab_proj_${v#*=}.log 2>&1
  rc=$?; echo "proj $v rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
done
for v in "BSLS_BB_FUSE_RR=1" "BSLS_BB_FUSE_RR=0"; do
  env $v timeout -k 10 300 python bench.py --legs c3 > $OUT/ab_c3_fuse${v#*=}.log 2>&1
  rc=$?; echo "c3 $v rc=$rc" | tee -a $OUT/ab.txt; fatal $rc
done
echo done | tee -a $OUT/ab.txt
