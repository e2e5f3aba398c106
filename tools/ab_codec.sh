#!/bin/bash
# A/B of the narrow colv codec on C3 (BSLS_VAL_CODEC=f64 keeps the doubles) and
# the 8-way rehearsal; each GPU step under its own timeout, stop at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bb.py tests/test_gpu_kernels.py tests/test_gpu_distributed.py -m gpu -q \
    --timeout 300 --timeout-method thread > $OUT/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
for c in auto f64; do
  BSLS_VAL_CODEC=$c timeout -k 10 300 python bench.py --legs c3 > $OUT/ab_c3_$c.log 2>&1
  rc=$?; echo "c3 $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --rehearse-shard 8 --steps 200 --warmup 20 > $OUT/ab_reh8.log 2>&1
echo "reh rc=$?"
