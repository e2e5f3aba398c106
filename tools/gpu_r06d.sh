#!/bin/bash
# round 6, step d: the tightened parity bounds measured (BSLS_PARITY_LOG), the
# near-tie K3 repair test, the SciPy bound of the fixed-point residual, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BSLS_PARITY_LOG=$PWD/gpurun_out/r6d_parity.jsonl
: > $BSLS_PARITY_LOG
T="python -u -m pytest -v --timeout 900 --timeout-method thread"
timeout -k 10 1100 $T tests/test_gpu_deep.py tests/test_gpu_shard_native.py > gpurun_out/r6d_tests.log 2>&1
rc=$?
timeout -k 10 400 $T tests/test_gpu_bb.py tests/test_gpu_lsq.py -k "near_ties or warm_start or dense_row" > gpurun_out/r6d_tests2.log 2>&1
rc2=$?
echo "tests2 rc=$rc2"
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6d_smoke.log 2>&1 || exit 1
