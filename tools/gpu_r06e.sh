#!/bin/bash
# round 6, step e: the whole GPU suite with the parity log (no -x: every
# measured error recorded), then smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BSLS_PARITY_LOG=$PWD/gpurun_out/r6e_parity.jsonl
: > $BSLS_PARITY_LOG
timeout -k 10 1100 python -u -m pytest -v -m gpu --timeout 900 --timeout-method thread tests > gpurun_out/r6e_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6e_smoke.log 2>&1 || exit 1
