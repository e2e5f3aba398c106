#!/bin/bash
# round 6, step h: the BB suites after sy_dr's retirement (K1 finish, K2's
# dz . dg, K3's dz hand-off), with the parity log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BSLS_PARITY_LOG=$PWD/gpurun_out/r6h_parity.jsonl
: > $BSLS_PARITY_LOG
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_bb.py tests/test_gpu_fullsize.py tests/test_gpu_plugins.py tests/test_gpu_c5.py tests/test_gpu_batch.py tests/test_gpu_distributed.py > gpurun_out/r6h_tests.log 2>&1 || exit 1
