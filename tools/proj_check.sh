#!/bin/bash
# Projection change check: bit-exact projection tests, C2 timing
# (tools/proj_time.py) and one PMC pass for LDS bank conflicts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_plugins.py -k "proj or simplex or ball" > gpurun_out/proj_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/proj_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/proj_time.py > gpurun_out/proj_time.log 2>&1
rc=$?; echo "time rc=$rc"; tail -8 gpurun_out/proj_time.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES \
    --output-format csv -d gpurun_out/proj_pmc -o pmc -- python3 tools/kprof.py --config C3 --iters 1 --proj 10 > gpurun_out/proj_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/proj_pmc > gpurun_out/proj_pmc_summary.txt 2>&1
grep -A7 proj_lds gpurun_out/proj_pmc_summary.txt
