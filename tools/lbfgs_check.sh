#!/bin/bash
# LBFGS.solve history kernels (csrc/lbfgs.hip): their parity tests, then the
# gdlbfgs bench leg under a rocprofv3 kernel trace.  A failing step ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_plugins.py -k "lbfgs or multi_dot or LBFGS" > gpurun_out/lbfgs_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/lbfgs_tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_gdl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gdl -o run \
    -- python3 bench.py --legs gdlbfgs > gpurun_out/prof_gdl.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_gdl -name '*kernel_stats.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/r03_gdlbfgs_kernel_stats.csv
grep '^{' gpurun_out/prof_gdl.log | tail -1
