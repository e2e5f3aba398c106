#!/bin/bash
# plugin-surface GPU tests, then a rocprofv3 kernel trace of the C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_plugins.py > gpurun_out/plugins.log 2>&1
rc=$?; echo "plugins rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run \
    -- python3 bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1
echo "prof rc=$?"
