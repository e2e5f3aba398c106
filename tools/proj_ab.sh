#!/bin/bash
# C2 projection A/B over BSLS_PROJ_WAVES (1 = one wave per workgroup, the
# default; 2 / 3 = staggered waves): projection tests under each setting, then
# tools/proj_waves.py per setting.  A failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WAVES:-2 3}; do
  BSLS_PROJ_WAVES=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_kernels.py -k "proj or simplex or ball" > gpurun_out/proj_tests_w$w.log 2>&1
  rc=$?; echo "tests w=$w rc=$rc"; tail -2 gpurun_out/proj_tests_w$w.log; [ $rc -eq 0 ] || exit $rc
done
for w in 1 ${WAVES:-2 3} 1; do
  BSLS_PROJ_WAVES=$w timeout -k 10 200 python -u tools/proj_waves.py >> gpurun_out/proj_waves.log 2>&1
  rc=$?; echo "time w=$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/proj_waves.log
