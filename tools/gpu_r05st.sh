#!/bin/bash
# round 5: K2 / K1 relaunched on one state right after the prologue, under a
# kernel trace -- does their early slowness need a changing iterate?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for st in 3 7; do
  rm -rf gpurun_out/st_$st
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st_$st -o run \
    -- python3 tools/window_probe.py --stage $st > gpurun_out/st_$st.log 2>&1 || exit 1
done
