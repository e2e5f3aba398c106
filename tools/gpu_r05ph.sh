#!/bin/bash
# round 5: per-dispatch trace of C3 iterations 1..205 (warmup 5, ten windows
# of 20) with and without ~100 ms of full-chip work before them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in cold preheat; do
  flag=""; [ $v = preheat ] && flag="--preheat"
  rm -rf gpurun_out/ph_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph_$v -o run \
    -- python3 tools/window_probe.py --steps 20 --warmup 5 --windows 10 $flag > gpurun_out/ph_$v.log 2>&1 || exit 1
done
