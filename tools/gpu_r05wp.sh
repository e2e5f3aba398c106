#!/bin/bash
# round 5: tools/window_probe.py -- host wall vs device time of short windows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
{ timeout -k 10 200 python -u tools/window_probe.py --steps 20 --warmup 400 &&
  timeout -k 10 200 python -u tools/window_probe.py --steps 20 --warmup 400 --hold &&
  timeout -k 10 200 python -u tools/window_probe.py --steps 200 --warmup 400 &&
  timeout -k 10 200 python -u tools/window_probe.py --steps 200 --warmup 400 --hold &&
  timeout -k 10 200 python -u tools/window_probe.py --steps 1 --warmup 400 --windows 50 &&
  timeout -k 10 200 python -u tools/window_probe.py --steps 1 --warmup 400 --windows 50 --hold; } > gpurun_out/r5wp2.log 2>&1
