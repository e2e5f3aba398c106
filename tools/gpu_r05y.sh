#!/bin/bash
# round 5, step y: where the driver's short windows lose against 200-step ones
# -- the early iterations (warmup 5 vs 400) or each window's fixed host ends
# (launch from an idle stream, completion detection in synchronize)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/sync_probe.py > gpurun_out/r5y_sync.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/sync_probe.py --spin-flag > gpurun_out/r5y_sync_spin.log 2>&1 || exit 1
ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 120 python -u tools/sync_probe.py > gpurun_out/r5y_sync_awt.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --legs main --steps 20 --warmup 5 --profile-iters 0 > gpurun_out/r5y_w5.$rep.json 2> gpurun_out/r5y_w5.$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --legs main --steps 20 --warmup 400 --profile-iters 0 > gpurun_out/r5y_w400.$rep.json 2> gpurun_out/r5y_w400.$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --legs main --steps 200 --warmup 5 --profile-iters 0 > gpurun_out/r5y_s200.$rep.json 2> gpurun_out/r5y_s200.$rep.err || exit 1
done
