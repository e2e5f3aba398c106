#!/bin/bash
# round 5, step r: the one-GPU fused loop against the sharded schedule on the
# same C3 problem (stages 10 / 15 / 14: atomic K1 in fixed point, r's
# initialisation in K3, no bb_k1_sum), twice each on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --legs main --steps 200 --windows 5 > gpurun_out/r5r_single.$rep.json 2> gpurun_out/r5r_single.$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --rehearse-workload C3 --steps 200 --windows 5 > gpurun_out/r5r_shard.$rep.json 2> gpurun_out/r5r_shard.$rep.err || exit 1
done
