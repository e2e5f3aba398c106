#!/bin/bash
# round 5, step w: rank 0 of the 8-way splits (C3 weak shard, C5 strong
# shard) through the native driver with and without a modelled exchange
# (11.25 us per MB + 10 us per all-reduce: SURVEY 8(e)'s single-link ring)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wl in C3 C5; do
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --rehearse-workload $wl --steps 200 --windows 5 \
    > gpurun_out/r5w_${wl}_plain.json 2> gpurun_out/r5w_${wl}_plain.err || exit 1
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --rehearse-workload $wl --steps 200 --windows 5 \
    --model-exchange 11.25,10 > gpurun_out/r5w_${wl}_model.json 2> gpurun_out/r5w_${wl}_model.err || exit 1
done
