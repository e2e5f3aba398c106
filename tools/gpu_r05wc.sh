#!/bin/bash
# round 5: the link-part pipeline on the weak-scaled C3 shard (rank 0 of 8,
# native driver): parts 1 / 2 / 4, with and without the modelled exchange
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for p in 1 2 4; do
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --rehearse-workload C3 --parts $p --steps 200 --windows 5 \
    > gpurun_out/r5wc_p${p}_plain.json 2> gpurun_out/r5wc_p${p}_plain.err || exit 1
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --rehearse-workload C3 --parts $p --steps 200 --windows 5 \
    --model-exchange 11.25,10 > gpurun_out/r5wc_p${p}_model.json 2> gpurun_out/r5wc_p${p}_model.err || exit 1
done
