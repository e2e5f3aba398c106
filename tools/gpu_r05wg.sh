#!/bin/bash
# round 5: K1 at C3 with two 1024-thread tiles per CU (lib/libbsls_hip_wg2.so:
# make VAR=_wg2 DEFS=-DBSLS_K1T_WGS=2, registers capped) and 16 column groups
# of the same tile height (same entries per tile column, twice the waves)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/block-simplex-least-squares_amd/lib
run() {  # run <tag> <lib> <plan or ''>
  BSLS_LIB=$L/$2 BSLS_TILE_PLAN_A=$3 timeout -k 10 300 python -u bench.py --legs main --steps 200 --windows 5 \
    > gpurun_out/r5wg_$1.json 2> gpurun_out/r5wg_$1.err || exit 1
}
for rep in 1 2; do
  run def.$rep libbsls_hip.so ""
  run wg2def.$rep libbsls_hip_wg2.so ""
  run wg2g16.$rep libbsls_hip_wg2.so 3125,16
  run wg2g16o0.$rep libbsls_hip_wg2.so 3125,16,0
done
