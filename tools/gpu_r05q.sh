#!/bin/bash
# round 5, step q: where K2's time goes at C3 and C5 -- the product build,
# the walk knocked out (KO 3) and the epilogue knocked out (KO 4), kernel
# table times from bench.py --legs main,c5 (results wrong by construction)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=block-simplex-least-squares_amd/lib
for v in "" _ko3 _ko4; do
  BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 300 python -u bench.py --legs main,c5 --steps 50 --windows 3 \
    > gpurun_out/r5q$v.json 2> gpurun_out/r5q$v.err || exit 1
done
