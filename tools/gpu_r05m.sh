#!/bin/bash
# round 5, step m: the persistent double-buffered LDS-DMA projection
# (BSLS_PROJ_PIPE_LDS=3) -- parity of every fast-projection test first (under
# a short time limit: a persistent kernel), then against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BSLS_PROJ_PIPE_LDS=3 timeout -k 10 180 python -u -m pytest -x -q --timeout 60 --timeout-method thread \
  tests/test_gpu_kernels.py -k fast_proj > gpurun_out/r5m_tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5m_def.$rep.json 2> gpurun_out/r5m_def.$rep.err || exit 1
  BSLS_PROJ_PIPE_LDS=3 timeout -k 10 240 python -u bench.py --legs proj > gpurun_out/r5m_dma.$rep.json 2> gpurun_out/r5m_dma.$rep.err || exit 1
done
