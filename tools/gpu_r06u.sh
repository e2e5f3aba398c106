#!/bin/bash
# round 6, step u: the sort-free C2 projection's range in/out by 16-B accesses
# (BSLS_PIPE_W16=1, lib/libbsls_hip_w16.so) against the shipped 8-B form:
# the projection tests on the variant, then bench.py's proj leg alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06u; mkdir -p $OUT
L=$PWD/block-simplex-least-squares_amd/lib
BSLS_LIB=$L/libbsls_hip_w16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "proj" --timeout 200 --timeout-method thread > $OUT/tests_w16.log 2>&1 || { echo "w16 tests failed"; tail -30 $OUT/tests_w16.log; exit 1; }
tail -2 $OUT/tests_w16.log
for rep in 1 2 3; do
  for v in "" _w16; do
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 120 python -u bench.py --legs proj > $OUT/proj$v.$rep.json 2> $OUT/proj$v.$rep.err || { echo "bench failed $v"; tail -5 $OUT/proj$v.$rep.err; exit 1; }
    python -c "
import json; d = json.loads(open('$OUT/proj$v.$rep.json').read().strip().splitlines()[-1])
for k in ('proj_simplex', 'proj_simplex_fast'):
    e = d[k]; print('lib%s rep $rep %s %.2f us frac %.3f floor %.2f bitexact %s rel %.1e' % ('$v' or '(shipped)', k, e['avg_us'], e['frac_hbm_peak'], e['same_size_scale_floor_us'], e['bit_exact_vs_oracle'], e['max_rel_diff_vs_oracle']))
" | tee -a $OUT/summary.txt
  done
done
