#!/bin/bash
# round 6, step w: the walks and bb_k1_sum branch on the stop flag only before their
# first global write (BSLS_LATE_STOP=1, lib/libbsls_hip_ls.so) against the shipped
# kernel: K2 / BB parity tests on the variant, then C3 + C5 bench lines and the
# 8-way C5 rank-0 rehearsal, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06w; mkdir -p $OUT
L=$PWD/block-simplex-least-squares_amd/lib
BSLS_LIB=$L/libbsls_hip_ls.so timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bb.py tests/test_gpu_c5.py tests/test_gpu_plugins.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_ls.log 2>&1 || { echo "pre tests failed"; tail -30 $OUT/tests_ls.log; exit 1; }
tail -2 $OUT/tests_ls.log
for rep in 1 2; do
  for v in "" _ls; do
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 200 python -u bench.py --legs main,c5 --steps 200 --warmup 20 > $OUT/main$v.$rep.json 2> $OUT/main$v.$rep.err || { echo "bench failed $v"; tail -5 $OUT/main$v.$rep.err; exit 1; }
    BSLS_LIB=$L/libbsls_hip$v.so timeout -k 10 200 python -u bench.py --rehearse-shard 8 --steps 100 --windows 5 > $OUT/reh$v.$rep.json 2> $OUT/reh$v.$rep.err || { echo "rehearsal failed $v"; tail -5 $OUT/reh$v.$rep.err; exit 1; }
    python -c "
import json
d = json.loads(open('$OUT/main$v.$rep.json').read().strip().splitlines()[-1])
r = json.loads(open('$OUT/reh$v.$rep.json').read().strip().splitlines()[-1])
k = lambda x: x['kernels']['K2_spmvT_Nt_dots']['avg_us']
print('lib%s rep $rep: C3 %.0f it/s (K2 %.2f us)  C5 %.1f it/s (K2 %.1f us)  C5/8 rank0 %.1f us/it (K2 %.1f us)' % ('$v' or '(shipped)', d['value'], k(d), d['c5']['value'], k(d['c5']), r['ms_per_step'] * 1e3, k(r)))
" | tee -a $OUT/summary.txt
  done
done
