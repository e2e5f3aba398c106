#!/bin/bash
# round 6, step c: bank_ubench round-robin lane assignment (perm 4) vs the
# shipped column order, timing and SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tools/bank_ubench
O=gpurun_out/r6c_bank.log
: > $O
for rep in 1 2; do
for R in 3125 3907; do
  for pk in "0 16 16" "4 16 16" "3 16 16" "1 16 16"; do
    set -- $pk
    timeout -k 5 60 $B 125000 62464 256 1 $1 $R $2 $3 >> $O || exit 1
  done
done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_LDS --kernel-trace --stats -d $R/gpurun_out/r6c_pmc_rr -o pmc -- $R/$B 125000 62464 256 1 4 3125 16 16 >> $R/$O 2>&1 || exit 1
