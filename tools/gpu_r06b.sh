#!/bin/bash
# round 6, step b: bank_ubench -- the dealt walk's ds_add_f64 bank conflicts
# vs the lane order inside an instruction (timing, then the SQ counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=tools/bank_ubench
O=gpurun_out/r6b_bank.log
: > $O
for R in 3125 3907; do
  for a in "0 0" "0 1" "1 0" "1 1"; do
    timeout -k 5 60 $B 125000 62464 256 $a $R >> $O || exit 1
  done
  for kg in "16 16" "32 32" "16 32" "32 16" "8 16"; do
    timeout -k 5 60 $B 125000 62464 256 1 2 $R $kg >> $O || exit 1
    timeout -k 5 60 $B 125000 62464 256 1 3 $R $kg >> $O || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "1 0 3125 16 16" "1 1 3125 16 16" "1 2 3125 16 16" "1 2 3125 32 32" "1 3 3125 16 16" "1 3 3125 32 32" "1 3 3125 16 32"; do
  set -- $cfg
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_LDS --kernel-trace --stats -d $R/gpurun_out/r6b_pmc_$1$2_$4_$5 -o pmc -- $R/$B 125000 62464 256 $1 $2 $3 $4 $5 >> $R/$O 2>&1 || exit 1
done
