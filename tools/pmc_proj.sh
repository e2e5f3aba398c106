#!/bin/bash
# PMC passes over tools/proj_ubench.py (one rocprofv3 run per counter group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export PROJ_UB_VARIANTS=${PROJ_UB_VARIANTS:-0,3,12}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/ppmc$i -o pmc \
      -- python3 tools/proj_ubench.py > $OUT/ppmc$i.log 2>&1
  rc=$?; echo "ppmc$i rc=$rc" | tee -a $OUT/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
