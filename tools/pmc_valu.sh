#!/bin/bash
# One rocprofv3 PMC pass per workload over tools/kprof.py: VALU occupancy of
# the BB kernels and the C2 projection (SQ_ACTIVE_INST_VALU against
# SQ_BUSY_CU_CYCLES, both quad-cycles summed per SE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-C3 C5}; do
    timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/valu_$cfg -o pmc -- python3 tools/kprof.py --config $cfg --iters 6 --proj 6 > gpurun_out/valu_$cfg.log 2>&1
    rc=$?; echo "valu $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 tools/pmc_summary.py gpurun_out/valu_$cfg > gpurun_out/valu_summary_$cfg.txt 2>&1
done
