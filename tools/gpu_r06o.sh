#!/bin/bash
# round 6: SQ counters of the iso_ubench variants (mode 0 product passes,
# 4 pair hand-over, 5 scan passes)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06o; mkdir -p $OUT
for m in "0 100" "4 1" "5 100"; do
  tag=$(echo $m | tr ' ' _)
  rm -rf $OUT/sq_$tag
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
     --output-format csv -d $OUT/sq_$tag -o pmc -- tools/iso_ubench $m 1 256 > $OUT/sq_$tag.log 2>&1
  rc=$?; echo "sq $tag rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
