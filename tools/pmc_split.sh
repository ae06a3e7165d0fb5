#!/bin/bash
# PMC passes of the pair remap, one lane per column against two: tools/pmc_split.sh <ncol>
set -u
export TMPDIR=/tmp
ncol=${1:-110592}
for split in 0 1; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmsp_${ncol}_${split}/p$i -o run -- python3 tools/mappm_split_pmc.py $split $ncol 3 > gpurun_out/pmsp_${ncol}_${split}_p$i.log 2>&1
    rc=$?; echo "split $split p$i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
