#!/bin/bash
# PMC passes of the coarsen kernel with 0 fields (pass 1 only) and 1 field
set -u
export TMPDIR=/tmp
for nf in 0 1; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmco_${nf}/p$i -o run -- python3 tools/coarsen_only.py $nf 3 > gpurun_out/pmco_${nf}_p$i.log 2>&1
    rc=$?; echo "nf $nf p$i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
