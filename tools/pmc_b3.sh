#!/bin/bash
# Instruction-mix PMC passes of one pmc_drive leg:  tools/pmc_b3.sh <leg> <tag>
set -u
export TMPDIR=/tmp
leg=$1; tag=$2
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_CVT SQ_BUSY_CYCLES" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmb_${tag}/p$i -o run -- python3 tools/pmc_drive.py $leg 3 > gpurun_out/pmb_${tag}_p$i.log 2>&1
  rc=$?; echo "$leg p$i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 tools/pmc_quick.py gpurun_out/pmb_${tag} dense_b3
