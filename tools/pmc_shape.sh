#!/bin/bash
# (FV3_B3_SHAPE=32 selected dense_b3w_kernel, built in commit d385025 and removed after this
# comparison: profiles/r05zd_b3_mfma32_pmc.txt; on later trees both passes run the default kernel)
# PMC passes of the emulator on both split-kernel shapes
set -u
export TMPDIR=/tmp FV3_VARIANTS=1
for shape in 16 32; do
  export FV3_B3_SHAPE=$shape
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pms_${shape}/p$i -o run -- python3 tools/b3_only.py emulator 3 > gpurun_out/pms_${shape}_p$i.log 2>&1
    rc=$?; echo "shape $shape p$i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
