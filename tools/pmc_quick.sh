#!/bin/bash
# tools-style quick PMC passes: /tmp/pmcq.sh <leg> <tag>
set -u
export TMPDIR=/tmp
leg=$1; tag=$2
i=0
for set in "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmq_${tag}/p$i -o run -- python3 tools/pmc_drive.py $leg 5 > gpurun_out/pmq_${tag}_p$i.log 2>&1
  rc=$?; echo "$leg p$i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 tools/pmc_quick.py gpurun_out/pmq_${tag} regrid
