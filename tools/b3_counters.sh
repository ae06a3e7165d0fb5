#!/usr/bin/env bash
# --pmc passes over the bf16x3 kernel only: tools/b3_counters.sh <tag> <dense|emulator>
set -euo pipefail
TAG=$1; WHAT=$2
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/cnt_${TAG}
mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 tools/b3_only.py $WHAT 5 > "$OUT/p$i.log" 2>&1 || echo "pass $i ($set) failed"
done
python3 tools/summarize_counters.py "$OUT"
