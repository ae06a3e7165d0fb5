#!/usr/bin/env bash
# Counter passes (each its own rocprofv3 run, --pmc only):  tools/counters_generic.sh <tag> <what> <n>
# SETS (env, optional): counter sets separated by ';' (default: the VALU/issue sets)
set -euo pipefail
TAG=$1; WHAT=$2; N=${3:-5}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/cnt_${TAG}
mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
DEFAULT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM;VALUBusy;ValuPipeIssueUtil;MemUnitBusy;VALUUtilization"
IFS=';' read -ra SETLIST <<< "${SETS:-$DEFAULT}"
for set in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 tools/valu_only.py $WHAT $N > "$OUT/p$i.log" 2>&1 || echo "pass $i ($set) failed"
done
python3 tools/summarize_counters.py "$OUT"
echo done
