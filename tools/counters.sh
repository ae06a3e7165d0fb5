#!/usr/bin/env bash
# SQ/TCC counter passes on the dense-only driver:  tools/counters.sh <tag> <res>
set -euo pipefail
TAG=${1:-c1}; RES=${2:-384}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/cnt_${TAG}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 tools/dense_only.py $RES 20 > "$OUT/t.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 tools/dense_only.py $RES 5 > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d "$OUT/p2" -o run -- python3 tools/dense_only.py $RES 5 > "$OUT/p2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/p3" -o run -- python3 tools/dense_only.py $RES 5 > "$OUT/p3.log" 2>&1
echo done
