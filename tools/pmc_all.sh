#!/usr/bin/env bash
# Per-kernel PMC passes over every bench leg:  tools/pmc_all.sh <tag> [legs...]
# Each (leg, counter set) is its own rocprofv3 --pmc run (no tracing domains), under its own
# time limit; a failed pass is recorded and the next one runs (a pass that exceeds the
# hardware's counter slots is killed by its timeout).  Summary: tools/pmc_collect.py.
set -uo pipefail
TAG=$1; shift
LEGS=("$@")
if [ ${#LEGS[@]} -eq 0 ]; then
  LEGS=(calib dense_c48 dense_c384 dense_c384_bf16x3 emulator_c384 emulator_c384_f32 mappm_c384_k1 mappm_c384_k10 mappm_c12
        coarsen_1f coarsen_4f stepper_c96 predict_mappm_c384 dense_c48_bf16x6 dense_c384_bf16x6 emulator_c384_bf16x6
        predict_mappm_c384_bf16x6 stepper_c96_r8 emulator_c384_r8 emulator_c384_f32_r8 predict_mappm_c384_r8
        predict_mappm_c384_bf16x6_r8 mappm_c384_k1_exact mappm_c384_k10_exact coarsen_1f_exact coarsen_4f_exact)
fi
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_${TAG}
# the calibration kernels of the "calib" leg (tools only; git-ignored build)
if [ ! -f tools/variants/libcalib.so ]; then
  mkdir -p tools/variants
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -o tools/variants/libcalib.so tools/calib.hip
fi
mkdir -p "$OUT"; export TMPDIR=/tmp
# the sources each profiled kernel was built from (bench.kernel_source_hash)
python3 -c "import json, bench; print(json.dumps({k: bench.kernel_source_hash(k) for k in
  ['dense_forward_kernel', 'dense_b3_kernel', 'mappm_ppm_kernel', 'mappm_cs_global_kernel', 'mappm_ppm_levels_kernel',
   'mappm_ppm_pair_kernel', 'mappm_ppm_pair_split_kernel', 'regrid_coarsen_cells_kernel', 'ml_epilogue_kernel',
   'ml_epilogue_levels_kernel']}))" > "$OUT/src_hashes.json"
SETS=("FETCH_SIZE"
      "WRITE_SIZE"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
      "VALUBusy VALUUtilization"
      "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU GRBM_GUI_ACTIVE")
for leg in "${LEGS[@]}"; do
  mkdir -p "$OUT/$leg"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/$leg/p$i" -o run -- \
        python3 tools/pmc_drive.py "$leg" 5 > "$OUT/$leg/p$i.log" 2>&1
    rc=$?
    echo "$leg pass $i rc=$rc" | tee -a "$OUT/status.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $leg pass $i rc=$rc"; exit $rc; fi
  done
done
python3 tools/pmc_collect.py "$OUT" > "$OUT/summary.json"
echo "pmc done: $OUT"
