#!/usr/bin/env bash
# Round-4: two column tiles per wave (FV3_B3_CPW=2, one wave per SIMD) now that the
# ds_read waits are counted (FV3_B3_GLDS_ASM variant): output hashes, then timings.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for v in base b3asm; do
  if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
  for cpw in 1 2; do
    echo "== $v cpw=$cpw" >> $OUT/b3_bitcheck_r04e.log
    FV3_B3_CPW=$cpw FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/b3_bitcheck.py >> $OUT/b3_bitcheck_r04e.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/b3_bitcheck_r04e.log
for round in 1 2; do
  for v in base b3asm b3asm_s1; do
    if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    for cpw in 1 2; do
      echo "== $v cpw=$cpw" >> $OUT/b3_cpw_r04e.log
      FV3_B3_CPW=$cpw B3_PRECS=bf16x3,bf16x6 B3_RES=384 FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/b3_time.py dense emulator \
          2>&1 | grep -v amdgpu.ids >> $OUT/b3_cpw_r04e.log || exit $?
    done
  done
done
cat $OUT/b3_cpw_r04e.log
echo done
