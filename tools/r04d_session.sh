#!/usr/bin/env bash
# Round-4: the split kernel with its LDS-DMA in inline asm (counted ds_read waits):
# output hashes vs the product library, the bf16 GPU tests on the variant, then A/B.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for v in base b3asm b3asm_s1 b3asm_fr6; do
  if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
  echo "== $v" >> $OUT/b3_bitcheck_r04d.log
  FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/b3_bitcheck.py >> $OUT/b3_bitcheck_r04d.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/b3_bitcheck_r04d.log
FV3NET_AMD_LIB=tools/variants/libb3asm.so timeout -k 10 500 python3 -u -m pytest tests/test_dense_b3_gpu.py \
    tests/test_emulator.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_b3asm_r04d.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_b3asm_r04d.log; echo "variant gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 bash tools/b3_ab.sh base b3asm b3asm_s1 b3asm_fr6 base b3asm > $OUT/b3_asm_ab_r04d.log 2>&1 || exit $?
cat $OUT/b3_asm_ab_r04d.log
FV3NET_AMD_LIB=tools/variants/libb3asm.so B3_PRECS=bf16x6 timeout -k 10 200 python3 tools/b3_time.py dense emulator \
    > $OUT/b3_asm_b6_r04d.log 2>&1 || exit $?
B3_PRECS=bf16x6 timeout -k 10 200 python3 tools/b3_time.py dense emulator >> $OUT/b3_asm_b6_r04d.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/b3_asm_b6_r04d.log
echo done
