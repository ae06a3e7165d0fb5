#!/usr/bin/env bash
# Round-4: where the split kernel's output layer goes (experiment builds, results invalid
# by construction): no output stores, no residual loads, no output epilogue; interleaved.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for rep in 1 2; do
  for v in base b3_noout b3_nores b3_noepi; do
    if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    echo "== $v"
    FV3NET_AMD_LIB=$lib B3_PRECS=bf16x3 timeout -k 10 120 python3 tools/b3_time.py dense emulator > $OUT/b3x_$v.txt 2>&1 || exit $?
    grep bf16x3 $OUT/b3x_$v.txt
  done
done | tee $OUT/b3_epi_ab_r04m.log
echo done
