#!/bin/bash
# A/B of the bf16x3 kernel's experiment builds (tools/build_variant.sh b3_<x> -DFV3_B3_EXP_<X>):
# each line is b3_time.py's figures under one library
set -o pipefail
export FV3_VARIANTS=1  # A/B tool: the library reads kernel-variant selectors only with this set
for v in "$@"; do
    echo "== $v"
    if [ "$v" = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    B3_PRECS=bf16x3 FV3NET_AMD_LIB=$lib timeout -k 10 120 python tools/b3_time.py dense emulator 2>&1 | grep bf16x3 || exit 1
done
