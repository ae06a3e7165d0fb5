#!/bin/bash
# A/B of the f32 dense kernel's experiment builds (tools/build_variant.sh d_<x> -DFV3_EXP_<X>)
set -o pipefail
for v in "$@"; do
    echo "== $v"
    if [ "$v" = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    FV3NET_AMD_LIB=$lib timeout -k 10 120 python tools/dense_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
