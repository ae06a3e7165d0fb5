#!/bin/bash
# A/B of library builds on tools/dense_res_time.py (f32 dense kernel, C48..C384)
set -o pipefail
for v in "$@"; do
    echo "== $v"
    if [ "$v" = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    FV3NET_AMD_LIB=$lib timeout -k 10 120 python tools/dense_res_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
