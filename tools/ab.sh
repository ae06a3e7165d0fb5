#!/bin/bash
# A/B of library builds on a timing script: tools/ab.sh <script.py> base|<variant>...
set -o pipefail
script=$1; shift
for v in "$@"; do
    echo "== $v"
    if [ "$v" = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    FV3NET_AMD_LIB=$lib timeout -k 10 120 python "$script" 2>&1 | grep -v amdgpu.ids || exit 1
done
