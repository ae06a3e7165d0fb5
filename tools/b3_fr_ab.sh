#!/usr/bin/env bash
# A/B of the split kernel's fragment-ring depth (FV3_B3_FR builds in tools/variants/),
# interleaved twice: C48 (4-wave blocks) and C384 (8-wave blocks), bf16x3 and bf16x6.
set -uo pipefail
export FV3_VARIANTS=1  # A/B tool: the library reads kernel-variant selectors only with this set
for rep in 1 2; do
  for v in base b3fr6 b3fr8; do
    if [ "$v" = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    echo "== $v ($rep)"
    FV3NET_AMD_LIB=$lib B3_RES=48,384 B3_PRECS=bf16x3,bf16x6 timeout -k 10 120 python tools/b3_time.py dense 2>&1 \
        | grep -v amdgpu.ids || exit 1
  done
done
