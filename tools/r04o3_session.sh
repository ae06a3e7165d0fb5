#!/usr/bin/env bash
# one rank's share of the C96 stepper: dense tile shape A/B (32-col 8-wave default,
# 16-col 4-wave, 32-col 4-wave), interleaved
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
L=$OUT/stepper_nc_r04o3.log; : > $L
for rep in 1 2 3; do
  for cfg in "default" "FV3_DENSE_NC=1" "FV3_DENSE_NW=4"; do
    if [ "$cfg" = default ]; then e=""; else e="$cfg"; fi
    echo -n "$cfg: " >> $L
    env $e timeout -k 10 120 python3 tools/stepper_trace.py 2000 2>&1 | grep -v amdgpu.ids >> $L || exit $?
  done
done
cat $L
