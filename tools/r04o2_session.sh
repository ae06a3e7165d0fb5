#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for r in 48 96; do
  timeout -k 10 200 python3 tools/h2h_c48_ab.py $r > $OUT/h2h_c${r}_r04o2.log 2>&1 || exit $?
  grep -v amdgpu.ids $OUT/h2h_c${r}_r04o2.log | tail -1
done
echo done
