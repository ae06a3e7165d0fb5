#!/usr/bin/env bash
# Round-4 profile session: the split kernel's phase trace (variant build), the bench's
# kernel trace + the headline's FETCH/WRITE passes, the host-boundary measurements.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
for w in "emulator bf16x3" "dense bf16x3" "emulator bf16x6"; do
  FV3NET_AMD_LIB=tools/variants/libb3trace.so timeout -k 10 120 python3 tools/b3_trace.py $w >> $OUT/b3_trace_r04c.log 2>&1 || exit $?
done
cat $OUT/b3_trace_r04c.log
timeout -k 10 180 python3 tools/h2h_register.py > $OUT/h2h_register_r04c.json 2> $OUT/h2h_register_r04c.err || exit $?
bash tools/profile.sh r04c || exit $?
echo done
