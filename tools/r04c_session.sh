#!/usr/bin/env bash
# Round-4: GPU tests of the touched files; kord-10 register-tail depth A/B; the split
# kernel's phase trace + pair-scheduling A/B; the bench's rank-share legs; host boundary.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_stepper.py tests/test_predictor.py tests/test_mappm_gpu.py \
    tests/test_mappm_multi_gpu.py tests/test_distributed.py tests/test_transfer.py -m gpu -q -x --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04c.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04c.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for nt in 0 16 32 48 0 32; do
  FV3_MAPPM_CS_NT=$nt timeout -k 10 120 python3 tools/mappm_nt_ab.py >> $OUT/mappm_nt_r04c.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/mappm_nt_r04c.log
for w in "emulator bf16x3" "dense bf16x3"; do
  FV3NET_AMD_LIB=tools/variants/libb3trace.so timeout -k 10 120 python3 tools/b3_trace.py $w >> $OUT/b3_trace_r04c.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/b3_trace_r04c.log
timeout -k 10 400 bash tools/b3_ab.sh base b3sched1 b3sched2 b3sched1fr6 base b3sched1 > $OUT/b3_sched_r04c.log 2>&1 || exit $?
cat $OUT/b3_sched_r04c.log
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share_r04c.json 2> $OUT/rank_share_r04c.err || exit $?
echo done
