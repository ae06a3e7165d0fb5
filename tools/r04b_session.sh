#!/usr/bin/env bash
# Round-4: stepper graphs, host-call path, kord>7 bounded scratch: the touched GPU tests,
# then timings (mappm kord 10 old grid vs new, rank-share legs, host call).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_stepper.py tests/test_predictor.py tests/test_mappm_gpu.py \
    tests/test_distributed.py tests/test_abi.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04b.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04b.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
FV3_MAPPM_CS_ROUNDS=1 timeout -k 10 120 python3 tools/mappm_time.py > $OUT/mappm_time_r04b_old.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/mappm_time.py > $OUT/mappm_time_r04b_new.log 2>&1 || exit $?
FV3_MAPPM_CS_ROUNDS=1 timeout -k 10 120 python3 tools/mappm_time.py > $OUT/mappm_time_r04b_old2.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/mappm_time.py > $OUT/mappm_time_r04b_new2.log 2>&1 || exit $?
head -2 $OUT/mappm_time_r04b_*.log
for b in 256 64 256 64; do FV3_MAPPM_BLOCK=$b timeout -k 10 120 python3 tools/mappm_block_ab.py >> $OUT/mappm_block_r04b.log 2>&1 || exit $?; done
cat $OUT/mappm_block_r04b.log
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share_r04b.json 2> $OUT/rank_share_r04b.err || exit $?
timeout -k 10 180 python3 tools/h2h_register.py > $OUT/h2h_register_r04b.json 2> $OUT/h2h_register_r04b.err || exit $?
echo done
