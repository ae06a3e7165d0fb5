#!/usr/bin/env bash
# Round-4: lazy bf16x6 packing and one-launch level sums: GPU tests, rank-share legs, and a
# kernel trace of the stepper rank share alone.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_stepper.py tests/test_distributed.py tests/test_plan.py \
    tests/test_dense_b3_gpu.py tests/test_emulator.py tests/test_reduce_gpu.py -m gpu -q -x --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04i.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04i.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share_r04i.json 2> $OUT/rank_share_r04i.err || exit $?
python3 -c "
import json;d=json.load(open('$OUT/rank_share_r04i.json'))
for k,v in d.items(): print(k, {x:(round(y,4) if isinstance(y,float) else y) for x,y in v.items() if x in ('ms_per_step','ms','predict_ms','ratio_to_full_over_world')})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stepper_trace_r04i -o run -- python3 $GRAFT_REPO_ROOT/tools/stepper_trace.py 300 || exit $?
echo done
