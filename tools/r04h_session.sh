#!/usr/bin/env bash
# Round-4: the stepper step as one native launch plan (csrc/plan.cpp): GPU tests, then the
# rank-share legs.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_stepper.py tests/test_distributed.py tests/test_mappm_multi_gpu.py \
    tests/test_abi.py tests/test_plan.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04h.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04h.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share_r04h.json 2> $OUT/rank_share_r04h.err || exit $?
python3 -c "
import json;d=json.load(open('$OUT/rank_share_r04h.json'))
for k,v in d.items(): print(k, {x:(round(y,4) if isinstance(y,float) else y) for x,y in v.items() if x!='note'})"
echo done
