#!/usr/bin/env bash
# Round-4: kord > 7 mappm with two-set blocked loads and buffer operations: GPU tests, A/B.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_mappm_gpu.py tests/test_stepper.py tests/test_reduce_gpu.py tests/test_distributed.py -m gpu -q -x --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04l.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04l.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 tools/mappm_pf_ab.py > $OUT/mappm_pf_r04l.log 2>&1 || exit $?
cat $OUT/mappm_pf_r04l.log | grep -v amdgpu.ids
echo done
