#!/usr/bin/env bash
# Round-4: level-parallel stepper epilogue and the kord > 7 mappm loads run ahead: GPU
# tests, then A/Bs of both (same box, interleaved).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_stepper.py tests/test_mappm_gpu.py tests/test_plan.py \
    tests/test_distributed.py tests/test_mappm_multi_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $OUT/gpu_tests_r04j.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04j.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/epi_ab.py > $OUT/epi_ab_r04j.log 2>&1 || exit $?
cat $OUT/epi_ab_r04j.log | grep -v amdgpu.ids
timeout -k 10 300 python3 tools/mappm_pf_ab.py > $OUT/mappm_pf_r04j.log 2>&1 || exit $?
cat $OUT/mappm_pf_r04j.log | grep -v amdgpu.ids
echo done
