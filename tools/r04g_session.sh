#!/usr/bin/env bash
# Round-4: one lane per (column, field) for the multi-field remap on mid-size grids; the
# split kernel's block shape on one rank's C384 band; mappm GPU tests.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_mappm_multi_gpu.py tests/test_mappm_gpu.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04g.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04g.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for f in pair lanes pair lanes; do
  FV3_MAPPM_FIELDS=$f timeout -k 10 120 python3 tools/mappm_fields_ab.py 2>&1 | grep -v amdgpu.ids >> $OUT/mappm_fields_r04g.log || exit $?
done
cat $OUT/mappm_fields_r04g.log
for w in 8 4 8 4; do
  FV3_B3_WAVES=$w timeout -k 10 200 python3 tools/b3_rank_waves.py 2>&1 | grep -v amdgpu.ids >> $OUT/b3_rank_waves_r04g.log || exit $?
done
cat $OUT/b3_rank_waves_r04g.log
echo done
