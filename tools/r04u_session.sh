#!/usr/bin/env bash
# Round-4: the two-field remap with level L + 4's loads carried one iteration ahead (as the
# one-field mappm kernel) vs read at each layer's start (libpair_nocarry.so).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_mappm_multi_gpu.py tests/test_mappm_gpu.py tests/test_coarsen.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04u.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04u.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in base pair_nocarry; do
    lib=fv3net_amd/_lib/libfv3net_amd.so
    if [ $v != base ]; then lib=tools/variants/lib$v.so; fi
    FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/pair_ab.py 2>&1 | grep " ms" || exit 1
  done
done | tee $OUT/pair_ab_r04u.log
echo done
