#!/usr/bin/env bash
# Round-4: the streaming remap's loads at each layer's start and the next output edge one
# call ahead (kord <= 7, two-field pair, coarsen): GPU tests, then an interleaved A/B of the
# product build against HEAD~ sources (tools/variants/libremap_head.so) and the same
# sources without the edge prefetch (libremap_noedge.so).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_mappm_gpu.py tests/test_mappm_multi_gpu.py tests/test_coarsen.py tests/test_coarsen_edges.py \
    tests/test_restarts.py tests/test_interpolate*.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04o.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04o.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in base remap_head remap_noedge; do
    if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/remap_ab.py 2>&1 | grep " ms" || exit 1
  done
done | tee $OUT/remap_ab_r04o.log
echo done
