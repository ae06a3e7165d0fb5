#!/usr/bin/env bash
# Round-4: kord > 7 mappm, next output edge loaded one call ahead: GPU tests, A/B against a
# build that loads it at the call (tools/variants/libmappm_noedge.so).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_mappm_gpu.py tests/test_mappm_multi_gpu.py tests/test_reduce_gpu.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04n.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04n.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in base mappm_noedge; do
    if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
    echo "== $v"
    FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/mappm_pf_ab.py "2:1,4:1" 2>&1 | grep -v amdgpu.ids | grep "rep\|PF" | head -4 || exit $?
  done
done | tee $OUT/mappm_edge_ab_r04n.log
echo done
