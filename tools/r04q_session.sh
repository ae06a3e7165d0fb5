#!/usr/bin/env bash
# Round-4: kord > 7 mappm with rolling subgrid flags and the kord-10 column: GPU tests, then
# an interleaved A/B (product; FV3_MAPPM_CS_KORD=0; the previous commit's build).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_mappm_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $OUT/gpu_tests_r04q.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04q.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for v in base nokord head2; do
    lib=fv3net_amd/_lib/libfv3net_amd.so; k=1
    if [ $v = nokord ]; then k=0; fi
    if [ $v = head2 ]; then lib=tools/variants/libremap_head2.so; fi
    echo "== $v"
    FV3_MAPPM_CS_KORD=$k FV3NET_AMD_LIB=$lib timeout -k 10 200 python3 tools/mappm_pf_ab.py "2:1,4:1" 2>&1 | grep "PF" | head -4 || exit 1
  done
done | tee $OUT/mappm_kord_ab_r04q.log
echo done
