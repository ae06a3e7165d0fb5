#!/usr/bin/env bash
# Round-4: kord > 7 register tail depth NT = 0 / 8 / 16 at load distance 4 with buffer
# operations (GPU tests of the kernel variants first), interleaved twice.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_mappm_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $OUT/gpu_tests_r04z2.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04z2.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 tools/mappm_pf_ab.py "4:1:0,4:1:8,4:1:16" > $OUT/mappm_nt_r04z2.log 2>&1 || exit $?
grep PF $OUT/mappm_nt_r04z2.log
echo done
