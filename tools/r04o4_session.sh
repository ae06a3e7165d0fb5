#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_mappm_conservation.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/conservation_r04o4.log 2>&1
rc=$?; tail -15 $OUT/conservation_r04o4.log; exit $rc
