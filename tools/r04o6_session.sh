#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest "tests/test_emulator.py::test_emulator_c384_columns_independent_of_position" "tests/test_mappm_conservation.py::test_c384_columns_independent_of_position" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/props_r04o6.log 2>&1
rc=$?; tail -12 $OUT/props_r04o6.log; exit $rc
