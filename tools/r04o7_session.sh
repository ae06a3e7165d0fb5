#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 300 python3 -u -m pytest "tests/test_stepper.py::test_stepper_c96_columns_independent_of_position" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/props_r04o7.log 2>&1
rc=$?; tail -8 $OUT/props_r04o7.log; exit $rc
