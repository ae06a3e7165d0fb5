#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest "tests/test_dense_gpu.py::test_c384_columns_independent_of_position" "tests/test_coarsen.py::test_kernel_c384_to_c48_constant_fields_preserved" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/props_r04o5.log 2>&1
rc=$?; tail -30 $OUT/props_r04o5.log; exit $rc
