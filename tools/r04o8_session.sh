#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 300 python3 -u -m pytest "tests/test_coarsen_edges.py::test_kernel_c384_to_c48_constant_winds_preserved" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/props_r04o8.log 2>&1
rc=$?; tail -8 $OUT/props_r04o8.log; exit $rc
