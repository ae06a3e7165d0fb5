#!/usr/bin/env bash
# Order-dependence check: every -m gpu test with the test files in reverse order (other
# kernels run before each test than in the usual order; LDS / allocator leftovers differ).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
FILES=$(ls tests/test_*.py | sort -r)
timeout -k 10 800 python3 -u -m pytest $FILES -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_reversed_r04z5.log 2>&1
rc=$?; tail -15 $OUT/gpu_tests_reversed_r04z5.log; exit $rc
