#!/usr/bin/env bash
# Order-dependence check: every -m gpu test with the test files in a fixed shuffled order.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
FILES=$(python3 -c "import glob, random; f = sorted(glob.glob('tests/test_*.py')); random.Random(4).shuffle(f); print(' '.join(f))")
echo "$FILES" > $OUT/order_r04z7.txt
timeout -k 10 800 python3 -u -m pytest $FILES -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_shuffled_r04z7.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_shuffled_r04z7.log; exit $rc
