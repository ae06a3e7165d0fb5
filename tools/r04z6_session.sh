#!/usr/bin/env bash
# Host-page registration opt-in (FV3_HOST_REGISTER=1): every -m gpu test with the test
# files in reverse order, then in the usual order, smoke, and the bench line.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
FILES=$(ls tests/test_*.py | sort -r)
timeout -k 10 800 python3 -u -m pytest $FILES -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_reversed_r04z6.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_reversed_r04z6.log; echo "reversed rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 800 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04z6.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04z6.log; echo "usual order rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r04z6.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 600 python3 bench.py > $OUT/bench_r04z6.json 2> $OUT/bench_r04z6.err || exit $?
echo done
