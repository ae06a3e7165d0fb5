#!/usr/bin/env bash
# Round-4 first session: smoke, the -m gpu tests, the full bench line (with the rank-share
# legs).  Each step under its own limit; stop at a crash.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r04a.log 2>&1 || exit $?
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04a.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04a.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python3 bench.py > $OUT/bench_r04a.json 2> $OUT/bench_r04a.err || exit $?
echo bench done
timeout -k 10 180 python3 tools/h2h_register.py > $OUT/h2h_register_r04a.json 2> $OUT/h2h_register_r04a.err || exit $?
echo h2h done
