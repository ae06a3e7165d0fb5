#!/usr/bin/env bash
# Round-4 closing session: smoke, every -m gpu test, the full bench line (rank-share legs
# included), then the headline's kernel trace + FETCH/WRITE passes (tools/profile.sh).
# Each step under its own limit; stop at a crash.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r04x.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 800 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04x.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04x.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 bench.py > $OUT/bench_r04x.json 2> $OUT/bench_r04x.err || exit $?
echo bench done
bash tools/profile.sh r04x || exit $?
echo done
