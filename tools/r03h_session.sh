#!/usr/bin/env bash
# Round-3 closing session: smoke, the full bench line, the -m gpu tests, then the
# split-kernel block-shape timings.  Each step under its own limit; stop at a crash.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r03h.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $OUT/bench_r03h.json 2> $OUT/bench_r03h.err || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r03h.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r03h.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cpw in 1 2; do
  FV3_B3_CPW=$cpw B3_RES=384 B3_PRECS=bf16x3,bf16x6 timeout -k 10 200 python -u tools/b3_time.py dense emulator \
      > $OUT/cpw_time_$cpw.log 2>&1 || exit $?
done
