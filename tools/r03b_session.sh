#!/usr/bin/env bash
# Round-3 measurement call: GPU tests, smoke, the default bench line, then the rocprof
# kernel trace and FETCH/WRITE passes (tools/profile.sh).  Each GPU step has its own limit;
# a crash, abort or time limit ends the call.
set -uo pipefail
TAG=${1:-r03b}
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/${TAG}_gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_gpu_tests.log"; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $?
cat "$OUT/${TAG}_smoke.log" | grep -v amdgpu.ids
timeout -k 10 600 python3 -u bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit $?
echo "bench rc=0"
bash tools/profile.sh "$TAG"
