#!/usr/bin/env bash
# One GPU call: the -m gpu tests, then the given follow-up commands (each under its own
# limit).  A test FAILURE (rc 1) still lets the follow-ups run; a crash, abort, fault or
# time limit (any other rc) ends the call there.
#   tools/gpu_session.sh <tag> [-- follow-up command ...]
set -uo pipefail
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/gpu_tests_${TAG}.log" 2>&1
rc=$?
tail -5 "$OUT/gpu_tests_${TAG}.log"
echo "gpu tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${1:-}" = "--" ]; then shift; bash -c "$*"; fi
