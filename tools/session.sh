#!/usr/bin/env bash
# One GPU call as a list of steps, each under its own time limit, output under gpurun_out/:
#   tools/session.sh <tag> 'name|seconds|command' ['name|seconds|command' ...]
# A step's stdout+stderr go to gpurun_out/<tag>_<name>.log.  The call stops at the first
# step that fails; a step named with a trailing '?' (a test run) may fail with rc 1 (test
# failures) and the call goes on, any other rc (a crash, abort, fault, time limit) ends it.
set -uo pipefail
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
for step in "$@"; do
    name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    soft=0
    if [ "${name: -1}" = "?" ]; then soft=1; name=${name%?}; fi
    log="$OUT/${TAG}_${name}.log"
    echo "== $name ($secs s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
    rc=$?
    echo "== $name rc=$rc in $(( $(date +%s) - start )) s"; tail -4 "$log"
    if [ $rc -ne 0 ]; then
        if [ $soft -eq 1 ] && [ $rc -eq 1 ]; then continue; fi
        exit $rc
    fi
done
echo "session $TAG done"
