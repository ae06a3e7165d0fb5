#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 200 python3 tools/tr_debug.py > $OUT/tr_debug.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/tr_debug.log | tail -40; exit $rc
