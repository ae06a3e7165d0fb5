#!/usr/bin/env bash
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 300 python3 tools/h2h_pipe_ab.py > $OUT/h2h_pipe_r04s.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/h2h_pipe_r04s.log; exit $rc
