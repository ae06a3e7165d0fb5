#!/usr/bin/env bash
# Round-4: MFMA-shape microbenchmark (tools only) for DESIGN.md §7 item 3.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 120 python3 tools/mfma_shape_bench.py > $OUT/mfma_shape_r04v.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/mfma_shape_r04v.log; exit $rc
