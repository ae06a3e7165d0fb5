#!/usr/bin/env bash
# Profile the bench on the GPU box:  tools/profile.sh <tag> [bench args...]
#   1) rocprofv3 --kernel-trace --stats  (per-kernel durations)
#   2) separate --pmc passes for FETCH_SIZE and WRITE_SIZE (HBM traffic, per
#      MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of wide coalesced bytes on gfx950)
# Every GPU step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
shift || true
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=("$@")
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline "${ARGS[@]}" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extra "${ARGS[@]}" > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extra "${ARGS[@]}" > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
echo "headline profile done: $OUT"
# the legs (bench.py runs them in a child process, which the trace above does not follow):
# their kernels traced in a run of the child mode itself
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/legs" -o legs -- \
    python3 bench.py --legs-only /tmp/bench_legs_profile.jsonl > "$OUT/legs.out" 2> "$OUT/legs.err"
echo "legs profile done: $OUT/legs"
