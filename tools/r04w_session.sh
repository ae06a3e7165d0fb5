#!/usr/bin/env bash
# Round-4: a second full bench line on another box (run-to-run spread of the extra legs).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 600 python3 bench.py > $OUT/bench_r04w.json 2> $OUT/bench_r04w.err || exit $?
python3 -c "
import json;d=json.loads(open('$OUT/bench_r04w.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print({k:round(v['ms_per_step'],4) for k,v in d['extra'].items() if 'ms_per_step' in v})"
echo done
