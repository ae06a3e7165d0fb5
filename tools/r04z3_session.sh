#!/usr/bin/env bash
# Round-4 closing verification (after the full-size property tests): smoke, every -m gpu
# test, the full bench line, then the predict + mappm host-to-host leg twice.
# Each step under its own limit; stop at a crash.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r04z3.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 800 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_r04z3.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04z3.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 bench.py > $OUT/bench_r04z3.json 2> $OUT/bench_r04z3.err || exit $?
echo bench done
timeout -k 10 300 python3 -c "
import json, torch, bench
dev = torch.device('cuda', 0)
for r in range(2):
    d = bench.predict_mappm_host_to_host(dev)
    print('predict_mappm_h2h', round(d['ms_per_step'], 2), d['bit_identical_to_device_resident'], flush=True)
" > $OUT/pm_h2h_r04z3.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/pm_h2h_r04z3.log

echo done
