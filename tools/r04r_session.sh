#!/usr/bin/env bash
# Round-4: the pipelined host call (DenseColumnModel.forward_host): GPU tests, then the
# host-to-host bench legs (C48, C384, the rank call, predict + mappm).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_predictor.py tests/test_transfer.py -m gpu -q -x --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04r.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04r.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "
import json, torch, bench
dev = torch.device('cuda', 0)
for r in range(2):
    print('c48', json.dumps(bench.host_to_host(dev, 48)['ms_per_step']), flush=True)
    print('c384', json.dumps(bench.host_to_host(dev, 384)['ms_per_step']), flush=True)
" > $OUT/h2h_r04r.log 2>&1 || exit $?
cat $OUT/h2h_r04r.log | grep -v amdgpu.ids
for k in 1 0; do
  FV3_D2H_KERNEL=$k timeout -k 10 300 python3 tools/h2h_pipe_ab.py > $OUT/h2h_pipe_r04r_k$k.log 2>&1 || exit $?
  echo "FV3_D2H_KERNEL=$k"; grep -v amdgpu.ids $OUT/h2h_pipe_r04r_k$k.log | tail -1
done
echo done
