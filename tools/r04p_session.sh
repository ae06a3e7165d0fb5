#!/usr/bin/env bash
# Round-4: the split kernel's transposed output layer (16-byte epilogue accesses): GPU tests
# of the split kernel, the emulator and the residual layouts, then an interleaved A/B
# against the row-per-lane output layer (FV3_B3_TR=0).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_dense_b3_gpu.py tests/test_emulator.py tests/test_dense_gpu.py \
    tests/test_stepper.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_r04p.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_r04p.log; echo "gpu tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for tr in 1 0; do
    echo "== FV3_B3_TR=$tr"
    FV3_B3_TR=$tr B3_PRECS=bf16x3,bf16x6 timeout -k 10 150 python3 tools/b3_time.py dense emulator 2>&1 | grep "bf16" || exit 1
  done
done | tee $OUT/b3_tr_ab_r04p.log
echo done
