#!/usr/bin/env bash
# Split-kernel block shapes on the box: the split-kernel GPU tests, then C384 timings of
# 8-wave blocks against 4-wave blocks with two column tiles per wave (FV3_B3_CPW=2).
set -uo pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_b3_gpu.py \
    tests/test_normalization_kat.py "tests/test_emulator.py::test_emulator_split_kernel_variants_agree" -m gpu \
    > gpurun_out/cpw_tests.log 2>&1 || exit $?
for cpw in 1 2; do
  FV3_B3_CPW=$cpw B3_RES=384 B3_PRECS=bf16x3,bf16x6 timeout -k 10 200 python -u tools/b3_time.py dense emulator \
      > gpurun_out/cpw_time_$cpw.log 2>&1 || exit $?
done
