# bf16x3: GPU tests of both staging pipelines, then interleaved timing (LDS-DMA default vs
# FV3_B3_STAGE=reg), all on one box
set -uo pipefail
mkdir -p gpurun_out/b3
timeout -k 10 300 python3 -u -m pytest tests/test_emulator.py tests/test_dense_b3_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/b3/tests.log 2>&1; rc=$?
tail -2 gpurun_out/b3/tests.log; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
FV3_B3_STAGE=reg timeout -k 10 300 python3 -u -m pytest tests/test_emulator.py tests/test_dense_b3_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/b3/tests_reg.log 2>&1; rc=$?
tail -2 gpurun_out/b3/tests_reg.log; echo "reg tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for v in glds reg; do
    echo "== $v"
    FV3_B3_STAGE=$v B3_PRECS=bf16x3 timeout -k 10 120 python3 tools/b3_time.py dense emulator 2>&1 | grep bf16x3 || exit 1
  done
done 2>&1 | tee gpurun_out/b3/ab.txt
echo done
