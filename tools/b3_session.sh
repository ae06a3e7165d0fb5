# bf16x3: the GPU tests, then interleaved timing of the default build against variants
set -uo pipefail
mkdir -p gpurun_out/b3
timeout -k 10 300 python3 -u -m pytest tests/test_emulator.py tests/test_dense_b3_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/b3/tests.log 2>&1; rc=$?
tail -2 gpurun_out/b3/tests.log; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 bash tools/b3_ab.sh base "$@" base "$@" 2>&1 | tee gpurun_out/b3/ab.txt
echo done
