set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r03e_gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
FV3_DENSE_NC=4 timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_predictor.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_nc4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03e_nc4_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for nc in 2 4; do FV3_DENSE_NC=$nc timeout -k 10 120 python3 -u tools/dense_time.py 2>&1 | grep -v amdgpu.ids; done | tee gpurun_out/r03e_nc_ab.txt
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err; echo bench rc=$?
