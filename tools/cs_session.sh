set -uo pipefail
mkdir -p gpurun_out/cs
timeout -k 10 300 python3 -u -m pytest tests/test_mappm_gpu.py tests/test_mappm_multi_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/cs/tests.log 2>&1; rc=$?
tail -3 gpurun_out/cs/tests.log; echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -u tools/cs_ab.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cs/ab.txt || exit 1
export TMPDIR=/tmp
for v in reg global; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cs/pmc_fetch_$v -o run -- python3 tools/cs_ab.py --only $v > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cs/pmc_write_$v -o run -- python3 tools/cs_ab.py --only $v > /dev/null 2>&1 || exit 1
done
echo done
