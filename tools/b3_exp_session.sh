# bf16x3 experiment builds (results invalid by construction): where the time goes
set -uo pipefail
mkdir -p gpurun_out/b3x
for v in b3_nobar b3_nofrag b3_nomfma; do
  echo "== $v"
  FV3NET_AMD_LIB=tools/variants/lib$v.so B3_PRECS=bf16x3 timeout -k 10 120 python3 tools/b3_time.py dense emulator > gpurun_out/b3x/$v.txt 2>&1
  echo "rc=$?"; grep bf16x3 gpurun_out/b3x/$v.txt; tail -3 gpurun_out/b3x/$v.txt | grep -v bf16x3
done
echo "== base"; B3_PRECS=bf16x3 timeout -k 10 120 python3 tools/b3_time.py dense emulator 2>&1 | grep bf16x3
echo done
