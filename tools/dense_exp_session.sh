# f32 dense experiment builds (results invalid by construction): where the C48 / C384 time goes
set -uo pipefail
mkdir -p gpurun_out/dx
for rep in 1 2; do
for v in base d_noin d_nostage d_nostore d_nowload d_l1w d_nomfma; do
  if [ $v = base ]; then lib=fv3net_amd/_lib/libfv3net_amd.so; else lib=tools/variants/lib$v.so; fi
  echo "== $v"
  FV3NET_AMD_LIB=$lib timeout -k 10 120 python3 tools/dense_time.py 2>&1 | grep "C48\|C384" || exit 1
done
done 2>&1 | tee gpurun_out/dx/ab.txt
echo done
