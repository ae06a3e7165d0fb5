set -o pipefail
export FV3_VARIANTS=1  # A/B tool: the library reads kernel-variant selectors only with this set
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_b3_gpu.py tests/test_normalization_kat.py -m gpu > gpurun_out/b6_tests.log 2>&1 || exit 1
for w in 4 8; do
  FV3_B3_WAVES=$w B3_RES=48 B3_PRECS=bf16x3,bf16x6 timeout -k 10 120 python -u tools/b3_time.py dense > gpurun_out/b6_time_w$w.log 2>&1 || exit 1
done
for st in glds g2 reg; do
  FV3_B3_STAGE=$st B3_RES=384 B3_PRECS=bf16x6 timeout -k 10 120 python -u tools/b3_time.py dense > gpurun_out/b6_time_$st.log 2>&1 || exit 1
done
B3_PRECS=f32,bf16x6 timeout -k 10 200 python -u tools/b3_time.py pm emulator > gpurun_out/b6_time_pm.log 2>&1
timeout -k 10 120 python -u tools/overlap_probe3.py > gpurun_out/b6_overlap.log 2>&1
