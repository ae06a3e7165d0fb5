"""Mean launch time of the dense kernels by precision: config #2 (2x256) at C48/C384 and
the config-#5 emulator at C384, f32 and bf16x3 (events around back-to-back launches,
after a clock-settle phase)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

F32_PEAK, BF16_PEAK = 157.3, 2516.6  # TFLOP/s dense (MI355X_MICROARCH.md)


def timed(step, n):
    t0 = time.time()
    while time.time() - t0 < 0.3:  # settle clocks
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def report(name, wl, t, prec):
    flop = wl.ncol * wl.flops_per_column / t / 1e12
    nm = {"bf16x3": 3, "bf16x6": 6}.get(prec)
    extra = f"{flop / F32_PEAK:.3f} of f32 MFMA peak" if prec == "f32" else \
        f"{nm * flop / BF16_PEAK:.3f} of bf16 MFMA peak ({nm} MFMAs/product)"
    print(f"{name:18s} {prec:6s}: {t * 1e6:9.1f} us  {wl.ncol / t:.3e} col/s  {flop:6.1f} f32-equiv TFLOP/s  {extra}",
          flush=True)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    which = sys.argv[1:] or ["dense", "emulator"]
    for prec in os.environ.get("B3_PRECS", "bf16x3,f32").split(","):
        if "dense" in which:
            for res, n in [(r, 200 if r < 384 else 10) for r in map(int, os.environ.get("B3_RES", "48,384").split(","))]:
                wl = W.make_dense_workload(res, seed=1, device=dev, precision=prec)
                report(f"dense C{res}", wl, timed(wl.step, n), prec)
        if "emulator" in which:
            wl = W.make_emulator_workload(384, seed=13, device=dev, precision=prec)
            report("emulator C384", wl, timed(wl.step, 10), prec)
        if "pm" in which:  # predict + two-field mappm on one C384 state
            wl = W.make_predict_mappm_workload(384, seed=21, device=dev, precision=prec)
            report("predict+mappm C384", wl, timed(wl.step, 10), prec)
