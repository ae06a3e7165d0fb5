"""Config #4 step at C96: predict on the exact-f32 kernel (float64 state read in place)
against the bf16x6 split kernel (state cast into bound float32 buffers), wall clock per
step after a clock settle."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for prec in ("f32", "bf16x6", "f32", "bf16x6"):
        wl = W.make_stepper_workload(96, seed=11, device=dev, precision=prec)
        t0 = time.time()
        while time.time() - t0 < 0.5:
            wl.step()
        torch.cuda.synchronize()
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            wl.step()
        torch.cuda.synchronize()
        print(f"stepper C96 {prec:7s}: {(time.perf_counter() - t0) / n * 1e3:.4f} ms/step", flush=True)
