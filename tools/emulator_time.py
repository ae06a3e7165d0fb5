"""Emulator (config #5) at C384 on one GPU: mean launch time."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    wl = W.make_emulator_workload(int(sys.argv[1]) if len(sys.argv) > 1 else 384, seed=13)
    wl.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        wl.step()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e-3
    print(f"emulator C384: {t * 1e3:.3f} ms, {wl.ncol / t:.3e} col/s, "
          f"{wl.ncol * wl.flops_per_column / t / 1e12:.1f} TFLOP/s", flush=True)
