"""Mean launch time of the fused C384 -> C48 coarsen (f = 8, 79 levels) for 1 and 4
fields, as fine columns/s and algorithmic HBM GB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    for nf in (1, 4):
        wl = W.make_coarsen_workload(384, 8, nf, seed=7, device=torch.device("cuda", 0))
        for _ in range(3):
            wl.step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        n = 10
        for _ in range(n):
            wl.step()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / n * 1e-3
        gbs = wl.bytes_per_column * wl.ncol_fine / t / 1e9
        print(f"coarsen C384->C48 {nf} field(s): {t * 1e3:.3f} ms, {wl.ncol_fine / t:.3e} fine col/s, "
              f"{gbs:.0f} GB/s ({gbs / 8000:.3f} of HBM peak)", flush=True)
