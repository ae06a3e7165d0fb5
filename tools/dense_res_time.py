"""Mean launch time of the f32 dense kernel (config #2 model) at several resolutions."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("FV3_DENSE"))
    for res, n in ((48, 200), (64, 100), (96, 50), (192, 20), (384, 10)):
        wl = W.make_dense_workload(res, seed=1, device=dev)
        wall, t = bench.timed_steps(wl.step, n, 5, settle_ms=150)
        tf = wl.ncol * wl.flops_per_column / t / 1e12
        print(f"[{tag or 'default'}] C{res}: {t * 1e6:9.1f} us  {tf / 157.3:.3f} of peak", flush=True)
