"""Mean launch time of the fused dense kernel at C48 and C384 (events around N
back-to-back launches); env knobs (FV3_DENSE_*) are read by the library per launch."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402


def time_res(res, n):
    wl = W.make_dense_workload(res, seed=1, device=torch.device("cuda", 0))
    import time
    t0 = time.time()
    while time.time() - t0 < 0.3:  # settle clocks (bench.py does the same)
        wl.step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        wl.step()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / n * 1e-3
    tf = wl.ncol * wl.flops_per_column / t / 1e12
    return t * 1e6, tf


if __name__ == "__main__":
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("FV3_DENSE"))
    for res, n in ((48, 200), (384, 10)):
        us, tf = time_res(res, n)
        print(f"[{tag or 'default'}] C{res}: {us:9.1f} us/launch  {tf:6.1f} TFLOP/s  ({tf / 157.3:.3f} of peak)",
              flush=True)
