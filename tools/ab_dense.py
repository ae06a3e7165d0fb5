"""A/B the dense kernel variants (FV3_DENSE_NC) in ONE process, interleaved rounds."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W
dev = torch.device("cuda", 0)
for res in (48, 96, 384):
    wl = W.make_dense_workload(res, seed=1, device=dev)
    res_t = {}
    for rnd in range(3):
        for nc in ("1", "2"):
            os.environ["FV3_DENSE_NC"] = nc
            for _ in range(3): wl.step()
            torch.cuda.synchronize()
            it = 50 if res < 384 else 10
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(it): wl.step()
            e1.record(); torch.cuda.synchronize()
            res_t.setdefault(nc, []).append(e0.elapsed_time(e1) / it)
    for nc, ts in res_t.items():
        ms = min(ts)
        print(f"C{res} NC={nc}: {ms*1e3:.1f} us/step  {wl.ncol/ms*1e3:.3e} col/s  {wl.ncol*wl.flops_per_column/ms/1e9:.1f} TFLOP/s  (rounds {['%.1f' % (t*1e3) for t in ts]})", flush=True)
    del wl
