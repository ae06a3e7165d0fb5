"""Marginal cost per hidden layer (steady-state MFMA efficiency) vs fixed per-tile overhead."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W
from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
dev = torch.device("cuda", 0)
for nc in ("1", "2"):
    os.environ["FV3_DENSE_NC"] = nc
    for res in (48, 384):
        ts = {}
        for depth in (2, 3, 4, 5):
            cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [79, 79], [79, 79], 256, depth)
            m = DenseColumnModel.random(cfg, seed=1)
            wl = W.make_dense_workload(res, seed=1, device=dev, model=m)
            for _ in range(3): wl.step()
            torch.cuda.synchronize()
            it = 30 if res < 384 else 5
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(it): wl.step()
            e1.record(); torch.cuda.synchronize()
            ts[depth] = e0.elapsed_time(e1) / it
            del wl
        ncol = W.c_columns(res)
        ideal_layer = ncol * 2 * 256 * 256 / 157.3e12 * 1e3  # ms
        d = np.diff([ts[k] for k in (2, 3, 4, 5)])
        print(f"NC={nc} C{res}: ms per depth {[round(ts[k],4) for k in (2,3,4,5)]}; marginal/layer {np.round(d,4)} ms; ideal {ideal_layer:.4f} ms -> eff {ideal_layer/np.mean(d):.2f}", flush=True)
