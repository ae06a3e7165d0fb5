"""The C384 host-to-host predict (float64 numpy T/q in, float32 numpy out, outputs reused):
DenseColumnModel.forward_host pipelined over the 6 tile blocks vs one call (the pipeline
threshold raised), interleaved.  ms per call."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    wl = W.make_dense_workload(384, seed=3, device=dev)
    T = wl.inputs[0].double().cpu().numpy()
    q = wl.inputs[1].double().cpu().numpy()
    out = [np.empty(T.shape, np.float32), np.empty(T.shape, np.float32)]
    m = wl.model
    res = {}
    for rep in range(4):
        for mode, thr in (("pipelined", 64 << 20), ("one call", 1 << 62)):
            m._PIPELINE_MIN_BYTES = thr
            m.forward_host([T, q], [1, 1], out=out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                m.forward_host([T, q], [1, 1], out=out)
            ms = (time.perf_counter() - t0) / 5 * 1e3
            res.setdefault(mode, []).append(ms)
            print(f"{mode} {ms:.2f} ms", flush=True)
    print({k: (round(min(v), 2), round(float(np.median(v)), 2)) for k, v in res.items()}, flush=True)
