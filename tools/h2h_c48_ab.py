"""C48 host-to-host predict (float64 numpy (6, 79, 48, 48) in, float32 out, outputs reused):
forward_host pipelined over the 6 tiles vs one call, interleaved.  ms per call."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    res = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    wl = W.make_dense_workload(res, seed=3, device=dev)
    T = wl.inputs[0].double().cpu().numpy()
    q = wl.inputs[1].double().cpu().numpy()
    out = [np.empty(T.shape, np.float32), np.empty(T.shape, np.float32)]
    m = wl.model
    res_ = {}
    for rep in range(3):
        for mode, thr in (("pipelined", 0), ("one call", 1 << 62)):
            m._PIPELINE_MIN_BYTES = thr
            for _ in range(3):
                m.forward_host([T, q], [1, 1], out=out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                m.forward_host([T, q], [1, 1], out=out)
            ms = (time.perf_counter() - t0) / 20 * 1e3
            res_.setdefault(mode, []).append(ms)
            print(f"C{res} {mode} {ms:.3f} ms", flush=True)
    print({k: (round(min(v), 3), round(float(np.median(v)), 3)) for k, v in res_.items()}, flush=True)
