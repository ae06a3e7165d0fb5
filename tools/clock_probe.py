"""Probe: the shader clock the dense kernel holds (in-kernel s_memtime / s_memrealtime
per tile, fv3_dense_set_trace) at C48 / C96 / C384, after back-to-back launches or
after an idle gap.  Timings only."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import _native, workloads as W  # noqa: E402


def traced_clock(wl, pre, gap_s):
    lib = _native.load()
    ntiles = (wl.ncol + 31) // 32
    buf = torch.zeros(ntiles * 8, dtype=torch.int64, device="cuda")
    for _ in range(pre):
        wl.step()
    torch.cuda.synchronize()
    if gap_s:
        time.sleep(gap_s)
    _native.check(lib.fv3_dense_set_trace(wl.model.handle(), buf.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    wl.step()
    e1.record()
    torch.cuda.synchronize()
    _native.check(lib.fv3_dense_set_trace(wl.model.handle(), None))
    t = buf.view(ntiles, 8).cpu().numpy().astype(np.float64)
    dur_us = (t[:, 4] - t[:, 5]) / 100.0
    ok = dur_us > 0.5
    ghz = t[ok, 6] / dur_us[ok] / 1e3
    return float(np.median(ghz)), e0.elapsed_time(e1) * 1e3


def bench_like():
    """bench.py's own timing (300 ms settle, 20 warmup, 200 timed launches), then one
    traced launch: the clock the headline runs at."""
    import bench

    wl = W.make_dense_workload(48, seed=1, device=torch.device("cuda", 0))
    wall, t = bench.timed_steps(wl.step, 200, 20, settle_ms=300.0)
    ghz, us = traced_clock(wl, 0, 0.0)
    print(f"bench-like C48: {t * 1e6:.2f} us/launch, then traced launch clock {ghz:.3f} GHz", flush=True)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "bench":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        bench_like()
        sys.exit(0)
    for res in (48, 96, 384):
        wl = W.make_dense_workload(res, seed=1, device=dev)
        wl.step()
        for pre, gap in ((300 if res < 384 else 20, 0.0), (3000 if res < 384 else 200, 0.0), (3, 0.05)):
            ghz, us = traced_clock(wl, pre, gap)
            print(f"C{res}: after {pre} launches, idle {gap * 1e3:.0f} ms: median tile clock {ghz:.3f} GHz, "
                  f"traced launch {us:.1f} us", flush=True)
        del wl
