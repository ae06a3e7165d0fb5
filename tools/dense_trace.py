"""Per-block phase timeline of the fused dense kernel (fv3_dense_set_trace).

    python tools/dense_trace.py [--res 48] [--nc 1|2]

Prints, over all blocks of one launch: phase durations (staging, layer 1, hidden,
output), block start-time spread, blocks per CU and the kernel span, in us."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import _native, workloads as W  # noqa: E402


def run(res, nc, wpe=2, warm=20):
    os.environ["FV3_DENSE_NC"] = str(nc)
    os.environ["FV3_DENSE_WPE"] = str(wpe)
    dev = torch.device("cuda", 0)
    wl = W.make_dense_workload(res, seed=1, device=dev)
    nblk = (wl.ncol + 16 * nc - 1) // (16 * nc)
    buf = torch.zeros(nblk * 8, dtype=torch.int64, device=dev)
    lib = _native.load()
    for _ in range(warm):
        wl.step()
    _native.check(lib.fv3_dense_set_trace(wl.model.handle(), buf.data_ptr()))
    wl.step()
    torch.cuda.synchronize()
    _native.check(lib.fv3_dense_set_trace(wl.model.handle(), None))
    t = buf.view(nblk, 8).cpu().numpy()
    ts = t[:, [0, 5, 1, 2, 3, 4]].astype(np.float64) / 100.0  # 100 MHz -> us
    t0 = ts[:, 0].min()
    ts -= t0
    d = np.diff(ts, axis=1)
    names = ["prolog", "stage", "layer1", "hidden", "output"]
    print(f"C{res} NC={nc} WPE={wpe}: {nblk} blocks, span {ts[:, 5].max():.1f} us, "
          f"block total mean {(ts[:, 5] - ts[:, 0]).mean():.1f} us (min {(ts[:, 5] - ts[:, 0]).min():.1f}, "
          f"max {(ts[:, 5] - ts[:, 0]).max():.1f})")
    for i, n in enumerate(names):
        print(f"   {n:7s} mean {d[:, i].mean():6.2f}  p10 {np.percentile(d[:, i], 10):6.2f}  "
              f"p90 {np.percentile(d[:, i], 90):6.2f}  max {d[:, i].max():6.2f}")
    cyc = t[:, 6].astype(np.float64)
    dur = ts[:, 5] - ts[:, 1]  # tile start (5) -> end (4), us
    ok = dur > 0
    print(f"   shader clock over tiles: median {np.median(cyc[ok] / dur[ok]) / 1e3:.3f} GHz "
          f"(p10 {np.percentile(cyc[ok] / dur[ok], 10) / 1e3:.3f}, p90 {np.percentile(cyc[ok] / dur[ok], 90) / 1e3:.3f})")
    starts = np.sort(ts[:, 0])
    print("   start times pct 0/25/50/75/90/100:",
          " ".join(f"{np.percentile(starts, q):.1f}" for q in (0, 25, 50, 75, 90, 100)))
    cu = t[:, 7]
    _, counts = np.unique(cu, return_counts=True)
    print(f"   CUs used {len(counts)}, blocks per CU: " +
          " ".join(f"{k}:{(counts == k).sum()}" for k in sorted(set(counts))))
    # concurrency: how many blocks are in flight on the busiest CUs at mid-kernel
    mid = ts[:, 5].max() / 2
    live = (ts[:, 0] <= mid) & (ts[:, 5] >= mid)
    print(f"   blocks live at mid-kernel: {live.sum()}")
    # per-CU occupancy over time: max / mean blocks in flight, and refill gaps
    span = ts[:, 5].max()
    conc_max, conc_mean, gaps = [], [], []
    for c in np.unique(cu):
        sel = cu == c
        st, en = ts[sel, 0], ts[sel, 4]
        ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        level = np.cumsum(ev[:, 1])
        conc_max.append(level.max())
        dt = np.diff(ev[:, 0])
        conc_mean.append((level[:-1] * dt).sum() / max(span, 1e-9))
        ss = np.sort(st)
        ee = np.sort(en)
        # gap: for each start after the first k, time since the most recent end before it
        for t_s in ss[3:]:
            prev = ee[ee <= t_s]
            if len(prev):
                gaps.append(t_s - prev[-1])
    # co-resident pairs: phase ends of the earlier- and later-finishing block of a 2-block CU
    pairs = [np.where(cu == c)[0] for c in np.unique(cu) if (cu == c).sum() == 2]
    if pairs:
        a = np.array([sorted(pp, key=lambda i: ts[i, 5]) for pp in pairs])
        for k, lab in ((0, "first-done"), (1, "second-done")):
            sel = a[:, k]
            print(f"   pair {lab:11s}: phase ends (us) " + " ".join(
                f"{n}={ts[sel, i + 1].mean():5.1f}" for i, n in enumerate(names)))
        single = np.array([np.where(cu == c)[0][0] for c in np.unique(cu) if (cu == c).sum() == 1])
        if len(single):
            print(f"   single-block CU  : phase ends (us) " + " ".join(
                f"{n}={ts[single, i + 1].mean():5.1f}" for i, n in enumerate(names)))
    g = np.array(gaps) if gaps else np.zeros(1)
    print(f"   per-CU blocks in flight: max {np.max(conc_max):.0f}, time-mean {np.mean(conc_mean):.2f}; "
          f"refill gap p50 {np.percentile(g, 50):.2f} p90 {np.percentile(g, 90):.2f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, nargs="+", default=[48, 384])
    ap.add_argument("--nc", type=int, nargs="+", default=[2, 1])
    ap.add_argument("--wpe", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--warm", type=int, nargs="+", default=[20], help="launches before the traced one")
    a = ap.parse_args()
    for res in a.res:
        for nc in a.nc:
            for wpe in a.wpe:
                for warm in a.warm:
                    print(f"-- after {warm} launches")
                    run(res, nc, wpe, warm)


if __name__ == "__main__":
    main()
