"""Probe: can the VALU-bound two-field mappm co-reside with the MFMA-bound dense predict
on one MI355X?  C384 (884,736 columns).  Times, with events on each stream:
  dense alone at several persistent grids (FV3_DENSE_GRID), mappm pair alone, the two
  back to back, and the two on two streams at once on independent buffers (an upper
  bound for any overlap scheme).  Results are timings only (no parity claims)."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402


def wall(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    wl = W.make_predict_mappm_workload(384, device=dev)
    wl.step()  # bind + first run
    bound, plan = wl._bound, wl._plans
    # a second, independent remap (other buffers) for the concurrency probe
    pe1, pe2 = wl.pe1.clone(), wl.pe2.clone()
    srcs = [o.view(o.shape[0], -1).clone() for o in wl.outputs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    plan2 = MappmMultiPlan(pe1, srcs, pe2, 1, 1, stream=s2)
    res = {}
    for g in ("", "256", "384", "512", "768"):
        if g:
            os.environ["FV3_DENSE_GRID"] = g
        else:
            os.environ.pop("FV3_DENSE_GRID", None)
        res[f"dense_grid{g or 'default'}"] = wall(lambda: bound())
    os.environ.pop("FV3_DENSE_GRID", None)
    res["mappm_pair"] = wall(lambda: plan2())
    res["sequential"] = wall(lambda: (bound(), plan()))

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            bound(stream=s1)
        plan2()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    for g in ("", "256"):
        for prio in ("0", "2", "3"):
            os.environ["FV3_DENSE_PRIO"] = prio
            if g:
                os.environ["FV3_DENSE_GRID"] = g
            else:
                os.environ.pop("FV3_DENSE_GRID", None)
            tag = f"grid{g or 'default'}_prio{prio}"
            res[f"dense_{tag}"] = wall(lambda: bound())
            res[f"concurrent_{tag}"] = wall(both)
    os.environ.pop("FV3_DENSE_PRIO", None)
    os.environ.pop("FV3_DENSE_GRID", None)
    for k, v in res.items():
        print(f"{k:28s} {v:8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
