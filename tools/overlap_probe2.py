"""Probe 2: when do the dense predict and an independent two-field mappm finish when
launched together on two streams (C384)?  Per-stream end events against one start
event; grid 256 (one 8-wave dense block per CU, room for mappm waves) and the default
grid.  Timings only."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    wl = W.make_predict_mappm_workload(384, device=dev)
    wl.step()
    bound = wl._bound
    srcs = [o.view(o.shape[0], -1).clone() for o in wl.outputs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    plan2 = MappmMultiPlan(wl.pe1.clone(), srcs, wl.pe2.clone(), 1, 1, stream=s2)
    for g in ("256", "", "128"):
        if g:
            os.environ["FV3_DENSE_GRID"] = g
        else:
            os.environ.pop("FV3_DENSE_GRID", None)
        res = []
        for it in range(8):
            cur = torch.cuda.current_stream()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e2 = torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(cur)
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            bound(stream=s1)
            e1.record(s1)
            plan2()
            e2.record(s2)
            torch.cuda.synchronize()
            if it >= 3:
                res.append((e0.elapsed_time(e1), e0.elapsed_time(e2)))
        d = sum(r[0] for r in res) / len(res)
        m = sum(r[1] for r in res) / len(res)
        print(f"grid {g or 'default':8s} dense ends {d:.3f} ms, mappm ends {m:.3f} ms", flush=True)
        # alone, same harness
        for name, fn, st in (("dense", lambda: bound(stream=s1), s1), ("mappm", plan2, s2)):
            ts = []
            for it in range(6):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(torch.cuda.current_stream())
                st.wait_stream(torch.cuda.current_stream())
                fn()
                e1.record(st)
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(e0.elapsed_time(e1))
            print(f"   {name} alone {sum(ts) / len(ts):.3f} ms", flush=True)
    os.environ.pop("FV3_DENSE_GRID", None)


if __name__ == "__main__":
    main()
