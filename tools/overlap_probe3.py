"""Probe 3: the bf16 split predict (bf16x6 by default) and an independent two-field mappm
launched together on two streams (C384), for both block shapes of the split kernel
(FV3_B3_WAVES=8: 8-wave blocks, 2 dense waves per SIMD and ~220 VGPRs each, no room for
remap waves; 4: one dense wave per SIMD, ~310 of the 512 registers, room for two 92-VGPR
remap waves).  Per-stream end events against one start event.  Timings only."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402


def span(fns, n=8, skip=3):
    out = []
    for it in range(n):
        cur = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        ends = [torch.cuda.Event(enable_timing=True) for _ in fns]
        torch.cuda.synchronize()
        e0.record(cur)
        for (fn, st), e in zip(fns, ends):
            st.wait_stream(cur)
            fn()
            e.record(st)
        torch.cuda.synchronize()
        if it >= skip:
            out.append([e0.elapsed_time(e) for e in ends])
    return [sum(r[i] for r in out) / len(out) for i in range(len(fns))]


def main():
    dev = torch.device("cuda", 0)
    prec = os.environ.get("PROBE_PREC", "bf16x6")
    wl = W.make_predict_mappm_workload(384, device=dev, precision=prec)
    wl.step()
    bound = wl._bound
    srcs = [o.view(o.shape[0], -1).clone() for o in wl.outputs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    plan2 = MappmMultiPlan(wl.pe1.clone(), srcs, wl.pe2.clone(), 1, 1, stream=s2)
    for _ in range(200):  # clock settle
        wl.step()
    for waves in ("8", "4"):
        os.environ["FV3_B3_WAVES"] = waves
        d, m = span([(lambda: bound(stream=s1), s1), (plan2, s2)])
        da, = span([(lambda: bound(stream=s1), s1)])
        ma, = span([(plan2, s2)])
        print(f"{prec} waves {waves}: together dense ends {d:.3f} ms, mappm ends {m:.3f} ms; "
              f"alone dense {da:.3f} ms, mappm {ma:.3f} ms (sum {da + ma:.3f})", flush=True)
    os.environ.pop("FV3_B3_WAVES", None)


if __name__ == "__main__":
    main()
