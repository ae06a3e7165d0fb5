"""Why the pipelined C384 host call does not overlap its two copy directions (DESIGN.md
§3.7): forward_host's loop (in-copies on the compute stream, out-copies on a side stream)
in variants that each change one thing, interleaved over rounds on one box.

Per variant: wall ms of the whole call, and host ms spent inside the in-copy calls (the
runtime's pageable H2D blocks the host until its staging is done), inside the out-copy
issue and in the final wait.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import _native, transfer  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = W.make_dense_workload(384, seed=3, device=dev)
    T4 = wl.inputs[0].double().cpu().numpy()
    q4 = wl.inputs[1].double().cpu().numpy()
    outs = [transfer.empty_host(T4.shape, np.float32) for _ in range(2)]
    wl.model.forward_host([T4, q4], [1, 1], out=outs)
    _, hb, hruns, hstreams = wl.model._host_call
    hs_out = hstreams[1]
    fresh_out = torch.cuda.Stream(device=dev)
    s_in = torch.cuda.Stream(device=dev)
    dev_out = [torch.empty(T4.shape, dtype=torch.float32, device=dev) for _ in range(2)]
    lib = _native.load()

    def loop(compute="real", out_stream=None, extra_kernel=False, idle_wait=False, pre_wait=True,
             in_stream=None, out_event="cur", sync_each=False):
        cur = torch.cuda.current_stream()
        so = out_stream or hs_out
        si = in_stream or cur
        t_in = t_out = 0.0
        if pre_wait:
            so.wait_stream(cur)
        for t in range(6):
            h0 = time.perf_counter()
            for a, b in zip((T4, q4), hb):
                transfer.host_copy(b[t], a[t], si.cuda_stream)
            t_in += time.perf_counter() - h0
            if si is not cur:
                e = torch.cuda.Event()
                e.record(si)
                cur.wait_event(e)
            if idle_wait:
                e = torch.cuda.Event()
                e.record(s_in)
                cur.wait_event(e)
            if compute == "real":
                o = hruns[t](cur)
            elif compute == "standin":
                for x in dev_out:
                    x[t].copy_(hb[0][t])
                o = [x[t] for x in dev_out]
            else:
                o = [x[t] for x in dev_out]
            if extra_kernel:
                dev_out[0][t, 0, 0, :1].add_(0)
            ev = torch.cuda.Event()
            ev.record(cur)
            so.wait_event(ev)
            h0 = time.perf_counter()
            for h_, oo in zip(outs, o):
                transfer.host_copy(h_[t], oo, so.cuda_stream)
            t_out += time.perf_counter() - h0
            if sync_each:
                so.synchronize()
        h0 = time.perf_counter()
        cur.wait_stream(so)
        cur.synchronize()
        return t_in, t_out, time.perf_counter() - h0

    variants = {
        "product_call": None,
        "real": dict(),
        "real_extra_kernel": dict(extra_kernel=True),
        "real_idle_wait": dict(idle_wait=True),
        "real_fresh_out_stream": dict(out_stream=fresh_out),
        "real_no_pre_wait": dict(pre_wait=False),
        "standin": dict(compute="standin"),
        "none": dict(compute="none"),
        "none_extra_kernel": dict(compute="none", extra_kernel=True),
        "real_in_side_stream": dict(in_stream=s_in),
        "real_sync_each": dict(sync_each=True),
    }
    res = {k: [] for k in variants}
    for rnd in range(3):
        names = list(variants) if rnd % 2 == 0 else list(reversed(list(variants)))
        for name in names:
            kw = variants[name]
            for rep in range(4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if kw is None:
                    wl.model.forward_host([T4, q4], [1, 1], out=outs)
                    parts = (0.0, 0.0, 0.0)
                else:
                    parts = loop(**kw)
                torch.cuda.synchronize()
                wall = time.perf_counter() - t0
                if rep:
                    res[name].append([wall * 1e3] + [p * 1e3 for p in parts])
        print(f"round {rnd} done", flush=True)
    summary = {}
    for k, v in res.items():
        a = np.median(np.array(v), axis=0)
        summary[k] = {"wall_ms": round(float(a[0]), 3), "in_calls_ms": round(float(a[1]), 3),
                      "out_issue_ms": round(float(a[2]), 3), "final_wait_ms": round(float(a[3]), 3),
                      "spread_ms": round(float(np.max(np.array(v)[:, 0]) - np.min(np.array(v)[:, 0])), 3)}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
