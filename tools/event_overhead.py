"""Wall time per dense step (C48) with and without per-launch HIP events, and with
the launch captured in a HIP graph — where do the microseconds between kernels go?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402


def wall(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device("cuda", 0)
    wl = W.make_dense_workload(48, seed=1, device=dev)
    n = 400
    for _ in range(50):
        wl.step()
    plain = wall(wl.step, n)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    it = iter(ev)

    def with_events():
        s, e = next(it)
        s.record()
        wl.step()
        e.record()

    evw = wall(with_events, n)
    kern = sum(s.elapsed_time(e) for s, e in ev) / n * 1e3

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        wl.step()
    e1.record()
    torch.cuda.synchronize()
    span = e0.elapsed_time(e1) / n * 1e3

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            wl.step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            wl.step()
    graph = wall(g.replay, n // 10) / 10
    print(f"plain wall {plain:.1f} us/step | with events {evw:.1f} us/step, event kernel {kern:.1f} us | "
          f"2-event span {span:.1f} us/step | graph(10 steps) {graph:.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
