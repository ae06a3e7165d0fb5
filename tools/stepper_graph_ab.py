"""One rank's C96 stepper step at world 8 (stubbed exchange) and the full C96 step:
the launch plan replayed by one C-ABI call per step against the same plan captured once
in a HIP graph (torch.cuda.CUDAGraph) and replayed, interleaved; ms per step.  Also
checks the graph replays give the plan's bits."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import _device  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402


def graphed(wl):
    wl.step()  # bind
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        wl._plan(_device.stream_handle(s))  # warm on the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            wl._plan(_device.stream_handle(s))
    torch.cuda.current_stream().wait_stream(s)
    return g


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    for name, mk in (("rank_of_8", lambda: W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev,
                                                                              stub_exchange=True)),
                     ("full", lambda: W.make_stepper_workload(96, seed=11, device=dev))):
        a, b = mk(), mk()
        ga = graphed(a)
        b.step()
        # same bits: replay the graph and the plan from equal states
        for k in a.state:
            a.state[k].copy_(b.state[k])
        ga.replay()
        b._plan(_device.stream_handle())
        torch.cuda.synchronize()
        same = all(torch.equal(a.state[k].view(torch.int64), b.state[k].view(torch.int64)) for k in a.state)
        for rnd in range(3):
            _, tg = bench.timed_steps(ga.replay, 300, 20, settle_ms=150)
            _, tp = bench.timed_steps(lambda: b._plan(_device.stream_handle()), 300, 20, settle_ms=150)
            out.setdefault(name, []).append({"graph_ms": round(tg * 1e3, 4), "plan_ms": round(tp * 1e3, 4)})
        print(name, "bit_identical", same, out[name], flush=True)
