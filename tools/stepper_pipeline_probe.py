"""Probe: one rank's share of the C96 stepper (world 8, stubbed exchange) with the step's
reductions (row partials + limiter counts, stub copy + fold) on a second stream,
overlapping the next step's predict, against the serial launch plan.  Python-issued
(torch streams + events): the host must stay ahead of the GPU for the wall clock to mean
anything, so the host time per step is printed too.  ``python tools/stepper_pipeline_probe.py [n]``."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402


def pipelined(wl, side):
    """step() with the reductions on ``side``: predict(n) overlaps reductions(n-1);
    epilogue(n) waits for them (they read the diagnostics it overwrites)."""
    main = torch.cuda.current_stream()
    h_main, h_side = main.cuda_stream, side.cuda_stream
    e_epi = torch.cuda.Event()
    e_red = torch.cuda.Event()
    first = [True]

    def step():
        wl.bound(h_main)
        if not first[0]:
            main.wait_event(e_red)
        first[0] = False
        wl._epi(h_main)
        e_epi.record(main)
        side.wait_event(e_epi)
        wl._diag(h_side)
        wl._fold(h_side)
        e_red.record(side)

    def finish():
        main.wait_event(e_red)

    return step, finish


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    side = torch.cuda.Stream(dev)
    for rnd in range(2):
        ref = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
        ref.step()  # binds
        wall, _ = bench.timed_steps(ref.step, n, 20, settle_ms=150)
        print(f"round {rnd} plan (serial): {wall / n * 1e3:.4f} ms/step", flush=True)
        pipe = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
        pipe.step()
        step, finish = pipelined(pipe, side)
        wall, _ = bench.timed_steps(step, n, 20, settle_ms=150)
        finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            step()
        host = (time.perf_counter() - t0) / 50
        finish()
        torch.cuda.synchronize()
        print(f"round {rnd} pipelined: {wall / n * 1e3:.4f} ms/step (host issue {host * 1e3:.4f} ms/step)", flush=True)
        # the same number of steps on both from the same state: identical bits
        a = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
        b = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
        for _ in range(5):
            ra = a.step()
        b.step()
        step, finish = pipelined(b, side)
        for _ in range(4):
            step()
        finish()
        torch.cuda.synchronize()
        same = torch.equal(ra.view(torch.int64), b._res.view(torch.int64)) and all(
            torch.equal(a.state[k].view(torch.int64), b.state[k].view(torch.int64)) for k in a.state)
        print(f"round {rnd} bit-identical after 5 steps: {same}", flush=True)
        del ref, pipe, a, b
