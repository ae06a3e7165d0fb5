"""Kernel times of the config #4 stepper step's pieces (events around N back-to-back
launches): the fused epilogue on a float64 C96 state, and the whole step's wall clock."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.stepper import ml_epilogue  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    wl = W.make_stepper_workload(96, seed=11, device=dev)
    T, q = wl.state["air_temperature"], wl.state["specific_humidity"]
    dq1, dq2 = wl.model.forward([T.to(torch.float32), q.to(torch.float32)], level_axes=[1, 1])
    dp = wl.state["pressure_thickness_of_atmospheric_layer"]
    Tc, qc = T.clone(), q.clone()
    step = lambda: ml_epilogue(dq1, dq2, qc, dp, Tc, wl.dt, wl.state["total_precipitation"], in_place=True, level_axis=1)
    wall, t = bench.timed_steps(step, 50, 5, settle_ms=100)
    print(f"epilogue (wall per call incl. host) {wall / 50 * 1e6:.1f} us, events {t * 1e6:.1f} us")
    wall, t = bench.timed_steps(wl.step, 50, 5, settle_ms=100)
    print(f"stepper step wall {wall / 50 * 1e3:.4f} ms")
