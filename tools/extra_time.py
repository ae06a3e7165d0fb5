"""Time the stepper (config #4, C96) and the f32 emulator legs of bench.py's extras."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    wl = W.make_stepper_workload(96, seed=11, device=dev)
    wall, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
    print(f"stepper_c96 {wall / 20 * 1e3:.4f} ms/step")
    wl = W.make_emulator_workload(384, seed=13, device=dev, precision="f32")
    wall, t = bench.timed_steps(wl.step, 10, 3, settle_ms=150)
    print(f"emulator_c384_f32 {t * 1e3:.4f} ms")
    wl = W.make_dense_workload(48, seed=1, device=dev)
    wall, t = bench.timed_steps(wl.step, 100, 10, settle_ms=300)
    print(f"dense_c48 {t * 1e6:.2f} us")
