"""The config #4 predict at C96 on the same state: float32 inputs vs the float64 state
read in place (events around back-to-back launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for res in (96, 384):
        wl = W.make_stepper_workload(res, seed=11, device=dev)
        T, q = wl.state["air_temperature"], wl.state["specific_humidity"]
        T32, q32 = T.to(torch.float32), q.to(torch.float32)
        b32 = wl.model.bind([T32, q32], level_axes=[1, 1])
        b64 = wl.model.bind([T, q], level_axes=[1, 1])
        for name, b in (("f32", b32), ("f64", b64)):
            wall, t = bench.timed_steps(b, 50, 5, settle_ms=100)
            print(f"C{res} predict {name} inputs: {t * 1e6:.1f} us", flush=True)
        del wl
