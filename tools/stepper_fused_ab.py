"""The stepper step with the predict and the epilogue fused into one launch (default
where it applies) against the two launches (FV3_STEPPER_FUSED=0, read at bind time):
one rank's share of C96 at world 8 (stubbed exchange) and the full C96 step,
interleaved on one box.  ms per step."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.stepper import BoundPredictEpilogue  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wls = {}
    for fused in ("1", "0"):
        os.environ["FV3_STEPPER_FUSED"] = fused
        rank = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
        full = W.make_stepper_workload(96, seed=11, device=dev)
        rank.step(), full.step()  # bind under this setting
        wls[fused] = (rank, full)
        print("fused" if fused == "1" else "pair", [type(op).__name__ for op in rank._plan._keep][:3], flush=True)
    for rep in range(3):
        for fused, (rank, full) in wls.items():
            _, tr = bench.timed_steps(rank.step, 300, 20, settle_ms=150)
            _, tf = bench.timed_steps(full.step, 100, 10, settle_ms=150)
            print(f"{'fused' if fused == '1' else 'pair '} stepper_c96_rank_of_8 {tr * 1e3:.4f} ms  "
                  f"stepper_c96 {tf * 1e3:.4f} ms", flush=True)
