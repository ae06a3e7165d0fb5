"""One rank's share of the C96 stepper at world 8 (stubbed exchange): the step's
reductions as one launch with the fold in it (default), the fold as its own launch
(FV3_STEP_FOLD_SPLIT=1), and every reduction apart (FV3_STEP_PARTIALS_SPLIT=1),
interleaved on one box.  ms per step."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rank = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
    variants = {"fused": {}, "fold_apart": {"FV3_STEP_FOLD_SPLIT": "1"}, "all_apart": {"FV3_STEP_PARTIALS_SPLIT": "1"}}
    for rep in range(3):
        for name, env in variants.items():
            for k in ("FV3_STEP_FOLD_SPLIT", "FV3_STEP_PARTIALS_SPLIT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            _, t = bench.timed_steps(rank.step, 300, 20, settle_ms=150)
            print(f"{name:12s} {t * 1e3:.4f} ms", flush=True)
