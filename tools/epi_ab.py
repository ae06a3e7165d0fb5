"""The stepper epilogue's two kernels (FV3_EPILOGUE_PATH=levels|columns, read per launch),
interleaved twice: one rank's share of C96 over 8 (bound step, stubbed exchange) and the
full C96 step.  ms per step."""
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
    full = W.make_stepper_workload(96, seed=11, device=dev)
    for rep in range(2):
        for path in ("levels", "levels-u3", "columns"):
            os.environ["FV3_EPILOGUE_PATH"] = path.split("-")[0]
            if path.endswith("u3"):
                os.environ["FV3_EPI_U"] = "3"
            else:
                os.environ.pop("FV3_EPI_U", None)
            _, tr = bench.timed_steps(rank.step, 200, 20, settle_ms=150)
            _, tf = bench.timed_steps(full.step, 50, 5, settle_ms=150)
            print(f"epilogue={path} stepper_c96_rank_of_8 {tr * 1e3:.4f} ms  stepper_c96 {tf * 1e3:.4f} ms", flush=True)
