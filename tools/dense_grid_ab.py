"""C48 headline kernel: persistent grid size and issue priority A/B (FV3_DENSE_GRID /
FV3_DENSE_PRIO, read per launch), interleaved: us per launch (bench.timed_steps)."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    wl = W.make_dense_workload(48, seed=1, device=dev)
    variants = {"default": {}, "grid256": {"FV3_DENSE_GRID": "256"}, "grid216": {"FV3_DENSE_GRID": "216"},
                "grid320": {"FV3_DENSE_GRID": "320"}, "prio1": {"FV3_DENSE_PRIO": "1"},
                "cfg_2_3": {"FV3_DENSE_CFG": "2,3"}}
    res = {}
    for rnd in range(3):
        for name, env in variants.items():
            for k in ("FV3_DENSE_GRID", "FV3_DENSE_PRIO", "FV3_DENSE_CFG"):
                os.environ.pop(k, None)
            os.environ.update(env)
            _, t = bench.timed_steps(wl.step, 300, 20, settle_ms=200)
            res.setdefault(name, []).append(round(t * 1e6, 2))
        print(rnd, json.dumps(res), flush=True)
