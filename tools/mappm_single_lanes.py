"""One field remapped 79 -> 79 (kord 1, iv 1): the level-parallel kernel
(FV3_MAPPM_PATH=levels), one lane per column (=serial) and the split kernels on two and
three lanes (FV3_MAPPM_SPLIT1=2|3), interleaved, us per call; every variant's output
compared bitwise with one lane's (sorted columns: the unsorted and NaN cases are the
GPU tests')."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd.mappm import MappmPlan  # noqa: E402

VARIANTS = {"levels": ("levels", None), "lanes1": ("serial", None), "lanes2": ("serial", "2"),
            "lanes3": ("serial", "3")}

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    km = 79
    sizes = [int(x) for x in sys.argv[1:]] or [6912, 13824, 27648, 55296, 82944, 110592, 147456, 221184]
    res = {}
    for ncol in sizes:
        base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
        pe = []
        for _ in range(2):
            delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
            pe.append(np.concatenate([np.full((1, ncol), 300, np.float32),
                                      300 + np.cumsum(delp, 0, dtype=np.float32)]))
        q = rng.normal(250, 10, (km, ncol)).astype(np.float32)
        d = [torch.from_numpy(a).to(dev) for a in (pe[0], q, pe[1])]
        line, outs = {}, {}
        for rnd in range(2):
            for name, (path, split) in VARIANTS.items():
                os.environ["FV3_MAPPM_PATH"] = path
                os.environ.pop("FV3_MAPPM_SPLIT1", None)
                if split:
                    os.environ["FV3_MAPPM_SPLIT1"] = split
                plan = MappmPlan(d[0], d[1], d[2], 1, 1)
                _, t = bench.timed_steps(plan, 50, 5, settle_ms=100)
                line.setdefault(name, []).append(round(t * 1e6, 1))
                outs[name] = plan.out.clone()
        ref = outs["lanes1"]
        same = {k: bool(torch.equal(v.view(torch.int32), ref.view(torch.int32))) for k, v in outs.items()}
        res[ncol] = line
        print(ncol, json.dumps(line), "bit-identical to one lane:", same, flush=True)
    print(json.dumps(res))
