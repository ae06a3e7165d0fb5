"""Two fields remapped 79 -> 79 (kord 1, iv 1) on small grids: the level-parallel kernel
(one field per launch, FV3_MAPPM_PATH=levels) against the pair kernel on one, two and three
lanes per column (FV3_MAPPM_PATH=serial, FV3_MAPPM_SPLIT=0|1|3), interleaved; us per call."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402

VARIANTS = {"levels": ("levels", "0"), "lanes1": ("serial", "0"), "lanes2": ("serial", "1"),
            "lanes3": ("serial", "3")}

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    km = 79
    res = {}
    sizes = [int(x) for x in sys.argv[1:]] or [13824, 27648, 55296, 65536, 82944]
    for ncol in sizes:
        base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
        pe = []
        for _ in range(2):
            delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
            pe.append(np.concatenate([np.full((1, ncol), 300, np.float32),
                                      300 + np.cumsum(delp, 0, dtype=np.float32)]))
        qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
        d = [torch.from_numpy(a).to(dev) for a in pe + qs]
        line = {}
        for rnd in range(2):
            for name, (path, split) in VARIANTS.items():
                os.environ["FV3_MAPPM_PATH"] = path
                os.environ["FV3_MAPPM_SPLIT"] = split
                plan = MappmMultiPlan(d[0], d[2:], d[1], 1, 1)
                _, t = bench.timed_steps(plan, 50, 5, settle_ms=100)
                line.setdefault(name, []).append(round(t * 1e6, 1))
        res[ncol] = line
        print(ncol, json.dumps(line), flush=True)
    print(json.dumps(res))
