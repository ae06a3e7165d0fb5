"""Two fields remapped 79 -> 79 (kord 1, iv 1) on C384-like columns: the pair kernel one
lane per column (FV3_MAPPM_SPLIT=0) against two lanes per column (=1), by column count:
picks csrc/mappm.hip kSplitMaxCols."""
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

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    km = 79
    res = {}
    for ncol in (65536, 110592, 147456, 221184, 262144, 331776, 442368, 884736):
        base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
        pe = []
        for _ in range(2):
            delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
            pe.append(np.concatenate([np.full((1, ncol), 300, np.float32),
                                      300 + np.cumsum(delp, 0, dtype=np.float32)]))
        qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
        d = [torch.from_numpy(a).to(dev) for a in pe + qs]
        plan = MappmMultiPlan(d[0], d[2:], d[1], 1, 1)
        line = {}
        for rnd in range(2):
            for split in ("0", "1"):
                os.environ["FV3_MAPPM_SPLIT"] = split
                _, t = bench.timed_steps(plan, 30, 3, settle_ms=100)
                line.setdefault(split, []).append(round(t * 1e6, 1))
        res[ncol] = line
        print(ncol, json.dumps(line), flush=True)
        del plan, d
    print(json.dumps(res))
