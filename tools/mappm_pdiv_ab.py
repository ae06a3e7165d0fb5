"""mappm kord 1 with and without the short pressure-only divisions (FV3_MAPPM_PDIV=0|1,
read per launch): one field and two fields (the pair kernel), C384 and one rank's
110,592 columns, interleaved; us per launch.  Also checks the two give the same bits."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan, MappmPlan  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    km = 79
    res = {}
    for ncol in (884736, 110592):
        base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
        pe = []
        for _ in range(2):
            delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
            pe.append(np.concatenate([np.full((1, ncol), 300, np.float32),
                                      300 + np.cumsum(delp, 0, dtype=np.float32)]))
        qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
        d = [torch.from_numpy(a).to(dev) for a in pe + qs]
        one = MappmPlan(d[0], d[2], d[1], 1, 1)
        pair = MappmMultiPlan(d[0], d[2:], d[1], 1, 1)
        line = {}
        outs = {}
        for rnd in range(2):
            for pdiv in ("0", "1"):
                os.environ["FV3_MAPPM_PDIV"] = pdiv
                for name, plan in (("one", one), ("pair", pair)):
                    _, t = bench.timed_steps(plan, 30, 3, settle_ms=100)
                    line.setdefault(f"{name}_pdiv{pdiv}", []).append(round(t * 1e6, 1))
                    r = plan()
                    r = r if isinstance(r, (list, tuple)) else [r]
                    outs.setdefault((name, pdiv), [x.clone() for x in r])
        same = all(torch.equal(a.view(torch.int32), b.view(torch.int32))
                   for name in ("one", "pair") for a, b in zip(outs[(name, "0")], outs[(name, "1")]))
        line["bit_identical"] = same
        res[ncol] = line
        print(ncol, json.dumps(line), flush=True)
        del one, pair, d
    print(json.dumps(res))
