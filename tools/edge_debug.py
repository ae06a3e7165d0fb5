"""Mismatch pattern of the edge-weighted coarsen kernel vs the oracle (f = 8)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import coarsen as OC  # noqa: E402
from fv3net_amd.coarsen import coarsen_edges_on_pressure  # noqa: E402
from test_coarsen_edges import _winds_state  # noqa: E402

for dtype in (np.float32, np.float64):
    for factor, n in ((8, 48), (8, 16), (4, 24)):
        rng = np.random.default_rng(factor * 10 + n)
        delp, u, v, dx, dy = _winds_state(rng, 40, n, dtype)
        for edge, sp, q in (("x", dx, u), ("y", dy, v)):
            o = coarsen_edges_on_pressure(delp, sp, {"q": q}, factor, edge)["q"].cpu().numpy()
            (r,) = OC.coarsen_edges_on_pressure(delp, sp, [q], factor, edge)
            bad = (o.view(np.uint32) != r.astype(np.float32).view(np.uint32)) & ~(np.isnan(o) & np.isnan(r))
            print(f"{dtype.__name__} f={factor} n={n} edge={edge}: bad {bad.sum()}/{bad.size}")
            if bad.any():
                print("   by tile", bad.sum(axis=(1, 2, 3)).tolist())
                print("   by coarse row", bad.sum(axis=(0, 1, 3)).tolist())
                print("   by coarse col", bad.sum(axis=(0, 1, 2)).tolist())
                print("   by level (first 12)", bad.sum(axis=(0, 2, 3))[:12].tolist())
                rel = np.abs(o[bad] - r[bad]) / np.abs(r[bad])
                print("   rel err max", rel.max(), "median", np.median(rel))
