"""Rough random columns (tests/test_remap_fast.py::test_random_columns_vs_oracle's data)
through every kord <= 7 x iv on the default arithmetic: max per-level error vs the C
oracle, per case (A/B of the fast arithmetic's variants via FV3NET_AMD_LIB)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fv3net_amd.mappm import mappm_device  # noqa: E402
from oracle.mappm import oracle_mappm  # noqa: E402
from tests.parity import per_level_errors  # noqa: E402

for delp_hi in (3000.0, 300.0):
    worst = []
    for kord in (1, 4, 6, 7):
        for iv in (-1, 0, 1, 2):
            rng = np.random.default_rng(100 + 10 * kord + iv)
            km, kn, ncol = 79, 50, 2000
            delp = rng.uniform(1, delp_hi, (km, ncol)).astype(np.float32)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
            q = (250 + rng.normal(0, 10, (km, ncol))).astype(np.float32)
            res = mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()
            rel, _ = per_level_errors(res.T, oracle_mappm(pe1, q, pe2, iv, kord).T)
            worst.append((kord, iv, float(np.nanmax(rel))))
    print("delp in [1, %g]:" % delp_hi, " ".join(f"k{k}iv{i}={e:.2e}" for k, i, e in worst), flush=True)
