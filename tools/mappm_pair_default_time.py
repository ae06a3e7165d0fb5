"""Two fields remapped 79 -> 79 (kord 1, iv 1) through the default path of fv3_mappm_multi,
by column count (us per call): checks the kernel selection (csrc/mappm.hip)."""
import os, sys, json
import numpy as np, torch
sys.path.insert(0, os.getcwd())
import bench
from fv3net_amd.mappm import MappmMultiPlan
dev = torch.device("cuda", 0); rng = np.random.default_rng(0); km = 79
for ncol in (6912, 13824, 55296, 82944, 110592, 221184):
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    pe = []
    for _ in range(2):
        delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
        pe.append(np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)]))
    qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
    d = [torch.from_numpy(a).to(dev) for a in pe + qs]
    plan = MappmMultiPlan(d[0], d[2:], d[1], 1, 1)
    _, t = bench.timed_steps(plan, 50, 5, settle_ms=100)
    print(ncol, round(t * 1e6, 1), flush=True)
