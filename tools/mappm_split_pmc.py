"""Launch only the two-field pair remap (kord 1, iv 1, 79 -> 79) on `ncol` C384-like
columns, one lane per column (split 0) or two (split 1), for --pmc passes:
mappm_split_pmc.py <split> <ncol> <n>  (data as tools/mappm_split_time.py)."""
import os
import sys

os.environ["FV3_VARIANTS"] = "1"
os.environ["FV3_MAPPM_SPLIT"] = sys.argv[1]
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402

if __name__ == "__main__":
    ncol, n = int(sys.argv[2]), int(sys.argv[3])
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    km = 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    pe = []
    for _ in range(2):
        delp = (base * rng.uniform(0.95, 1.05, (km, ncol))).astype(np.float32)
        pe.append(np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)]))
    qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
    d = [torch.from_numpy(a).to(dev) for a in pe + qs]
    plan = MappmMultiPlan(d[0], d[2:], d[1], 1, 1)
    for _ in range(n):
        out = plan()
    torch.cuda.synchronize()
    import hashlib
    h = hashlib.sha1(b"".join(o.cpu().numpy().tobytes() for o in out)).hexdigest()[:16]
    print("ok", sys.argv[1:], "outputs sha1", h)
