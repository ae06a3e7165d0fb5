"""Time the C384 -> C48 edge-weighted coarsen (u on x edges, 79 levels) on both remap
paths: input-driven through the scratch column (default) and the cursor."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd.coarsen import coarsen_edges_on_pressure  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    n, nz = 384, 79
    delp = 1000.0 + 200.0 * torch.rand((6, nz, n, n), device=dev, generator=g)
    dx = 2.0e4 + 1.0e3 * torch.rand((6, n + 1, n), device=dev, generator=g)
    u = 10.0 * torch.randn((6, nz, n + 1, n), device=dev, generator=g)
    for path in ("scratch", "cursor"):
        if path == "cursor":
            os.environ["FV3_COARSEN_CURSOR"] = "1"
        step = lambda: coarsen_edges_on_pressure(delp, dx, {"u": u}, 8, "x")  # noqa: E731
        wall, t = bench.timed_steps(step, 20, 3, settle_ms=150)
        print(f"edge_c384_to_c48_{path} {t * 1e3:.4f} ms (wall {wall / 20 * 1e3:.4f} ms/step)")
