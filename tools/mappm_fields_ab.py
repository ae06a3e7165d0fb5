"""Two-field kord-1 mappm (the predict+mappm step's remap) and the single-field kernel at
one rank's C384 band over 8 GPUs (110,592 columns) and the full grid (884,736), under the
multi-field scheme FV3_MAPPM_FIELDS selects (pair | lanes; unset: the library's choice).
Mean launch ms."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan, MappmPlan  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tag = os.environ.get("FV3_MAPPM_FIELDS", "default")
    for ncol in (W.c_columns(384) // 8, W.c_columns(384)):
        wl = W.make_mappm_workload(ncol, 79, 79, 1, seed=5, device=dev)
        q2 = wl.q1.clone()
        single = MappmPlan(wl.pe1, wl.q1, wl.pe2, 1, 1)
        pair = MappmMultiPlan(wl.pe1, [wl.q1, q2], wl.pe2, 1, 1)
        _, t1 = bench.timed_steps(single, 20, 3, settle_ms=150)
        _, t2 = bench.timed_steps(pair, 20, 3, settle_ms=150)
        print(f"fields={tag} ncol={ncol} single {t1 * 1e3:.4f} ms pair {t2 * 1e3:.4f} ms", flush=True)
        del wl
