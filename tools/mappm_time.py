"""Mean launch time of the standalone mappm (C384 fine columns, 79 -> 79, kord 1 and 10)
and the fused C384 -> C48 coarsen (1 field): the VALU-bound remap legs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for kord in (1, 10):
        wl = W.make_mappm_workload(W.c_columns(384), 79, 79, kord, seed=5, device=dev)
        wall, t = bench.timed_steps(wl.step, 10, 3, settle_ms=150)
        print(f"mappm_c384_kord{kord} {t * 1e3:.4f} ms", flush=True)
        del wl
    wl = W.make_coarsen_workload(384, 8, 1, seed=7, device=dev)
    wall, t = bench.timed_steps(wl.step, 10, 3, settle_ms=150)
    print(f"coarsen_c384_1field {t * 1e3:.4f} ms", flush=True)
    # two fields on the same edges: two single-field launches vs one two-field pass
    from fv3net_amd.mappm import MappmMultiPlan, MappmPlan  # noqa: E402

    wl = W.make_mappm_workload(W.c_columns(384), 79, 79, 1, seed=5, device=dev)
    q2 = wl.q1.clone() if hasattr(wl, "q1") else None
    if q2 is not None:
        singles = [MappmPlan(wl.pe1, q, wl.pe2, 1, 1) for q in (wl.q1, q2)]
        pair = MappmMultiPlan(wl.pe1, [wl.q1, q2], wl.pe2, 1, 1)
        _, t1 = bench.timed_steps(lambda: [p() for p in singles], 10, 3, settle_ms=150)
        _, t2 = bench.timed_steps(pair, 10, 3, settle_ms=150)
        print(f"mappm_c384_2fields single x2 {t1 * 1e3:.4f} ms, pair {t2 * 1e3:.4f} ms", flush=True)
