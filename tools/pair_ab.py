"""The two-field streaming remap (mappm_ppm_pair_kernel, predict + mappm's second kernel)
at C384 79 -> 79 and one rank's band over 8, under the library FV3NET_AMD_LIB selects.
Mean launch ms."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.mappm import MappmMultiPlan  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tag = os.path.basename(os.environ.get("FV3NET_AMD_LIB", "base"))
    for n in (W.c_columns(384), W.c_columns(384) // 8):
        wl = W.make_mappm_workload(n, 79, 79, 1, seed=5, device=dev)
        q2 = wl.q1 * 1.5 + 3.0
        plan = MappmMultiPlan(wl.pe1, [wl.q1, q2], wl.pe2, 1, 1)
        _, t = bench.timed_steps(plan, 20, 3, settle_ms=150)
        print(f"{tag} pair ncol={n} {t * 1e3:.4f} ms", flush=True)
        del wl, plan
