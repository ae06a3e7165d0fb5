"""The streaming remap kernels under one library build (FV3NET_AMD_LIB selects it): mappm
kord 1 and kord 10 at C384 (79 -> 79), the two-field remap of predict + mappm's step
(mappm_device_multi on the pair kernel) and the pressure-level coarsen C384 -> C48 with
1 and 4 fields.  Mean launch ms, one line each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tag = os.path.basename(os.environ.get("FV3NET_AMD_LIB", "base"))
    n = W.c_columns(384)
    legs = [("mappm_kord1", lambda: W.make_mappm_workload(n, 79, 79, 1, seed=5, device=dev)),
            ("mappm_kord10", lambda: W.make_mappm_workload(n, 79, 79, 10, seed=5, device=dev)),
            ("coarsen_1field", lambda: W.make_coarsen_workload(384, 8, 1, seed=3, device=dev)),
            ("coarsen_4field", lambda: W.make_coarsen_workload(384, 8, 4, seed=3, device=dev))]
    for name, mk in legs:
        wl = mk()
        _, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
        print(f"{tag} {name} {t * 1e3:.4f} ms", flush=True)
        del wl
