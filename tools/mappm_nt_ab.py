"""kord-10 mappm (C384, 79 -> 79, and one rank's C384 band over 8) under the register-tail
depth FV3_MAPPM_CS_NT selects (unset: the library default).  Mean launch ms."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    tag = os.environ.get("FV3_MAPPM_CS_NT", "default")
    for ncol in (W.c_columns(384), W.c_columns(384) // 8):
        wl = W.make_mappm_workload(ncol, 79, 79, 10, seed=5, device=dev)
        _, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
        print(f"NT={tag} ncol={ncol} kord10 {t * 1e3:.4f} ms", flush=True)
        del wl
