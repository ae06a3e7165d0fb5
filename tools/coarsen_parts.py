"""Coarsen C384 -> C48 (f = 8, 79 levels) launch time with 0 fields (pass 1 only: the
coarse delp / phalf), 1 and 4 fields; the remap's share is the difference.
FV3_COARSEN_PATH=cells|rows|cursor in the environment selects the kernel path."""
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
    for nf in (0, 1, 4):
        wl = W.make_coarsen_workload(384, 8, nf, seed=7, device=dev)
        wall, t = bench.timed_steps(wl.step, 10, 3, settle_ms=100)
        print(f"coarsen_c384_{nf}field {t * 1e3:.4f} ms", flush=True)
        del wl
