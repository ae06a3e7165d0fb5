"""kord 1 mappm launch time vs column count on both kernels (FV3_MAPPM_PATH): picks
the level-parallel kernel's ncol threshold (csrc/mappm.hip kLevelsMaxCols)."""
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
    for res, kn in ((12, 50), (12, 79), (24, 79), (48, 79), (96, 79)):
        ncol = W.c_columns(res)
        for kord in (1, 7):
            wl = W.make_mappm_workload(ncol, 79, kn, kord, seed=5, device=dev)
            line = []
            for path in ("serial", "levels"):
                os.environ["FV3_MAPPM_PATH"] = path
                wall, t = bench.timed_steps(wl.step, 20, 3, settle_ms=100)
                line.append(f"{path} {t * 1e6:8.1f} us")
            print(f"C{res} ncol {ncol:6d} 79->{kn} kord {kord}: " + ", ".join(line), flush=True)
            del wl
