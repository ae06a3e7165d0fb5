"""kord-10 mappm (C384, 79 -> 79, and one rank's C384 band over 8) under each load
distance FV3_MAPPM_CS_PF of the kord > 7 kernel (read per launch), interleaved twice.
Mean launch ms."""
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
    # PF[:C32[:NT]] settings (NT unset: the library default by grid size)
    pfs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0:0", "2:0", "0:1", "2:1", "4:1", "8:1"]
    wls = {n: W.make_mappm_workload(n, 79, 79, 10, seed=5, device=dev) for n in (W.c_columns(384), W.c_columns(384) // 8)}
    for rep in range(2):
        for v in pfs:
            parts = v.split(":")
            pf = parts[0]
            c32 = parts[1] if len(parts) > 1 else "1"
            nt = parts[2] if len(parts) > 2 else ""
            os.environ["FV3_MAPPM_CS_PF"] = pf
            os.environ["FV3_MAPPM_CS_C32"] = c32
            if nt:
                os.environ["FV3_MAPPM_CS_NT"] = nt
            else:
                os.environ.pop("FV3_MAPPM_CS_NT", None)
            for n, wl in wls.items():
                _, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
                print(f"PF={pf} C32={c32} NT={nt or 'default'} ncol={n} kord10 {t * 1e3:.4f} ms", flush=True)
