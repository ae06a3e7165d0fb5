"""A/B of the kord > 7 (cs_profile) mappm kernels at C384 79 -> 79: the edge values in
registers (default, mappm_cs_reg_kernel) vs both planes in the global scratch
(FV3_MAPPM_CS=global).  `--only reg|global --launches N` runs just N launches of one
variant (for a rocprofv3 --pmc pass)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--kord", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.make_mappm_workload(W.c_columns(384), 79, 79, a.kord, seed=5, device=dev)
    if a.only:
        os.environ["FV3_MAPPM_CS"] = a.only
        for _ in range(a.launches):
            wl.step()
        torch.cuda.synchronize()
        print(f"ran {a.launches} launches of {a.only}", flush=True)
        sys.exit(0)
    for rep in range(2):
        for v in ("reg", "global"):
            os.environ["FV3_MAPPM_CS"] = v
            wall, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
            print(f"mappm_c384_kord{a.kord} {v} {t * 1e3:.4f} ms", flush=True)
