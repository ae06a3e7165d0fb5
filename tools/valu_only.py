"""Drivers for counter passes: `mappm` (C384 79->79 kord 1) or `coarsen` (C384 -> C48,
1 field) or `dense` (C48) / `dense384`, N launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    what, n = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    if what == "mappm":
        wl = W.make_mappm_workload(W.c_columns(384), 79, 79, 1, seed=5, device=dev)
    elif what == "coarsen":
        wl = W.make_coarsen_workload(384, 8, 1, seed=7, device=dev)
    elif what == "dense384":
        wl = W.make_dense_workload(384, seed=1, device=dev)
    else:
        wl = W.make_dense_workload(48, seed=1, device=dev)
    for _ in range(n):
        wl.step()
    torch.cuda.synchronize()
