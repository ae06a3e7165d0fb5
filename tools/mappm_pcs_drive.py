"""A short driver for a PC-sampling pass over one kernel: the config #3 mappm (C384,
79 -> 79, kord 1, the default arithmetic) or the 1-field coarsen, launched N times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

which, n = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
wl = (W.make_mappm_workload(W.c_columns(384), 79, 79, 1, seed=5, device=dev) if which == "mappm"
      else W.make_coarsen_workload(384, 8, 1, seed=7, device=dev))
for _ in range(n):
    wl.step()
torch.cuda.synchronize()
print("done", which, n, flush=True)
