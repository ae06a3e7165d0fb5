"""Launch only the coarsen kernel (C384 -> C48, f = 8, 79 levels) with nf fields, n times
(for --pmc passes): coarsen_only.py <nf> <n>."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    nf, n = int(sys.argv[1]), int(sys.argv[2])
    wl = W.make_coarsen_workload(384, 8, nf, seed=7, device=torch.device("cuda", 0))
    for _ in range(n):
        wl.step()
    torch.cuda.synchronize()
    print("ok", nf, n)
