"""Launch only the bf16x3 dense kernel (for --pmc passes): b3_only.py <dense|emulator> <n>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    what, n = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    if what == "dense":
        wl = W.make_dense_workload(384, seed=1, device=dev, precision="bf16x3")
    else:
        wl = W.make_emulator_workload(384, seed=13, device=dev, precision="bf16x3")
    for _ in range(n):
        wl.step()
    torch.cuda.synchronize()
    print("ok", what, n)
