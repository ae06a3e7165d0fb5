"""Run only the fused dense kernel (for rocprofv3 counter passes):  python tools/dense_only.py RES ITERS"""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W
res = int(sys.argv[1]) if len(sys.argv) > 1 else 48
it = int(sys.argv[2]) if len(sys.argv) > 2 else 50
wl = W.make_dense_workload(res, seed=1, device=torch.device("cuda", 0))
torch.cuda.synchronize()
for _ in range(it):
    wl.step()
torch.cuda.synchronize()
print("done", res, it)
