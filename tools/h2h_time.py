"""Host -> device -> host predict (bench.host_to_host) at C48 and C384, with the
product's pinned staging, beside torch's pageable copies of the same bytes."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    for res in (48, 384):
        r = bench.host_to_host(dev, res)
        print(f"C{res} staged: {r['ms_per_step']:.3f} ms, {r['pcie_inclusive_gbs']:.1f} GB/s", flush=True)
        n = 6 * 79 * res * res
        a = np.random.default_rng(0).normal(size=n)
        d = torch.empty(n, dtype=torch.float64, device=dev)
        for _ in range(2):
            d.copy_(torch.from_numpy(a))
            b = d.cpu().numpy()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            d.copy_(torch.from_numpy(a))
            b = d.cpu().numpy()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(f"C{res} pageable torch round trip of one f64 field: {2 * a.nbytes / dt / 1e9:.1f} GB/s", flush=True)
        from fv3net_amd import transfer
        t0 = time.perf_counter()
        for _ in range(5):
            transfer.h2d(a, out=d)
            transfer.d2h(d, out=b)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(f"C{res} staged round trip of one f64 field: {2 * a.nbytes / dt / 1e9:.1f} GB/s", flush=True)
