"""One rank's share of the C96 stepper at world 8 (stubbed exchange), n steps back to back
after a settle phase: for a rocprofv3 kernel trace of the step's launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rank = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
    _, t = bench.timed_steps(rank.step, n, 20, settle_ms=150)
    print(f"rank step {t * 1e3:.4f} ms", flush=True)
