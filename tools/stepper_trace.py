"""One rank's share of the C96 stepper at world 8 (bench.py's stepper_c96_rank_of_8 leg),
stepped N times with nothing else, for a rocprofv3 kernel trace of the step's launches:
    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/stepper_trace.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fv3net_amd import workloads as W  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = W.make_sharded_stepper_workload(96, 0, 8, seed=11, device=dev, stub_exchange=True)
    for _ in range(20):
        wl.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.step()
    torch.cuda.synchronize()
    print(f"stepper rank-of-8 {1e3 * (time.perf_counter() - t0) / steps:.4f} ms/step over {steps}", flush=True)
