"""The split kernel on one rank's C384 band over 8 GPUs (110,592 columns: 864 tiles of
128 columns for 256 CUs, 3.4 per CU) under the block shape FV3_B3_WAVES selects (8:
128-column tiles; 4: 64-column tiles, 6.75 per CU).  Mean launch ms."""
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
    tag = os.environ.get("FV3_B3_WAVES", "default")
    for prec in ("bf16x3", "bf16x6"):
        wl = W.make_emulator_workload(384, seed=13, device=dev, precision=prec, world=8)
        _, t = bench.timed_steps(wl.step, 20, 3, settle_ms=150)
        print(f"waves={tag} emulator r8 {prec} {t * 1e3:.4f} ms", flush=True)
        del wl
        wl = W.make_predict_mappm_workload(384, 0, 8, seed=21, device=dev, precision=prec)
        wl.step()
        _, t = bench.timed_steps(wl._bound, 20, 3, settle_ms=150)
        print(f"waves={tag} dense r8 {prec} {t * 1e3:.4f} ms", flush=True)
        del wl
