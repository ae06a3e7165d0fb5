"""Per-tile phase timeline of the bf16 split kernel (dense_b3.hip) from the trace variant:
    tools/build_b3_variant.sh b3trace -DFV3_B3_TRACE
    FV3NET_AMD_LIB=tools/variants/libb3trace.so python3 tools/b3_trace.py [emulator|dense] [bf16x3|bf16x6]
The trace variant's clock reads are scheduling barriers (its instruction order differs
from the product kernel's), so the phase split is indicative; its launch time is printed
beside the product's from the same process for comparison.  Per tile: layer 1, hidden
layers, output layer (us), shader clock, and the fraction of the tile wave 0 spent in the
chunk waits (vmcnt + barrier)."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fv3net_amd import _native, workloads as W  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "emulator"
    prec = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    dev = torch.device("cuda", 0)
    if what == "emulator":
        wl = W.make_emulator_workload(384, seed=13, device=dev, precision=prec)
        model = wl.emulator.model
    else:
        wl = W.make_dense_workload(384, seed=3, device=dev, precision=prec)
        model = wl.model
    _, t = bench.timed_steps(wl.step, 10, 3, settle_ms=150)
    ntiles = -(-wl.ncol // 128)
    buf = torch.zeros(ntiles * 8 + 64, dtype=torch.int64, device=dev)
    lib = _native.load()
    _native.check(lib.fv3_dense_set_trace(model.handle(), buf.data_ptr()))
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    _native.check(lib.fv3_dense_set_trace(model.handle(), None))
    r = buf[: ntiles * 8].view(ntiles, 8).cpu().numpy().astype(np.float64)
    wall = r[:, :4] / 100.0  # us
    d = np.diff(wall, axis=1)
    cyc = r[:, 6] - r[:, 5]
    dur = wall[:, 3] - wall[:, 0]
    ok = dur > 0
    clk = cyc[ok] / dur[ok] / 1e3
    waitf = r[ok, 7] / cyc[ok]
    print(f"{what} {prec}: {wl.ncol} columns, {ntiles} tiles of 128, launch {t * 1e3:.3f} ms (trace variant)")
    for i, n in enumerate(("layer1", "hidden", "output")):
        print(f"   {n:7s} mean {d[ok, i].mean():7.2f} us  p10 {np.percentile(d[ok, i], 10):7.2f}  "
              f"p90 {np.percentile(d[ok, i], 90):7.2f}")
    print(f"   tile   mean {dur[ok].mean():7.2f} us; clock {np.median(clk):.3f} GHz; "
          f"wave-0 chunk-wait fraction mean {waitf.mean():.3f} (p10 {np.percentile(waitf, 10):.3f}, "
          f"p90 {np.percentile(waitf, 90):.3f})")
    span = wall[ok, 3].max() - wall[ok, 0].min()
    print(f"   span {span:.1f} us; tiles per CU {ntiles / len(np.unique(r[ok, 4])):.1f}")


if __name__ == "__main__":
    main()
