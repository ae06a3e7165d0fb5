"""The bf16x3 split kernel on 16x16x32 MFMAs (dense_b3_kernel, the default) against the
32x32x16 kernel (dense_b3w_kernel, FV3_B3_SHAPE=32): output agreement and mean launch
time, interleaved on one box (config #5 emulator at C384, the 2x256 DenseModel at C384 and
C96).  The 32x32x16 kernel was built in commit d385025 and removed after this A/B
(profiles/r05zc_b3_mfma32_ab.log); run it against that tree."""
import os
import sys
import time

os.environ["FV3_VARIANTS"] = "1"
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fv3net_amd import workloads as W  # noqa: E402

BF16_PEAK = 2516.6


def timed(step, n):
    t0 = time.time()
    while time.time() - t0 < 0.3:
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def outputs(wl):
    return [v.clone() for v in (wl.out.values() if hasattr(wl, "out") else wl.outputs)]


def main():
    dev = torch.device("cuda", 0)
    cases = {"emulator_c384": W.make_emulator_workload(384, seed=13, device=dev, precision="bf16x3"),
             "dense_c384": W.make_dense_workload(384, seed=1, device=dev, precision="bf16x3"),
             "dense_c96": W.make_dense_workload(96, seed=1, device=dev, precision="bf16x3")}
    shapes = sys.argv[1:] or ["16", "32"]
    for name, wl in cases.items():
        outs = {}
        for s in shapes:
            os.environ["FV3_B3_SHAPE"] = s
            wl.step()
            torch.cuda.synchronize()
            outs[s] = outputs(wl)
        ref = outs[shapes[0]]
        for s in shapes[1:]:
            worst = max(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item() for a, b in zip(outs[s], ref))
            nan = sum(int(torch.isnan(a).sum().item()) for a in outs[s])
            print(f"{name} shape {s} vs {shapes[0]}: worst rel diff {worst:.3e}, NaNs {nan}", flush=True)
    res = {n: {s: [] for s in shapes} for n in cases}
    for rnd in range(3):
        order = shapes if rnd % 2 == 0 else shapes[::-1]
        for name, wl in cases.items():
            n = 10 if "c384" in name else 100
            for s in order:
                os.environ["FV3_B3_SHAPE"] = s
                res[name][s].append(timed(wl.step, n) * 1e6)
    for name, wl in cases.items():
        for s in shapes:
            t = sorted(res[name][s])[1] * 1e-6
            frac = 3 * wl.ncol * wl.flops_per_column / t / 1e12 / BF16_PEAK
            print(f"{name:14s} shape {s}: {[round(x, 1) for x in res[name][s]]} us, median {t * 1e6:.1f} us, "
                  f"{frac:.3f} of bf16 peak", flush=True)


if __name__ == "__main__":
    main()
