"""The tolerance-contract remap (FV3_ARITH_FAST) against the exact one and the flang
golden vectors: per-level errors (max |fast - ref| / max |ref| per output level), the
positions that moved by more than 1e-5 of their level's scale (limiter-branch flips),
and kernel times of both arithmetics.  Prints one JSON line per item."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fv3net_amd import workloads as W  # noqa: E402
from fv3net_amd.coarsen import coarsen_on_pressure  # noqa: E402
from fv3net_amd.mappm import mappm_device  # noqa: E402


def level_err(got, ref, axis_level=0):
    g = got.double()
    r = ref.double()
    dims = [d for d in range(g.dim()) if d != axis_level]
    err = (g - r).abs().amax(dim=dims)
    scale = r.abs().amax(dim=dims)
    rel = torch.where(scale > 0, err / scale.clamp_min(1e-300), err)
    flips = ((g - r).abs() > 1e-5 * scale.reshape([-1 if d == axis_level else 1 for d in range(g.dim())])).sum()
    return float(rel.max()), float(rel.median()), int(flips)


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(ROOT, "tests", "golden", "mappm_golden.npz"))
    worst = {}
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = mappm_device(pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord))
                    exp = torch.as_tensor(g[f"c{ci}_{qn}_k{kord}_iv{iv}"], device=dev)
                    mx, med, fl = level_err(res, exp)
                    worst[f"c{ci}_{qn}_k{kord}_iv{iv}"] = (mx, med, fl)
    vals = sorted(worst.items(), key=lambda kv: -kv[1][0])
    print(json.dumps({"item": "golden", "n": len(vals), "over_1e-6": sum(v[0] > 1e-6 for _, v in vals),
                      "over_1e-5": sum(v[0] > 1e-5 for _, v in vals), "worst": vals[:12]}), flush=True)
    for kord in (1, 10):
        wl = W.make_mappm_workload(W.c_columns(384), 79, 79, kord, seed=5, device=dev)
        fast = mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord)
        exact = mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord, exact=True)
        mx, med, fl = level_err(fast, exact)
        tf = timeit(lambda: mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord, out=fast))
        te = timeit(lambda: mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord, out=exact, exact=True))
        print(json.dumps({"item": f"mappm_c384_kord{kord}", "max_rel": mx, "median_rel": med, "flips": fl,
                          "ms_fast": tf, "ms_exact": te}), flush=True)
        del wl
    for nf in (1, 4):
        wl = W.make_coarsen_workload(384, 8, nf, seed=7, device=dev)
        fa, _ = coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8)
        ex, _ = coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8, exact=True)
        errs = [level_err(fa[k], ex[k], 1) for k in fa]
        tf = timeit(lambda: coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8))
        te = timeit(lambda: coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8, exact=True))
        print(json.dumps({"item": f"coarsen_c384_{nf}field", "max_rel": max(e[0] for e in errs),
                          "flips": sum(e[2] for e in errs), "ms_fast": tf, "ms_exact": te}), flush=True)
        del wl


if __name__ == "__main__":
    main()
