"""CPU study: which bf16 split of the emulator's three matmul stages (layer 1, hidden,
output) keeps the config #5 contract (1e-3 rel, per output level)?
   S3:  xh@wh + xh@wl + xl@wh  (the bf16x3 kernel)
   S2w: xh@wh + xl@wh          (weights rounded to bf16, activations split)
   S2x: xh@wh + xh@wl          (activations rounded, weights split)
   S1:  xh@wh                  (plain bf16)
Per-level errors vs the float64 graph, as tests/parity.py measures them."""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import emulator as OE  # noqa: E402
from parity import per_level_errors  # noqa: E402

b = OE.to_bf16


def split(a):
    a = np.asarray(a, np.float32)
    h = b(a)
    return h.astype(np.float64), b(a - h).astype(np.float64)


def mm(x, W, scheme):
    xh, xl = split(x)
    wh, wl = split(W)
    r = xh @ wh
    if scheme in ("S3", "S2x"):
        r = r + xh @ wl
    if scheme in ("S3", "S2w"):
        r = r + xl @ wh
    return r.astype(np.float32)


def forward(raw, spec, P, schemes):
    xs = OE.model_inputs({k: np.asarray(v, np.float32) for k, v in raw.items()}, spec)
    feats = [(x - np.float32(P["in_center"][f["name"]])) / np.float32(P["in_scale"][f["name"]])
             for f, x in zip(spec["features"], xs)]
    h = np.concatenate(feats, axis=-1).astype(np.float32)
    for li, (W, bb) in enumerate(zip(P["hidden_kernels"], P["hidden_biases"])):
        h = np.maximum(mm(h, W, schemes[0] if li == 0 else schemes[1]) + np.float32(bb), 0).astype(np.float32)
    out = {}
    for o in spec["outputs"]:
        y = mm(h, P["out_kernels"][o["name"]], schemes[2]) + np.float32(P["out_biases"][o["name"]])
        out[o["name"]] = y * np.float32(P["out_scale"][o["name"]]) + np.float32(P["out_center"][o["name"]])
    return out


if __name__ == "__main__":
    from fv3net_amd.emulator import MicrophysicsEmulator, zhao_carr_outputs

    raw = OE.synthetic_raw(2048, seed=1)
    rng = np.random.default_rng(2)
    sample_out = {}
    for o in zhao_carr_outputs():
        s = 1e-3 if o.name == "total_precipitation" else (1e-5 if ("humid" in o.name or "cloud" in o.name) else 0.5)
        sample_out[o.name] = rng.normal(0, s, (4096, o.nz)).astype(np.float32)
    emu = MicrophysicsEmulator.random(raw, sample_out, seed=1, precision="bf16x3")
    P = emu.params_by_name()
    spec = OE.zhao_carr_spec()
    ref = OE.forward(raw, spec, P, np.float64)
    for schemes in itertools.product(("S3", "S2w", "S2x"), repeat=3):
        got = forward(raw, spec, P, schemes)
        worst = max(np.nanmax(per_level_errors(got[o["name"]], ref[o["name"]])[0]) for o in spec["outputs"])
        print(" ".join(schemes), f"{worst:.2e}", flush=True)
