"""Debug: the split kernel's transposed output layer (FV3_B3_TR=1) against the row-per-lane
one (0) on the emulator's 2,048 columns: per output, the levels and columns that differ."""
import os as _os

_os.environ.setdefault("FV3_VARIANTS", "1")  # A/B tool: kernel-variant selectors on
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_emulator import _emulator  # noqa: E402
from oracle import emulator as OE  # noqa: E402

emu, raw = _emulator(precision="bf16x3")
state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}
outs = {}
for tr in ("0", "1"):
    os.environ["FV3_B3_TR"] = tr
    got = emu(state)
    outs[tr] = {k: v.cpu().numpy().copy() for k, v in got.items()}
ref = OE.forward(raw, OE.zhao_carr_spec(), emu.params_by_name(), np.float64)
for o in OE.zhao_carr_spec()["outputs"]:
    name = o.get("after") or o["name"]
    a, b = outs["0"][name], outs["1"][name]
    r = ref[name]
    r = r[:, 0] if o["nz"] == 1 else r.T
    d = np.abs(a.astype(np.float64) - b)
    scale = np.abs(r).max(axis=-1, keepdims=True) if r.ndim == 2 else np.abs(r).max()
    rel = d / np.maximum(scale, 1e-30)
    print(name, a.shape, "max rel diff tr0/tr1", float(rel.max()), flush=True)
    if rel.max() > 1e-4 and a.ndim == 2:
        lev, col = np.nonzero(rel > 1e-4)
        print("  levels", np.unique(lev)[:20], "n cols", len(np.unique(col)), "cols", np.unique(col)[:24],
              "col%16", np.unique(col % 16), flush=True)
        k = lev[0]; c = col[0]
        print("  e.g. level", k, "col", c, "tr0", a[k, c], "tr1", b[k, c], "ref", r[k, c], flush=True)
        e0 = np.abs(a - r).max(axis=1) / np.maximum(np.abs(r).max(axis=1), 1e-30)
        e1 = np.abs(b - r).max(axis=1) / np.maximum(np.abs(r).max(axis=1), 1e-30)
        print("  oracle rel err per level tr0 max", e0.max(), "tr1 max", e1.max(), "tr1 worst level", int(e1.argmax()))
