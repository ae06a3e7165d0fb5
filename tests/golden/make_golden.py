"""Generate the committed golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the .npz files).

* mappm_golden.npz — outputs of the REFERENCE Fortran mappm (mappm.f90 compiled
  unmodified by oracle/Makefile into oracle/_ref/libmappm_ref.so) on seeded
  synthetic columns, for kord in {1,4,7,9,...,17} x iv in {0,1,-1,2}, plus a full
  C12 79->50 case for kord 1 and 10.
* coarsen_kat.npz — expected coarse fields from the reference's own regression
  data, external/vcm/tests/_coarsen_restarts_regression_tests/reference/
  pressure-level-without-agrid-winds-{fv_core.res,fv_tracer.res}.json (the
  values, not the files), for the masked-area-weighted pressure-level variables.
* coarsen_edge_kat.npz — the same data's coarse D-grid winds u and v (the
  edge-weighted pressure-level path, regridz.py:58-112).
* restarts_kat.npz — EVERY variable of the same data's fv_core.res, fv_tracer.res and
  fv_srf_wnd.res categories, for both pressure-level tags (with and without A-grid
  winds): the whole coarsen_restarts_on_pressure output except sfc_data.
  Inputs are regenerated in the tests exactly as external/synth does
  (np.random.seed(0); uniform(lo, hi, shape) per single-chunk variable,
  synth/core.py:63-67), so only the expected values are stored.

Usage:  python tests/golden/make_golden.py [--edge-kat | --restarts-kat]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.mappm import build, reference_available, reference_mappm  # noqa: E402

REF_JSON = "/root/reference/external/vcm/tests/_coarsen_restarts_regression_tests/reference"

KORDS = [1, 4, 7, 9, 10, 11, 12, 13, 14, 15, 16, 17]
IVS = [0, 1, -1, 2]


def synthetic_columns(rng, ncol, km, kn, kind):
    """config #1 style columns: delp ~ U(500,1500) Pa, 300 Pa top."""
    delp = rng.uniform(500.0, 1500.0, size=(km, ncol)).astype(np.float32)
    pe1 = np.empty((km + 1, ncol), np.float32)
    pe1[0] = 300.0
    pe1[1:] = 300.0 + np.cumsum(delp, axis=0, dtype=np.float32)
    if kind == "uniform":  # kn+1 edges evenly spanning the old column
        pe2 = np.linspace(pe1[0], pe1[-1], kn + 1).astype(np.float32)
    elif kind == "coarse_on_fine":  # a neighbour's edges, shared 300 Pa top
        d2 = delp * rng.uniform(0.95, 1.05, size=delp.shape).astype(np.float32)
        pe2 = np.empty((km + 1, ncol), np.float32)
        pe2[0] = 300.0
        pe2[1:] = 300.0 + np.cumsum(d2, axis=0, dtype=np.float32)
        if kn != km:
            raise ValueError("coarse_on_fine needs kn == km")
    elif kind == "overhang":  # edges above the old top and below the old surface
        pe2 = np.linspace(pe1[0] * 0.5, pe1[-1] * 1.05, kn + 1).astype(np.float32)
    else:
        raise ValueError(kind)
    q_smooth = (250.0 + 10.0 * np.sin(np.arange(km)[:, None] * 0.3)
                + rng.normal(0.0, 1.0, (km, ncol))).astype(np.float32)
    q_rough = (rng.normal(0.0, 1.0, (km, ncol))
               * rng.choice([1e-3, 1.0, 100.0], size=(km, ncol))).astype(np.float32)
    return pe1, pe2, q_smooth, q_rough


def make_mappm_golden():
    rng = np.random.default_rng(20250418)
    out = {}
    cases = [("uniform", 79, 50), ("coarse_on_fine", 79, 79), ("overhang", 79, 50), ("uniform", 7, 5)]
    for ci, (kind, km, kn) in enumerate(cases):
        pe1, pe2, qs, qr = synthetic_columns(rng, 32, km, kn, kind)
        out[f"c{ci}_pe1"], out[f"c{ci}_pe2"] = pe1, pe2
        out[f"c{ci}_qs"], out[f"c{ci}_qr"] = qs, qr
        for kord in KORDS:
            for iv in IVS:
                for qn, q in (("qs", qs), ("qr", qr)):
                    out[f"c{ci}_{qn}_k{kord}_iv{iv}"] = reference_mappm(pe1, q, pe2, iv, kord)
    out["cases"] = np.array([f"{k}:{a}:{b}" for k, a, b in cases])
    out["kords"] = np.array(KORDS)
    out["ivs"] = np.array(IVS)
    # full C12 (6*12*12 columns) 79 -> 50, q ~ N(250, 10), SURVEY §8(d) config #1
    rng = np.random.default_rng(12)
    ncol = 6 * 12 * 12
    pe1, pe2, _, _ = synthetic_columns(rng, ncol, 79, 50, "uniform")
    q = rng.normal(250.0, 10.0, (79, ncol)).astype(np.float32)
    out["c12_pe1"], out["c12_pe2"], out["c12_q"] = pe1, pe2, q
    for kord in (1, 10):
        out[f"c12_k{kord}_iv1"] = reference_mappm(pe1, q, pe2, 1, kord)
    np.savez_compressed(os.path.join(HERE, "mappm_golden.npz"), **out)


def make_coarsen_kat():
    out = {}
    for cat in ("fv_core.res", "fv_tracer.res"):
        with open(os.path.join(REF_JSON, f"pressure-level-without-agrid-winds-{cat}.json")) as f:
            d = json.load(f)
        for name, var in d["data_vars"].items():
            dims = var["dims"]
            if "zaxis_1" not in dims or "xaxis_1" not in dims:
                continue
            if name in ("delp", "DZ", "u", "v"):
                continue  # not on the masked area-weighted pressure path
            out[f"{cat}/{name}"] = np.asarray(var["data"], dtype=np.float64)
            out[f"{cat}/{name}/dims"] = np.array(dims)
    np.savez_compressed(os.path.join(HERE, "coarsen_kat.npz"), **out)


def make_coarsen_edge_kat():
    """coarsen_edge_kat.npz: the reference's coarse D-grid winds u (edge "x") and v
    (edge "y") of the same regression data (regrid_to_edge_weighted_pressure path)."""
    with open(os.path.join(REF_JSON, "pressure-level-without-agrid-winds-fv_core.res.json")) as f:
        d = json.load(f)
    out = {}
    for name in ("u", "v"):
        var = d["data_vars"][name]
        out[f"fv_core.res/{name}"] = np.asarray(var["data"], dtype=np.float64)
        out[f"fv_core.res/{name}/dims"] = np.array(var["dims"])
    np.savez_compressed(os.path.join(HERE, "coarsen_edge_kat.npz"), **out)


def make_restarts_kat():
    out = {}
    for tag in ("pressure-level-without-agrid-winds", "pressure-level-with-agrid-winds"):
        for cat in ("fv_core.res", "fv_tracer.res", "fv_srf_wnd.res"):
            with open(os.path.join(REF_JSON, f"{tag}-{cat}.json")) as f:
                d = json.load(f)
            for name, var in d["data_vars"].items():
                out[f"{tag}/{cat}/{name}"] = np.asarray(var["data"], dtype=np.float64)
                out[f"{tag}/{cat}/{name}/dims"] = np.array(var["dims"])
    np.savez_compressed(os.path.join(HERE, "restarts_kat.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["--edge-kat"]:  # JSON values only; no reference build needed
        make_coarsen_edge_kat()
        raise SystemExit(0)
    if sys.argv[1:] == ["--restarts-kat"]:  # JSON values only; no reference build needed
        make_restarts_kat()
        raise SystemExit(0)
    build()
    if not reference_available():
        raise SystemExit("reference mappm not built (needs /root/reference + flang)")
    make_mappm_golden()
    make_coarsen_kat()
    make_coarsen_edge_kat()
    make_restarts_kat()
    print("golden fixtures written to", HERE)
