"""The default remap arithmetic (FV3_ARITH_FAST, csrc/mappm_core.h: reciprocal divisions,
FMA within an expression, hardware MAX / MIN) held to north_star's floating-point
contract against the same references the exact path matches bit for bit.

Bound: per output level, max |fast - ref| <= rtol * max |ref| (tests/parity.py), with
rtol 1e-5 (north_star: tendencies within 1e-5 rel of the CPU reference).  Tighter
measured bounds are asserted where the data allow it (golden vectors 1e-6), so a
regression in the arithmetic shows before it reaches the contract.  The reference
itself does not promise bit reproducibility across platforms for this routine
(external/vcm/tests/test_coarsen_restarts.py:115-122 compares with assert_allclose).

kord > 7 (cs_profile) is exact whatever the request: its limiter switches on flags of
the solved edges, which 1-ulp changes flip (mappm.hip, launch_arith).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coarsen as OC
from oracle import restarts as OR
from oracle.mappm import oracle_mappm
from tests.parity import assert_per_level, per_level_errors

pytestmark = pytest.mark.gpu


def _rel(got, ref, axis=0):
    """Max per-level error of [level, ...] arrays (levels on ``axis``)."""
    g = np.moveaxis(np.asarray(got, np.float64), axis, -1).reshape(-1, np.shape(got)[axis])
    r = np.moveaxis(np.asarray(ref, np.float64), axis, -1).reshape(-1, np.shape(ref)[axis])
    rel, zero = per_level_errors(g, r)
    assert (zero == 0).all()
    return float(np.nanmax(rel)) if np.isfinite(rel).any() else 0.0


def test_golden_vectors_within_1e6(gpu):
    """Every golden case (flang build of mappm.f90), kord x iv x field: kord <= 7 within
    1e-6 per level (measured 3.4e-7), kord > 7 bit-identical (the exact path)."""
    from fv3net_amd.mappm import mappm_device

    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    worst = 0.0
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = mappm_device(pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord)).cpu().numpy()
                    exp = g[f"c{ci}_{qn}_k{kord}_iv{iv}"]
                    if kord > 7:
                        assert (res.view(np.uint32) == exp.view(np.uint32)).all(), (ci, qn, kord, iv)
                    else:
                        e = _rel(res, exp)
                        worst = max(worst, e)
                        assert e <= 1e-6, (ci, qn, kord, iv, e)
    assert worst > 0.0  # the fast path did run (it is not the exact kernel)
    for kord in (1, 10):
        res = mappm_device(g["c12_pe1"], g["c12_q"], g["c12_pe2"], 1, kord).cpu().numpy()
        assert_per_level(res.T, g[f"c12_k{kord}_iv1"].T, 1e-6, f"C12 kord {kord}")


def test_f2py_mirror_is_exact(gpu):
    """mappm.mappm (the f2py signature) keeps the reference's arithmetic: a NaN column
    gives NaN as in test_mappm.py:33-44, and golden vectors come back bit for bit."""
    from fv3net_amd import mappm as M

    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    r = M.mappm(g["c12_pe1"].T, g["c12_q"].T, g["c12_pe2"].T, 1, g["c12_pe1"].shape[1], 1, 1, 0.0)
    assert (r.T.view(np.uint32) == g["c12_k1_iv1"].view(np.uint32)).all()


@pytest.mark.parametrize("kord", [1, 4, 6, 7])
@pytest.mark.parametrize("iv", [-1, 0, 1, 2])
def test_random_columns_vs_oracle(gpu, kord, iv):
    """Rough random columns (values over 7 decades, overhanging output edges) through
    every kord <= 7 x iv: within 1e-5 per level of the C restatement (bit-exact to the
    reference, tests/test_mappm_oracle.py)."""
    from fv3net_amd.mappm import mappm_device

    rng = np.random.default_rng(100 + 10 * kord + iv)
    km, kn, ncol = 79, 50, 2000
    delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
    q = (250 + rng.normal(0, 10, (km, ncol))).astype(np.float32)
    res = mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()
    assert_per_level(res.T, oracle_mappm(pe1, q, pe2, iv, kord).T, 1e-5, f"kord {kord} iv {iv}")


@pytest.mark.parametrize("kord", [1, 10])
def test_c384_grid_vs_exact(gpu, kord):
    """The bench's config #3 columns (C384, 884,736 columns, 79 -> 79): the default
    arithmetic against the exact kernel over the whole grid (kord 1 measured 4.2e-7 per
    level with no flip; kord 10 runs exact: identical)."""
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.mappm import mappm_device

    wl = W.make_mappm_workload(W.c_columns(384), 79, 79, kord, seed=5, device=torch.device("cuda", 0))
    fast = mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord)
    exact = mappm_device(wl.pe1, wl.q1, wl.pe2, 1, kord, exact=True)
    rel = (fast.double() - exact.double()).abs() / exact.double().abs().amax(1, keepdim=True)
    if kord > 7:
        assert rel.max().item() == 0.0
    else:  # flips as in test_coarsen_c384_vs_exact: counted, at most 2 of 69.9 M values
        assert int((rel > 1e-5).sum()) <= 2 and rel.max().item() <= 1e-3
        assert 0.0 < rel[rel <= 1e-5].max().item() <= 1e-6


def test_pairs_and_split_lanes_vs_single(gpu):
    """Two fields per pass (mappm_device_multi) and the two- and three-lane kernels the
    host picks by size: within 1e-6 per level of the single-field fast kernel."""
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.mappm import mappm_device, mappm_device_multi

    dev = torch.device("cuda", 0)
    for ncol in (13824, 65536, 110592, 200000):  # levels / three / two lanes / one lane
        wl = W.make_mappm_workload(ncol, 79, 79, 1, seed=ncol, device=dev)
        t = wl.q1 * 0.5 + 3.0
        outs = mappm_device_multi(wl.pe1, [wl.q1, t], wl.pe2, 1, 1)
        for q, o in zip((wl.q1, t), outs):
            ref = mappm_device(wl.pe1, q, wl.pe2, 1, 1, exact=True)
            err = ((o.double() - ref.double()).abs().amax(1) / ref.double().abs().amax(1)).max().item()
            assert err <= 1e-5, (ncol, err)


@pytest.mark.parametrize("factor", [1, 2, 4, 8])
@pytest.mark.parametrize("nfields", [1, 3])
def test_coarsen_vs_oracle(gpu, factor, nfields):
    """The fused pressure-level coarsen under the default arithmetic against
    oracle/coarsen.py (bit-exact to the reference's numpy + mappm chain)."""
    from fv3net_amd.coarsen import coarsen_on_pressure

    rng = np.random.default_rng(7 * factor + nfields)
    n, km = 8 * factor, 79
    base = np.linspace(200, 1800, km)[None, :, None, None]
    delp = (base * rng.uniform(0.9, 1.1, (6, km, n, n))).astype(np.float32)
    delp[:, -4:] *= rng.uniform(0.3, 2.0, (6, 1, n, n)).astype(np.float32)
    area = rng.uniform(0.5, 1.0, (6, n, n)).astype(np.float32)
    fields = {f"f{i}": (250 + rng.normal(0, 10, (6, km, n, n))).astype(np.float32) for i in range(nfields)}
    got, dc = coarsen_on_pressure(delp, area, fields, factor)
    exp, exp_dc = OC.coarsen_on_pressure(delp, area, list(fields.values()), factor)
    assert (dc.cpu().numpy() == exp_dc).all()  # pass 1 (coarse delp) keeps the reference's arithmetic
    for (name, g), e in zip(got.items(), exp):
        assert _rel(g.cpu().numpy(), e, axis=1) <= 1e-5, name


@pytest.mark.parametrize("nfields", [1, 4])
def test_coarsen_c384_vs_exact(gpu, nfields):
    """Config #3 at full size (C384 -> C48, 1,092,096 coarse values per field): the
    default arithmetic against the exact kernel.  The reference's limiter flattens a
    layer when its dc is exactly 0 (ppm_limiters lmt 0, `dm == 0`); a layer whose dc
    sits within an ulp of that switch can take the other branch, which moves that one
    fine value by its curvature term.  Such flips are counted: at most 2 coarse values
    per field beyond 1e-5 of their level's scale (measured: 0 or 1), none beyond 1e-4,
    and every other value within 2e-6 (measured 1.6e-6)."""
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.coarsen import coarsen_on_pressure

    wl = W.make_coarsen_workload(384, 8, nfields, seed=7, device=torch.device("cuda", 0))
    fast, _ = coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8)
    exact, _ = coarsen_on_pressure(wl.delp, wl.area, wl.fields, 8, exact=True)
    for k in fast:
        f, e = fast[k].double(), exact[k].double()
        rel = (f - e).abs() / e.abs().amax((0, 2, 3), keepdim=True)
        flips = int((rel > 1e-5).sum())
        assert flips <= 2 and rel.max().item() <= 1e-4, (k, flips, rel.max().item())
        assert rel[rel <= 1e-5].max().item() <= 2e-6, k


@pytest.mark.parametrize("edge", ["x", "y"])
def test_coarsen_edges_vs_oracle(gpu, edge):
    from fv3net_amd.coarsen import coarsen_edges_on_pressure

    rng = np.random.default_rng(3 if edge == "x" else 4)
    n, km, f = 16, 79, 4
    base = np.linspace(200, 1800, km)[None, :, None, None]
    delp = (base * rng.uniform(0.9, 1.1, (6, km, n, n))).astype(np.float32)
    es = (6, n + 1, n) if edge == "x" else (6, n, n + 1)
    spacing = rng.uniform(0.5, 1.0, es).astype(np.float32)
    u = rng.normal(0, 10, (6, km) + es[1:]).astype(np.float32)
    got = coarsen_edges_on_pressure(delp, spacing, {"u": u}, f, edge)["u"].cpu().numpy()
    exp = OC.coarsen_edges_on_pressure(delp, spacing, [u], f, edge)[0]
    assert _rel(got, exp, axis=1) <= 1e-5


@pytest.mark.parametrize("tag,agrid", [("pressure-level-without-agrid-winds", False),
                                       ("pressure-level-with-agrid-winds", True)])
def test_restarts_reference_regression_data(gpu, tag, agrid):
    """Every variable of both reference regression files at the reference test's own
    tolerance (assert_allclose rtol 1e-5), on the default arithmetic."""
    from fv3net_amd.restarts import coarsen_restarts_on_pressure
    from tests.test_restarts import _check_against_reference, _expected, _golden, _to_np

    grid, restarts = OR.kat_inputs()
    got = _to_np(coarsen_restarts_on_pressure(2, grid, restarts, coarsen_agrid_winds=agrid))
    _check_against_reference(got, _expected(_golden(), tag))


def test_regrid_vertical_default_vs_oracle(gpu):
    """regridz.regrid_vertical (z last) on the default arithmetic: within 1e-6 per level
    of the oracle on rough columns, and exact=True bit-identical to it."""
    from fv3net_amd.coarsen import regrid_vertical

    rng = np.random.default_rng(31)
    km, kn = 79, 40
    delp = rng.uniform(1, 3000, (6, 8, km))
    p_in = 300 + np.concatenate([np.zeros((6, 8, 1)), np.cumsum(delp, -1)], -1)
    f_in = 250 + rng.normal(0, 10, (6, 8, km))
    p_out = np.sort(rng.uniform(p_in[..., :1] * 0.9, p_in[..., -1:] * 1.05, (6, 8, kn + 1)), -1)
    col = lambda a: np.ascontiguousarray(a.reshape(-1, a.shape[-1]).T).astype(np.float32)  # noqa: E731
    ref = oracle_mappm(col(p_in), col(f_in), col(p_out)).T.reshape(6, 8, kn)
    got = regrid_vertical(p_in, f_in, p_out).cpu().numpy()
    assert _rel(got, ref, axis=2) <= 1e-6
    exact = regrid_vertical(p_in, f_in, p_out, exact=True).cpu().numpy()
    assert (exact.view(np.uint32) == ref.view(np.uint32)).all()


def test_prepared_plans_default_arithmetic(gpu):
    """MappmPlan / MappmMultiPlan on their default arithmetic: bit-identical to
    mappm_device / mappm_device_multi on the same buffers (the same fast kernels), and
    exact=True bit-identical to the exact calls."""
    import torch

    from fv3net_amd.mappm import MappmMultiPlan, MappmPlan, mappm_device, mappm_device_multi

    rng = np.random.default_rng(32)
    km, kn, ncol = 79, 79, 30000
    delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    pe2 = np.sort(rng.uniform(pe1[0] * 0.9, pe1[-1] * 1.05, (kn + 1, ncol)), 0).astype(np.float32)
    qa = (250 + rng.normal(0, 10, (km, ncol))).astype(np.float32)
    qb = (rng.normal(0, 1e-3, (km, ncol))).astype(np.float32)
    d1, da, db, d2 = (torch.from_numpy(a).cuda() for a in (pe1, qa, qb, pe2))
    eq = lambda x, y: torch.equal(x.view(torch.int32), y.view(torch.int32))  # noqa: E731
    for exact in (False, True):
        assert eq(MappmPlan(d1, da, d2, 1, 1, exact=exact)(), mappm_device(d1, da, d2, 1, 1, exact=exact))
        outs = MappmMultiPlan(d1, [da, db], d2, 1, 1, exact=exact)()
        want = mappm_device_multi(d1, [da, db], d2, 1, 1, exact=exact)
        assert all(eq(o, w) for o, w in zip(outs, want))
    fast = mappm_device(d1, da, d2, 1, 1)
    ref = mappm_device(d1, da, d2, 1, 1, exact=True)
    assert not torch.equal(fast, ref)  # the default is the fast kernel
    assert ((fast.double() - ref.double()).abs().amax(1) / ref.double().abs().amax(1)).max().item() <= 1e-6
