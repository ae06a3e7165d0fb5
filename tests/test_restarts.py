"""coarsen_restarts_on_pressure: the whole fv_core / fv_tracer /
fv_srf_wnd output against the reference's regression data, and the device path
against the oracle.

Reference KAT: external/vcm/tests/test_coarsen_restarts.py:103-122 (tags
"pressure-level-with-agrid-winds" and "pressure-level-without-agrid-winds"), data
_coarsen_restarts_regression_tests/reference/*.json (values in
tests/golden/restarts_kat.npz, tests/golden/make_golden.py --restarts-kat).  Inputs are
regenerated as external/synth does (oracle/restarts.py kat_inputs).  Tolerance: the
reference test's xarray.testing.assert_allclose defaults, rtol 1e-5, atol 1e-8.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import coarsen as OC
from oracle import restarts as OR

TAGS = [("pressure-level-without-agrid-winds", False), ("pressure-level-with-agrid-winds", True)]
# log() enters DZ and phis through hydrostatic_dz: the device libm and numpy's may differ
# in the last ulp, so those two are compared to the oracle at 1e-12, everything else bitwise
LOG_VARS = {("fv_core.res", "DZ"), ("fv_core.res", "phis")}


def _golden():
    return np.load(os.path.join(GOLDEN, "restarts_kat.npz"))


def _expected(g, tag):
    out = {}
    for k in g.files:
        if k.startswith(tag + "/") and not k.endswith("/dims"):
            _, cat, name = k.split("/")
            out.setdefault(cat, {})[name] = g[k]
    return out


def _check_against_reference(result, expected):
    assert sorted(result) == sorted(expected)
    for cat, names in expected.items():
        assert sorted(result[cat]) == sorted(names), cat
        for name, e in names.items():
            got = np.asarray(result[cat][name])
            assert got.shape == e.shape, (cat, name, got.shape, e.shape)
            np.testing.assert_allclose(got, e, rtol=1e-5, atol=1e-8, err_msg=f"{cat}/{name}")


@pytest.mark.parametrize("tag,agrid", TAGS)
def test_oracle_matches_reference_regression_data(tag, agrid):
    grid, restarts = OR.kat_inputs()
    result = OR.coarsen_restarts_on_pressure(2, grid, restarts, agrid)
    _check_against_reference(result, _expected(_golden(), tag))


def test_oracle_tracer_set_is_the_reference_list():
    """_coarse_grain_fv_tracer_on_pressure (coarsen_restarts.py:859-887) returns exactly
    FRACTION_TRACERS + NON_FRACTION_TRACERS: an extra tracer is dropped, a missing one
    is a KeyError."""
    grid, restarts = OR.kat_inputs()
    extra = dict(restarts["fv_tracer.res"], extra_tracer=restarts["fv_tracer.res"]["sphum"])
    result = OR.coarsen_restarts_on_pressure(2, grid, dict(restarts, **{"fv_tracer.res": extra}))
    assert list(result["fv_tracer.res"]) == OR.FRACTION_TRACERS + OR.NON_FRACTION_TRACERS
    short = {k: v for k, v in restarts["fv_tracer.res"].items() if k != "o3mr"}
    with pytest.raises(KeyError):
        OR.coarsen_restarts_on_pressure(2, grid, dict(restarts, **{"fv_tracer.res": short}))


@pytest.mark.gpu
def test_device_tracer_set_is_the_reference_list(gpu):
    from tests.remap_exact import FRACTION_TRACERS, NON_FRACTION_TRACERS, coarsen_restarts_on_pressure

    grid, restarts = OR.kat_inputs()
    extra = dict(restarts["fv_tracer.res"], extra_tracer=restarts["fv_tracer.res"]["sphum"])
    result = coarsen_restarts_on_pressure(2, grid, dict(restarts, **{"fv_tracer.res": extra}))
    assert list(result["fv_tracer.res"]) == FRACTION_TRACERS + NON_FRACTION_TRACERS
    short = {k: v for k, v in restarts["fv_tracer.res"].items() if k != "o3mr"}
    with pytest.raises(KeyError):
        coarsen_restarts_on_pressure(2, grid, dict(restarts, **{"fv_tracer.res": short}))


def test_oracle_hydrostatic_dz_closed_form():
    """hydrostatic_dz on an isothermal dry column: dz = -Rd T / g * log(p[k+1]/p[k])."""
    delp = np.full((1, 5, 1, 1), 1000.0)
    T = np.full((1, 5, 1, 1), 250.0, np.float32)
    q = np.zeros_like(T)
    dz = OR.hydrostatic_dz(T, q, delp)
    p = 300.0 + 1000.0 * np.arange(6)
    np.testing.assert_allclose(dz[0, :, 0, 0], -OR.RDGAS * 250.0 / OR.GRAVITY * np.diff(np.log(p)), rtol=1e-14)


def _to_np(result):
    return {cat: {n: t.cpu().numpy() for n, t in d.items()} for cat, d in result.items()}


def _compare_to_oracle(got, ref):
    for cat, names in ref.items():
        for name, r in names.items():
            g = got[cat][name]
            assert g.dtype == r.dtype and g.shape == r.shape, (cat, name, g.dtype, r.dtype, g.shape, r.shape)
            if (cat, name) in LOG_VARS:
                np.testing.assert_allclose(g, r, rtol=1e-12, atol=0, err_msg=f"{cat}/{name}")
            else:
                bad = ~((g == r) | (np.isnan(g) & np.isnan(r)))
                assert not bad.any(), f"{cat}/{name}: {bad.sum()} of {bad.size} differ"


@pytest.mark.gpu
@pytest.mark.parametrize("tag,agrid", TAGS)
def test_device_matches_reference_regression_data(gpu, tag, agrid):
    """Every variable of both regression files, at the reference test's tolerance, and
    the device result against the oracle (bitwise except the log-based DZ / phis)."""
    from tests.remap_exact import coarsen_restarts_on_pressure

    grid, restarts = OR.kat_inputs()
    got = _to_np(coarsen_restarts_on_pressure(2, grid, restarts, coarsen_agrid_winds=agrid))
    _check_against_reference(got, _expected(_golden(), tag))
    _compare_to_oracle(got, OR.coarsen_restarts_on_pressure(2, grid, restarts, agrid))


def _random_restarts(rng, n, km, with_time):
    base = np.linspace(200, 1800, km)[None, :, None, None]
    s3 = (6, km, n, n)
    core = {
        "delp": base * rng.uniform(0.9, 1.1, s3),
        "T": 250 + 30 * np.sin(np.arange(km) / 10.0)[None, :, None, None] + rng.normal(0, 1, s3),
        "W": rng.normal(0, 0.5, s3),
        "DZ": -np.linspace(2000, 20, km)[None, :, None, None] * rng.uniform(0.95, 1.05, s3),
        "phis": rng.uniform(0, 3e4, (6, n, n)),
        "u": rng.normal(0, 10, (6, km, n + 1, n)),
        "v": rng.normal(0, 10, (6, km, n, n + 1)),
        "ua": rng.normal(0, 10, s3),
        "va": rng.normal(0, 10, s3),
    }
    core["delp"][:, -4:] *= rng.uniform(0.3, 2.0, (6, 1, n, n))  # the mask drops fine columns near the surface
    tracer = {t: rng.uniform(0, 0.02, s3) for t in OR.NON_FRACTION_TRACERS + OR.FRACTION_TRACERS}
    srf = {"u_srf": rng.normal(0, 5, (6, n, n)), "v_srf": rng.normal(0, 5, (6, n, n))}
    grid = {"area": rng.uniform(0.5, 1.0, (6, n, n)).astype(np.float32),
            "dx": rng.uniform(0.5, 1.0, (6, n + 1, n)).astype(np.float32),
            "dy": rng.uniform(0.5, 1.0, (6, n, n + 1)).astype(np.float32)}
    restarts = {"fv_core.res": core, "fv_tracer.res": tracer, "fv_srf_wnd.res": srf}
    with_t = {c: {k: v[:, None] for k, v in d.items()} for c, d in restarts.items()}
    return grid, (with_t if with_time else restarts), with_t


@pytest.mark.gpu
@pytest.mark.parametrize("with_time", [True, False])
def test_device_matches_oracle_79_levels(gpu, with_time):
    """A C32 -> C8 (f = 4) 79-level restart set with strongly varying surface pressure:
    every output variable against the oracle; inputs with or without the Time axis."""
    import torch

    from tests.remap_exact import coarsen_restarts_on_pressure

    grid, restarts, with_t = _random_restarts(np.random.default_rng(32), 32, 79, with_time)
    got = coarsen_restarts_on_pressure(4, grid, restarts, coarsen_agrid_winds=True)
    torch.cuda.synchronize()
    got = _to_np(got)
    if not with_time:
        got = {c: {k: v[:, None] for k, v in d.items()} for c, d in got.items()}
    _compare_to_oracle(got, OR.coarsen_restarts_on_pressure(4, grid, with_t, True))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("factor", [1, 2, 3, 8])
def test_weighted_block_average_bitwise(gpu, dtype, factor):
    """fv3_weighted_block_average[_f64] vs numpy's nansum order, NaN inputs skipped."""
    from tests.remap_exact import weighted_block_average

    rng = np.random.default_rng(factor)
    n = 8 * factor
    obj3 = rng.normal(0, 100, (6, 5, n, n)).astype(dtype)
    obj3[0, 1, 0, 0] = np.nan
    obj2 = rng.normal(0, 100, (6, n, n)).astype(dtype)
    w = rng.uniform(0.5, 1.0, (6, n, n)).astype(np.float32)
    got = weighted_block_average({"a": obj3, "b": obj2}, w, factor)
    ra = OC.weighted_block_average(obj3, w[:, None], factor)
    rb = OC.weighted_block_average(obj2, w, factor)
    for g, r in ((got["a"], ra), (got["b"], rb)):
        g = g.cpu().numpy()
        assert g.dtype == r.dtype
        assert (g == r).all()


@pytest.mark.gpu
def test_errors_match_reference(gpu):
    from tests.remap_exact import coarsen_restarts_on_pressure

    grid, restarts = OR.kat_inputs()
    no_ua = dict(restarts)
    no_ua["fv_core.res"] = {k: v for k, v in restarts["fv_core.res"].items() if k != "ua"}
    with pytest.raises(ValueError, match="'ua' and 'va'"):
        coarsen_restarts_on_pressure(2, grid, no_ua, coarsen_agrid_winds=True)
    with pytest.raises(NotImplementedError, match="sfc_data"):
        coarsen_restarts_on_pressure(2, grid, dict(restarts, sfc_data={}))
    with pytest.raises(ValueError):
        coarsen_restarts_on_pressure(3, grid, restarts)
