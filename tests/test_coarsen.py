"""Pressure-level coarse-graining: oracle pinned by the reference's own regression
data, HIP kernel checked against the oracle and the same data.

Reference KAT: external/vcm/tests/test_coarsen_restarts.py:103-122 with
_coarsen_restarts_regression_tests/reference/pressure-level-without-agrid-winds-*.json
(values copied into tests/golden/coarsen_kat.npz by tests/golden/make_golden.py).
Inputs are regenerated as external/synth does (seed 0 per single-chunk variable):
delp ~ U(3,5) f8, area ~ U(0.5,1) f4, T/W/tracers ~ U(-1000,1000) f8, C4 -> C2, 7 levels.
Tolerance: xarray.testing.assert_allclose defaults (rtol 1e-5, atol 1e-8), as the
reference test uses (its comment: mappm is not bit-for-bit across platforms).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, set_variant
from oracle import coarsen as OC

FACTOR = 2


def _kat_inputs():
    shape = (6, 1, 7, 4, 4)  # fv_core.res-schema.json: (tile, Time, zaxis_1, yaxis_2, xaxis_1)
    delp = OC.synth_uniform(3, 5, shape, np.float64)[:, 0]
    T = OC.synth_uniform(-1000, 1000, shape, np.float64)[:, 0]
    area = OC.synth_uniform(0.5, 1, (6, 4, 4), np.float32)  # grid-schema.json area
    return delp, area, T


def _expected(name="fv_core.res/T"):
    g = np.load(os.path.join(GOLDEN, "coarsen_kat.npz"))
    return g[name][:, 0]  # drop Time


def test_oracle_reproduces_reference_kat():
    delp, area, T = _kat_inputs()
    (Tc,), _ = OC.coarsen_on_pressure(delp, area, [T], FACTOR)
    np.testing.assert_allclose(Tc, _expected(), rtol=1e-5, atol=1e-8)


def test_kat_tracers_share_the_t_path():
    """All tracers (and W) are generated from the same seed/range as T, so the
    reference's coarse tracers equal its coarse T: the JSON must agree with itself."""
    g = np.load(os.path.join(GOLDEN, "coarsen_kat.npz"))
    ref = g["fv_core.res/T"]
    for k in g.files:
        if k.endswith("/dims") or k == "fv_core.res/T":
            continue
        np.testing.assert_allclose(g[k], ref, rtol=1e-6)


def test_oracle_block_average_kat():
    """test_cubedsphere.py:207-236 weighted_block_average KAT: constant 3 -> 3."""
    obj = np.full((1, 4, 4), 3.0)
    w = np.random.default_rng(0).uniform(0.5, 1.0, (1, 4, 4))
    np.testing.assert_allclose(OC.weighted_block_average(obj, w, 2), np.full((1, 2, 2), 3.0))


def test_oracle_mask_weights_kat():
    """test_regridz.py:113-129 _mask_weights KAT (as (tile, z, y, x) with x singleton)."""
    weights = np.arange(4, dtype=np.float32).reshape(2, 2)[:, :, None]  # (x=2 -> tile, y=2, x=1)
    pc = np.zeros((2, 3, 2, 1), np.float32)
    pf = np.zeros((2, 3, 2, 1), np.float32)
    pc[:, 0], pc[:, 1], pc[:, 2] = 1.0, 2.0, 3.0
    pf[:, 0], pf[:, 1] = 1.0, 2.0
    pf[0, 2], pf[1, 2] = 2.5, 3.5
    got = OC.mask_weights(weights, pc, pf)
    expected = np.broadcast_to(weights[:, None], (2, 2, 2, 1)).copy()
    expected[0, 1] = 0.0
    np.testing.assert_allclose(got, expected)


def _bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    assert a.shape == b.shape
    bad = a.view(np.uint32) != b.view(np.uint32)
    assert not bad.any(), f"{bad.sum()} / {bad.size} differ, e.g. {a[bad][:4]} vs {b[bad][:4]}"


@pytest.mark.gpu
def test_kernel_reproduces_reference_kat(gpu):
    """float64 delp (as in the restart files): within the reference test's own
    tolerance of its regression data, and bit-identical to the oracle."""
    from tests.remap_exact import coarsen_on_pressure

    delp, area, T = _kat_inputs()
    out, delp_c = coarsen_on_pressure(delp, area, {"T": T, "W": T}, FACTOR)
    got = out["T"].cpu().numpy()
    np.testing.assert_allclose(got, _expected(), rtol=1e-5, atol=1e-8)
    np.testing.assert_array_equal(got, out["W"].cpu().numpy())
    (ref,), ref_dc = OC.coarsen_on_pressure(delp, area, [T], FACTOR)
    _bits_equal(got, ref)
    _bits_equal(delp_c.cpu().numpy(), ref_dc)


def _smooth_state(rng, nt, km, ny, nx):
    base = np.linspace(200, 1800, km)[None, :, None, None]
    delp = (base * rng.uniform(0.95, 1.05, (nt, km, ny, nx))).astype(np.float32)
    area = rng.uniform(0.5, 1.0, (nt, ny, nx)).astype(np.float32)
    T = (250 + 30 * np.sin(np.arange(km) / 10.0)[None, :, None, None]
         + rng.normal(0, 1, (nt, km, ny, nx))).astype(np.float32)
    q = rng.uniform(0, 0.02, (nt, km, ny, nx)).astype(np.float32)
    return delp, area, T, q


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["cells", "rows", "cursor"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("factor,n", [(1, 4), (2, 16), (3, 12), (4, 24), (8, 48)])
def test_kernel_vs_oracle_random(gpu, factor, n, dtype, path, monkeypatch):
    """Bit-identical to the oracle for every factor (numpy's block-sum order) and
    both delp dtypes (the arithmetic follows delp's dtype, as the reference does), on
    every kernel path (FV3_COARSEN_PATH): whole cells per wave with the per-wave output
    ring (default, f >= 2), f-wave row segments with a per-lane scratch column, and
    the row segments with the scratch-free output-driven cursor."""
    from tests.remap_exact import coarsen_on_pressure

    set_variant(monkeypatch, "FV3_COARSEN_PATH", path)

    rng = np.random.default_rng(factor * 100 + n)
    delp, area, T, q = _smooth_state(rng, 6, 79, n, n)
    delp = delp.astype(dtype)
    out, delp_c = coarsen_on_pressure(delp, area, {"T": T, "q": q}, factor)
    ref, ref_dc = OC.coarsen_on_pressure(delp, area, [T, q], factor)
    for name, r in zip(("T", "q"), ref):
        _bits_equal(out[name].cpu().numpy(), r)
    _bits_equal(delp_c.cpu().numpy(), ref_dc)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["cells", "rows"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_kernel_steep_cells_overflow_columns(gpu, path, dtype, monkeypatch):
    """Fine columns of one coarse cell with very different surface pressures (steep
    terrain: the lowest 40 of 79 layers scaled by 0.05 .. 4 per column), so within a
    cell some columns emit their remapped levels dozens of levels ahead of others: the
    cells path's per-wave ring (16 levels) overflows into the per-lane global columns.
    Still bit-identical to the oracle, on both paths."""
    from tests.remap_exact import coarsen_on_pressure

    set_variant(monkeypatch, "FV3_COARSEN_PATH", path)
    rng = np.random.default_rng(11)
    delp, area, T, q = _smooth_state(rng, 6, 79, 16, 16)
    delp[:, -40:] *= rng.uniform(0.05, 4.0, (6, 1, 16, 16)).astype(np.float32)
    delp = delp.astype(dtype)
    for f in (8, 4):
        out, delp_c = coarsen_on_pressure(delp, area, {"T": T, "q": q}, f)
        ref, ref_dc = OC.coarsen_on_pressure(delp, area, [T, q], f)
        for name, r in zip(("T", "q"), ref):
            _bits_equal(out[name].cpu().numpy(), r)
        _bits_equal(delp_c.cpu().numpy(), ref_dc)


@pytest.mark.gpu
def test_kernel_masked_levels_and_kord(gpu):
    """Strongly varying surface pressure so the mask drops fine columns at the lowest
    coarse levels; iv/kord variants of the PPM path; kord > 7 is refused loudly."""
    from tests.remap_exact import coarsen_on_pressure

    rng = np.random.default_rng(7)
    delp, area, T, q = _smooth_state(rng, 2, 40, 16, 16)
    delp[:, -5:] *= rng.uniform(0.2, 3.0, (2, 1, 16, 16)).astype(np.float32)
    for iv, kord in ((1, 1), (0, 4), (1, 6), (-1, 7)):
        out, _ = coarsen_on_pressure(delp, area, {"q": q}, 4, iv=iv, kord=kord)
        (r,), _ = OC.coarsen_on_pressure(delp, area, [q], 4, iv=iv, kord=kord)
        _bits_equal(out["q"].cpu().numpy(), r)
    with pytest.raises(NotImplementedError):
        coarsen_on_pressure(delp, area, {"q": q}, 4, kord=9)
    with pytest.raises(ValueError):
        coarsen_on_pressure(delp[..., :15], area[..., :15], {"q": q[..., :15]}, 4)


@pytest.mark.gpu
def test_kernel_c384_to_c48_sampled_and_deterministic(gpu):
    """BASELINE config #3 size: C384 -> C48, f = 8, 79 levels.  Deterministic across
    runs (fixed reduction order) and sampled tiles match the oracle."""
    import torch

    from tests.remap_exact import coarsen_on_pressure

    rng = np.random.default_rng(384)
    delp, area, T, _ = _smooth_state(rng, 6, 79, 384, 384)
    out1, _ = coarsen_on_pressure(delp, area, {"T": T}, 8)
    out2, _ = coarsen_on_pressure(delp, area, {"T": T}, 8)
    torch.cuda.synchronize()
    a, b = out1["T"].cpu().numpy(), out2["T"].cpu().numpy()
    assert (a.view(np.uint32) == b.view(np.uint32)).all()
    assert np.isfinite(a).all()
    sl = (slice(2, 3), slice(None), slice(64, 128), slice(192, 256))  # one tile, 8x8 coarse cells
    (r,), _ = OC.coarsen_on_pressure(delp[sl], area[2:3, 64:128, 192:256], [T[sl]], 8)
    _bits_equal(a[2:3, :, 8:16, 24:32], r)


def test_oracle_preserves_constant_fields():
    """A size-independent property (pinned here on the oracle): the pressure regrid of a
    constant profile is that constant (its PPM parabola is flat) and the area-weighted
    block average of a constant is that constant, to float32 rounding (measured 2.4e-7)."""
    rng = np.random.default_rng(5)
    delp, area, _, _ = _smooth_state(rng, 1, 79, 32, 32)
    for c in (273.15, 0.0123):
        (r,), _ = OC.coarsen_on_pressure(delp, area, [np.full_like(delp, c)], 8)
        assert np.isfinite(r).all()
        assert np.abs(r / np.float32(c) - 1).max() <= 1e-6


@pytest.mark.gpu
def test_kernel_c384_to_c48_constant_fields_preserved(gpu):
    """The same property at BASELINE config #3's full size (C384 -> C48, 79 levels), every
    coarse cell, with two fields in one call (the kernel's two-field pass)."""
    import torch

    from tests.remap_exact import coarsen_on_pressure

    rng = np.random.default_rng(3843)
    delp, area, _, _ = _smooth_state(rng, 6, 79, 384, 384)
    consts = {"T": 273.15, "q": 0.0123}
    fields = {k: np.full_like(delp, c) for k, c in consts.items()}
    out, _ = coarsen_on_pressure(delp, area, fields, 8)
    torch.cuda.synchronize()
    for k, c in consts.items():
        r = out[k].cpu().numpy()
        assert r.shape == (6, 79, 48, 48)
        assert np.isfinite(r).all(), k
        assert np.abs(r / np.float32(c) - 1).max() <= 1e-6, k


@pytest.mark.gpu
def test_regrid_vertical_device_matches_oracle(gpu):
    """regridz.regrid_vertical semantics (z last, new-nlevels, error paths)."""
    from tests.remap_exact import regrid_vertical
    from oracle.mappm import oracle_mappm

    rng = np.random.default_rng(1)
    p_in = np.sort(rng.uniform(0, 100, (4, 4, 6)), axis=-1)
    f_in = rng.normal(0, 1, (4, 4, 5))
    p_out = np.sort(rng.uniform(0, 100, (4, 4, 3)), axis=-1)
    got = regrid_vertical(p_in, f_in, p_out).cpu().numpy()
    assert got.shape == (4, 4, 2) and got.dtype == np.float32
    col = lambda a: a.reshape(-1, a.shape[-1]).T
    ref = oracle_mappm(col(p_in), col(f_in), col(p_out)).T.reshape(4, 4, 2)
    assert (got.view(np.uint32) == ref.view(np.uint32)).all()
    with pytest.raises(ValueError, match="one shorter"):
        regrid_vertical(p_in, f_in[..., :3], p_out)
    with pytest.raises(ValueError, match="same size"):
        regrid_vertical(p_in, f_in[:3], p_out)


@pytest.mark.gpu
def test_side_stream_host_and_float64_inputs(gpu):
    """``stream=`` with host float64 inputs: the device copies and the outputs are
    allocated on the current stream and used on the side stream, so they must be kept
    alive for it (record_stream).  Churning the allocator on the current stream while
    the side stream still runs must not change a bit of the results."""
    import torch

    from tests.remap_exact import coarsen_on_pressure
    from tests.remap_exact import weighted_block_average

    rng = np.random.default_rng(21)
    delp, area, T, q = _smooth_state(rng, 6, 79, 96, 96)
    ref, ref_dc = coarsen_on_pressure(delp.astype(np.float64), area, {"T": T.astype(np.float64), "q": q}, 8)
    wref = weighted_block_average({"T": T.astype(np.float64)}, area, 8)["T"]
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    for _ in range(3):
        out, dc = coarsen_on_pressure(delp.astype(np.float64), area, {"T": T.astype(np.float64), "q": q}, 8,
                                      stream=side)
        w = weighted_block_average({"T": T.astype(np.float64)}, area, 8, stream=side)["T"]
        # reuse whatever the caching allocator frees on the current stream
        junk = [torch.full((6, 79, 96, 96), float("nan"), device="cuda") for _ in range(4)]
        del junk
        side.synchronize()
        for k in ref:
            assert torch.equal(out[k], ref[k]), k
        assert torch.equal(dc, ref_dc) and torch.equal(w, wref)
