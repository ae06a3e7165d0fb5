"""GPU parity tests for the HIP mappm (through the C ABI) against the reference
golden vectors (flang build of mappm.f90) and the C oracle.  Bar: bit-exact.

Reference: external/mappm/mappm/mappm.f90:10-126; KATs external/vcm/tests/test_mappm.py.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, require_variant_kernels, set_variant
from oracle.mappm import oracle_mappm

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["serial", "levels"])
def mappm_path(request, monkeypatch):
    """Every test runs on both kord <= 7 kernels: one lane per column (`serial`) and
    one block per column, one lane per level (`levels`, the small-ncol default)."""
    set_variant(monkeypatch, "FV3_MAPPM_PATH", request.param)
    return request.param


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return bool(same.all())


def test_reference_kats_through_f2py_signature(gpu):
    from fv3net_amd import mappm as mappm_mod

    # test_mappm.py:5-16
    r = mappm_mod.mappm(np.asarray([0.0, 1.0, 2.0, 3.0, 4.0, 5.0])[None, :],
                        np.asarray([0.0, 1.0, 2.0, 3.0, 4.0])[None, :],
                        np.asarray([0.5, 1.2, 2.4, 2.8, 3.2, 4.5])[None, :], 1, 1.0, 1.0, 1.0, 0.0)
    assert r.dtype == np.float32 and r.shape == (1, 5)
    np.testing.assert_almost_equal(r, np.asarray([[0.35, 1.3, 2.1, 2.5, 3.35]], np.float32), decimal=5)
    # test_mappm.py:19-30
    r = mappm_mod.mappm(np.asarray([1.0, 2.0, 3.0, 4.0, 5.0])[None, :],
                        np.asarray([1.5, 2.5, 3.5, 4.5])[None, :],
                        np.asarray([0.0, 2.5, 3.5, 4.5, 50.0])[None, :], 1, 1.0, 1.0, 1.0, 0.0)
    np.testing.assert_almost_equal(r, np.asarray([[1.5, 3.0, 4.0, 4.502747]], np.float32), decimal=5)
    # test_mappm.py:33-44
    r = mappm_mod.mappm(np.asarray([1.0, 2.0, 3.0, 2.0, 5.0])[None, :],
                        np.asarray([np.nan] * 4)[None, :],
                        np.asarray([0.0, 2.5, 3.5, 4.5, 50.0])[None, :], 1, 1.0, 1.0, 1.0, 0.0)
    assert np.isnan(r).all()


def test_golden_vectors_bit_exact(gpu):
    from tests.remap_exact import mappm_device

    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = mappm_device(pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord)).cpu().numpy()
                    assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv)
    for kord in (1, 10):
        res = mappm_device(g["c12_pe1"], g["c12_q"], g["c12_pe2"], 1, kord).cpu().numpy()
        assert _bits_equal(res, g[f"c12_k{kord}_iv1"])


def _columns(rng, km, kn, ncol):
    delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
    m = min(km, kn) + 1
    pe2[: m // 2] = pe1[: m // 2]
    pe2 = np.sort(pe2, 0)
    q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
    return pe1, q, pe2


@pytest.mark.parametrize("km,kn,ncol", [(4, 3, 1), (5, 9, 257), (79, 50, 1000), (79, 79, 777), (127, 40, 300)])
def test_random_vs_oracle_bit_exact(gpu, km, kn, ncol):
    from tests.remap_exact import mappm_device

    rng = np.random.default_rng(km + kn + ncol)
    pe1, q, pe2 = _columns(rng, km, kn, ncol)
    for kord in (1, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17):
        for iv in (0, 1, -1, 2):
            res = mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()
            assert _bits_equal(res, oracle_mappm(pe1, q, pe2, iv, kord)), (kord, iv)


@pytest.mark.parametrize("km,kn,ncol", [(5, 9, 257), (79, 79, 777), (127, 40, 300)])
def test_cs_lds_path_vs_oracle_bit_exact(gpu, km, kn, ncol, monkeypatch):
    """kord > 7 with the edge-solve scratch in LDS (FV3_MAPPM_LDS=1) instead of the
    default global scratch: the same arithmetic, bit-identical."""
    from tests.remap_exact import mappm_device

    require_variant_kernels()
    set_variant(monkeypatch, "FV3_MAPPM_LDS", "1")
    rng = np.random.default_rng(km * kn + ncol)
    pe1, q, pe2 = _columns(rng, km, kn, ncol)
    for kord in (8, 10, 13, 17):
        for iv in (0, 1, -1, 2):
            res = mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()
            assert _bits_equal(res, oracle_mappm(pe1, q, pe2, iv, kord)), (kord, iv)


@pytest.mark.parametrize("nt,pf,c32,kspec", [(0, 0, 0, 1), (0, 2, 0, 1), (0, 0, 1, 1), (0, 2, 1, 1), (0, 4, 1, 1),
                                              (0, 8, 1, 1), (48, 0, 1, 1), (48, 8, 1, 1), (48, 4, 1, 1),
                                              (48, 4, 1, 0), (48, 4, 0, 1)])
def test_cs_kernel_variants_vs_oracle_bit_exact(gpu, nt, pf, c32, kspec, monkeypatch, mappm_path):
    """Every build of the global-scratch kord > 7 kernel: register tail depth NT, load
    distance PF (two register sets of PF levels in the solve), buffer operations at 32-bit
    offsets or 64-bit addresses, the column specialised for kord 10 (the default load
    distances with buffer operations) or not: the same bits as the oracle, on level counts
    around the blocks' remainders."""
    from tests.remap_exact import mappm_device

    if mappm_path != "serial":
        pytest.skip("kord > 7 has one kernel family; run once")
    if pf != 4 or nt not in (0, 48):  # the product keeps PF 4 at NT 0 / 48
        require_variant_kernels()
    set_variant(monkeypatch, "FV3_MAPPM_CS_NT", str(nt))
    set_variant(monkeypatch, "FV3_MAPPM_CS_PF", str(pf))
    set_variant(monkeypatch, "FV3_MAPPM_CS_C32", str(c32))
    set_variant(monkeypatch, "FV3_MAPPM_CS_KORD", str(kspec))
    for km, kn, ncol in ((5, 9, 257), (17, 12, 333), (50, 60, 300), (79, 79, 777), (127, 40, 300)):
        rng = np.random.default_rng(km * 31 + kn + ncol + pf)
        pe1, q, pe2 = _columns(rng, km, kn, ncol)
        for kord in (8, 9, 10, 11, 12, 13, 14, 15, 16, 17):
            for iv in (0, 1, -1, 2):
                res = mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()
                assert _bits_equal(res, oracle_mappm(pe1, q, pe2, iv, kord)), (km, kn, kord, iv)


def test_c384_scale_kord10_sampled_bit_exact(gpu):
    """config #3's kord 10 leg at its C384 size (884,736 columns, 79->79) through the
    default (global-scratch) kernel: the first / last wave and 4,096 sampled columns
    bit-exact against the oracle."""
    import torch

    from tests.remap_exact import mappm_device

    rng = np.random.default_rng(3841)
    ncol, km = 6 * 384 * 384, 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    delp = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    d2 = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
    pe2 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(d2, 0, dtype=np.float32)])
    q = rng.normal(250, 10, (km, ncol)).astype(np.float32)
    res = mappm_device(pe1, q, pe2, 1, 10)
    torch.cuda.synchronize()
    res = res.cpu().numpy()
    assert np.isfinite(res).all()
    idx = np.sort(np.concatenate([np.arange(64), rng.choice(ncol, 4096, replace=False), np.arange(ncol - 64, ncol)]))
    idx = np.unique(idx)
    ref = oracle_mappm(pe1[:, idx], q[:, idx], pe2[:, idx], 1, 10)
    assert _bits_equal(res[:, idx], ref)


def test_tile_layout_in_place(gpu):
    """(tile, z, y, x) restart-shaped arrays remapped in place via fv3_mappm_ex."""
    import torch

    from fv3net_amd import _device, _native

    rng = np.random.default_rng(7)
    ntile, km, ny, nx = 6, 79, 12, 12
    ncol = ntile * ny * nx
    pe1, q, pe2 = _columns(rng, km, km, ncol)
    # [lev, ncol] -> (tile, lev, y, x)
    to_t = lambda a: np.ascontiguousarray(a.reshape(a.shape[0], ntile, ny * nx).transpose(1, 0, 2)
                                          .reshape(ntile, a.shape[0], ny, nx))
    dev = [_device.to_device_f32(to_t(a)) for a in (pe1, q, pe2)]
    out = torch.empty((ntile, km, ny, nx), dtype=torch.float32, device="cuda")
    lays = [_device.level_layout(t, 1)[0] for t in dev + [out]]
    lib = _native.load()
    st = lib.fv3_mappm_ex(dev[0].data_ptr(), lays[0], dev[1].data_ptr(), lays[1], dev[2].data_ptr(), lays[2],
                          out.data_ptr(), lays[3], ncol, km, km, 1, 1, 0.0, _native.ARITH_EXACT,
                          _device.stream_handle())
    _native.check(st)
    got = out.cpu().numpy().reshape(ntile, km, ny * nx).transpose(1, 0, 2).reshape(km, ncol)
    assert _bits_equal(got, oracle_mappm(pe1, q, pe2, 1, 1))


def test_empty_and_errors(gpu):
    import torch

    from tests.remap_exact import mappm_device

    e = mappm_device(np.zeros((80, 0)), np.zeros((79, 0)), np.zeros((51, 0)))
    assert tuple(e.shape) == (50, 0)
    with pytest.raises(ValueError, match="one shorter"):
        mappm_device(np.zeros((80, 3)), np.zeros((78, 3)), np.zeros((51, 3)))
    with pytest.raises(ValueError, match="same size"):
        mappm_device(np.zeros((80, 3)), np.zeros((79, 3)), np.zeros((51, 4)))
    with pytest.raises(ValueError, match="km must be >= 4"):
        mappm_device(np.zeros((4, 3)), np.zeros((3, 3)), np.zeros((4, 3)))
    torch.cuda.synchronize()


def test_c384_scale_sampled_bit_exact(gpu):
    """BASELINE config #3 size (6*384*384 fine columns, 79->79): sampled columns
    bit-exact against the oracle, plus whole-array finiteness."""
    import torch

    from tests.remap_exact import mappm_device

    rng = np.random.default_rng(384)
    ncol, km = 6 * 384 * 384, 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    delp = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    d2 = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
    pe2 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(d2, 0, dtype=np.float32)])
    q = rng.normal(250, 10, (km, ncol)).astype(np.float32)
    res = mappm_device(pe1, q, pe2, 1, 1)
    torch.cuda.synchronize()
    res = res.cpu().numpy()
    assert np.isfinite(res).all()
    idx = np.sort(rng.choice(ncol, 4096, replace=False))
    ref = oracle_mappm(pe1[:, idx], q[:, idx], pe2[:, idx], 1, 1)
    assert _bits_equal(res[:, idx], ref)


def test_unsorted_edges_fall_back_per_column(gpu, monkeypatch):
    """Columns whose pe1 or pe2 are not non-decreasing (or hold NaN) take the serial
    streaming code inside the level-parallel kernel; sorted neighbours in the same launch
    do not.  Both kernels agree bit for bit.  A negative layer thickness with sorted pe2
    also matches the oracle; out-of-order or NaN pe2 hits the reference's failed search
    (mappm.f90:58-124 leaves q2 undefined), where the product writes NaN, so there only
    the two kernels are compared."""

    from tests.remap_exact import mappm_device

    rng = np.random.default_rng(5)
    km, kn, ncol = 79, 50, 300
    pe1, q, pe2 = _columns(rng, km, kn, ncol)
    pe1[40, 1::7] = pe1[39, 1::7] - 5  # a negative layer thickness
    bad2 = pe2.copy()
    bad2[10, ::3] = bad2[20, ::3]      # pe2 out of order in every third column
    bad2[5, 2::11] = np.nan
    for kord in (1, 4, 6, 7):
        for iv in (0, 1, -1):
            for p2, vs_oracle in ((pe2, True), (bad2, False)):
                set_variant(monkeypatch, "FV3_MAPPM_PATH", "levels")
                a = mappm_device(pe1, q, p2, iv, kord).cpu().numpy()
                set_variant(monkeypatch, "FV3_MAPPM_PATH", "serial")
                b = mappm_device(pe1, q, p2, iv, kord).cpu().numpy()
                assert _bits_equal(a, b), (kord, iv, vs_oracle)
                if vs_oracle:
                    assert _bits_equal(a, oracle_mappm(pe1, q, p2, iv, kord)), (kord, iv)


def test_prepared_plan_matches_and_tracks_contents(gpu):
    """MappmPlan re-issues the same call on the same buffers: bit-identical to
    mappm_device, and it sees in-place updates of the inputs."""
    import torch

    from tests.remap_exact import MappmPlan, mappm_device

    rng = np.random.default_rng(21)
    pe1, q, pe2 = _columns(rng, 79, 50, 864)
    d = [torch.from_numpy(a).cuda() for a in (pe1, q, pe2)]
    plan = MappmPlan(*d, 1, 4)
    assert _bits_equal(plan().cpu().numpy(), oracle_mappm(pe1, q, pe2, 1, 4))
    d[1].mul_(2.0)
    got = plan().cpu().numpy()
    assert _bits_equal(got, mappm_device(*d, 1, 4).cpu().numpy())
    assert _bits_equal(got, oracle_mappm(pe1, q * 2, pe2, 1, 4))


def test_prepared_plan_refuses_copies(gpu):
    """A plan bound to a copy (float64 input, host array) would keep remapping a stale
    snapshot: MappmPlan refuses it."""
    import torch

    from tests.remap_exact import MappmPlan

    rng = np.random.default_rng(22)
    pe1, q, pe2 = _columns(rng, 79, 50, 64)
    d = [torch.from_numpy(a).cuda() for a in (pe1, q, pe2)]
    with pytest.raises(ValueError, match="copy"):
        MappmPlan(d[0], d[1].double(), d[2], 1, 1)
    with pytest.raises(ValueError, match="copy"):
        MappmPlan(d[0], q, d[2], 1, 1)


def test_f2py_signature_column_count(gpu):
    """pe1(i1:i2, km+1): the arrays hold exactly columns i1..i2 (f2py), so any
    i1 > 1 call passes i2-i1+1 columns; a mismatch is an error, not a silent slice."""
    from fv3net_amd import mappm as mappm_mod

    rng = np.random.default_rng(23)
    pe1, q, pe2 = _columns(rng, 79, 50, 10)
    full = mappm_mod.mappm(pe1.T, q.T, pe2.T, 1, 10, 1, 1, 0.0)
    part = mappm_mod.mappm(pe1.T[3:7], q.T[3:7], pe2.T[3:7], 4, 7, 1, 1, 0.0)
    assert _bits_equal(part, full[3:7])
    with pytest.raises(ValueError, match="columns"):
        mappm_mod.mappm(pe1.T, q.T, pe2.T, 4, 7, 1, 1, 0.0)
