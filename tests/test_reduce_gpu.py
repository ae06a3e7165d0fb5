"""Reductions behind the stepper diagnostics (csrc/reduce.hip) vs float64 numpy."""
import ctypes

import numpy as np
import pytest

from fv3net_amd import dataset as DS


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 2304, 13824, 884736])
def test_area_weighted_partials(gpu, n):
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(n)
    x = rng.normal(0, 1, (3, n)).astype(np.float32)
    a = rng.uniform(0.5, 1, n).astype(np.float32)
    xt = [torch.from_numpy(v).cuda() for v in x]
    at = torch.from_numpy(a).cuda()
    p1 = D.area_weighted_partials(xt, at).cpu().numpy()
    p2 = D.area_weighted_partials(xt, at).cpu().numpy()
    assert (p1.view(np.uint64) == p2.view(np.uint64)).all()  # deterministic
    a64 = a.astype(np.float64)
    for d in range(3):
        np.testing.assert_allclose(p1[d, 0], np.sum(a64 * x[d].astype(np.float64)), rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(p1[d, 1], np.sum(a64), rtol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 300, 55296])
@pytest.mark.parametrize("n_diag", [1, 9, 17])
def test_area_weighted_partials_f64(gpu, n, n_diag):
    """float64 diagnostics (the stepper's dtype) run the float64 kernel, with an float32
    area widened exactly, as numpy's area * ds promotes; diags in chunks of 8."""
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(n + n_diag)
    x = rng.normal(0, 1, (n_diag, n)) * 10.0 ** rng.integers(-8, 3, (n_diag, 1))
    a = rng.uniform(0.5, 1, n).astype(np.float32)
    xt = [torch.from_numpy(v).cuda() for v in x]
    p1 = D.area_weighted_partials(xt, torch.from_numpy(a).cuda()).cpu().numpy()
    p2 = D.area_weighted_partials(xt, torch.from_numpy(a.astype(np.float64)).cuda()).cpu().numpy()
    assert (p1.view(np.uint64) == p2.view(np.uint64)).all()
    a64 = a.astype(np.float64)
    for d in range(n_diag):
        np.testing.assert_allclose(p1[d, 0], np.sum(a64 * x[d]), rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(p1[d, 1], np.sum(a64), rtol=1e-13)


@pytest.mark.gpu
def test_level_sums_on_views(gpu):
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(3)
    f = rng.normal(0, 1, (6, 79, 48, 48)).astype(np.float32)
    ft = torch.from_numpy(f).cuda()
    seg = D.Segment(2, 8, 20)
    got = D.level_sums(D.segment_view(ft, seg)).cpu().numpy()  # strided (z, rows, x) view in place
    ref = f[2, :, 8:20].astype(np.float64).sum(axis=(1, 2))
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-10)


@pytest.mark.gpu
def test_column_integral_matches_mass_integrate(gpu):
    """vcm.mass_integrate (vertically_dependent.py:18-22): sum_z x * delp / g."""
    import torch

    from fv3net_amd import _native

    rng = np.random.default_rng(4)
    x = rng.normal(0, 1e-4, (79, 48, 48)).astype(np.float32)
    dp = rng.uniform(200, 1800, (79, 48, 48)).astype(np.float32)
    xt, dt = torch.from_numpy(x).cuda(), torch.from_numpy(dp).cuda()
    out = torch.empty((48, 48), device="cuda")
    lay = _native.layout(2304, 2304, 79 * 2304)
    g = 9.80665
    st = _native.load().fv3_column_integral(xt.data_ptr(), lay, dt.data_ptr(), lay, out.data_ptr(), 2304, 79,
                                            1.0 / g, None)
    _native.check(st)
    ref = (x.astype(np.float64) * dp.astype(np.float64) / g).sum(axis=0)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_metrics_mirrors_single_rank(gpu):
    """globally_average_2d_diagnostics / globally_sum_3d_diagnostics (metrics.py:33-55)
    without a process group: 2-D (x, y) vars incl. area averaged, 3-D excluded."""
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(5)
    area = rng.uniform(0.5, 1, (12, 12)).astype(np.float32)
    pr = rng.normal(0, 1, (12, 12)).astype(np.float32)
    t3 = rng.normal(0, 1, (7, 12, 12)).astype(np.float32)
    diags = {"area": DS.DataArray(torch.from_numpy(area).cuda(), ["y", "x"]),
             "precip": DS.DataArray(torch.from_numpy(pr).cuda(), ["y", "x"]),
             "skip": DS.DataArray(torch.from_numpy(pr).cuda(), ["y", "x"]),
             "T": DS.DataArray(torch.from_numpy(t3).cuda(), ["z", "y", "x"])}
    avg = D.globally_average_2d_diagnostics(diags, exclude=["skip"])
    assert set(avg) == {"area", "precip"}
    a64 = area.astype(np.float64)
    np.testing.assert_allclose(avg["precip"], np.sum(a64 * pr) / np.sum(a64), rtol=1e-12)
    np.testing.assert_allclose(avg["area"], np.sum(a64 * a64) / np.sum(a64), rtol=1e-12)
    sums = D.globally_sum_3d_diagnostics(diags, include=["T"])
    np.testing.assert_allclose(sums["T_global_sum"], t3.astype(np.float64).sum(axis=(1, 2)), rtol=1e-12,
                               atol=1e-10)


@pytest.mark.gpu
def test_level_sums_keep_dtype(gpu):
    """float64 fields are summed without a float32 rounding and the uint8
    limiter flag is read in place; the sums equal numpy's in float64."""
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(9)
    f = rng.normal(0, 1, (79, 24, 24)) * (1 + 1e-9 * rng.normal(size=(79, 24, 24)))
    got = D.level_sums(torch.from_numpy(f).cuda()).cpu().numpy()
    np.testing.assert_allclose(got, f.sum(axis=(1, 2)), rtol=1e-13, atol=1e-12)
    flag = (rng.uniform(size=(79, 24, 24)) < 0.3).astype(np.uint8)
    got = D.level_sums(torch.from_numpy(flag).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, flag.sum(axis=(1, 2)).astype(np.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("ncol", [1, 15, 16, 17, 255, 6912, 6913, 32768, 40000, 100000])
def test_level_sums_u8_counts_exact(gpu, ncol):
    """uint8 level sums: one band in one launch (16-byte loads summed by v_sad_u8 when the
    rows are 16-byte aligned, the scalar kernel on a misaligned view), several slices past
    32,768 columns; arbitrary byte values, not only 0/1 flags: exact integers."""
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(ncol)
    v = rng.integers(0, 256, size=(9, ncol), dtype=np.uint8)
    t = torch.from_numpy(v).cuda()
    got = D.level_sums(t).cpu().numpy()
    np.testing.assert_array_equal(got, v.sum(axis=1, dtype=np.int64).astype(np.float64))
    if ncol > 1:  # a view starting one byte in: rows not 16-byte aligned
        got = D.level_sums(t[:, 1:]).cpu().numpy()
        np.testing.assert_array_equal(got, v[:, 1:].sum(axis=1, dtype=np.int64).astype(np.float64))
