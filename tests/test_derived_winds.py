"""vcm.DerivedMapping's D-grid wind rotation, wind-parallel projections and solar zenith
angle (derived_mapping.py:114-187, cubedsphere/rotate.py:9-56, coarsen.py:54-75,
calc/_zenith_angle.py) on csrc/derived.hip, against the numpy restatement in
oracle/derived.py, which the reference's own KATs pin (CPU tests below):
external/vcm/tests/test__rotate.py, test_derived_mapping.py:33-90 and
test__zenith_angle.py.
"""
import datetime

import numpy as np
import pytest

from fv3net_amd import dataset as D
from fv3net_amd import predictor as P
from oracle import derived as OD

NZ = 79
COEFFS = ("eastward_wind_u_coeff", "eastward_wind_v_coeff", "northward_wind_u_coeff", "northward_wind_v_coeff")


def _bits(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (what, a.shape, b.shape, a.dtype, b.dtype)
    u = np.uint64 if a.dtype.itemsize == 8 else np.uint32
    same = (a.view(u) == b.view(u)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{what}: {(~same).sum()} differ, e.g. {a[~same][:3]} vs {b[~same][:3]}"


# ----------------------------------------------------------- oracle vs reference KATs
def test_oracle_rotate_xy_winds_kat():
    """test__rotate.py:7-34: axes 45 degrees from x/y, unit x and y winds."""
    c = np.sqrt(2.0) / 2.0
    coeffs = [(np.array([[v]]), ("x", "y")) for v in (c, c, -c, c)]
    one = np.ones((2, 1, 1))
    east, north = OD.rotate_xy_winds(coeffs, one, one, ("time", "x", "y"))
    assert (east == np.sqrt(2.0)).all() and (north == 0.0).all()


def test_oracle_rotated_winds_zero_coefficients_kat():
    """test_derived_mapping.py:64-90: zero coefficients give zero winds and tendencies."""
    ny, nx = 1, 2
    coeffs = [(np.zeros((ny, nx)), ("y", "x"))] * 4
    (e, ed), (n, nd) = OD.center_and_rotate_xy_winds(coeffs, np.ones((ny + 1, nx)), ("y_interface", "x"),
                                                     np.ones((ny, nx + 1)), ("y", "x_interface"))
    assert ed == nd == ("y", "x") and e.shape == (ny, nx)
    np.testing.assert_array_almost_equal(0.0, e)
    np.testing.assert_array_almost_equal(0.0, n)
    with pytest.raises(ValueError, match="Variable to shift to center"):
        OD.shift_edge_var_to_center(np.ones((2, 2)), ("y", "x"))


# test_derived_mapping.py:33-58's five cases.  That test asserts
# ``pytest.approx(value, projection)``, an always-true approx object (the expected value
# passed as the tolerance), so its "projection" column pins nothing: the values below are
# what derived_mapping.py:177-187's expression gives (the norm is of both whole arrays).
PROJECTION_CASES = [(1.0, 0.0, 1.0, 0.0, 1.0), (1.0, 0.0, -1.0, 0.0, -1.0), (1.0, 1.0, 1.0, 1.0, np.sqrt(2)),
                    (1.0, 0.0, 1.0, 1.0, 1 / np.sqrt(2)), (-1.0, 0.0, 1.0, 1.0, -1 / np.sqrt(2))]


@pytest.mark.parametrize("dqu, dqv, east, north, projection", PROJECTION_CASES)
def test_oracle_horizontal_projection_kats(dqu, dqv, east, north, projection):
    a = lambda v: np.array([v])  # noqa: E731
    got = OD.horizontal_wind_tendency_parallel_to_horizontal_wind(a(east), a(dqu), a(north), a(dqv))
    assert got.item() == pytest.approx(projection, rel=1e-15)


ZENITH_KATS = [((2020, 3, 21, 12), 0.0, 0.0, 1.0), ((2020, 3, 21, 18), -90.0, 0.0, 1.0),
               ((2020, 3, 21, 18), 270.0, 0.0, 1.0), ((2020, 7, 6, 12), -90.0, 0.0, -0.0196310),
               ((2020, 7, 6, 9), 40.0, 40.0, 0.9501915), ((2020, 7, 6, 12), 0.0, 90.0, 0.3843733)]


@pytest.mark.parametrize("calendar", ["julian", "gregorian"])
@pytest.mark.parametrize("case", range(len(ZENITH_KATS)))
def test_oracle_zenith_kats(calendar, case):
    """test__zenith_angle.py:9-31 (abs 1e-3, both calendars)."""
    t, lon, lat, expected = ZENITH_KATS[case]
    time = OD.JulianDate(*t) if calendar == "julian" else datetime.datetime(*t)
    assert OD.cos_zenith_angle(time, lon, lat) == pytest.approx(expected, abs=1e-3)


class _NoLeap:  # a calendar the reference refuses (cftime.DatetimeNoLeap)
    def __init__(self, *a):
        pass


def test_zenith_invalid_calendar_raises():
    """test__zenith_angle.py:34-44, oracle and the product's host part."""
    from fv3net_amd.derived import solar_terms

    for bad in (_NoLeap(2000, 1, 1), np.array([_NoLeap(2000, 1, 1), _NoLeap(2000, 2, 1)])):
        with pytest.raises(ValueError, match="model_time has an invalid date type"):
            OD.cos_zenith_angle(bad, 0.0, 0.0)
        with pytest.raises(ValueError, match="model_time has an invalid date type"):
            solar_terms(bad)


def test_product_solar_terms_match_oracle():
    """The product's per-time factors (host numpy) are the oracle's, bit for bit, for
    Gregorian and Julian times (emulation.JulianTime stands in for cftime.DatetimeJulian)."""
    from fv3net_amd.derived import solar_terms
    from fv3net_amd.emulation import JulianTime

    greg = [datetime.datetime(1999, 12, 31, 3), datetime.datetime(2020, 7, 6, 9, 30, 15),
            datetime.datetime(2101, 2, 28, 23, 59, 59)]
    jul = [JulianTime(t.year, t.month, t.day, t.hour, t.minute, t.second) for t in greg]
    for times, types in ((greg, ()), (jul, (JulianTime,))):
        got = solar_terms(np.array(times, dtype=object))
        days = OD.days_from_2000(np.array(times, dtype=object), julian_types=types or (OD.JulianDate,))
        ra, dec = OD._right_ascension_declination(days)
        _bits(got, np.stack([OD._gmst(days), ra, np.sin(dec), np.cos(dec)]), "solar terms")


# ------------------------------------------------------------------------------ GPU
def _rotation_case(rng, wdt, cdts, tile=True, transposed=False, n=12, nz=7):
    """D-grid winds (tile, z, y_interface, x) / (tile, z, y, x_interface) and (tile, y, x)
    coefficients of the given dtypes; ``transposed``: the x wind as (x, y_interface, z, tile)."""
    lead = (("tile", 2),) if tile else ()
    xdims = tuple(d for d, _ in lead) + ("z", "y_interface", "x")
    ydims = tuple(d for d, _ in lead) + ("z", "y", "x_interface")
    xs = tuple(s for _, s in lead) + (nz, n + 1, n)
    ys = tuple(s for _, s in lead) + (nz, n, n + 1)
    x = rng.normal(0, 10, xs).astype(wdt[0])
    y = rng.normal(0, 10, ys).astype(wdt[1])
    x.flat[5] = np.nan
    cdims = tuple(d for d, _ in lead) + ("y", "x")
    cs = tuple(s for _, s in lead) + (n, n)
    coeffs = [rng.uniform(-1, 1, cs).astype(dt) for dt in cdts]
    if transposed:
        perm = list(reversed(range(len(xdims))))
        x = np.ascontiguousarray(np.transpose(x, perm))
        xdims = tuple(xdims[p] for p in perm)
    return (x, xdims), (y, ydims), [(c, cdims) for c in coeffs]


DTYPES = [((np.float64, np.float64), (np.float64,) * 4), ((np.float32, np.float32), (np.float32,) * 4),
          ((np.float32, np.float32), (np.float64,) * 4), ((np.float64, np.float32), (np.float32, np.float64) * 2),
          ((np.float32, np.float64), (np.float32,) * 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("dts", range(len(DTYPES)))
@pytest.mark.parametrize("layout", ["tile", "plain", "transposed"])
@pytest.mark.parametrize("device", [True, False])
def test_rotation_bitwise_vs_oracle(gpu, dts, layout, device):
    """dQu / dQv / eastward_wind / northward_wind through DerivedMapping: the fused
    centre-and-rotate kernel equals the numpy restatement bit for bit (numpy's dtype flow
    for every mix of float32 / float64 winds and coefficients, NaN, transposed layouts)."""
    import torch

    from fv3net_amd.derived import DerivedMapping

    rng = np.random.default_rng(dts + 10 * len(layout))
    wdt, cdts = DTYPES[dts]
    (x, xd), (y, yd), coeffs = _rotation_case(rng, wdt, cdts, tile=layout != "plain",
                                              transposed=layout == "transposed")
    conv = (lambda a: torch.from_numpy(a).cuda()) if device else (lambda a: a)
    data = {"dQxwind": D.DataArray(conv(x), xd), "dQywind": D.DataArray(conv(y), yd),
            "x_wind": D.DataArray(conv(x), xd),
            "y_wind": D.DataArray(conv(y), yd)}
    for name, (c, cd) in zip(COEFFS, coeffs):
        data[name] = D.DataArray(conv(c), cd)
    dm = DerivedMapping(D.Dataset(data))
    (e, ed), (nn, nd) = OD.center_and_rotate_xy_winds(coeffs, x, xd, y, yd)
    for name, ref, dims in (("dQu", e, ed), ("dQv", nn, nd), ("eastward_wind", e, ed), ("northward_wind", nn, nd)):
        got = dm[name]
        assert got.dims == dims, (name, got.dims, dims)
        assert hasattr(got.data, "is_cuda") == device
        _bits(got.values, ref, name)


@pytest.mark.gpu
def test_rotated_winds_kats_and_errors(gpu):
    """test_derived_mapping.py:64-97 through DerivedMapping on the device: zero
    coefficients give zeros; existing dQu is used as is; winds on cell centres raise the
    reference's ValueError; missing coefficients a KeyError."""
    from fv3net_amd.derived import DerivedMapping

    ny, nx = 1, 2
    rot = {k: D.DataArray(np.zeros((ny, nx)), ["y", "x"]) for k in COEFFS}
    data = D.Dataset({"dQxwind": D.DataArray(np.ones((ny + 1, nx)), ["y_interface", "x"]),
                      "dQywind": D.DataArray(np.ones((ny, nx + 1)), ["y", "x_interface"]),
                      "x_wind": D.DataArray(np.ones((ny + 1, nx)), ["y_interface", "x"]),
                      "y_wind": D.DataArray(np.ones((ny, nx + 1)), ["y", "x_interface"]), **rot})
    dm = DerivedMapping(data)
    for v in ("dQu", "dQv", "eastward_wind", "northward_wind"):
        np.testing.assert_array_almost_equal(0.0, dm[v].values)
    existing = DerivedMapping(D.Dataset({"dQu": D.DataArray(np.ones((3, 2)), ["y", "x"])}))
    np.testing.assert_array_almost_equal(existing["dQu"].values, 1.0)
    centred = D.Dataset({"dQxwind": D.DataArray(np.ones((ny, nx)), ["y", "x"]),
                         "dQywind": D.DataArray(np.ones((ny, nx)), ["y", "x"]), **rot})
    with pytest.raises(ValueError, match="Variable to shift to center"):
        DerivedMapping(centred)["dQu"]
    with pytest.raises(KeyError):
        DerivedMapping(D.Dataset({"dQxwind": data["dQxwind"], "dQywind": data["dQywind"]}))["dQv"]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_wind_parallel_projections(gpu, dtype):
    """dQu_parallel_to_eastward_wind / dQv_parallel_to_northward_wind bit for bit (zeros,
    signed zeros, NaN, inf), and the horizontal projection (its norm sums BLAS's way in
    numpy: rtol 1e-13 at float64, 1e-6 at float32) with test_derived_mapping.py:33-58's
    five cases (PROJECTION_CASES)."""
    import torch

    from fv3net_amd.derived import DerivedMapping

    rng = np.random.default_rng(4)
    shape = (NZ, 10, 12)
    E, N = rng.normal(0, 10, shape).astype(dtype), rng.normal(0, 10, shape).astype(dtype)
    dqu, dqv = rng.normal(0, 1e-3, shape).astype(dtype), rng.normal(0, 1e-3, shape).astype(dtype)
    E.flat[:6] = [0.0, -0.0, 1.0, np.nan, np.inf, 0.0]
    dqu.flat[:6] = [1.0, 1.0, 0.0, 1.0, 2.0, 0.0]
    dims = ["z", "y", "x"]
    dm = DerivedMapping(D.Dataset({k: D.DataArray(torch.from_numpy(v).cuda(), dims) for k, v in (
        ("eastward_wind", E), ("northward_wind", N), ("dQu", dqu), ("dQv", dqv))}))
    _bits(dm["dQu_parallel_to_eastward_wind"].values, OD.parallel_to_wind(E, dqu), "dQu parallel")
    _bits(dm["dQv_parallel_to_northward_wind"].values, OD.parallel_to_wind(N, dqv), "dQv parallel")
    E[np.isnan(E) | np.isinf(E)] = 1.0
    dm = DerivedMapping(D.Dataset({k: D.DataArray(torch.from_numpy(v).cuda(), dims) for k, v in (
        ("eastward_wind", E), ("northward_wind", N), ("dQu", dqu), ("dQv", dqv))}))
    got = dm["horizontal_wind_tendency_parallel_to_horizontal_wind"].values
    ref = OD.horizontal_wind_tendency_parallel_to_horizontal_wind(E, dqu, N, dqv)
    assert got.dtype == ref.dtype
    np.testing.assert_allclose(got, ref, rtol=1e-13 if dtype == np.float64 else 1e-6, atol=0)
    for dqu1, dqv1, east, north, projection in PROJECTION_CASES:
        one = DerivedMapping(D.Dataset({k: D.DataArray(np.array([v]), ["x"]) for k, v in (
            ("dQu", dqu1), ("dQv", dqv1), ("eastward_wind", east), ("northward_wind", north))}))
        v = one["horizontal_wind_tendency_parallel_to_horizontal_wind"].values.item()
        assert v == pytest.approx(projection, rel=1e-15)


@pytest.mark.gpu
def test_cos_zenith_kats_and_oracle(gpu):
    """test__zenith_angle.py on the device: the twelve points (abs 1e-3), DataArray inputs
    (name, dims, the radian-units conversion identical to degrees), and random points and
    times against the oracle (sin / cos of the device library vs glibc: abs 1e-14)."""
    from fv3net_amd.derived import cos_zenith_angle
    from fv3net_amd.emulation import JulianTime

    for t, lon, lat, expected in ZENITH_KATS:
        for time in (JulianTime(*t), datetime.datetime(*t)):
            got = cos_zenith_angle(time, lon, lat)
            assert float(got) == pytest.approx(expected, abs=1e-3)
            # scalar inputs give a numpy float64 scalar, not a 0-d array (_star_cos_zenith)
            assert isinstance(got, np.float64) and not isinstance(got, np.ndarray)
    time = JulianTime(2020, 3, 21, 12)
    da = cos_zenith_angle(D.DataArray(np.array(time, dtype=object), []), D.DataArray(np.array([0]), ["x"]),
                          D.DataArray(np.array([0]), ["x"]))
    assert isinstance(da, D.DataArray) and da.name == "cos_zenith_angle" and da.dims == ("x",)
    assert da.values.item() == pytest.approx(float(cos_zenith_angle(time, 0.0, 0.0)))
    ref = None
    for lon_u in ("degrees", "radians"):
        for lat_u in ("degrees", "radians"):
            lon = np.deg2rad(10) if lon_u == "radians" else 10
            lat = np.deg2rad(10) if lat_u == "radians" else 10
            r = cos_zenith_angle(D.DataArray(np.array(time, dtype=object), []),
                                 D.DataArray(np.array([lon]), ["x"], attrs={"units": lon_u}),
                                 D.DataArray(np.array([lat]), ["x"], attrs={"units": lat_u})).values
            ref = r if ref is None else ref
            _bits(r, ref, f"{lon_u}/{lat_u}")
    rng = np.random.default_rng(1)
    times = np.array([datetime.datetime(2016, 1, 1) + datetime.timedelta(hours=float(h))
                      for h in rng.uniform(0, 24 * 366, 5)], dtype=object)
    lon = rng.uniform(-180, 360, (6, 20, 24))
    lat = rng.uniform(-90, 90, (6, 20, 24))
    got = cos_zenith_angle(D.DataArray(times, ["time"]), D.DataArray(lon, ["tile", "y", "x"]),
                           D.DataArray(lat, ["tile", "y", "x"]))
    assert got.dims == ("time", "tile", "y", "x")
    ref = OD.cos_zenith_angle(times[:, None, None, None], lon[None], lat[None])
    np.testing.assert_allclose(got.values, ref, rtol=0, atol=1e-14)
    lat32 = lat.astype(np.float32)  # float32 lat / lon: their radians and sin / cos in float32
    got = cos_zenith_angle(times[2], lon.astype(np.float32), lat32)
    ref = OD.cos_zenith_angle(times[2], lon.astype(np.float32), lat32)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_derived_mapping_cos_zenith_from_time_coordinate(gpu):
    """test_derived_mapping.py:9-31, 102-105: "cos_zenith_angle" from a Dataset whose time
    is a coordinate: a DataArray over (time, y, x) equal to the oracle."""
    from fv3net_amd.derived import DerivedMapping
    from fv3net_amd.emulation import JulianTime

    nt, nx, ny = 3, 2, 1
    rng = np.random.default_rng(0)
    times = np.array([JulianTime(2016, 1, 1, 6 * k) for k in range(nt)], dtype=object)
    lat, lon = rng.random((ny, nx)), rng.random((ny, nx))
    ds = D.Dataset({"lat": D.DataArray(lat, ["y", "x"]), "lon": D.DataArray(lon, ["y", "x"]),
                    "T": D.DataArray(rng.random((ny, nx, nt)), ["y", "x", "time"], coords={"time": times})})
    out = DerivedMapping(ds)["cos_zenith_angle"]
    assert isinstance(out, D.DataArray) and out.dims == ("time", "y", "x")
    jt = np.array([OD.JulianDate(2016, 1, 1, 6 * k) for k in range(nt)], dtype=object)
    np.testing.assert_allclose(out.values, OD.cos_zenith_angle(jt[:, None, None], lon[None], lat[None]), atol=1e-14,
                               rtol=0)


def _dense(inputs, output, seed):
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    cfg = DenseModelConfig(list(inputs), [output], [NZ, NZ], [NZ], width=64, depth=2)
    rng = np.random.default_rng(seed)
    s = [rng.normal(260, 15, (512, NZ)).astype(np.float32), rng.uniform(0, 0.02, (512, NZ)).astype(np.float32)]
    m = DenseColumnModel.random(cfg, seed=seed, sample_inputs=s, bias_scale=0.1)
    return P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)


def _write(path, name, config_file, config):
    import yaml

    path.mkdir()
    with open(path / config_file, "w") as f:
        yaml.safe_dump(config, f)
    with open(path / "name", "w") as f:
        f.write(name)


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False])
def test_dqu_dqv_from_dense_predictions_on_staggered_grids(gpu, device):
    """Two mi355x-dense predictors, one on the y-staggered grid predicting dQxwind, one on
    the x-staggered grid predicting dQywind (each sees its own Dataset: PureKerasModel.predict
    stacks every dim of its input, pure_keras.py:110, so one model cannot take both grids),
    merged with the grid's rotation coefficients into a DerivedMapping, as the prognostic
    run's derived state does: dQu / dQv are the oracle's centre-and-rotate of the
    predictions, bit for bit, and the predictions pass through unchanged."""
    import torch

    from fv3net_amd.derived import DerivedMapping
    from fv3net_amd.stepper import merge

    n = 24
    rng = np.random.default_rng(3)
    a, b = _dense(["Ta", "qa"], "dQxwind", 1), _dense(["Tb", "qb"], "dQywind", 2)
    conv = (lambda v: torch.from_numpy(v).cuda()) if device else (lambda v: v)
    Xa = D.Dataset({k: D.DataArray(conv(rng.normal(260, 15, (NZ, n + 1, n)) if k == "Ta" else
                                        rng.uniform(0, 0.02, (NZ, n + 1, n))), ["z", "y_interface", "x"])
                    for k in ("Ta", "qa")})
    Xb = D.Dataset({k: D.DataArray(conv(rng.normal(260, 15, (NZ, n, n + 1)) if k == "Tb" else
                                        rng.uniform(0, 0.02, (NZ, n, n + 1))), ["z", "y", "x_interface"])
                    for k in ("Tb", "qb")})
    coeffs = [rng.uniform(-1, 1, (n, n)) for _ in COEFFS]
    rot = D.Dataset({k: D.DataArray(conv(c), ["y", "x"]) for k, c in zip(COEFFS, coeffs)})
    xw, yw = a.predict(Xa)["dQxwind"], b.predict(Xb)["dQywind"]
    dm = DerivedMapping(merge([D.Dataset({"dQxwind": xw, "dQywind": yw}), rot]))
    (e, ed), (nn, nd) = OD.center_and_rotate_xy_winds([(c, ("y", "x")) for c in coeffs], xw.values, xw.dims,
                                                      yw.values, yw.dims)
    got_u, got_v = dm["dQu"], dm["dQv"]
    assert got_u.dims == ed and got_v.dims == nd
    _bits(got_u.values, e, "dQu")
    _bits(got_v.values, nn, "dQv")
    _bits(dm["dQxwind"].values, xw.values, "dQxwind passes through")


@pytest.mark.gpu
def test_derived_model_dqu_dqv_through_the_registry(gpu, tmp_path):
    """derived_model(dQu, dQv) over a combined_output_model loaded by path (yaml + name
    files, models.py:19-62, 110-220): members predicting dQxwind on the y-staggered grid,
    dQywind on the x-staggered grid and the rotation coefficients on cell centres
    (constant-output predictors, which stack only their own inputs, testing.py:70-73).
    dQu / dQv equal the oracle's centre-and-rotate of the members' predictions, bit for
    bit, on host arrays."""
    from fv3net_amd.derived import DerivedModel

    n = 6
    rng = np.random.default_rng(8)
    members = []
    for name, inp, outs in (("u", "u_grid", {"dQxwind": rng.normal(0, 1e-3, NZ)}),
                            ("v", "v_grid", {"dQywind": rng.normal(0, 1e-3, NZ)}),
                            ("c", "grid", dict(zip(COEFFS, (0.8, -0.6, 0.6, 0.8))))):
        m = P.ConstantOutputPredictor([inp], list(outs))
        m.set_outputs(**outs)
        P.dump(m, str(tmp_path / name))
        members.append(str(tmp_path / name))
    _write(tmp_path / "combined", "combined_output_model", "combined_output_model.yaml", {"models": members})
    _write(tmp_path / "derived", "derived_model", "derived_model.yaml",
           {"model": str(tmp_path / "combined"), "derived_output_variables": ["dQu", "dQv"]})
    model = P.load(str(tmp_path / "derived"))
    assert isinstance(model, DerivedModel) and {"dQu", "dQv"} <= set(model.output_variables)
    X = D.Dataset({"u_grid": D.DataArray(np.zeros((n + 1, n)), ["y_interface", "x"]),
                   "v_grid": D.DataArray(np.zeros((n, n + 1)), ["y", "x_interface"]),
                   "grid": D.DataArray(np.zeros((n, n)), ["y", "x"])})
    out = model.predict(X)
    xw, yw = out["dQxwind"], out["dQywind"]
    coeffs = [(out[k].transpose("y", "x").values, ("y", "x")) for k in COEFFS]
    (e, ed), (nn, nd) = OD.center_and_rotate_xy_winds(coeffs, xw.values, xw.dims, yw.values, yw.dims)
    assert out["dQu"].dims == ed and out["dQv"].dims == nd
    _bits(out["dQu"].values, e, "dQu")
    _bits(out["dQv"].values, nn, "dQv")
