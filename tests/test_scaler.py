"""StandardScaler: the reference's own test_scalers.py cases
(external/fv3fit/tests/test_scalers.py:17-80) against fv3net_amd.normalization, whose
normalize / denormalize run on the GPU (csrc/scaler.hip); fit, dump/load and the
RuntimeError of an unfitted scaler need no GPU."""
import io
import zipfile

import numpy as np
import pytest

from fv3net_amd.normalization import StandardScaler, fit_mean_std

SEED = 1


def test_standard_scaler_not_fit_before_call():
    scaler = StandardScaler()
    with pytest.raises(RuntimeError):
        scaler.normalize(np.array([0.0, 1.0]))
    with pytest.raises(RuntimeError):
        scaler.denormalize(np.array([0.0, 1.0]))


@pytest.mark.parametrize("std_epsilon", [1e-12, 1e-8])
def test_standard_scaler_fit_constant_features(std_epsilon):
    scaler = StandardScaler(std_epsilon)
    const = 10.0
    y = np.vstack([np.arange(5.0), np.full(5, const), np.full(5, 2 * const)]).T
    scaler.fit(y)
    assert scaler.mean.dtype == np.float64 and scaler.std.dtype == np.float64
    assert (scaler.std[1:] == std_epsilon).all()
    np.testing.assert_array_equal(scaler.std[0], np.std(np.arange(5.0)) + std_epsilon)


def test_dump_load_is_the_reference_npz():
    """The file is an npz of mean/std (scaler.py:86-100): readable by numpy alone, and
    a zip of them per variable is the PytorchPredictor's scalers.zip."""
    rng = np.random.default_rng(SEED)
    scaler = StandardScaler()
    scaler.fit(rng.uniform(0, 10, (10, 5)))
    buf = io.BytesIO()
    scaler.dump(buf)
    buf.seek(0)
    z = np.load(buf, allow_pickle=False)
    assert sorted(z.files) == ["mean", "std"]
    np.testing.assert_array_equal(z["std"], scaler.std)
    buf.seek(0)
    assert StandardScaler.load(buf) == scaler
    zb = io.BytesIO()
    with zipfile.ZipFile(zb, "w") as archive:
        with archive.open("air_temperature", "w") as f:
            scaler.dump(f)
    zb.seek(0)
    with zipfile.ZipFile(zb, "r") as archive:
        assert StandardScaler.load(archive.open("air_temperature", "r")) == scaler
    unfit = StandardScaler()
    b2 = io.BytesIO()
    unfit.dump(b2)
    b2.seek(0)
    loaded = StandardScaler.load(b2)
    assert loaded.mean is None and loaded.std is None


def test_fit_mean_std_is_population_std_float32():
    """PerFeatureStd (emulation/layers/normalization.py:90-94): ddof 0, float32."""
    x = np.random.default_rng(0).normal(3, 2, (100, 6)).astype(np.float32)
    m, s = fit_mean_std(x)
    assert m.dtype == np.float32 and s.dtype == np.float32
    np.testing.assert_allclose(s, x.std(axis=0, ddof=0), rtol=1e-6)


# --------------------------------------------------------------- GPU (csrc/scaler.hip)
@pytest.mark.gpu
@pytest.mark.parametrize("std_epsilon", [1e-12, 1e-8])
def test_standard_scaler_constant_scaling(gpu, std_epsilon):
    scaler = StandardScaler(std_epsilon)
    const = 10.0
    y = np.vstack([np.arange(5.0), np.full(5, const), np.full(5, 2 * const)]).T
    scaler.fit(y)
    assert (scaler.normalize(np.array([3.0, const, const * 2.0]))[1:] == 0.0).all()
    d = scaler.denormalize(np.array([3.0, 0.0, 0.0]))
    assert d[1] == const and d[2] == const * 2.0


@pytest.mark.gpu
@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_standard_scaler_normalize_then_denormalize(gpu, n_samples, n_features):
    np.random.seed(SEED)
    X = np.random.uniform(0, 10, size=[n_samples, n_features])
    scaler = StandardScaler()
    scaler.fit(X)
    np.testing.assert_almost_equal(scaler.denormalize(scaler.normalize(X)), X)


@pytest.mark.gpu
@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_standard_scaler_normalize(gpu, n_samples, n_features):
    np.random.seed(SEED)
    X = np.random.uniform(0, 10, size=[n_samples, n_features])
    scaler = StandardScaler()
    scaler.fit(X)
    r = scaler.normalize(X)
    np.testing.assert_almost_equal(np.mean(r, axis=0), 0)
    np.testing.assert_almost_equal(np.std(r, axis=0), 1)


@pytest.mark.gpu
@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_normalize_then_denormalize_on_reloaded_scaler(gpu, n_samples, n_features):
    np.random.seed(SEED)
    X = np.random.uniform(0, 10, size=[n_samples, n_features])
    scaler = StandardScaler()
    scaler.fit(X)
    r = scaler.normalize(X)
    buf = io.BytesIO()
    scaler.dump(buf)
    buf.seek(0)
    loaded = StandardScaler.load(buf)
    np.testing.assert_almost_equal(loaded.denormalize(r), X)
    np.testing.assert_array_equal(loaded.mean, scaler.mean)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_device_arithmetic_is_numpy_float64(gpu, dtype):
    """Bitwise numpy: (x - mean) / std in float64 (and its float32 rounding for the
    PytorchPredictor pack), y * std + mean in float64; features last or first, 2-D
    (scalar) statistics, torch in -> torch out."""
    import torch

    rng = np.random.default_rng(3)
    X = rng.normal(250, 20, (300, 79)).astype(dtype)
    scaler = StandardScaler()
    scaler.fit(X.astype(np.float64))
    ref = (X.astype(np.float64) - scaler.mean) / scaler.std
    got = scaler.normalize(X)
    assert got.dtype == np.float64 and (got == ref).all()
    assert (scaler.normalize(X, out_f32=True) == ref.astype(np.float32)).all()
    got_t = scaler.normalize(torch.from_numpy(np.ascontiguousarray(X.T)).cuda(), feature_axis=0)
    assert torch.is_tensor(got_t) and (got_t.cpu().numpy() == ref.T).all()
    y = rng.normal(0, 1, (300, 79)).astype(np.float32)
    assert (scaler.denormalize(y) == y.astype(np.float64) * scaler.std + scaler.mean).all()
    s2 = StandardScaler()
    s2.fit(X[:, 0].astype(np.float64))  # a 2-D variable: scalar statistics
    col = X[:, 0]
    assert (s2.normalize(col) == (col.astype(np.float64) - s2.mean) / s2.std).all()


@pytest.mark.gpu
def test_reassigned_statistics_are_not_served_stale(gpu):
    """scaler.py:86-100 loads by assigning ``mean`` / ``std``: after a normalize has
    cached device copies, a reassigned or in-place edited statistic must be used."""
    scaler = StandardScaler()
    x = np.random.default_rng(4).normal(3, 2, (50, 6))
    scaler.fit(x)
    scaler.normalize(x)
    scaler.mean = scaler.mean + 1.0
    np.testing.assert_array_equal(scaler.normalize(x), (x - scaler.mean) / scaler.std)
    scaler.std *= 2.0
    np.testing.assert_array_equal(scaler.normalize(x), (x - scaler.mean) / scaler.std)
