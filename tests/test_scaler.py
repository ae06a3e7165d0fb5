"""StandardScaler mirror: the reference's own test_scalers.py cases
(external/fv3fit/tests/test_scalers.py:17-80) against fv3net_amd.normalization."""
import io

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
def test_standard_scaler_constant_scaling(std_epsilon):
    scaler = StandardScaler(std_epsilon)
    const = 10.0
    y = np.vstack([np.arange(5.0), np.full(5, const), np.full(5, 2 * const)]).T
    scaler.fit(y)
    assert (scaler.std[1:] == std_epsilon).all()
    assert (scaler.normalize(np.array([3.0, const, const * 2.0]))[1:] == 0.0).all()
    d = scaler.denormalize(np.array([3.0, 0.0, 0.0]))
    assert d[1] == const and d[2] == const * 2.0


@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_standard_scaler_normalize_then_denormalize(n_samples, n_features):
    np.random.seed(SEED)
    X = np.random.uniform(0, 10, size=[n_samples, n_features])
    scaler = StandardScaler()
    scaler.fit(X)
    np.testing.assert_almost_equal(scaler.denormalize(scaler.normalize(X)), X)


@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_standard_scaler_normalize(n_samples, n_features):
    np.random.seed(SEED)
    X = np.random.uniform(0, 10, size=[n_samples, n_features])
    scaler = StandardScaler()
    scaler.fit(X)
    r = scaler.normalize(X)
    np.testing.assert_almost_equal(np.mean(r, axis=0), 0)
    np.testing.assert_almost_equal(np.std(r, axis=0), 1)


@pytest.mark.parametrize("n_samples, n_features", [(10, 1), (10, 5)])
def test_normalize_then_denormalize_on_reloaded_scaler(n_samples, n_features):
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


def test_fit_mean_std_is_population_std_float32():
    """PerFeatureStd (emulation/layers/normalization.py:90-94): ddof 0, float32."""
    x = np.random.default_rng(0).normal(3, 2, (100, 6)).astype(np.float32)
    m, s = fit_mean_std(x)
    assert m.dtype == np.float32 and s.dtype == np.float32
    np.testing.assert_allclose(s, x.std(axis=0, ddof=0), rtol=1e-6)
