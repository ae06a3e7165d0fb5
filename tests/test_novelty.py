"""The out-of-sample composite (OutOfSampleModel, "out_of_sample") with the min-max
novelty detector ("minmax") and the three tapers, over the build's predictor.

Reference KATs mirrored: external/fv3fit/tests/test_taper.py:19-105 (mask / ramp /
decay values, the loaded model's default and ramp tapers) and
test_out_of_sample.py:24-72 (constant predictor and detector, cutoffs -1 / 1, five output
variables, is_novelty == 1 - taper_values).  The oracle (oracle/novelty.py) is pinned by
those KATs and by scikit-learn's MinMaxScaler (importable here); the kernels
(csrc/novelty.hip) are compared with it bit for bit.
"""
import os

import numpy as np
import pytest
import yaml

from fv3net_amd import dataset as D
from fv3net_amd import predictor as P
from oracle import novelty as ON

SCORES = np.asarray([[1, 3, 5], [6, 4, 2]])


# --------------------------------------------------------------------------- oracle
def test_oracle_taper_kats():
    """test_taper.py:19-60."""
    np.testing.assert_almost_equal(ON.taper_mask(SCORES, cutoff=3), [[1, 1, 0], [0, 0, 1]])
    np.testing.assert_almost_equal(ON.taper_ramp(SCORES, ramp_min=2, ramp_max=5), [[1, 2 / 3, 0], [0, 1 / 3, 1]])
    np.testing.assert_almost_equal(ON.taper_decay(SCORES, threshold=2, rate=0.5),
                                   [[1, 2 ** -1, 2 ** -3], [2 ** -4, 2 ** -2, 1]])
    assert ON.taper_mask(SCORES.astype(np.float32), 3).dtype == np.int64


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_minmax_fit_and_oracle_match_sklearn(dtype):
    """The detector's fit (scale_, min_) and the oracle's transform against scikit-learn's
    MinMaxScaler on the same data, bit for bit (a constant feature included)."""
    from sklearn.preprocessing import MinMaxScaler

    from fv3net_amd.novelty import MinMaxNoveltyDetector

    rng = np.random.default_rng(1)
    X = rng.normal(0, 3, (500, 12)).astype(dtype)
    X[:, 4] = 2.5  # zero range: scale 1
    sk = MinMaxScaler().fit(X)
    det = MinMaxNoveltyDetector.fit(X, ["a"])
    assert det.scale.dtype == sk.scale_.dtype and np.array_equal(det.scale, sk.scale_)
    assert np.array_equal(det.min, sk.min_)
    Y = rng.normal(0, 5, (300, 12)).astype(dtype)
    scaled = sk.transform(Y)
    ref = np.maximum(scaled.max(axis=1) - 1, 0) + np.maximum(-1 * scaled.min(axis=1), 0)
    got = ON.minmax_scores(Y, det.scale, det.min)
    assert got.dtype == ref.dtype and np.array_equal(got, ref)


def test_minmax_dump_load_and_pickle_refusal(tmp_path):
    from fv3net_amd.novelty import MinMaxNoveltyDetector

    det = MinMaxNoveltyDetector.fit(np.random.default_rng(0).normal(0, 1, (50, 7)).astype(np.float32), ["a", "b"],
                                    clip={"a": {"start": 1, "stop": 4}})
    P.dump(det, str(tmp_path / "m"))
    back = P.load(str(tmp_path / "m"))
    assert isinstance(back, MinMaxNoveltyDetector) and back.input_variables == ["a", "b"]
    assert np.array_equal(back.scale, det.scale) and back.scale.dtype == np.float32 and back.clip == det.clip
    os.makedirs(tmp_path / "pkl")
    (tmp_path / "pkl" / "minmax.pkl").write_bytes(b"not loaded")
    with pytest.raises(ValueError, match="pickled"):
        MinMaxNoveltyDetector.load(str(tmp_path / "pkl"))


def _write_oos(path, base_path, novelty_path, **extra):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "out_of_sample_model.yaml"), "w") as f:
        yaml.safe_dump({"base_model_path": base_path, "novelty_detector_path": novelty_path, **extra}, f)
    with open(os.path.join(path, "name"), "w") as f:
        print("out_of_sample", file=f)


def test_out_of_sample_load_taper_configs(tmp_path):
    """OutOfSampleModel.load's default tapering config (models.py:424-436): a mask at the
    cutoff, or the yaml's own taper (test_taper.py:80-105 loads these two)."""
    from fv3net_amd.novelty import ConstantOutputNoveltyDetector, OutOfSampleModel

    base, det = P.ConstantOutputPredictor([], []), ConstantOutputNoveltyDetector([])
    P.dump(base, str(tmp_path / "base"))
    P.dump(det, str(tmp_path / "novelty"))
    _write_oos(str(tmp_path / "a"), str(tmp_path / "base"), str(tmp_path / "novelty"))
    m = P.load(str(tmp_path / "a"))
    assert isinstance(m, OutOfSampleModel) and (m.taper.name, m.taper.p0) == ("taper_mask", 0.0)
    _write_oos(str(tmp_path / "b"), str(tmp_path / "base"), str(tmp_path / "novelty"),
               tapering_function={"name": "taper_ramp", "ramp_min": -1, "ramp_max": 2})
    m = P.load(str(tmp_path / "b"))
    assert (m.taper.name, m.taper.p0, m.taper.p1) == ("taper_ramp", -1.0, 2.0)
    with pytest.raises(ValueError, match="Incorrect tapering name"):
        _write_oos(str(tmp_path / "c"), str(tmp_path / "base"), str(tmp_path / "novelty"),
                   tapering_function={"name": "taper_none"})
        P.load(str(tmp_path / "c"))
    with pytest.raises(NotImplementedError):
        m.dump(str(tmp_path / "d"))


# ---------------------------------------------------------------------------- device
def _bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["f32", "f64", "mixed", "f32_scale64"])
def test_minmax_scores_kernel_vs_oracle(gpu, case):
    """fv3_minmax_scores bit for bit: (z, y, x) and 2-D inputs, a clipped variable, the
    scaler's dtype against X's, NaN columns."""
    import torch

    from fv3net_amd.novelty import MinMaxNoveltyDetector

    rng = np.random.default_rng(len(case))
    nz, ny, nx = 19, 6, 7
    ta = np.float64 if case in ("f64", "mixed") else np.float32
    tb = np.float64 if case == "f64" else np.float32
    a = rng.normal(250, 10, (nz, ny, nx)).astype(ta)
    b = rng.normal(0, 1, (ny, nx)).astype(tb)
    c = rng.normal(5, 2, (nz, ny, nx)).astype(tb)
    a[:, 0, 0] *= 3.0  # out of range
    c[3, 1, 1] = np.nan
    feats = lambda a, b, c: [a[2:15].reshape(13, -1).T, b.reshape(1, -1).T, c.reshape(nz, -1).T]  # noqa: E731
    train = ON.pack(feats(a, b, c)).astype(np.float32)
    det = MinMaxNoveltyDetector.fit(np.nan_to_num(train) * 0.9, ["a", "b", "c"], clip={"a": {"start": 2, "stop": 15}})
    if case == "f32_scale64":
        det = MinMaxNoveltyDetector(["a", "b", "c"], det.scale.astype(np.float64), det.min.astype(np.float64),
                                    det.clip)
    X = D.Dataset({"a": D.DataArray(torch.from_numpy(a).cuda(), ["z", "y", "x"]),
                   "b": D.DataArray(torch.from_numpy(b).cuda(), ["y", "x"]),
                   "c": D.DataArray(c, ["z", "y", "x"])})
    out = det.predict(X)
    got = out["novelty_score"].values
    ref = ON.minmax_scores(ON.pack(feats(a, b, c)), det.scale, det.min).reshape(ny, nx)
    assert out["novelty_score"].dims == ("y", "x")
    _bits(got, ref)
    assert np.isnan(got[1, 1]) and got[0, 0] > 0
    _bits(out["centered_score"].values, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name,params", [("taper_mask", {"cutoff": 0.3}),
                                         ("taper_ramp", {"ramp_min": 0.1, "ramp_max": 0.7}),
                                         ("taper_decay", {"threshold": 0.2, "rate": 0.5})])
@pytest.mark.parametrize("sdt,odt", [(np.float32, np.float32), (np.float32, np.float64), (np.float64, np.float32)])
def test_taper_kernel_vs_oracle(gpu, name, params, sdt, odt):
    """fv3_taper_columns: taper values and outputs * taper in numpy's dtype flow, for
    (tile, z, y, x) and 2-D outputs (decay: the device pow against numpy's, 1 ulp)."""
    import torch

    from fv3net_amd.novelty import get_taper_function

    rng = np.random.default_rng(3)
    s = rng.uniform(-0.2, 1.2, (6, 5, 4)).astype(sdt)
    s[0, 0, 0] = np.nan
    o3 = rng.normal(0, 1, (6, 9, 5, 4)).astype(odt)
    o2 = rng.normal(0, 1, (6, 5, 4)).astype(odt)
    taper = get_taper_function(name, params)
    scores = D.DataArray(torch.from_numpy(s).cuda(), ["tile", "y", "x"])
    values, (t3, t2) = taper.run(scores, [D.DataArray(torch.from_numpy(o3).cuda(), ["tile", "z", "y", "x"]),
                                          D.DataArray(o2, ["tile", "y", "x"])])
    ref = ON.TAPERS[name](s, **params)
    got = values.values
    if name == "taper_decay":
        assert got.dtype == ref.dtype
        np.testing.assert_allclose(got, ref, rtol=4e-7 if sdt == np.float32 else 1e-15, equal_nan=True)
        ref = got  # the products below on the device's taper values
    else:
        _bits(got, ref)
    assert t3.dims == ("tile", "z", "y", "x") and t2.dims == ("tile", "y", "x")
    _bits(t3.values, o3 * ref[:, None])
    _bits(t2.values, o2 * ref)


@pytest.mark.gpu
def test_taper_loading_kats(gpu, tmp_path):
    """test_taper.py:80-105 on the device."""
    from fv3net_amd.novelty import ConstantOutputNoveltyDetector

    P.dump(P.ConstantOutputPredictor([], []), str(tmp_path / "base"))
    P.dump(ConstantOutputNoveltyDetector([]), str(tmp_path / "novelty"))
    _write_oos(str(tmp_path / "a"), str(tmp_path / "base"), str(tmp_path / "novelty"))
    m = P.load(str(tmp_path / "a"))
    np.testing.assert_allclose(m.taper(np.asarray([-1e-5, 1e-5])).values, [1, 0])
    _write_oos(str(tmp_path / "b"), str(tmp_path / "base"), str(tmp_path / "novelty"),
               tapering_function={"name": "taper_ramp", "ramp_min": -1, "ramp_max": 2})
    m = P.load(str(tmp_path / "b"))
    np.testing.assert_allclose(m.taper(np.asarray([-1, 0.5, 2])).values, [1, 0.5, 0])


@pytest.mark.gpu
@pytest.mark.parametrize("base_value,novelty_cutoff,output", [(1, -1, 0), (1, 1, 1)])
@pytest.mark.parametrize("different_inputs", [False, True])
def test_out_of_sample_model_kats(gpu, base_value, novelty_cutoff, output, different_inputs):
    """test_out_of_sample.py:24-72."""
    from fv3net_amd.novelty import ConstantOutputNoveltyDetector, NoveltyDetector, OutOfSampleModel

    if different_inputs:
        base = P.ConstantOutputPredictor(["shared_input", "base_input"], ["output"])
        det = ConstantOutputNoveltyDetector(["shared_input", "novelty_input"])
        X = D.Dataset({"shared_input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"]),
                       "base_input": D.DataArray(np.ones([3, 3]), ["x", "y"]),
                       "novelty_input": D.DataArray(np.ones([3, 3, 5]), ["x", "y", "z"])})
    else:
        base = P.ConstantOutputPredictor(["input"], ["output"])
        det = ConstantOutputNoveltyDetector(["input"])
        X = D.Dataset({"input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"])})
    base.set_outputs(output=base_value)
    model = OutOfSampleModel(base, det, novelty_cutoff)
    out = model.predict(X)
    assert len(out.data_vars) == 5
    np.testing.assert_allclose(out[NoveltyDetector._NOVELTY_OUTPUT_VAR].values,
                               1 - out[OutOfSampleModel._TAPER_VALUES_OUTPUT_VAR].values)
    assert "output" in out.data_vars
    np.testing.assert_almost_equal(out["output"].values, output)


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False])
def test_dense_predictor_nested_in_out_of_sample(gpu, tmp_path, device):
    """An mi355x-dense predictor and a min-max detector fitted on its training columns,
    dumped and loaded through the registry as an out_of_sample model: in-sample columns
    keep the base prediction, scaled-up columns (x 3) are masked, bit for bit against
    the base prediction times the oracle's mask of the oracle's scores."""
    import torch

    from fv3net_amd.novelty import MinMaxNoveltyDetector, OutOfSampleModel
    from tests.test_composite import _dense_predictor

    base = _dense_predictor()
    rng = np.random.default_rng(5)
    nz, n = 79, 24
    T = rng.normal(260, 15, (nz, n, n))
    q = rng.uniform(0, 0.02, (nz, n, n))
    train = ON.pack([T.reshape(nz, -1).T, q.reshape(nz, -1).T]).astype(np.float32)
    det = MinMaxNoveltyDetector.fit(train, ["air_temperature", "specific_humidity"])
    T[:, :4] *= 3.0  # rows 0..3 out of range
    P.dump(base, str(tmp_path / "base"))
    P.dump(det, str(tmp_path / "novelty"))
    _write_oos(str(tmp_path / "oos"), str(tmp_path / "base"), str(tmp_path / "novelty"), cutoff=0)
    model = P.load(str(tmp_path / "oos"))
    assert isinstance(model, OutOfSampleModel)
    conv = (lambda a: torch.from_numpy(a).cuda()) if device else (lambda a: a)
    X = D.Dataset({"air_temperature": D.DataArray(conv(T), ["z", "y", "x"]),
                   "specific_humidity": D.DataArray(conv(q), ["z", "y", "x"])})
    out = model.predict(X)
    plain = base.predict(X)
    score = ON.minmax_scores(ON.pack([T.reshape(nz, -1).T, q.reshape(nz, -1).T]), det.scale, det.min).reshape(n, n)
    mask = ON.taper_mask(score, 0)
    assert mask[:4].sum() == 0 and mask[4:].sum() > 0
    _bits(out["taper_values"].values, mask)
    _bits(out["novelty_score"].values, score)
    for v in ("dQ1", "dQ2"):
        _bits(out[v].values, plain[v].values * mask)
