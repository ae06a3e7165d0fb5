"""Composite predictors over the build's predictor, and the online transformer Adapter
(SURVEY.md 8(b) "Composition", 8(b) Callers: transformers/fv3fit.py).

Reference KATs mirrored: external/fv3fit/tests/test_ensemble.py:8-28,
test_tapered_model.py:12-60, test_combined_output_model.py:12-88.  The composites load
their members through the name-file registry from subdirectories, so the build's
``mi355x-dense`` predictor is checked as a nested base_model: it must predict exactly as
when loaded directly.  Composite arithmetic (csrc/composite.hip) and the Adapter
(fv3_adapter_apply) are compared bit for bit with oracle/composite.py.
"""
import os

import numpy as np
import pytest
import yaml

from fv3net_amd import dataset as D
from fv3net_amd import predictor as P
from oracle import composite as OC


def _bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    assert np.array_equal(a, b, equal_nan=True) and (np.signbit(a) == np.signbit(b)).all()


# --------------------------------------------------------------------------- oracle
@pytest.mark.parametrize("values,reduction,output", [((0.0, 3.0, 5.0), "median", 3.0),
                                                     ((0.0, 3.0, 5.0), "mean", 8.0 / 3)])
def test_oracle_ensemble_kat(values, reduction, output):
    """test_ensemble.py:8-28 on the restatement."""
    members = [np.full((3, 3, 5), v) for v in values]
    np.testing.assert_almost_equal(OC.member_reduce(members, reduction), output)


def test_oracle_taper_factors():
    s = OC.vertical_tapering_scale_factors(10, 3, 5.0)
    np.testing.assert_allclose(s[:3], np.exp((np.arange(3) - 3) / 5.0))
    assert (s[3:] == 1).all() and s.dtype == np.float64


def test_oracle_adapter_limits_and_sums():
    rng = np.random.default_rng(0)
    q = rng.uniform(0, 1e-3, (5, 7))
    T = rng.normal(260, 5, (5, 7))
    pred = {"dq_a": rng.normal(0, 1e-6, (5, 7)).astype(np.float32),
            "dq_b": rng.normal(0, 1e-6, (5, 7)).astype(np.float32),
            "dT": rng.normal(0, 1e-4, (5, 7)).astype(np.float32)}
    pred["dq_a"][0, 0] = -1.0  # drives the humidity negative: limited
    up = OC.adapter_predict(pred, {"specific_humidity": q, "air_temperature": T},
                            {"dq_a": "specific_humidity", "dq_b": "specific_humidity", "dT": "air_temperature"}, {},
                            900.0)
    assert up["specific_humidity"].dtype == np.float64 and (up["specific_humidity"] >= 0).all()
    assert up["specific_humidity"][0, 0] == 0.0
    with pytest.raises(NotImplementedError):
        OC.adapter_predict(pred, {"air_temperature": T}, {"dT": "air_temperature"}, {}, 900.0)


# ------------------------------------------------------------- registry / no arithmetic
def _constant(tmp_path, name, inputs, outputs, **values):
    m = P.ConstantOutputPredictor(inputs, outputs)
    m.set_outputs(**values)
    path = str(tmp_path / name)
    P.dump(m, path)
    return m, path


def _write_composite(path, registry_name, config_file, config):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, config_file), "w") as f:
        yaml.safe_dump(config, f)
    with open(os.path.join(path, "name"), "w") as f:
        print(registry_name, file=f)  # the reference tests write the name with a newline


def test_combined_output_model_loads_members_through_the_registry(tmp_path):
    """test_combined_output_model.py:12-88."""
    from fv3net_amd.composite import CombinedOutputModel

    m0, p0 = _constant(tmp_path, "predictor0", ["in0", "in1"], ["out0a", "out0b"], out0a=np.ones(10),
                       out0b=np.ones(10))
    m1, p1 = _constant(tmp_path, "predictor1", ["in1", "in2"], ["out1a", "out1b"], out1a=np.ones(10) * 2,
                       out1b=np.ones(10) * 2)
    da = D.DataArray(np.ones((5, 10)), ["x", "z"])
    X = D.Dataset({"in0": da, "in1": da, "in2": da})
    direct = CombinedOutputModel([m0, m1])
    assert set(direct.input_variables) == {"in0", "in1", "in2"}
    assert set(direct.output_variables) == {"out0a", "out0b", "out1a", "out1b"}
    pred = direct.predict(X)
    np.testing.assert_array_equal(pred["out0a"].values, m0.predict(X)["out0a"].values)
    np.testing.assert_array_equal(pred["out1a"].values, m1.predict(X)["out1a"].values)
    path = str(tmp_path / "combined")
    _write_composite(path, "combined_output_model", "combined_output_model.yaml", {"models": [p0, p1]})
    loaded = P.load(path)
    assert isinstance(loaded, CombinedOutputModel)
    assert {"out0a", "out0b", "out1a", "out1b"} == set(loaded.predict(X).data_vars)
    with pytest.raises(ValueError):
        CombinedOutputModel([m0, P.ConstantOutputPredictor(["in1"], ["out0a"])])


def test_composite_argument_errors():
    from fv3net_amd.composite import EnsembleModel, TaperConfig, TaperedModel

    m = P.ConstantOutputPredictor(["in0"], ["out0"])
    with pytest.raises(NotImplementedError):
        EnsembleModel([m], reduction="max")
    with pytest.raises(ValueError):
        EnsembleModel([m, P.ConstantOutputPredictor(["in0"], ["other"])], reduction="mean")
    with pytest.raises(KeyError):
        TaperedModel(m, {"missing": TaperConfig(cutoff=3, rate=5.0)})


def test_adapter_config_validation():
    from fv3net_amd.transformers import Config

    with pytest.raises(ValueError):
        Config(url=[], state_predictions={"a": "x", "b": "x"})
    with pytest.raises(ValueError):
        Config(url=[], tendency_predictions={"a": "x"}, state_predictions={"b": "x"})


# -------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("values,reduction,output", [((0.0, 3.0, 5.0), "median", 3.0),
                                                     ((0.0, 3.0, 5.0), "mean", 8.0 / 3)])
def test_ensemble_model_kat(gpu, values, reduction, output):
    """test_ensemble.py:8-28 through the device reduction."""
    from fv3net_amd.composite import EnsembleModel

    models = []
    for v in values:
        m = P.ConstantOutputPredictor(["input"], ["output"])
        m.set_outputs(output=v)
        models.append(m)
    ensemble = EnsembleModel(models, reduction=reduction)
    ds_in = D.Dataset({"input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"])})
    ds_out = ensemble.predict(ds_in)
    assert list(ds_out.data_vars) == ["output"]
    np.testing.assert_almost_equal(ds_out["output"].values, output)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n_members", [1, 2, 3, 4, 7, 9])
def test_member_reduce_bitwise_vs_numpy(gpu, dtype, n_members):
    """fv3_member_reduce against np.nanmean / np.nanmedian over the member axis: NaNs
    (some and all members), ties, signed zeros and infinities."""
    import torch

    from fv3net_amd.composite import EnsembleModel

    rng = np.random.default_rng(n_members)
    shape = (6, 79, 17)
    members = [rng.normal(0, 1, shape).astype(dtype) for _ in range(n_members)]
    for j, m in enumerate(members):
        m[0, j % 79] = np.nan
        m[1, :3] = np.round(m[1, :3])  # ties
        m[2, 0, :] = -0.0 if j % 2 else 0.0
        m[3, 5, j % 17] = np.inf if j % 2 else -np.inf
    for m in members:
        m[4, 7] = np.nan  # every member NaN
    for reduction in ("mean", "median"):
        got = EnsembleModel._reduce([torch.from_numpy(m).cuda() for m in members], reduction)
        _bits(got.cpu().numpy(), OC.member_reduce(members, reduction))


@pytest.mark.gpu
def test_tapered_model_kat(gpu, tmp_path):
    """test_tapered_model.py:12-60: the taper of constant outputs equals
    TaperConfig.apply of the base prediction; load through the name file."""
    from fv3net_amd.composite import TaperConfig, TaperedModel

    model, base = _constant(tmp_path, "predictor", ["in0", "in1"], ["out0", "out1"], out1=np.ones(10),
                            out0=np.ones(10))
    c0, c1 = TaperConfig(cutoff=3, rate=5.0, taper_dim="z"), TaperConfig(cutoff=6, rate=3.0, taper_dim="z")
    tapered = TaperedModel(model, {"out0": c0, "out1": c1})
    da = D.DataArray(np.ones((5, 10)), ["x", "z"])
    X = D.Dataset({"in0": da, "in1": da})
    out = tapered.predict(X)
    for name, c in (("out0", c0), ("out1", c1)):
        base_pred = model.predict(X)[name]
        assert out[name].dims == ("z", "x")  # scaling * data: the scaling's dim first
        _bits(out[name].values, OC.taper(base_pred.values, base_pred.dims.index("z"), c.cutoff, c.rate))
        _bits(out[name].values, c.apply(base_pred).values)
    path = str(tmp_path / "tapered_model")
    _write_composite(path, "tapered_model", "tapered_model.yaml",
                     {"tapering": {"out0": {"cutoff": 3, "rate": 5}, "out1": {"cutoff": 2, "rate": 6}},
                      "model": base})
    loaded = P.load(path)
    assert isinstance(loaded, TaperedModel)
    assert np.mean(loaded.predict(X)["out0"].values) < 1.0


def _dense_predictor(seed=2, nz=79):
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    cfg = DenseModelConfig(["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [nz, nz], [nz, nz],
                           width=256, depth=3)
    rng = np.random.default_rng(seed)
    sT = rng.normal(260, 15, (4096, nz)).astype(np.float32)
    sq = rng.uniform(0, 0.02, (4096, nz)).astype(np.float32)
    out = [rng.normal(0, 1e-4, (4096, nz)).astype(np.float32), rng.normal(0, 3e-8, (4096, nz)).astype(np.float32)]
    m = DenseColumnModel.random(cfg, seed=seed, sample_inputs=[sT, sq], sample_outputs=out, bias_scale=0.1)
    return P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)


def _c48_rank_state(rng, nz=79, n=48, device=True):
    import torch

    T = rng.normal(260, 15, (nz, n, n))
    q = rng.uniform(0, 0.02, (nz, n, n))
    conv = (lambda a: torch.from_numpy(a).cuda()) if device else (lambda a: a)
    return D.Dataset({"air_temperature": D.DataArray(conv(T), ["z", "y", "x"]),
                      "specific_humidity": D.DataArray(conv(q), ["z", "y", "x"])})


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False])
def test_dense_predictor_nested_in_composites(gpu, tmp_path, device):
    """The build's predictor dumped into subdirectories and loaded by EnsembleModel,
    TaperedModel and CombinedOutputModel through the registry (recursive load, as
    fv3fit's io.load): an ensemble of the same model predicts exactly the direct load,
    the taper is the oracle's taper of the direct prediction."""
    from fv3net_amd.composite import CombinedOutputModel, EnsembleModel, TaperedModel

    pred = _dense_predictor()
    P.dump(pred, str(tmp_path / "base_a"))
    P.dump(pred, str(tmp_path / "base_b"))
    X = _c48_rank_state(np.random.default_rng(1), device=device)
    direct = P.load(str(tmp_path / "base_a")).predict(X)
    for reduction in ("mean", "median"):
        path = str(tmp_path / f"ensemble_{reduction}")
        _write_composite(path, "ensemble", "ensemble_model.yaml",
                         {"models": [str(tmp_path / "base_a"), str(tmp_path / "base_b")], "reduction": reduction})
        ens = P.load(path)
        assert isinstance(ens, EnsembleModel)
        got = ens.predict(X)
        for k in ("dQ1", "dQ2"):
            assert got[k].dims == direct[k].dims
            _bits(got[k].values, direct[k].values)
    path = str(tmp_path / "tapered")
    _write_composite(path, "tapered_model", "tapered_model.yaml",
                     {"model": str(tmp_path / "base_a"), "tapering": {"dQ2": {"cutoff": 20, "rate": 4.0}}})
    tap = P.load(path)
    assert isinstance(tap, TaperedModel)
    got = tap.predict(X)
    _bits(got["dQ1"].values, direct["dQ1"].values)
    _bits(got["dQ2"].values, OC.taper(direct["dQ2"].values, 0, 20, 4.0))
    # a composite of composites: the tapered model combined with a constant predictor
    _, const = _constant(tmp_path, "const", ["air_temperature"], ["ml_flag"], ml_flag=1.0)
    path = str(tmp_path / "combined")
    _write_composite(path, "combined_output_model", "combined_output_model.yaml",
                     {"models": [str(tmp_path / "tapered"), const]})
    comb = P.load(path)
    assert isinstance(comb, CombinedOutputModel)
    got = comb.predict(X)
    _bits(got["dQ2"].values, OC.taper(direct["dQ2"].values, 0, 20, 4.0))
    assert (got["ml_flag"].values == 1.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("limit", [True, False])
@pytest.mark.parametrize("state_dtype", [np.float64, np.float32])
def test_adapter_matches_oracle(gpu, tmp_path, limit, state_dtype):
    """transformers/fv3fit.py Adapter over two models loaded from paths: dQ1 and a
    second model's output both mapped to air_temperature (summed), dQ2 to the
    humidity (limited, MSE-conserving), a state prediction passed through; bit for bit
    against oracle.composite.adapter_predict on the models' own predictions."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from fv3net_amd.transformers import Adapter, Config

    rng = np.random.default_rng(3)
    nz, n = 79, 48
    pa = _dense_predictor(seed=4)
    cfg_b = DenseModelConfig(["air_temperature"], ["dT_extra", "surface_flux"], [nz], [nz, 1], width=64, depth=2)
    mb = DenseColumnModel.random(cfg_b, seed=5, bias_scale=0.1,
                                 sample_inputs=[rng.normal(260, 15, (512, nz)).astype(np.float32)],
                                 sample_outputs=[rng.normal(0, 1e-5, (512, nz)).astype(np.float32),
                                                 rng.normal(0, 1, (512, 1)).astype(np.float32)])
    pb = P.DenseColumnPredictor(cfg_b.input_variables, cfg_b.output_variables, mb)
    P.dump(pa, str(tmp_path / "a"))
    P.dump(pb, str(tmp_path / "b"))
    config = Config(url=[str(tmp_path / "a"), str(tmp_path / "b")],
                    tendency_predictions={"dQ1": "air_temperature", "dT_extra": "air_temperature",
                                          "dQ2": "specific_humidity"},
                    state_predictions={"surface_flux": "surface_flux_state"}, limit_negative_humidity=limit)
    adapter = Adapter(config, 900.0)
    assert set(adapter.input_variables) == {"air_temperature", "specific_humidity"}
    T = rng.normal(260, 15, (nz, n, n)).astype(state_dtype)
    q = rng.uniform(0, 2e-5, (nz, n, n)).astype(state_dtype)  # dry enough for the limiter to fire
    attrs = {"units": "K"}
    inputs = {"air_temperature": D.DataArray(torch.from_numpy(T).cuda(), ["z", "y", "x"], attrs=attrs),
              "specific_humidity": D.DataArray(torch.from_numpy(q).cuda(), ["z", "y", "x"])}
    updates = adapter.predict(inputs)
    ds = D.Dataset(inputs)
    prediction = {}
    for m in adapter.model.models:
        p = m.predict(ds)
        prediction.update({k: p[k].values for k in p})
    ref = OC.adapter_predict(prediction, {"air_temperature": T, "specific_humidity": q},
                             config.tendency_predictions, config.state_predictions, 900.0, limit)
    assert sorted(updates) == sorted(ref)
    for k, r in ref.items():
        _bits(updates[k].values, r)
    assert updates["air_temperature"].attrs == attrs and updates["air_temperature"].dims == ("z", "y", "x")
    if limit:  # q + (-q / dt) * dt: zero up to the rounding of the reference's own expression
        assert (updates["specific_humidity"].values >= -1e-6 * np.abs(q).max()).all()
        raw = q + (prediction["dQ2"] * 900.0)
        assert (raw < 0).any()  # the limiter had something to do
    state = dict(inputs)
    adapter.apply(updates, state)
    assert state["air_temperature"] is updates["air_temperature"]


@pytest.mark.gpu
def test_adapter_limit_needs_humidity(gpu, tmp_path):
    from fv3net_amd.transformers import Adapter, Config

    pa = _dense_predictor(seed=4)
    adapter = Adapter(Config(url=[], tendency_predictions={"dQ1": "air_temperature"}), 900.0, models=[pa])
    X = _c48_rank_state(np.random.default_rng(0))
    with pytest.raises(NotImplementedError):
        adapter.predict({k: X[k] for k in X})


@pytest.mark.gpu
def test_ensemble_reduction_dispatch_is_case_sensitive(gpu):
    """models.py:239-260 validates ``reduction.lower()`` but dispatches on
    ``self._reduction == "median"``: a 'Median' config reduces with the mean."""
    from fv3net_amd.composite import EnsembleModel

    models = []
    for v in (0.0, 3.0, 5.0):
        m = P.ConstantOutputPredictor(["input"], ["output"])
        m.set_outputs(output=v)
        models.append(m)
    ds_in = D.Dataset({"input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"])})
    np.testing.assert_almost_equal(EnsembleModel(models, reduction="Median").predict(ds_in)["output"].values, 8.0 / 3)
    np.testing.assert_almost_equal(EnsembleModel(models, reduction="median").predict(ds_in)["output"].values, 3.0)


def test_oracle_adapter_float64_predictions_keep_float64():
    """A TaperedModel returns float64 (scaling * data): the sum, the limiter and the
    state update stay float64 even over a float32 state (numpy promotion)."""
    rng = np.random.default_rng(1)
    q = rng.uniform(0, 1e-5, (4, 6)).astype(np.float32)
    T = rng.normal(260, 5, (4, 6)).astype(np.float32)
    pred = {"dQ2": rng.normal(0, 1e-8, (4, 6)), "dQ1": rng.normal(0, 1e-4, (4, 6)).astype(np.float32)}
    up = OC.adapter_predict(pred, {"specific_humidity": q, "air_temperature": T},
                            {"dQ1": "air_temperature", "dQ2": "specific_humidity"}, {}, 900.0)
    assert up["specific_humidity"].dtype == np.float64 and up["air_temperature"].dtype == np.float64
    up = OC.adapter_predict(pred, {"specific_humidity": q, "air_temperature": T},
                            {"dQ1": "air_temperature", "dQ2": "specific_humidity"}, {}, 900.0, False)
    assert up["specific_humidity"].dtype == np.float64 and up["air_temperature"].dtype == np.float32


@pytest.mark.gpu
@pytest.mark.parametrize("limit", [True, False])
@pytest.mark.parametrize("state_dtype", [np.float64, np.float32])
def test_adapter_over_tapered_model_matches_oracle(gpu, tmp_path, limit, state_dtype):
    """The usual prognostic setup: Adapter over a TaperedModel nesting the
    build's predictor.  The taper returns float64 dQ2 (dQ1 untapered stays float32); a
    second model's float32 output is summed onto air_temperature after dQ1.  Each
    target's sum, limiter and update keep numpy's dtype flow (float64 humidity update
    over a float32 state), bit for bit against the oracle."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from fv3net_amd.transformers import Adapter, Config

    rng = np.random.default_rng(8)
    nz, n = 79, 32
    P.dump(_dense_predictor(seed=4), str(tmp_path / "base"))
    _write_composite(str(tmp_path / "tapered"), "tapered_model", "tapered_model.yaml",
                     {"model": str(tmp_path / "base"), "tapering": {"dQ2": {"cutoff": 30, "rate": 5.0}}})
    cfg_b = DenseModelConfig(["air_temperature"], ["dT_extra"], [nz], [nz], width=64, depth=2)
    mb = DenseColumnModel.random(cfg_b, seed=5, bias_scale=0.1,
                                 sample_inputs=[rng.normal(260, 15, (512, nz)).astype(np.float32)],
                                 sample_outputs=[rng.normal(0, 1e-5, (512, nz)).astype(np.float32)])
    P.dump(P.DenseColumnPredictor(cfg_b.input_variables, cfg_b.output_variables, mb), str(tmp_path / "b"))
    config = Config(url=[str(tmp_path / "tapered"), str(tmp_path / "b")],
                    tendency_predictions={"dQ1": "air_temperature", "dT_extra": "air_temperature",
                                          "dQ2": "specific_humidity"}, limit_negative_humidity=limit)
    adapter = Adapter(config, 900.0)
    T = rng.normal(260, 15, (nz, n, n)).astype(state_dtype)
    q = rng.uniform(0, 2e-5, (nz, n, n)).astype(state_dtype)
    inputs = {"air_temperature": D.DataArray(torch.from_numpy(T).cuda(), ["z", "y", "x"]),
              "specific_humidity": D.DataArray(torch.from_numpy(q).cuda(), ["z", "y", "x"])}
    updates = adapter.predict(inputs)
    ds = D.Dataset(inputs)
    prediction = {}
    for m in adapter.model.models:
        p = m.predict(ds)
        prediction.update({k: p[k].transpose("z", "y", "x").values for k in p})
    assert prediction["dQ2"].dtype == np.float64 and prediction["dQ1"].dtype == np.float32
    ref = OC.adapter_predict(prediction, {"air_temperature": T, "specific_humidity": q},
                             config.tendency_predictions, config.state_predictions, 900.0, limit)
    assert sorted(updates) == sorted(ref)
    for k, r in ref.items():
        _bits(updates[k].values, r)
