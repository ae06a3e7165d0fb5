"""DerivedModel / TransformedPredictor (SURVEY.md 8(b) "Composition") over the build's
predictor, with the vcm.DerivedMapping / DataTransform entries computed by
csrc/derived.hip, bit for bit against the numpy restatement oracle/derived.py.

Reference KATs mirrored: external/fv3fit/tests/test_derived_model.py,
external/fv3fit/tests/test_transformed_predictor.py.
"""
import numpy as np
import pytest
import yaml

from fv3net_amd import dataset as D
from fv3net_amd import predictor as P
from oracle import derived as OD

NZ = 79
SW_OVERRIDE = "override_for_time_adjusted_total_sky_downward_shortwave_flux_at_surface"


def _bits(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (what, a.shape, b.shape, a.dtype, b.dtype)
    same = (a.view(np.uint64 if a.dtype.itemsize == 8 else np.uint32)
            == b.view(np.uint64 if b.dtype.itemsize == 8 else np.uint32))
    assert same.all(), f"{what}: {(~same).sum()} differ, e.g. {a[~same][:3]} vs {b[~same][:3]}"


# ------------------------------------------------------------------ bookkeeping (CPU)
def _constant(inputs, outputs, **values):
    m = P.ConstantOutputPredictor(inputs, outputs)
    m.set_outputs(**values)
    return m


def test_wrap_another_derived_model():
    """test_derived_model.py:21-49 (inputs / outputs / the flattened base model)."""
    from fv3net_amd.derived import DerivedModel

    base_outputs = [SW_OVERRIDE, "dQ2"]
    base = _constant(["input"], base_outputs, **{SW_OVERRIDE: 1.0, "dQ2": 1.0})
    m0 = DerivedModel(base, derived_output_variables=["net_shortwave_sfc_flux_derived"])
    m1 = DerivedModel(m0, derived_output_variables=["Q2"])
    assert not isinstance(m1.base_model, DerivedModel)
    assert set(m1.input_variables) == {"input", "surface_diffused_shortwave_albedo",
                                       "pressure_thickness_of_atmospheric_layer", "pQ2"}
    assert set(m1.output_variables) == set(base_outputs) | {"Q2", "net_shortwave_sfc_flux_derived"}


def test_get_additional_inputs_and_errors():
    """test_derived_model.py:52-96."""
    from fv3net_amd.derived import DerivedModel

    base = _constant(["input"], [SW_OVERRIDE], **{SW_OVERRIDE: 1.0})
    m = DerivedModel(base, derived_output_variables=["net_shortwave_sfc_flux_derived"])
    assert m._additional_input_variables == ["surface_diffused_shortwave_albedo"]
    with pytest.raises(KeyError):
        m.predict(D.Dataset({"input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"])}))
    with pytest.raises(ValueError):
        DerivedModel(base, derived_output_variables=["variable_not_in_DerivedMapping"])


def test_transformed_predictor_variables():
    """test_transformed_predictor.py:55-67 and the ChainedDataTransform bookkeeping."""
    from fv3net_amd.derived import ChainedDataTransform, DataTransform, TransformedPredictor

    t = [DataTransform("Qm_from_Q1_Q2")]
    m = TransformedPredictor(_constant(["input"], ["Q1", "Q2"], Q1=1.0, Q2=2.0), t)
    assert m.input_variables == ["input"] and m.output_variables == ["Q1", "Q2", "Qm"]
    m = TransformedPredictor(_constant(["input"], ["Q1"]), t)
    assert m.input_variables == ["Q2", "input"] and m.output_variables == ["Q1", "Qm"]
    chain = ChainedDataTransform([DataTransform("Q1_from_dQ1_pQ1"), DataTransform("Q2_from_dQ2_pQ2"),
                                  DataTransform("Qm_from_Q1_Q2"), DataTransform("Q2_flux_from_Q2_tendency")])
    assert chain.input_variables == sorted(["dQ1", "pQ1", "dQ2", "pQ2", OD.DELP, OD.LHF])
    assert chain.output_variables == sorted(["Q1", "Q2", "Qm", "Q2_flux", "implied_surface_precipitation_rate"])
    with pytest.raises(ValueError):
        DataTransform("not_a_transform")


def test_registry_names_match_the_reference():
    """Every vcm.DerivedMapping entry (derived_mapping.py:114-410) and DataTransform
    (data_transform.py:24-41) is known under the reference's name."""
    from fv3net_amd.derived import DATA_TRANSFORM_REGISTRY, DerivedMapping

    assert set(DerivedMapping.VARIABLES) == {
        "cos_zenith_angle", "evaporation", "dQu", "dQv", "eastward_wind", "northward_wind",
        "dQu_parallel_to_eastward_wind", "dQv_parallel_to_northward_wind",
        "horizontal_wind_tendency_parallel_to_horizontal_wind", "net_shortwave_sfc_flux_derived",
        "downward_shortwave_sfc_flux_via_transmissivity", "net_shortwave_sfc_flux_via_transmissivity", "is_land",
        "is_sea", "is_sea_ice", "Q1", "Q2", "pQ1", "pQ2", "internal_energy", "column_integrated_dQ1",
        "column_integrated_dQ2", "column_integrated_Q1", "column_integrated_Q2", "water_vapor_path",
        "upward_heat_flux_at_surface", "incloud_water_mixing_ratio", "incloud_ice_mixing_ratio"}
    assert set(DATA_TRANSFORM_REGISTRY) == {
        "Q1_from_Qm_Q2", "Qm_from_Q1_Q2", "Q1_from_Qm_Q2_temperature_dependent",
        "Qm_from_Q1_Q2_temperature_dependent", "Q1_from_dQ1_pQ1", "Q2_from_dQ2_pQ2", "Qm_flux_from_Qm_tendency",
        "Q2_flux_from_Q2_tendency", "Qm_tendency_from_Qm_flux", "Q2_tendency_from_Q2_flux",
        "implied_surface_precipitation_rate", "implied_downward_radiative_flux_at_surface", "tapered_dQ1",
        "tapered_dQ2", "cloud_water_mixing_ratio_from_incloud", "cloud_ice_mixing_ratio_from_incloud"}


def test_oracle_pairwise_order_matches_numpy():
    """The z-last mass integral is numpy's pairwise sum (what the kernel replays)."""
    rng = np.random.default_rng(0)
    x = rng.normal(0, 1e3, (6, 79)).astype(np.float32)
    d = rng.uniform(100, 2000, (6, 79)).astype(np.float32)
    seq = OD.mass_integrate(x.T, d.T)
    pw = np.nansum(x * d / OD.GRAVITY, axis=-1)
    assert not np.array_equal(seq, pw)  # the order matters at float32


# ------------------------------------------------------------------------------ GPU
def _dense_predictor(seed=2):
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    cfg = DenseModelConfig(["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [NZ, NZ], [NZ, NZ],
                           width=128, depth=3)
    rng = np.random.default_rng(seed)
    sT = rng.normal(260, 15, (2048, NZ)).astype(np.float32)
    sq = rng.uniform(0, 0.02, (2048, NZ)).astype(np.float32)
    out = [rng.normal(0, 1e-4, (2048, NZ)).astype(np.float32), rng.normal(0, 3e-8, (2048, NZ)).astype(np.float32)]
    m = DenseColumnModel.random(cfg, seed=seed, sample_inputs=[sT, sq], sample_outputs=out, bias_scale=0.1)
    return P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)


def _state(rng, dtype, n=24, device=True, nans=True):
    """(z, y, x) state + 2-D surface fields, as a Dataset (device or host arrays)."""
    import torch

    f3 = lambda a: a.astype(dtype)  # noqa: E731
    base = np.linspace(200, 1800, NZ)[:, None, None]
    st = {"air_temperature": f3(rng.normal(260, 15, (NZ, n, n))),
          "specific_humidity": f3(rng.uniform(0, 0.02, (NZ, n, n))),
          OD.DELP: f3(base * rng.uniform(0.95, 1.05, (NZ, n, n))),
          "pQ1": f3(rng.normal(0, 1e-4, (NZ, n, n))),
          "pQ2": f3(rng.normal(0, 1e-8, (NZ, n, n))),
          "cloud_amount": f3(rng.uniform(-0.01, 1.0, (NZ, n, n))),
          "cloud_water_mixing_ratio": f3(rng.uniform(0, 1e-4, (NZ, n, n))),
          "cloud_ice_mixing_ratio": f3(rng.uniform(0, 1e-5, (NZ, n, n)))}
    st["cloud_amount"][:, 0, :5] = [0.0, 1e-3, 2e-3, 0.05, 0.06]  # the climit edges
    if nans:
        st["specific_humidity"][3, 1, 2] = np.nan
    sfc = {k: rng.normal(100, 50, (n, n)).astype(dtype) for k in (
        OD.LHF, OD.SHF, OD.USW_SFC, OD.ULW_SFC, OD.ULW_TOA, OD.USW_TOA, OD.DSW_TOA, OD.COL_T_NUDGE, SW_OVERRIDE,
        "total_sky_downward_shortwave_flux_at_surface", "total_sky_downward_longwave_flux_at_surface")}
    sfc["surface_diffused_shortwave_albedo"] = rng.uniform(0, 1, (n, n)).astype(dtype)
    sfc["shortwave_transmissivity_of_atmospheric_column"] = rng.uniform(0, 1, (n, n)).astype(dtype)
    sfc["land_sea_mask"] = rng.integers(0, 3, (n, n)).astype(dtype)
    sfc["land_sea_mask"][0, :3] = [1.00001, 2.0001, np.nan]  # close / not close / NaN
    conv = (lambda a: torch.from_numpy(a).cuda()) if device else (lambda a: a)
    ds = D.Dataset({k: D.DataArray(conv(v), ["z", "y", "x"]) for k, v in st.items()})
    for k, v in sfc.items():
        ds[k] = D.DataArray(conv(v), ["y", "x"])
    return ds, {**st, **sfc}


DERIVED = ["Q1", "Q2", "pQ2", "internal_energy", "column_integrated_dQ1", "column_integrated_dQ2",
           "water_vapor_path", "evaporation", "upward_heat_flux_at_surface", "incloud_water_mixing_ratio",
           "incloud_ice_mixing_ratio", "net_shortwave_sfc_flux_derived",
           "net_shortwave_sfc_flux_via_transmissivity", "is_land", "is_sea", "is_sea_ice"]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("device", [True, False])
def test_derived_model_over_dense_predictor(gpu, tmp_path, dtype, device):
    """An mi355x-dense predictor nested in a DerivedModel, dumped and loaded through the
    registry: the base prediction passes through bit-identically and every derived
    variable equals the numpy restatement over (state + prediction), bit for bit."""
    from fv3net_amd.derived import DerivedModel

    rng = np.random.default_rng(5)
    X, arrays = _state(rng, dtype, device=device)
    base = _dense_predictor()
    model = DerivedModel(base, DERIVED)
    P.dump(model, str(tmp_path / "derived"))
    loaded = P.load(str(tmp_path / "derived"))
    assert isinstance(loaded, DerivedModel) and loaded.output_variables == model.output_variables
    assert set(model.input_variables) >= {"air_temperature", "specific_humidity", OD.DELP, "pQ1"}
    out = loaded.predict(X)
    direct = base.predict(X)
    m = dict(arrays)
    for k in ("dQ1", "dQ2"):
        _bits(out[k].values, direct[k].values, k)
        m[k] = direct[k].values
    for name in DERIVED:
        _bits(out[name].values, OD.derived(name, m), name)
        assert hasattr(out[name].data, "is_cuda") == device, name  # device in, device out
    # without pQ2 in the data: pQ2 = zeros_like(delp), Q2 = dQ2 + 0 in promote(dQ2, delp)
    from fv3net_amd.derived import DerivedMapping

    mp = DerivedMapping(D.Dataset({"dQ2": out["dQ2"], OD.DELP: X[OD.DELP]}))
    m.pop("pQ2")
    _bits(mp["Q2"].values, OD.derived("Q2", m), "Q2 with pQ2 = zeros_like(delp)")
    _bits(mp["pQ2"].values, np.zeros_like(arrays[OD.DELP]), "pQ2 = zeros_like(delp)")


@pytest.mark.gpu
def test_derived_column_integrals_z_last_pairwise(gpu):
    """A (y, x, z) prediction: numpy sums the contiguous last axis pairwise, and the kernel
    replays that order (it differs from the level-ordered sum at float32)."""
    import torch

    from fv3net_amd.derived import DerivedMapping

    rng = np.random.default_rng(9)
    n = 16
    for nz in (3, 8, 79, 128):
        dq = rng.normal(0, 1e3, (n, n, nz)).astype(np.float32)
        dq[2, 3, nz // 2] = np.nan
        dp = rng.uniform(100, 2000, (n, n, nz)).astype(np.float32)
        ds = D.Dataset({"dQ1": D.DataArray(torch.from_numpy(dq).cuda(), ["y", "x", "z"]),
                        "dQ2": D.DataArray(torch.from_numpy(dq).cuda(), ["y", "x", "z"]),
                        OD.DELP: D.DataArray(torch.from_numpy(dp).cuda(), ["y", "x", "z"])})
        dm = DerivedMapping(ds)
        got = dm["column_integrated_dQ1"].values
        ref = (OD.CP - OD.RDGAS) * np.nansum(dq * dp / OD.GRAVITY, axis=-1)
        _bits(got, ref, f"z-last nz={nz}")
        got = dm["column_integrated_dQ2"].values
        ref = -(OD.KG_M2S_TO_MM_DAY * np.nansum(dq * -1 * dp / OD.GRAVITY, axis=-1))
        _bits(got, ref, f"z-last moistening nz={nz}")


TRANSFORM_CHAINS = [
    [("Q1_from_dQ1_pQ1", {}), ("Q2_from_dQ2_pQ2", {}), ("Qm_from_Q1_Q2", {}), ("Q2_flux_from_Q2_tendency", {}),
     ("Qm_flux_from_Qm_tendency", {}), ("Q2_tendency_from_Q2_flux", {}), ("Qm_tendency_from_Qm_flux", {}),
     ("Q1_from_Qm_Q2", {})],
    [("Q1_from_dQ1_pQ1", {}), ("Q2_from_dQ2_pQ2", {}), ("Qm_from_Q1_Q2_temperature_dependent", {}),
     ("implied_surface_precipitation_rate", {"rectify": False}),
     ("implied_downward_radiative_flux_at_surface", {"include_temperature_nudging": False}),
     ("Q1_from_Qm_Q2_temperature_dependent", {}), ("tapered_dQ1", {"cutoff": 25, "rate": 5.0}),
     ("tapered_dQ2", {"cutoff": 10, "rate": 2.0}), ("cloud_water_mixing_ratio_from_incloud", {}),
     ("cloud_ice_mixing_ratio_from_incloud", {})],
    [("Q2_from_dQ2_pQ2", {}), ("Q2_flux_from_Q2_tendency", {"rectify_surface_precipitation_rate": False}),
     ("Q2_tendency_from_Q2_flux", {}), ("Q1_from_dQ1_pQ1", {}), ("Qm_from_Q1_Q2", {}),
     ("Qm_flux_from_Qm_tendency", {"rectify_downward_radiative_flux": False,
                                   "include_temperature_nudging": False})],
]


@pytest.mark.gpu
@pytest.mark.parametrize("chain", range(len(TRANSFORM_CHAINS)))
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_transformed_predictor_over_dense_predictor(gpu, tmp_path, chain, dtype):
    """An mi355x-dense predictor nested in a TransformedPredictor, dumped and loaded:
    every transform of the chain (flux form and back, MSE and back, tapers, condensate)
    bit for bit against the numpy restatement applied to the same prediction."""
    from fv3net_amd.derived import DataTransform, TransformedPredictor

    rng = np.random.default_rng(chain + 3)
    X, arrays = _state(rng, dtype, nans=False)
    arrays["incloud_water_mixing_ratio"] = arrays["cloud_water_mixing_ratio"] * 3
    arrays["incloud_ice_mixing_ratio"] = arrays["cloud_ice_mixing_ratio"] * 3
    import torch

    for k in ("incloud_water_mixing_ratio", "incloud_ice_mixing_ratio"):
        X[k] = D.DataArray(torch.from_numpy(arrays[k]).cuda(), ["z", "y", "x"])
    base = _dense_predictor(seed=7)
    transforms = [DataTransform(name, kw) for name, kw in TRANSFORM_CHAINS[chain]]
    model = TransformedPredictor(base, transforms)
    P.dump(model, str(tmp_path / "transformed"))
    with open(tmp_path / "transformed" / "output_transformed_model.yaml") as f:
        assert [t["name"] for t in yaml.safe_load(f)["transforms"]] == [n for n, _ in TRANSFORM_CHAINS[chain]]
    loaded = P.load(str(tmp_path / "transformed"))
    out = loaded.predict(X)
    pred = base.predict(X)
    ds = dict(arrays)
    ds.update({k: pred[k].values for k in pred})
    for name, kw in TRANSFORM_CHAINS[chain]:
        ds = OD.apply_transform(name, ds, **kw)
    assert sorted(out) == sorted(set(pred) | set(model.output_transform.output_variables))
    for k in model.output_transform.output_variables:
        _bits(out[k].values, ds[k], k)


@pytest.mark.gpu
def test_transformed_prediction_kats(gpu):
    """test_transformed_predictor.py:18-52 on constant predictors (host arrays)."""
    from fv3net_amd.derived import DataTransform, TransformedPredictor

    t = [DataTransform("Qm_from_Q1_Q2")]
    m = TransformedPredictor(_constant(["input"], ["Q1", "Q2"], Q1=1.0, Q2=2.0), t)
    out = m.predict(D.Dataset({"input": D.DataArray(np.array([0.0, 1.0, 2.0]), ["x"])}))
    assert "Qm" in out
    np.testing.assert_array_equal(out["Qm"].values, OD.moist_static_energy_tendency(np.ones(3), np.full(3, 2.0)))
    base = _constant(["input"], ["Q1"], Q1=np.array([5.0, 6.0, 7.0]))
    m = TransformedPredictor(base, t)
    X = D.Dataset({"input": D.DataArray(np.array([0.0, 1.0, 2.0]), ["x"]),
                   "Q2": D.DataArray(np.array([0.0, 1.0, 2.0]), ["z"]),
                   "Qm": D.DataArray(np.array([3.0, 4.0, 5.0]), ["z"])})
    out = m.predict(X)
    assert "Qm" in out and "Q2" not in out
    q1 = base.predict(X)["Q1"].transpose("z", "x").values
    ref = OD.moist_static_energy_tendency(q1, np.array([0.0, 1.0, 2.0])[:, None])
    np.testing.assert_array_equal(out["Qm"].transpose("z", "x").values, ref)


@pytest.mark.gpu
def test_derived_prediction_kat(gpu, tmp_path):
    """test_derived_model.py:63-130: prediction, dump and load, on host arrays."""
    from fv3net_amd.derived import DerivedModel

    base = _constant(["input"], [SW_OVERRIDE], **{SW_OVERRIDE: 1.0})
    m = DerivedModel(base, derived_output_variables=["net_shortwave_sfc_flux_derived"])
    X = D.Dataset({"input": D.DataArray(np.zeros([3, 3, 5]), ["x", "y", "z"]),
                   "surface_diffused_shortwave_albedo": D.DataArray(np.full([3, 3], 0.25), ["x", "y"])})
    pred = m.predict(X)
    np.testing.assert_array_equal(pred["net_shortwave_sfc_flux_derived"].values, np.full([3, 3], 0.75))
    P.dump(m, str(tmp_path / "d"))
    again = P.load(str(tmp_path / "d")).predict(X)
    for k in pred:
        np.testing.assert_array_equal(again[k].values, pred[k].values)
