"""The microphysics emulator hook's classifier head and masks: the
oracle against the reference's own KATs, and the HIP kernels against the oracle.

Reference KATs: external/emulation/tests/test_zhao_carr.py:15-66, 107-147,
test_mask.py:7-50, test_models.py:7-50."""
import numpy as np
import pytest

from oracle import emulation as OE


# ------------------------------------------------------------------ oracle vs KATs
def test_oracle_limit_net_condensation_kat():
    qv = np.array([[1, 1, 1], [0, 0, 0]], dtype=np.float64)
    qc = np.array([[0, 0, 0], [1, 1, 0]], dtype=np.float64)
    net = np.array([[1.5, 0.5, 0], [-1.5, -0.5, 0]], dtype=np.float64)
    got = OE.limit_net_condensation({OE.QC_IN: qc, OE.QV_IN: qv}, net)
    np.testing.assert_array_equal(got, [[1, 0.5, 0], [-1, -0.5, 0]])


@pytest.mark.parametrize("t,cloud,expected", [
    ([[10, 0, -10, -15, -16]], [[0, 0, 0, 1, 0]], [[0, 0, 0.0, 1.0, 1.0]]),
    ([[-14, -16]], [[0, 0]], [[0, 1.0]]),
])
def test_oracle_ice_water_flag_kats(t, cloud, expected):
    t, cloud = np.array(t, np.float64), np.array(cloud, np.float64)
    np.testing.assert_array_equal(OE.ice_water_flag(t, cloud), expected)
    np.testing.assert_array_equal(OE.ice_water_flag_fast(t, cloud), expected)


def test_oracle_ice_flag_fast_matches_loop():
    rng = np.random.default_rng(0)
    t = rng.uniform(-20, 5, (7, 300))
    cloud = np.where(rng.uniform(size=t.shape) < 0.8, 1e-5, 0.0)
    np.testing.assert_array_equal(OE.ice_water_flag(t, cloud), OE.ice_water_flag_fast(t, cloud))


def test_oracle_strict_precip_kat():
    c_to_p = np.array([[1.0], [-2.0], [3.0]])
    p_to_v = np.array([[4.0], [-1.0], [2.0]])
    c, p, total = OE.strict_precip(c_to_p, p_to_v)
    np.testing.assert_equal(c, [[1.0], [0.0], [3.0]])
    np.testing.assert_equal(p, [[2.0], [0.0], [2.0]])
    np.testing.assert_equal(total, np.zeros_like(total))


def _zc_states(shp=(5, 10)):
    state = {OE.QC_GS: np.ones(shp) * 4, OE.QV_GS: np.ones(shp), OE.T_GS: np.ones(shp) * 10, OE.DELP: np.ones(shp)}
    emulator = {OE.QC_PR: np.ones(shp) * 2, OE.QV_PR: np.ones(shp) * 2}
    return state, emulator


def test_oracle_enforce_conservative_overwrite_kat():
    state, _ = _zc_states()
    dummy = -1 * np.ones_like(state[OE.QV_GS])
    emulator = {OE.QC_PR: dummy * -10, OE.QV_PR: dummy, OE.T_PR: dummy, OE.PRECIP: dummy}
    result = {**emulator, **OE.precpd_conservative(state, emulator)}
    for v in result.values():
        assert not np.any(v == -1)
    assert not np.any(result[OE.QC_PR] == 10)


def test_oracle_range_and_level_mask_kats():
    assert OE.range_mask(np.float64(1.5), 0, 1) == 1.0 and OE.range_mask(np.float64(-1.5), 0, 1) == 0
    ones, zeros = np.ones((4, 2)), np.zeros((4, 2))
    for start, stop in [(2, 3), (2, 5), (None, 2), (None, None)]:
        r = OE.level_mask(ones, zeros, start, stop)
        np.testing.assert_array_equal(r[slice(start, stop)], zeros[slice(start, stop)])
        assert r.sum() == r.size - zeros[slice(start, stop)].size


# -------------------------------------------------------------------- device vs oracle
def _state(rng, dtype, nz=79, ncol=3000):
    lev = np.linspace(0, 1, nz)[:, None]
    s = {
        OE.T_IN: (200 + 100 * lev + rng.normal(0, 10, (nz, ncol))).astype(dtype),
        OE.QV_IN: (0.02 * np.exp(-6 * lev) * rng.uniform(0, 1, (nz, ncol))).astype(dtype),
        OE.QC_IN: (1e-4 * rng.uniform(0, 1, (nz, ncol)) * (rng.uniform(size=(nz, ncol)) < 0.5)).astype(dtype),
        OE.DELP: (200 + 1600 * lev * rng.uniform(0.95, 1.05, (nz, ncol))).astype(dtype),
    }
    s[OE.QC_GS] = (s[OE.QC_IN] * rng.uniform(0, 2, (nz, ncol)) * (rng.uniform(size=(nz, ncol)) < 0.7)).astype(dtype)
    s[OE.QC_GS][:, :50] = s[OE.QC_IN][:, :50]  # identical clouds
    s[OE.QV_GS] = (s[OE.QV_IN] + rng.normal(0, 1e-5, (nz, ncol))).astype(dtype)
    s[OE.T_GS] = (s[OE.T_IN] + rng.normal(0, 0.1, (nz, ncol))).astype(dtype)
    emu = {
        OE.QC_GS: (s[OE.QC_IN] + rng.normal(0, 5e-5, (nz, ncol))).astype(dtype),
        OE.QV_GS: (s[OE.QV_IN] + rng.normal(0, 1e-5, (nz, ncol))).astype(dtype),
        OE.QC_PR: (s[OE.QC_GS] + rng.normal(0, 5e-5, (nz, ncol))).astype(dtype),
        OE.QV_PR: (s[OE.QV_GS] + rng.normal(0, 1e-5, (nz, ncol))).astype(dtype),
        "gscond_classes": rng.normal(0, 1, (4, nz, ncol)).astype(dtype),
        "precpd_classes": rng.normal(0, 1, (4, nz, ncol)).astype(dtype),
    }
    emu["gscond_classes"][:, 0, :5] = 1.0  # ties: every class maximal
    emu[OE.QC_GS][3, 7] = np.nan
    return s, emu


def _dev(d):
    import torch

    return {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in d.items()}


def _bits(got, ref):
    got = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert got.dtype == ref.dtype, (got.dtype, ref.dtype)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref)) if got.dtype.kind == "f" else (got == ref)
    assert same.all(), f"{(~same).sum()} of {same.size} differ"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_gscond_masks_match_oracle(gpu, dtype):
    from fv3net_amd import emulation as E

    rng = np.random.default_rng(1)
    s, emu = _state(rng, dtype)
    ds, de = _dev(s), _dev(emu)
    cases = [
        (E.enforce_conservative_gscond, OE.gscond_update(s, emu[OE.QC_GS])),
        (E.mask_where_fortran_cloud_identical,
         OE.gscond_update(s, np.where(s[OE.QC_GS] == s[OE.QC_IN], s[OE.QC_IN], emu[OE.QC_GS]))),
        (E.mask_where_fortran_cloud_vanishes_gscond,
         OE.gscond_update(s, np.where(s[OE.QC_GS] < 1e-15, 0, emu[OE.QC_GS]))),
        (E.mask_zero_cloud_classifier,
         OE.gscond_update(s, np.where(OE.classify(emu["gscond_classes"])["zero_cloud"], 0, emu[OE.QC_GS]))),
        (E.mask_zero_tend_classifier,
         OE.gscond_update(s, np.where(OE.classify(emu["gscond_classes"])["zero_tendency"], s[OE.QC_IN],
                                      emu[OE.QC_GS]))),
        (E.enforce_conservative_phase_dependent, OE.phase_dependent(s, emu)),
    ]
    for fn, ref in cases:
        got = fn(ds, de)
        for k, r in ref.items():
            _bits(got[k], r)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_cloud_fixers_match_oracle(gpu, dtype):
    from fv3net_amd import emulation as E

    rng = np.random.default_rng(2)
    s, emu = _state(rng, dtype)
    ds, de = _dev(s), _dev(emu)
    _bits(E.infer_gscond_cloud_from_conservation(ds, de)[OE.QC_GS], OE.infer_cloud(s, emu))
    got = E.squash_gscond(ds, de, 2e-5)
    c, h = OE.squash(emu[OE.QC_GS], emu[OE.QV_GS], 2e-5)
    _bits(got[OE.QC_GS], c)
    _bits(got[OE.QV_GS], h)
    got = E.squash_precpd(ds, de, 2e-5)
    c, h = OE.squash(emu[OE.QC_PR], emu[OE.QV_PR], 2e-5)
    _bits(got[OE.QC_PR], c)
    _bits(got[OE.QV_PR], h)
    got = E.mask_zero_cloud_classifier_precpd(ds, de)
    _bits(got[OE.QC_PR], np.where(OE.classify(emu["precpd_classes"])["zero_cloud"], 0, emu[OE.QC_PR]))
    got = E.enforce_conservative_precpd(ds, de)
    for k, r in OE.precpd_conservative(s, {k: v.copy() for k, v in emu.items()}).items():
        _bits(got[k], r)
    _bits(E.conservative_precip_simple(ds, de)[OE.PRECIP], OE.precip_simple(s, emu))
    got = E.RangeMask(OE.QV_PR, min=0.0, max=0.015)(ds, de)
    _bits(got[OE.QV_PR], OE.range_mask(emu[OE.QV_PR], 0.0, 0.015))
    got = E.LevelMask(OE.QC_PR, 70, None, fill_value=OE.QC_GS)(ds, de)  # levels from state[fill_value]
    _bits(got[OE.QC_PR], OE.level_mask(emu[OE.QC_PR], s[OE.QC_GS], 70, None))
    got = E.LevelMask(OE.QC_GS, None, 5)(ds, de)  # levels from the Fortran state's own field
    _bits(got[OE.QC_GS], OE.level_mask(emu[OE.QC_GS], s[OE.QC_GS], None, 5))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_classify_and_ice_flag_match_oracle(gpu, dtype):
    """One-hot decoding (ties, NaN logits) and the ice-water recurrence across chunk
    boundaries: rows of 5000 with long cloudy runs in the middle temperature band."""
    import torch

    from fv3net_amd import emulation as E

    rng = np.random.default_rng(3)
    logits = rng.normal(0, 1, (4, 9, 700)).astype(dtype)
    logits[:, 1, 3] = 0.5
    logits[2, 2, 4] = np.nan
    got = E.classify_output(torch.from_numpy(logits).cuda())
    for k, r in OE.classify(logits).items():
        _bits(got[k], r.astype(np.uint8))
    got = E.classify_output(torch.from_numpy(np.ascontiguousarray(np.moveaxis(logits, 0, -1))).cuda(), one_hot_axis=-1)
    for k, r in OE.classify(logits).items():
        _bits(got[k], r.astype(np.uint8))
    z = 5000
    t = rng.uniform(258.16 - 20, 273.16 + 2, (6, z)).astype(dtype)
    t[:, 1000:2600] = 265.0  # a long middle-band run: the flag propagates over chunks
    t[:, 2599] = 250.0
    cloud = np.where(rng.uniform(size=(6, z)) < 0.97, 1e-5, 0.0).astype(dtype)
    cloud[:, 1000:2600] = 1e-5
    iw = E.ice_water_flag(torch.from_numpy(t).cuda(), torch.from_numpy(cloud).cuda())
    _bits(iw, OE.ice_water_flag_fast(t - dtype(273.16) if dtype == np.float32 else t - 273.16, cloud))
    assert iw.cpu().numpy()[:, 1000:2600].all()


@pytest.mark.gpu
def test_mask_config_composition_matches_oracle(gpu):
    """MaskConfig builds the reference's mask chain in config.py's order."""
    from fv3net_amd import emulation as E

    rng = np.random.default_rng(4)
    s, emu = _state(rng, np.float32)
    cfg = E.MaskConfig(ranges={OE.QV_PR: E.Range(min=0.0)}, gscond_cloud_conservative=True, cloud_squash=1e-6,
                       mask_gscond_zero_cloud=True, enforce_conservative=True,
                       enforce_strict_precpd_conservative=True,
                       mask_emulator_levels={OE.QC_PR: E.LevelSlice(75, None, 0.0)})
    got = cfg.build_mask()(_dev(s), _dev(emu))
    ref = dict(emu)
    ref[OE.QV_PR] = OE.range_mask(ref[OE.QV_PR], 0.0)
    ref[OE.QC_GS] = OE.infer_cloud(s, ref)
    ref[OE.QC_GS], ref[OE.QV_GS] = OE.squash(ref[OE.QC_GS], ref[OE.QV_GS], 1e-6)
    ref[OE.QC_PR], ref[OE.QV_PR] = OE.squash(ref[OE.QC_PR], ref[OE.QV_PR], 1e-6)
    ref.update(OE.gscond_update(s, np.where(s[OE.QC_GS] < np.float32(1e-15), 0, ref[OE.QC_GS])))
    ref.update(OE.gscond_update(s, ref[OE.QC_GS]))
    ref.update(OE.precpd_conservative(s, {k: v.copy() for k, v in ref.items()}))
    ref[OE.QC_PR] = ref[OE.QC_PR].copy()
    ref[OE.QC_PR][75:] = 0.0
    for k in (OE.QC_GS, OE.QV_GS, OE.T_GS, OE.QC_PR, OE.QV_PR, OE.T_PR, OE.PRECIP):
        _bits(got[k], ref[k])
    with pytest.raises(ValueError):
        E.MaskConfig(enforce_conservative=True, enforce_conservative_phase_dependent=True)


@pytest.mark.gpu
def test_model_with_classifier(gpu):
    """models.py:14-53 (test_models.py:7-50): the classifier's logits decoded into one-hot
    class masks that reach the regressor's inputs and the outputs; no classifier: the
    regressor alone; inputs_to_ignore dropped."""
    import torch

    from fv3net_amd import emulation as E
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    rng = np.random.default_rng(5)
    nz, ncol = 79, 1000
    a = rng.normal(0, 1, (nz, ncol)).astype(np.float32)
    cfg = DenseModelConfig(["a"], ["gscond_classes"], [nz], [4 * nz], width=32, depth=2)
    clf = E.ClassifierModel(DenseColumnModel.random(cfg, seed=3, sample_inputs=[a.T]))
    seen = {}

    def regressor(x):
        seen.update(x)
        return {"air_temperature_output": x["a"]}

    model = E.combine_classifier_and_regressor(clf, regressor)
    out = model({"a": torch.from_numpy(a).cuda(), "rank": 0})
    assert "rank" not in seen and set(E.CLASS_NAMES) <= set(seen) and "nontrivial_tendency" in seen
    assert set(E.CLASS_NAMES) <= set(out) and "air_temperature_after_precpd" in out
    logits = clf({"a": torch.from_numpy(a).cuda()})["gscond_classes"].cpu().numpy()
    assert logits.shape == (4, nz, ncol)
    for k, r in OE.classify(logits).items():
        _bits(out[k], r.astype(np.uint8))
    plain = E.ModelWithClassifier(regressor, classifier=None)({"a": torch.from_numpy(a).cuda()})
    assert set(plain) == {"air_temperature_output"}


# ---- TimeMask / IntervalSchedule (_emulate/microphysics.py:23-47) ----------------------
def test_interval_schedule_reference_kats():
    """test_microphysics.py:47-56, on the Julian calendar the reference's cftime uses."""
    import datetime

    from fv3net_amd.emulation import IntervalSchedule, JulianTime

    scheduler = IntervalSchedule(datetime.timedelta(hours=3), JulianTime(2000, 1, 1))
    assert scheduler(JulianTime(2000, 1, 1)) == 1
    assert scheduler(JulianTime(2000, 1, 1, 1)) == 1
    assert scheduler(JulianTime(2000, 1, 1, 1, 30)) == 0
    assert scheduler(JulianTime(2000, 1, 1, 2)) == 0
    assert scheduler(JulianTime(2000, 1, 20)) == 1
    # Julian-calendar day counts: 1900 is a leap year there (not in the Gregorian one)
    assert JulianTime(1900, 3, 1) - JulianTime(1900, 2, 28) == datetime.timedelta(days=2)
    assert JulianTime(2001, 1, 1) - JulianTime(2000, 1, 1) == datetime.timedelta(days=366)


@pytest.mark.parametrize("weight", [0.0, 0.5, 1.0])
def test_time_mask_reference_kat(weight):
    """test_microphysics.py:58-64: Python numbers blend as Python does; only the keys
    both dicts hold are returned; model_time[3] is skipped (_time.py:6-13)."""
    from fv3net_amd.emulation import TimeMask

    mask = TimeMask(schedule=lambda time: weight)
    left = {"a": 0.0, "model_time": [2021, 1, 1, 0, 0, 0]}
    right = {"a": 1.0}
    assert mask(left, right) == {"a": 1 - weight}


def test_mask_config_time_mask_first():
    """config.py:176-177: the online schedule's TimeMask is the first mask."""
    from fv3net_amd.emulation import MaskConfig, Range, RangeMask, TimeMask

    def schedule(time):
        return 1.0

    masks = list(MaskConfig(ranges={"x": Range(min=0.0)}, online_schedule=schedule).build_masks())
    assert isinstance(masks[0], TimeMask) and masks[0].schedule is schedule
    assert isinstance(masks[1], RangeMask)
    assert not any(isinstance(m, TimeMask) for m in MaskConfig().build_masks())


@pytest.mark.gpu
@pytest.mark.parametrize("ds,de", [(np.float64, np.float64), (np.float64, np.float32), (np.float32, np.float64),
                                   (np.float32, np.float32)])
def test_time_mask_blend_matches_numpy(gpu, ds, de):
    """fv3_time_blend: bitwise numpy's `state * alpha + emulator * (1 - alpha)` (NumPy 2
    weak scalars: each product in its array's dtype, the sum promoted), NaN / inf
    included; keys only one side holds are left out, as in the reference."""
    import datetime

    import torch

    from fv3net_amd.emulation import IntervalSchedule, JulianTime, TimeMask

    rng = np.random.default_rng(11)
    s = rng.normal(0, 1, (79, 1000)).astype(ds)
    e = rng.normal(0, 1, (79, 1000)).astype(de)
    s[0, :3] = [np.nan, np.inf, -0.0]
    e[1, :3] = [np.inf, np.nan, 0.0]
    for alpha in (0.0, 1.0, 0.5, 0.3):
        mask = TimeMask(schedule=lambda t, a=alpha: a)
        out = mask({"x": torch.from_numpy(s).cuda(), "model_time": [2021, 1, 1, 0, 0, 0], "only_state": 1.0},
                   {"x": torch.from_numpy(e).cuda(), "only_emulator": 2.0})
        assert set(out) == {"x"}
        ref = s * alpha + e * (1 - alpha)
        got = out["x"].cpu().numpy()
        assert got.dtype == ref.dtype
        assert ((got.view(np.uint8) == ref.view(np.uint8)).all()), alpha
    # the interval schedule picks the state in the first half of each period
    sched = IntervalSchedule(datetime.timedelta(hours=3), JulianTime(2021, 1, 1))
    st = {"x": torch.from_numpy(s).cuda(), "model_time": [2021, 1, 1, 0, 2, 0]}  # hour 2: second half
    got = TimeMask(sched)(st, {"x": torch.from_numpy(e).cuda()})["x"].cpu().numpy()
    ref = s * 0.0 + e * 1.0
    assert (got.view(np.uint8) == ref.view(np.uint8)).all()
