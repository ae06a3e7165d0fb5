"""Zhao-Carr microphysics emulator (BASELINE config #5): the fused
kernel vs the numpy restatement of the inference graph (oracle/emulator.py).
Contract: 1e-3 rel (north_star, bf16 MFMA); the bf16x3 path (the config's default) is
held to 1e-4 on every output level, the exact-f32 MFMA path to 1e-5 (tests/parity.py:
max over columns / max |ref| of each level)."""
import numpy as np
import pytest

from conftest import set_variant

from oracle import emulator as OE
from tests.parity import assert_per_level


def test_product_spec_matches_the_reference_restatement():
    from fv3net_amd import emulator as E

    spec = OE.zhao_carr_spec()
    assert [f.name for f in E.zhao_carr_features()] == [f["name"] for f in spec["features"]]
    assert [f.source for f in E.zhao_carr_features()] == [f["source"] for f in spec["features"]]
    assert [f.log_eps for f in E.zhao_carr_features()] == [f.get("log_eps") for f in spec["features"]]
    assert [(o.name, o.nz, o.residual_of, o.after) for o in E.zhao_carr_outputs()] == \
        [(o["name"], o["nz"], o.get("residual_of"), o.get("after")) for o in spec["outputs"]]


def test_norm_fits_match_oracle():
    from fv3net_amd import emulator as E

    x = np.random.default_rng(0).normal(3, 2, (500, 79)).astype(np.float32)
    np.testing.assert_array_equal(E.fit_center_per_feature(x), OE.fit_center_per_feature(x))
    assert E.fit_scale_all(x) == OE.fit_scale_all(x)


def test_oracle_bf16_rounding():
    # bf16 keeps 7 explicit mantissa bits: ulp(1) = 2**-7
    x = np.array([1.0078125, 1.00390625, 1.01171875, 1.001953125, -3.14159, np.nan], np.float32)
    r = OE.to_bf16(x)
    assert r[0] == 1.0078125                      # representable
    assert r[1] == 1.0 and r[2] == 1.015625       # ties go to the even mantissa
    assert r[3] == 1.0                            # below half an ulp
    assert r[4] == -3.140625 and np.isnan(r[5])


def _emulator(ncol=2048, seed=1, precision="bf16x3"):
    from fv3net_amd.emulator import MicrophysicsEmulator, zhao_carr_outputs

    raw = OE.synthetic_raw(ncol, seed=seed)
    rng = np.random.default_rng(seed + 1)
    sample_out = {}
    for o in zhao_carr_outputs():
        s = 1e-3 if o.name == "total_precipitation" else (1e-5 if ("humid" in o.name or "cloud" in o.name) else 0.5)
        sample_out[o.name] = rng.normal(0, s, (4096, o.nz)).astype(np.float32)
    emu = MicrophysicsEmulator.random(raw, sample_out, seed=seed, precision=precision)
    return emu, raw


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rtol", [("bf16x3", 1e-4), ("bf16x6", 1e-5), ("f32", 1e-5)])
def test_emulator_matches_oracle(gpu, precision, rtol):
    import torch

    emu, raw = _emulator(precision=precision)
    ref = OE.forward(raw, OE.zhao_carr_spec(), emu.params_by_name(), np.float64)
    state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}  # [feature, sample]
    got = emu(state)
    for o in OE.zhao_carr_spec()["outputs"]:
        name = o.get("after") or o["name"]
        g = got[name].cpu().numpy()
        r = ref[name]
        r = r[:, 0] if o["nz"] == 1 else r.T
        assert_per_level(g.T if g.ndim == 2 else g, r.T if r.ndim == 2 else r, rtol, name)
        if o.get("residual_of"):  # the difference itself, recovered from the after-state
            d = g.astype(np.float64) - raw[o["residual_of"]].T.astype(np.float64)
            derr = np.abs(d - ref[o["name"]].T).max() / np.abs(ref[o["name"]]).max()
            assert derr <= 1e-3, (o["name"], derr)


def _check_columns(got, raw, emu, cols, rtol, scale=None):
    """got: the emulator's outputs ([nz, ncol] / [ncol] device tensors) over the whole
    grid; cols: column indices checked against the float64 oracle (per level)."""
    import torch

    idx = torch.as_tensor(cols, device="cuda")
    sub = {k: v[:, idx].T.cpu().numpy() if torch.is_tensor(v) else v[cols] for k, v in raw.items()}
    ref = OE.forward(sub, OE.zhao_carr_spec(), emu.params_by_name(), np.float64)
    for o in OE.zhao_carr_spec()["outputs"]:
        name = o.get("after") or o["name"]
        g = got[name]
        g = (g[idx] if g.ndim == 1 else g[:, idx].T).cpu().numpy()
        r = ref[name][:, 0] if o["nz"] == 1 else ref[name]
        sc = None if scale is None else scale.get(name)
        assert_per_level(g, r, rtol, f"{name} columns {cols[0]}..{cols[-1]}", scale=sc)
        if o.get("residual_of"):  # the difference, recovered from the after-state
            d = g.astype(np.float64) - sub[o["residual_of"]].astype(np.float64)
            derr = np.abs(d - ref[o["name"]]).max() / np.abs(ref[o["name"]]).max()
            assert derr <= 1e-3, (o["name"], derr)
    return ref


def _device_raw(ncol, nz=79, seed=5):
    """oracle.emulator.synthetic_raw's distributions, drawn on the device ([nz, ncol],
    the hook's Fortran [feature, sample] layout) so a C384 state is cheap to make."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(seed)
    dev = "cuda"
    shape = (nz, ncol)

    def u(lo, hi):
        return torch.rand(shape, generator=g, device=dev) * (hi - lo) + lo

    prof = torch.linspace(200.0, 300.0, nz, device=dev)[:, None]
    T = prof + 5 * torch.randn(shape, generator=g, device=dev)
    q = 0.02 * torch.exp(-torch.linspace(0, 6, nz, device=dev))[:, None] * u(0.2, 1.0)
    qc = torch.where(torch.rand(shape, generator=g, device=dev) < 0.3, u(0, 1e-4), torch.zeros((), device=dev))
    delp = torch.linspace(200, 1800, nz, device=dev)[:, None] * u(0.98, 1.02)
    return {
        "air_temperature_input": T.contiguous(),
        "specific_humidity_input": q.contiguous(),
        "cloud_water_mixing_ratio_input": qc.contiguous(),
        "pressure_thickness_of_atmospheric_layer": delp.contiguous(),
        "air_temperature_after_last_gscond": (T + 0.1 * torch.randn(shape, generator=g, device=dev)).contiguous(),
        "specific_humidity_after_last_gscond": (q * u(0.95, 1.05)).contiguous(),
    }


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rtol", [("bf16x3", 1e-4), ("bf16x6", 1e-5), ("f32", 1e-5)])
def test_emulator_c384_full_grid(gpu, precision, rtol):
    """BASELINE config #5 at its real size: 884,736 columns, so every persistent block
    walks many tiles (bf16x3: 6,912 tiles of 128 on one block per CU; f32: 27,648 tiles
    of 32).  Columns from the first, a middle and the last tile, plus a stride through
    every block's tiles, are checked per level against the float64 oracle; the whole
    grid must be finite and reproducible launch to launch."""
    import torch

    ncol = 6 * 384 * 384
    emu, _ = _emulator(precision=precision)
    raw = _device_raw(ncol)
    a = emu(raw)
    b = emu(raw)
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
        assert torch.isfinite(a[k]).all(), k
    # level magnitudes from the strided sample, applied to the contiguous blocks too
    strided = np.arange(7, ncol, 97)
    ref = _check_columns(a, raw, emu, strided, rtol)
    scale = {}
    for o in OE.zhao_carr_spec()["outputs"]:
        name = o.get("after") or o["name"]
        r = ref[name][:, 0] if o["nz"] == 1 else ref[name]
        scale[name] = np.abs(r).max(axis=0)
    for c0 in (0, ncol // 2 - 1024, ncol - 2048):
        _check_columns(a, raw, emu, np.arange(c0, c0 + 2048), rtol, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3", "f32"])
def test_emulator_c384_columns_independent_of_position(gpu, precision):
    """Config #5 at its full size, a size-independent property: 37 template columns
    (37 is prime to every tile width) repeated over all 884,736 columns, and every copy's
    outputs carry exactly its template's bits, wherever it falls (lane, wave, tile,
    block, the residual reads one tile ahead)."""
    import torch

    ncol, nt = 6 * 384 * 384, 37
    emu, _ = _emulator(precision=precision)
    pick = torch.arange(ncol, device="cuda") % nt
    raw = {k: v[:, pick].contiguous() for k, v in _device_raw(nt, seed=9).items()}
    out = emu(raw)
    torch.cuda.synchronize()
    for k, v in out.items():
        tmpl = v[:nt] if v.ndim == 1 else v[:, :nt]
        want = tmpl[pick] if v.ndim == 1 else tmpl[:, pick]
        assert torch.equal(v, want), k


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rtol", [("bf16x3", 1e-4), ("bf16x6", 1e-5)])
def test_emulator_split_kernel_variants_agree(gpu, monkeypatch, precision, rtol):
    """The split kernel's staging pipelines (LDS-DMA, the default, and register staging,
    FV3_B3_STAGE=reg) and block shapes (8-wave and 4-wave blocks) run the same arithmetic in the same order per column:
    bit-identical outputs on a ragged grid forced to 4 persistent blocks (every block
    walks >= 4 tiles, so the cross-tile input DMA, the residual reads and the weight ring
    wrap around), and within the oracle bound."""
    import torch

    emu, raw = _emulator(ncol=2085, seed=11, precision=precision)
    state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}
    set_variant(monkeypatch, "FV3_B3_GRID", "4")
    runs = {}
    for name, env in (("glds-w8", {"FV3_B3_STAGE": "glds", "FV3_B3_WAVES": "8"}),
                      ("reg-w8", {"FV3_B3_STAGE": "reg", "FV3_B3_WAVES": "8"}),
                      ("glds-w4", {"FV3_B3_STAGE": "glds", "FV3_B3_WAVES": "4"})):
        for k in ("FV3_B3_STAGE", "FV3_B3_WAVES"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        runs[name] = emu(state)
    torch.cuda.synchronize()
    ref = runs.pop("glds-w8")
    for name, out in runs.items():
        for k in ref:
            assert torch.equal(ref[k], out[k]), (name, k)
    _check_columns(ref, state, emu, np.arange(2085), rtol)


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rtol,env", [("bf16x3", 1e-4, "FV3_B3_GRID"), ("bf16x6", 1e-5, "FV3_B3_GRID"),
                                                ("f32", 1e-5, "FV3_DENSE_GRID")])
def test_emulator_forced_multi_tile_blocks(gpu, precision, rtol, env, monkeypatch):
    """A ragged grid (2,085 columns) on 4 persistent blocks: every block walks >= 4 tiles
    (bf16x3: 17 tiles of 128; f32: 66 of 32), so the cross-tile prefetch of the LDS
    input-group table, the LogTransform inputs and the residual reads run with the
    emulator's features; must equal the default grid bit for bit."""
    import torch

    emu, raw = _emulator(ncol=2085, seed=9, precision=precision)
    state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}
    base = emu(state)
    set_variant(monkeypatch, env, "4")
    forced = emu(state)
    torch.cuda.synchronize()
    monkeypatch.delenv(env)
    for k in base:
        assert torch.equal(base[k], forced[k]), k
    _check_columns(forced, state, emu, np.arange(2085), rtol)


@pytest.mark.gpu
def test_microphysics_hook_updates_state_in_place(gpu):
    import torch

    from fv3net_amd.emulator import MicrophysicsHook

    emu, raw = _emulator(ncol=300, seed=3)
    state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}
    hook = MicrophysicsHook(emu)
    hook.microphysics(state)
    assert "air_temperature_after_precpd" in state and state["total_precipitation"].shape == (300,)
    with pytest.raises(KeyError):
        emu({"air_temperature_input": state["air_temperature_input"]})


@pytest.mark.gpu
def test_emulator_workload_c12(gpu):
    import torch

    from fv3net_amd import workloads as W

    wl = W.make_emulator_workload(12, seed=1)
    res = wl.step()
    torch.cuda.synchronize()
    assert res["total_precipitation"].shape == (W.c_columns(12),)
    assert all(torch.isfinite(v).all() for v in res.values())
    assert wl.flops_per_column == 2 * (711 * 256 + 256 * 256 + 256 * 396)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["torch", "numpy"])
def test_emulator_as_registered_predictor(gpu, tmp_path, kind):
    """The emulator as the drop-in for the reference's all-keras-dict model
    (PureKerasDictPredictor, pure_keras.py:181-258): ``emulator.predictor()`` predicts on a
    (z, y, x) dataset of the raw variables, and after dump / load through the registry,
    bit for bit what the emulator gives on the same columns (device tensors and host
    numpy arrays); the loaded predictor keeps bf16x3 and rebuilds the same emulator."""
    import torch

    from fv3net_amd import dataset as D
    from fv3net_amd.emulator import MicrophysicsEmulator
    from fv3net_amd.predictor import dump, load

    emu, raw = _emulator(ncol=24 * 24, seed=4)
    state = {k: torch.from_numpy(np.ascontiguousarray(v.T)).cuda() for k, v in raw.items()}  # [nz, ncol]
    want = {k: v.clone() for k, v in emu(state).items()}
    torch.cuda.synchronize()
    ds = D.Dataset()
    for k, v in state.items():
        arr = v.reshape(v.shape[0], 24, 24)
        ds[k] = D.DataArray(arr if kind == "torch" else arr.cpu().numpy(), ["z", "y", "x"])
    pred = emu.predictor()
    dump(pred, str(tmp_path))
    loaded = load(str(tmp_path))
    assert loaded.model.precision == "bf16x3"
    for p in (pred, loaded):
        out = p.predict(ds)
        for name, w in want.items():
            got = out[name].data
            got = got if isinstance(got, torch.Tensor) else torch.from_numpy(np.asarray(got)).cuda()
            assert tuple(out[name].dims) == (("z", "y", "x") if w.dim() == 2 else ("y", "x")), name
            assert torch.equal(got.reshape(w.shape).contiguous().view(torch.int32), w.view(torch.int32)), name
    again = MicrophysicsEmulator.from_predictor(loaded)(state)
    for name, w in want.items():
        assert torch.equal(again[name].view(torch.int32), w.view(torch.int32)), name
