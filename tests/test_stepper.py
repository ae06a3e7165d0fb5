"""ML stepper epilogue (limiter + diagnostics + apply): HIP kernel vs the numpy
restatement of the reference's dtype flow, bit for bit (oracle/stepper.py)."""
import numpy as np
import pytest

from conftest import set_variant

from oracle import stepper as OS


def _state(rng, nz=79, ncol=1000, dtype=np.float64):
    base = np.linspace(200, 1800, nz)[:, None]
    delp = (base * rng.uniform(0.95, 1.05, (nz, ncol))).astype(dtype)
    T = (250 + rng.normal(0, 10, (nz, ncol))).astype(dtype)
    q = rng.uniform(0, 0.02, (nz, ncol)).astype(dtype)
    q[rng.uniform(size=q.shape) < 0.1] = 0.0  # dry points: the limiter engages
    dq1 = rng.normal(0, 1e-4, (nz, ncol)).astype(np.float32)
    dq2 = rng.normal(0, 3e-7, (nz, ncol)).astype(np.float32)
    precip = rng.uniform(0, 1e-3, ncol).astype(dtype)
    return dq1, dq2, q, delp, T, precip


def test_oracle_mass_integrate_is_nansum():
    rng = np.random.default_rng(0)
    x = rng.normal(0, 1, (79, 50))
    d = rng.uniform(100, 2000, (79, 50))
    x[3, 4] = np.nan
    assert (OS.mass_integrate(x, d) == np.nansum(x * d / OS.GRAVITY, axis=0)).all()


def test_oracle_limiter_keeps_humidity_non_negative():
    rng = np.random.default_rng(1)
    dq1, dq2, q, delp, T, _ = _state(rng)
    q1n, q2n = OS.limiter(q, dq1, dq2, 900.0, True)
    assert (q + q2n * 900.0 >= -1e-18).all()
    assert q1n.dtype == np.float64 and q2n.dtype == np.float64


def _bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (a.shape, b.shape, a.dtype, b.dtype)
    ia = a.view(np.uint64 if a.dtype.itemsize == 8 else (np.uint32 if a.dtype.itemsize == 4 else np.uint8))
    ib = b.view(ia.dtype)
    bad = ia != ib
    assert not bad.any(), f"{bad.sum()} differ, e.g. {a[bad][:3]} vs {b[bad][:3]}"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("mse", [True, False])
@pytest.mark.parametrize("hydrostatic", [False, True])
@pytest.mark.parametrize("path", ["levels", "levels-u3", "columns"])
def test_epilogue_bit_identical_to_oracle(gpu, dtype, mse, hydrostatic, path, monkeypatch):
    """Both epilogue kernels: level-parallel (the default; 5 levels per lane per pass, and
    round 4's 3) and one thread per column."""
    import torch

    set_variant(monkeypatch, "FV3_EPILOGUE_PATH", path.split("-")[0])
    if path.endswith("u3"):
        set_variant(monkeypatch, "FV3_EPI_U", "3")

    from fv3net_amd.stepper import ml_epilogue

    rng = np.random.default_rng(7)
    dq1, dq2, q, delp, T, precip = _state(rng, dtype=dtype)
    dq1[5, 17] = np.nan  # NaN predictions: fillna + NaN-skipping sums
    dq2[40, 3] = np.nan
    ref = OS.epilogue(dq1, dq2, q, delp, T, precip, 900.0, mse, hydrostatic)
    got = ml_epilogue(*(torch.from_numpy(a).cuda() for a in (dq1, dq2, q, delp, T)), 900.0,
                      torch.from_numpy(precip).cuda(), mse, hydrostatic, label="ml")
    names = {"net_moistening": "net_moistening_due_to_ml", "column_heating": "column_heating_due_to_ml"}
    for k, r in ref.items():
        g = got[names.get(k, k)].cpu().numpy()
        if k.endswith("filled_frac"):
            r = r.astype(dtype)
        _bits(g, r)


@pytest.mark.gpu
@pytest.mark.parametrize("nz", [1, 3, 5, 8, 9, 16, 17, 24, 33, 47, 48, 49, 79, 80, 81, 95, 96, 130])
@pytest.mark.parametrize("path", ["levels", "columns"])
def test_epilogue_level_batches(gpu, nz, path, monkeypatch):
    """The column kernel fetches levels in double-buffered batches of 8, the level-parallel
    one in batches of 5 per level lane of 16 (and hands nz > 95 to the column kernel):
    every remainder of nz (fewer levels than one batch, exact multiples, one past) stays
    bit-identical, on 130 columns (a partial block of 16)."""
    import torch

    set_variant(monkeypatch, "FV3_EPILOGUE_PATH", path)

    from fv3net_amd.stepper import ml_epilogue

    rng = np.random.default_rng(nz)
    dq1, dq2, q, delp, T, precip = _state(rng, nz=nz, ncol=130)
    dq2[nz - 1, 5] = -1.0  # limiter active at the last level
    dq1[0, 7] = np.nan
    ref = OS.epilogue(dq1, dq2, q, delp, T, precip, 900.0, True, False)
    got = ml_epilogue(*(torch.from_numpy(a).cuda() for a in (dq1, dq2, q, delp, T)), 900.0,
                      torch.from_numpy(precip).cuda(), True, False, label="ml")
    names = {"net_moistening": "net_moistening_due_to_ml", "column_heating": "column_heating_due_to_ml"}
    for k, r in ref.items():
        g = got[names.get(k, k)].cpu().numpy()
        if k.endswith("filled_frac"):
            r = r.astype(np.float64)
        _bits(g, r)


@pytest.mark.gpu
def test_epilogue_in_place_on_tile_state(gpu):
    """(tile, z, y, x) state updated in place; columns = (tile, y, x)."""
    import torch

    from fv3net_amd.stepper import ml_epilogue

    rng = np.random.default_rng(3)
    dq1, dq2, q, delp, T, _ = _state(rng, ncol=6 * 12 * 12)
    as4 = lambda a: np.ascontiguousarray(a.reshape(79, 6, 12, 12).transpose(1, 0, 2, 3))
    ref = OS.epilogue(dq1, dq2, q, delp, T, np.zeros(864), 450.0)
    # the kernel takes [z][col] arrays; a (tile, z, y, x) state is passed per tile
    qt, Tt = torch.from_numpy(as4(q)).cuda(), torch.from_numpy(as4(T)).cuda()
    for t in range(6):
        ml_epilogue(torch.from_numpy(as4(dq1)[t]).cuda(), torch.from_numpy(as4(dq2)[t]).cuda(), qt[t],
                    torch.from_numpy(as4(delp)[t]).cuda(), Tt[t], 450.0, in_place=True)
    _bits(qt.cpu().numpy(), as4(ref["specific_humidity"]))
    _bits(Tt.cpu().numpy(), as4(ref["air_temperature"]))


@pytest.mark.gpu
def test_stepper_workload_step(gpu):
    """Config #4 step (predict -> epilogue in place -> global means) on a C12 state."""
    import torch

    from fv3net_amd import workloads as W

    wl = W.make_stepper_workload(12, seed=2)
    q0 = wl.state["specific_humidity"].clone()
    sums = wl.step()
    torch.cuda.synchronize()
    q1 = wl.state["specific_humidity"]
    assert not torch.equal(q0, q1)
    assert (q1 >= -1e-15).all()  # the limiter keeps humidity non-negative
    assert sums.shape == (3, 2) and torch.isfinite(sums).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["full", "rank_of_4_stub", "full_bf16x6"])
def test_bound_stepper_steps_bit_identical_to_unbound_calls(gpu, kind):
    """The stepper workloads marshal every launch once (BoundForward, BoundEpilogue with
    the precipitation accumulated in place in its column buffer, bound partials / level
    counts / fold).  Four steps give, bit for bit, what the per-call product functions
    (forward, ml_epilogue, area_weighted_partials / area_row_partials, level_sums,
    fold_rows) give on a copy of the same state: the state, the accumulated
    precipitation, the global sums and the limiter profile."""
    import torch

    from fv3net_amd import distributed as D
    from fv3net_amd import workloads as W
    from fv3net_amd.stepper import ml_epilogue

    sharded = kind == "rank_of_4_stub"
    if sharded:
        wl = W.make_sharded_stepper_workload(12, 1, 4, seed=4, stub_exchange=True)
    else:
        wl = W.make_stepper_workload(12, seed=4, precision="bf16x6" if "bf16x6" in kind else "f32")
    ref = {k: v.clone() for k, v in wl.state.items()}
    ax = 0 if sharded else 1
    names = ("net_moistening_due_to_machine_learning", "column_heating_due_to_machine_learning", "total_precipitation")
    for step in range(4):
        got = wl.step()
        T, q = ref["air_temperature"], ref["specific_humidity"]
        bf6 = "bf16x6" in kind  # the workload casts the state into float32 buffers for the split kernel
        ins = [T.float(), q.float()] if bf6 else [T, q]
        dq1, dq2 = wl.model.forward(ins, level_axes=[ax, ax], precision="bf16x6" if bf6 else None)
        res = ml_epilogue(dq1, dq2, q, ref["pressure_thickness_of_atmospheric_layer"], T, wl.dt,
                          ref["total_precipitation"], in_place=True, level_axis=ax)
        ref["total_precipitation"] = res["total_precipitation"]
        if sharded:
            local = D.area_row_partials([res[n] for n in names], wl.area,
                                        out=torch.empty((wl.area.shape[0], 6), dtype=torch.float64, device=q.device))
            lim = D.level_sums(res["specific_humidity_limiter_active"])
            want = torch.cat([D.fold_rows(local.repeat(4, 1)), lim])
        else:
            want = D.area_weighted_partials([res[n] for n in names], wl.area)
        torch.cuda.synchronize()
        assert torch.equal(got.view(torch.int64), want.view(torch.int64)), step
        for k in ref:
            assert torch.equal(wl.state[k].reshape(-1).view(torch.int64), ref[k].reshape(-1).view(torch.int64)), (step, k)


@pytest.mark.gpu
def test_stepper_workload_bf16x6_predict(gpu):
    """The config #4 step with the predict on the bf16x6 split kernel (the float64 state
    cast into bound float32 buffers each step): its tendencies agree with the exact-f32
    kernel's to 2e-5 per level (each within 1e-5 of the float64 graph), and two steps
    re-read the updated state."""
    import torch

    from fv3net_amd import workloads as W
    from tests.parity import assert_per_level

    a = W.make_stepper_workload(12, seed=2)
    b = W.make_stepper_workload(12, seed=2, precision="bf16x6")
    for _ in range(2):
        sa, sb = a.step(), b.step()
        torch.cuda.synchronize()
        for ta, tb in zip(a.bound.outputs, b.bound.outputs):
            ref = ta.permute(1, 0, 2, 3).reshape(ta.shape[1], -1).T.double().cpu().numpy()
            got = tb.permute(1, 0, 2, 3).reshape(tb.shape[1], -1).T.double().cpu().numpy()
            assert_per_level(got, ref, 2e-5, "bf16x6 vs f32 tendencies")
        assert torch.isfinite(sb).all() and torch.isfinite(sa).all()
    assert (b.state["specific_humidity"] >= -1e-15).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x6", "f32"])
def test_stepper_workload_c96_matches_oracle(gpu, precision):
    """Config #4 at its size (C96, 79 levels, float64 state): one step of the stepper
    workload with the predict on the bf16x6 split kernel (and the exact-f32 kernel beside
    it).  The predicted dQ1/dQ2 are held to north_star's 1e-5 per level against the
    float64 DenseModel graph (oracle/dense.py) on the state's float32 inputs, and the
    epilogue's state update to oracle/stepper.py applied to the kernel's own prediction,
    bit for bit."""
    import torch

    from fv3net_amd import workloads as W
    from oracle.dense import dense_predict
    from tests.parity import assert_per_level

    wl = W.make_stepper_workload(96, seed=3, precision=precision)
    st0 = {k: v.clone() for k, v in wl.state.items()}
    wl.step()
    torch.cuda.synchronize()
    zc = lambda a: a.permute(1, 0, 2, 3).reshape(a.shape[1], -1).cpu().numpy()  # noqa: E731
    T0, q0 = zc(st0["air_temperature"]), zc(st0["specific_humidity"])
    ref = dense_predict([T0.T.astype(np.float32), q0.T.astype(np.float32)], wl.model.oracle_params(), np.float64)
    pred = [zc(o) for o in wl.bound.outputs]
    for i, (g, r) in enumerate(zip(pred, ref)):
        assert_per_level(g.T.astype(np.float64), r, 1e-5, f"{precision} C96 dQ{i + 1} vs float64 graph")
    r = OS.epilogue(pred[0], pred[1], q0, zc(st0["pressure_thickness_of_atmospheric_layer"]), T0,
                    st0["total_precipitation"].reshape(-1).cpu().numpy(), wl.dt)
    _bits(zc(wl.state["air_temperature"]), r["air_temperature"])
    _bits(zc(wl.state["specific_humidity"]), r["specific_humidity"])
    _bits(wl.state["total_precipitation"].reshape(-1).cpu().numpy(), r["total_precipitation"])


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "bf16x6"])
def test_stepper_c96_columns_independent_of_position(gpu, precision):
    """Config #4 at its full size, a size-independent property: the state is 37 template
    columns repeated over the 55,296 columns (37 is prime to every tile width), and after
    two steps every copy of the updated state, the predicted tendencies and the column
    diagnostics carries exactly its template's bits."""
    import torch

    from fv3net_amd import workloads as W

    wl = W.make_stepper_workload(96, seed=5, precision=precision)
    ncol, nt = wl.ncol, 37
    pick = torch.arange(ncol, device="cuda") % nt

    def cols(t):
        if t.dim() == 4:  # (tile, z, y, x)
            return t.permute(1, 0, 2, 3).reshape(t.shape[1], -1)
        assert t.numel() % ncol == 0
        return t.reshape(-1, ncol)

    for v in wl.state.values():
        c = cols(v)
        rep = c[:, :nt][:, pick]
        if v.dim() == 4:
            v.copy_(rep.reshape(v.shape[1], v.shape[0], v.shape[2], v.shape[3]).permute(1, 0, 2, 3))
        else:
            v.copy_(rep.reshape(v.shape))
    for _ in range(2):
        wl.step()
    torch.cuda.synchronize()
    checked = dict(wl.state)
    checked.update({f"dQ{i + 1}": o for i, o in enumerate(wl.bound.outputs)})
    checked.update({f"out:{k}": v for k, v in wl._epi.out.items() if torch.is_tensor(v)})
    for k, v in checked.items():
        c = cols(v)
        assert torch.equal(c, c[:, :nt][:, pick]), k


@pytest.mark.gpu
def test_pure_ml_stepper_mirror(gpu):
    """PureMLStepper (machine_learning.py:239-315) over a DenseColumnPredictor: the
    tendencies/diagnostics equal the oracle epilogue applied to the model's own
    prediction."""
    import torch

    from fv3net_amd import dataset as D
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from fv3net_amd.predictor import DenseColumnPredictor
    from fv3net_amd.stepper import PureMLStepper

    rng = np.random.default_rng(9)
    nz, ny, nx = 79, 12, 12
    dq1, dq2, q, delp, T, precip = _state(rng, nz, ny * nx)
    to3 = lambda a: a.reshape(nz, ny, nx)
    state = {"air_temperature": D.DataArray(torch.from_numpy(to3(T)).cuda(), ("z", "y", "x")),
             "specific_humidity": D.DataArray(torch.from_numpy(to3(q)).cuda(), ("z", "y", "x")),
             "pressure_thickness_of_atmospheric_layer": D.DataArray(torch.from_numpy(to3(delp)).cuda(),
                                                                    ("z", "y", "x")),
             "total_precipitation": D.DataArray(torch.from_numpy(precip.reshape(ny, nx)).cuda(), ("y", "x"))}
    cfg = DenseModelConfig(["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [nz, nz], [nz, nz],
                           width=64, depth=3)
    model = DenseColumnModel.random(cfg, seed=4, sample_inputs=[T.T.astype(np.float32), q.T.astype(np.float32)])
    pred = DenseColumnPredictor(cfg.input_variables, cfg.output_variables, model)
    stepper = PureMLStepper(pred, 900.0)
    tend, diags, updates = stepper(None, state)
    # the model's prediction on the same float32 inputs
    X = D.Dataset({"air_temperature": D.DataArray(torch.from_numpy(to3(T).astype(np.float32)).cuda(), ("z", "y", "x")),
                   "specific_humidity": D.DataArray(torch.from_numpy(to3(q).astype(np.float32)).cuda(),
                                                    ("z", "y", "x"))})
    p = pred.predict(X)
    d1 = p["dQ1"].data.cpu().numpy().reshape(nz, -1)
    d2 = p["dQ2"].data.cpu().numpy().reshape(nz, -1)
    ref = OS.epilogue(d1, d2, q, delp, T, precip, 900.0)
    _bits(tend["dQ1"].data.cpu().numpy().reshape(nz, -1), ref["dQ1"])
    _bits(tend["dQ2"].data.cpu().numpy().reshape(nz, -1), ref["dQ2"])
    net, _ = stepper.get_diagnostics(state, tend)
    _bits(net["net_moistening_due_to_machine_learning"].data.cpu().numpy().reshape(-1), ref["net_moistening"])
    updated, fracs = stepper.apply()
    _bits(updated["specific_humidity"].cpu().numpy().reshape(nz, -1), ref["specific_humidity"])
    _bits(updated["total_precipitation"].cpu().numpy().reshape(-1), ref["total_precipitation"])


@pytest.mark.gpu
def test_in_place_refuses_copies(gpu):
    """in_place=True with a state the kernel would read through a copy (mixed dtypes,
    host arrays) would leave the caller's state unchanged: refused."""
    import torch

    from fv3net_amd.stepper import ml_epilogue

    rng = np.random.default_rng(4)
    dq1, dq2, q, delp, T, _ = _state(rng, ncol=64)
    qd = torch.from_numpy(q).cuda()
    with pytest.raises(ValueError, match="in_place"):
        ml_epilogue(dq1, dq2, qd, delp, torch.from_numpy(T).cuda().float(), 450.0, in_place=True)
    with pytest.raises(ValueError, match="in_place"):
        ml_epilogue(dq1, dq2, qd, delp, T, 450.0, in_place=True)


# ------------------------------------------------------------------ adapters (a1)
def _host_ds(**vs):
    from fv3net_amd import dataset as D

    return D.Dataset({k: D.DataArray(v, ("z", "y", "x")) for k, v in vs.items()})


class _Echo:
    """Predictor stand-in: returns its inputs renamed out_<name> (host arrays)."""

    def __init__(self, inputs, outputs):
        self.input_variables = list(inputs)
        self.outputs = dict(outputs)

    def predict(self, X):
        from fv3net_amd import dataset as D

        return D.Dataset({o: D.DataArray(X[i].data.astype(np.float32), X[i].dims) for o, i in self.outputs.items()})


def test_renaming_adapter_renames_inputs_and_outputs():
    """machine_learning.py:106-147: rename_in maps standard -> model names,
    rename_out standard -> model output names (inverted on the way out)."""
    from fv3net_amd.stepper import RenamingAdapter

    model = _Echo(["T_model"], {"Q1_model": "T_model"})
    ad = RenamingAdapter(model, {"air_temperature": "T_model"}, {"dQ1": "Q1_model"})
    assert ad.input_variables == {"air_temperature"}
    x = np.arange(24.0).reshape(2, 3, 4)
    out = ad.predict(_host_ds(air_temperature=x))
    assert list(out) == ["dQ1"] and out["dQ1"].dims == ("z", "y", "x")
    np.testing.assert_array_equal(out["dQ1"].data, x.astype(np.float32))


def test_multi_model_adapter_merges_and_scales():
    """machine_learning.py:150-179: union of the models' inputs, merged outputs, scaling
    in float32; a name two models predict differently is a merge conflict."""
    from fv3net_amd.stepper import MultiModelAdapter, RenamingAdapter

    a = RenamingAdapter(_Echo(["air_temperature"], {"dQ1": "air_temperature"}), {})
    b = RenamingAdapter(_Echo(["specific_humidity"], {"dQ2": "specific_humidity"}), {})
    ad = MultiModelAdapter([a, b], scaling={"dQ2": 0.5})
    assert ad.input_variables == {"air_temperature", "specific_humidity"}
    t, q = np.full((2, 2, 2), 3.0), np.full((2, 2, 2), 0.1)
    out = ad.predict(_host_ds(air_temperature=t, specific_humidity=q))
    assert sorted(out) == ["dQ1", "dQ2"]
    np.testing.assert_array_equal(out["dQ2"].data, np.float32(0.1) * 0.5)
    assert out["dQ2"].data.dtype == np.float32
    c = RenamingAdapter(_Echo(["specific_humidity"], {"dQ1": "specific_humidity"}), {})
    with pytest.raises(ValueError, match="conflicting"):
        MultiModelAdapter([a, c]).predict(_host_ds(air_temperature=t, specific_humidity=q))


def test_tendency_split_matches_names():
    """names.py:54-65."""
    from fv3net_amd.stepper import is_state_update_variable, is_tendency_variable

    state = {"air_temperature": 1, "total_precipitation": 2}
    assert is_state_update_variable("total_precipitation", state)
    assert is_state_update_variable("total_precipitation_rate", state)
    assert is_state_update_variable("air_temperature", state)  # a predicted state variable
    assert not is_state_update_variable("dQ1", {"dQ1": 1})
    assert all(is_tendency_variable(k) for k in ("dQ1", "dQ2", "dQu", "dQv", "dQp", "dQx_wind", "dQy_wind"))
    assert not is_tendency_variable("total_precipitation")


def _two_model_stepper(rng, res, nz=79, ntile=6, mse=True, hydrostatic=False):
    """A C<res> (tile, z, y, x) float64 state and two DenseColumnPredictors behind the
    adapters: model A (dQ1, dQ2 from T, q), model B (dQu, dQv, dQp from its own input
    names, renamed by rename_in/rename_out, plus a diagnostic 'ml_diag')."""
    import torch

    from fv3net_amd import dataset as D
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from fv3net_amd.predictor import DenseColumnPredictor
    from fv3net_amd.stepper import MultiModelAdapter, PureMLStepper, RenamingAdapter

    shape = (ntile, nz, res, res)
    base = np.linspace(200, 1800, nz)[None, :, None, None]
    st = {"air_temperature": 250 + rng.normal(0, 10, shape),
          "specific_humidity": rng.uniform(0, 0.02, shape),
          "pressure_thickness_of_atmospheric_layer": base * rng.uniform(0.95, 1.05, shape)}
    st["specific_humidity"][rng.uniform(size=shape) < 0.1] = 0.0
    ncol = ntile * res * res
    flat = lambda a: a.transpose(0, 2, 3, 1).reshape(-1, nz).astype(np.float32)
    T, q = flat(st["air_temperature"]), flat(st["specific_humidity"])
    cfg_a = DenseModelConfig(["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [nz, nz], [nz, nz],
                             width=64, depth=3)
    out_a = [rng.normal(0, 1e-4, (4096, nz)).astype(np.float32), rng.normal(0, 3e-7, (4096, nz)).astype(np.float32)]
    model_a = DenseColumnModel.random(cfg_a, seed=4, sample_inputs=[T[:4096], q[:4096]], sample_outputs=out_a)
    cfg_b = DenseModelConfig(["temp", "delp"], ["u_tend", "v_tend", "p_tend", "ml_diag"], [nz, nz],
                             [nz, nz, nz, 1], width=32, depth=2)
    D_ = flat(st["pressure_thickness_of_atmospheric_layer"])
    out_b = [rng.normal(0, 1e-3, (4096, nz)).astype(np.float32)] * 2 + [
        rng.normal(0, 1e-2, (4096, nz)).astype(np.float32), rng.normal(0, 1, (4096, 1)).astype(np.float32)]
    model_b = DenseColumnModel.random(cfg_b, seed=5, sample_inputs=[T[:4096], D_[:4096]], sample_outputs=out_b)
    pa = DenseColumnPredictor(cfg_a.input_variables, cfg_a.output_variables, model_a)
    pb = DenseColumnPredictor(cfg_b.input_variables, cfg_b.output_variables, model_b)
    adapter = MultiModelAdapter([
        RenamingAdapter(pa, {}),
        RenamingAdapter(pb, {"air_temperature": "temp", "pressure_thickness_of_atmospheric_layer": "delp"},
                        {"dQu": "u_tend", "dQv": "v_tend", "dQp": "p_tend"}),
    ])
    dims = ("tile", "z", "y", "x")
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    state = {k: D.DataArray(dev(v), dims) for k, v in st.items()}
    state["total_precipitation"] = D.DataArray(dev(rng.uniform(0, 1e-3, (ntile, res, res))), ("tile", "y", "x"))
    stepper = PureMLStepper(adapter, 900.0, hydrostatic=hydrostatic, mse_conserving_limiter=mse)
    return stepper, state, adapter, ncol


def _zc(a):
    """(tile, z, y, x) -> [z, col]; (tile, y, x) -> [col]."""
    a = np.asarray(a)
    return a.transpose(1, 0, 2, 3).reshape(a.shape[1], -1) if a.ndim == 4 else a.reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("res,mse,hydrostatic", [(96, True, False), (12, False, True)])
def test_two_model_stepper_matches_oracle(gpu, res, mse, hydrostatic):
    """Config #4 size (C96, 79 levels): a PureMLStepper over TWO models behind
    MultiModelAdapter/RenamingAdapter (dQ1/dQ2 + dQu/dQv/dQp + a diagnostic) against
    oracle/stepper.py pure_ml_step on the adapter's own prediction: tendencies,
    diagnostics, get_diagnostics (incl. momentum and mass) and apply, bit for bit."""
    import torch

    from fv3net_amd.stepper import predict

    rng = np.random.default_rng(res)
    stepper, state, adapter, ncol = _two_model_stepper(rng, res, mse=mse, hydrostatic=hydrostatic)
    st_np = {k: _zc(v.data.cpu().numpy()) for k, v in state.items()}
    tend, diags, updates = stepper(None, state)
    torch.cuda.synchronize()
    pred = {k: _zc(v.data.cpu().numpy()) for k, v in predict(adapter, state).items()}
    r_tend, r_diags, r_upd, r_sd, (r_app, r_frac) = OS.pure_ml_step(pred, st_np, 900.0, mse, hydrostatic)
    assert sorted(tend) == sorted(r_tend) == ["dQ1", "dQ2", "dQp", "dQu", "dQv"]
    for k, r in r_tend.items():
        _bits(_zc(tend[k].data.cpu().numpy()), r.astype(np.float64) if k in ("dQ1", "dQ2") else r)
    assert sorted(diags) == sorted(r_diags)
    for k, r in r_diags.items():
        _bits(_zc(diags[k].data.cpu().numpy()), r)
    assert updates == {} and r_upd == {}
    sd, net = stepper.get_diagnostics(state, tend)
    for k, r in r_sd.items():
        _bits(_zc(sd[k].data.cpu().numpy()), r)
    applied, fracs = stepper.apply()
    assert sorted(applied) == sorted(r_app)
    for k, r in r_app.items():
        _bits(_zc(applied[k].cpu().numpy()), r)
    for k, r in r_frac.items():
        _bits(_zc(fracs[k].cpu().numpy()), r.astype(np.float64))


@pytest.mark.gpu
def test_stepper_without_dq1_leaves_temperature(gpu):
    """A model predicting only dQ2 (machine_learning.py:258-259 limits zeros for dQ1):
    temperature unchanged, no dQ1 diagnostics, column heating zero — as the oracle."""
    import torch

    from fv3net_amd.stepper import ml_epilogue

    rng = np.random.default_rng(11)
    dq1, dq2, q, delp, T, precip = _state(rng, ncol=300)
    q[2, :5] = -1e-6  # negative humidity: the limiter rewrites the zero dQ2 too
    z = np.zeros_like(dq1)
    ref = OS.pure_ml_step({"dQ2": dq2}, {"specific_humidity": q, "pressure_thickness_of_atmospheric_layer": delp,
                                         "air_temperature": T, "total_precipitation": precip}, 900.0)
    got = ml_epilogue(*(torch.from_numpy(a).cuda() for a in (z, dq2, q, delp, T)), 900.0,
                      torch.from_numpy(precip).cuda(), has_dq1=False)
    _bits(got["air_temperature"].cpu().numpy(), T)
    _bits(got["specific_humidity"].cpu().numpy(), ref[4][0]["specific_humidity"])
    _bits(got["column_heating_due_to_machine_learning"].cpu().numpy(), ref[3]["column_heating_due_to_machine_learning"])
    _bits(got["total_precipitation"].cpu().numpy(), ref[4][0]["total_precipitation"])
    _bits(got["dQ2"].cpu().numpy(), ref[0]["dQ2"])


@pytest.mark.gpu
def test_tendency_columns_nan_and_dtypes(gpu):
    """fv3_tendency_columns: NaN predictions (fillna, filled fraction, NaN-skipping
    integrals) for dQu (float64 state) and dQp (float32 state) vs the oracle."""
    import torch

    from fv3net_amd.stepper import tendency_columns

    rng = np.random.default_rng(5)
    for dtype in (np.float64, np.float32):
        _, _, _, delp, _, _ = _state(rng, ncol=200, dtype=dtype)
        t = rng.normal(0, 1e-3, delp.shape).astype(np.float32)
        t[0, 3] = t[78, 3] = t[40, 199] = np.nan
        ref = OS.pure_ml_step({"dQu": t, "dQp": t}, {"specific_humidity": np.zeros_like(delp),
                                                     "pressure_thickness_of_atmospheric_layer": delp,
                                                     "air_temperature": np.zeros_like(delp)}, 900.0)
        w = tendency_columns(torch.from_numpy(t).cuda(), torch.from_numpy(delp).cuda(), 900.0, "wind")
        m = tendency_columns(torch.from_numpy(t).cuda(), torch.from_numpy(delp).cuda(), 900.0, "mass")
        _bits(w["integral"].cpu().numpy(), ref[3]["column_integrated_dQu_stress"])
        _bits(w["filled"].cpu().numpy(), ref[4][0]["dQu"])
        _bits(w["filled_frac"].cpu().numpy(), ref[4][1]["dQu_filled_frac"].astype(dtype))
        _bits(m["integral"].cpu().numpy(), ref[3]["net_mass_tendency_due_to_machine_learning"])
        _bits(m["state"].cpu().numpy(), ref[4][0]["pressure_thickness_of_atmospheric_layer"])
