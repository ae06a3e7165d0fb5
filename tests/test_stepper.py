"""ML stepper epilogue (limiter + diagnostics + apply): HIP kernel vs the numpy
restatement of the reference's dtype flow, bit for bit (oracle/stepper.py)."""
import numpy as np
import pytest

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
def test_epilogue_bit_identical_to_oracle(gpu, dtype, mse, hydrostatic):
    import torch

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
@pytest.mark.parametrize("nz", [1, 3, 8, 9, 16, 17, 24, 33])
def test_epilogue_level_batches(gpu, nz):
    """The kernel fetches levels in double-buffered batches of 8: every remainder of nz
    (fewer levels than one batch, exact multiples, one past) stays bit-identical."""
    import torch

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
    _bits(tend["dQ1"].cpu().numpy().reshape(nz, -1), ref["dQ1"])
    _bits(tend["dQ2"].cpu().numpy().reshape(nz, -1), ref["dQ2"])
    net, _ = stepper.get_diagnostics(state, tend)
    _bits(net["net_moistening_due_to_machine_learning"].cpu().numpy().reshape(-1), ref["net_moistening"])
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
