"""The stepper's predict and epilogue as one launch (the dense kernel's fused epilogue,
fv3_dense_stepper_f64in / stepper.BoundPredictEpilogue) against the two launches it
replaces (fv3_dense_forward_f64in + fv3_ml_epilogue_ex): the updated state, the limited
tendencies, the limiter flags and the column diagnostics (precipitation accumulated in
place) bit for bit, over several steps; MSE-conserving and legacy limiters, hydrostatic
or not, NaN tendencies (inputs that make the model emit NaN), ragged column counts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(model, state, dt, mse, hydro, level_axis):
    import torch

    from fv3net_amd.stepper import BoundEpilogue

    T, q = state["air_temperature"], state["specific_humidity"]
    bound = model.bind([T, q], level_axes=[level_axis, level_axis])
    precip = state["total_precipitation"]
    column = torch.empty((7, precip.numel()), dtype=precip.dtype, device=precip.device)
    column[6].copy_(precip.reshape(-1))
    state["total_precipitation"] = column[6].view(precip.shape)
    epi = BoundEpilogue(*bound.outputs, q, state["pressure_thickness_of_atmospheric_layer"], T, dt,
                        state["total_precipitation"], mse_conserving=mse, hydrostatic=hydro, in_place=True,
                        level_axis=level_axis, column=column)
    return bound, epi, column


def _bits(a, b, what):
    import torch

    assert a.shape == b.shape, what
    assert torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8)), what


@pytest.mark.parametrize("mse,hydro", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("res,band", [(12, None), (48, None), (12, (13, 31))])
def test_fused_predict_epilogue_bit_identical_to_two_launches(gpu, mse, hydro, res, band):
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.stepper import BoundPredictEpilogue

    wl = W.make_stepper_workload(res, seed=res + int(mse) + 2 * int(hydro))
    state = wl.state
    level_axis = 1
    if band is not None:  # a (z, rows, x) band of the flattened (tile, y) rows: ragged tiles
        r0, r1 = band
        b3 = lambda a: a.permute(1, 0, 2, 3).reshape(a.shape[1], -1, res)[:, r0:r1].contiguous()  # noqa: E731
        state = {k: (b3(v) if v.dim() == 4 else v.reshape(-1, res)[r0:r1].contiguous()) for k, v in state.items()}
        level_axis = 0
    # NaN inputs in a few columns: the model's tendencies there are NaN (the filled counts)
    T = state["air_temperature"]
    if level_axis == 1:
        T[0, 3:6, 2, 2] = float("nan")
    else:
        T[3:6, 1, 2] = float("nan")
    a = {k: v.clone() for k, v in state.items()}
    b = {k: v.clone() for k, v in state.items()}
    ba, ea, ca = _pair(wl.model, a, wl.dt, mse, hydro, level_axis)
    bb, eb, cb = _pair(wl.model, b, wl.dt, mse, hydro, level_axis)
    fused = BoundPredictEpilogue(bb, eb)
    for step in range(3):
        ba(), ea()
        out = fused()
        torch.cuda.synchronize()
        for k in a:
            _bits(a[k], b[k], (step, k))
        _bits(ca, cb, (step, "column"))
        for k in ("dQ1", "dQ2", "specific_humidity_limiter_active"):
            _bits(ea.out[k], out[k], (step, k))
    assert torch.isnan(ca[0]).sum() == 0  # NaN-skipping sums
    assert (ca[4] > 0).any()  # some filled levels were counted


def test_fused_predict_epilogue_refuses_what_it_cannot_fuse(gpu):
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.stepper import BoundEpilogue, BoundPredictEpilogue

    wl = W.make_stepper_workload(12, seed=1)
    T, q = wl.state["air_temperature"], wl.state["specific_humidity"]
    T32, q32 = T.float(), q.float()
    b32 = wl.model.bind([T32, q32], level_axes=[1, 1])  # float32 inputs: not the f64 kernel
    e32 = BoundEpilogue(*b32.outputs, q, wl.state["pressure_thickness_of_atmospheric_layer"], T, wl.dt,
                        in_place=True, level_axis=1)
    ok, why = BoundPredictEpilogue.supported(b32, e32)
    assert not ok and "float64" in why
    with pytest.raises(NotImplementedError):
        BoundPredictEpilogue(b32, e32)
    b64 = wl.model.bind([T, q], level_axes=[1, 1])
    other = [torch.empty_like(o) for o in b64.outputs]  # an epilogue that reads other buffers
    e2 = BoundEpilogue(*other, q, wl.state["pressure_thickness_of_atmospheric_layer"], T, wl.dt, in_place=True,
                       level_axis=1)
    assert not BoundPredictEpilogue.supported(b64, e2)[0]
