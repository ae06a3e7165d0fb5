"""The native launch plan (csrc/plan.cpp, fv3net_amd/plan.py): a recorded sequence of
bound launches issued by one C-ABI call gives the bits of issuing them one by one."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_plan_replays_bound_launches_bit_identically(gpu):
    """predict (float64 state read in place) -> fused epilogue (precipitation accumulated
    in its column buffer) -> area partials -> copies -> fold, recorded once and run three
    times, against the same launches issued one by one on a copy of the state."""
    import torch

    from fv3net_amd import distributed as D
    from fv3net_amd import workloads as W
    from fv3net_amd.plan import LaunchPlan
    from fv3net_amd.stepper import BoundEpilogue

    def build(seed):
        wl = W.make_stepper_workload(12, seed=seed)
        T, q = wl.state["air_temperature"], wl.state["specific_humidity"]
        bound = wl.model.bind([T, q], level_axes=[1, 1])
        precip = wl.state["total_precipitation"]
        column = torch.empty((7, precip.numel()), dtype=precip.dtype, device=precip.device)
        column[6].copy_(precip.reshape(-1))
        wl.state["total_precipitation"] = column[6].view(precip.shape)
        epi = BoundEpilogue(*bound.outputs, q, wl.state["pressure_thickness_of_atmospheric_layer"], T, wl.dt,
                            wl.state["total_precipitation"], level_axis=1, column=column)
        out = epi.out
        diags = [out["net_moistening_due_to_machine_learning"], out["column_heating_due_to_machine_learning"],
                 out["total_precipitation"]]
        part = D.bind_area_weighted_partials(diags, wl.area)
        rows = torch.empty((4, 3, 2), dtype=torch.float64, device=q.device)
        fold = D.bind_fold_rows(rows)
        return wl, bound, epi, part, rows, fold

    a = build(6)
    b = build(6)
    plan = LaunchPlan([a[1], a[2], a[3]])
    for r in range(4):
        plan.copy(a[4][r], a[3].result)
    plan.add(a[5])
    assert len(plan) == 8
    for _ in range(3):
        plan()
        b[1](), b[2](), b[3]()
        for r in range(4):
            b[4][r].copy_(b[3].result)
        b[5]()
        torch.cuda.synchronize()
        assert torch.equal(a[5].result.view(torch.int64), b[5].result.view(torch.int64))
        for k in a[0].state:
            assert torch.equal(a[0].state[k].view(torch.int64), b[0].state[k].view(torch.int64)), k
    # on a side stream: ordered after the current stream's work, same bits
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        plan()
    b[1](), b[2](), b[3]()
    for r in range(4):
        b[4][r].copy_(b[3].result)
    b[5]()
    torch.cuda.synchronize()
    assert torch.equal(a[5].result.view(torch.int64), b[5].result.view(torch.int64))


def test_plan_refuses_unknown_ops(gpu):
    import torch

    from fv3net_amd import distributed as D
    from fv3net_amd.plan import LaunchPlan

    plan = LaunchPlan()
    assert len(plan) == 0
    plan()  # an empty plan is a no-op
    f32 = D.bind_level_sums(torch.zeros((3, 8), device="cuda"))  # the float32 sums have no plan op
    with pytest.raises(NotImplementedError):
        plan.add(f32)
    with pytest.raises(ValueError):
        plan.copy(torch.zeros(3, device="cuda"), torch.zeros(4, device="cuda"))
    x = torch.from_numpy(np.arange(10.0)).cuda()
    y = torch.zeros_like(x)
    plan.copy(y, x)
    z = torch.zeros((3, 10), dtype=torch.float64, device="cuda")
    plan.repeat(z, x, 3)
    with pytest.raises(ValueError):
        plan.repeat(torch.zeros((2, 10), dtype=torch.float64, device="cuda"), x, 3)
    plan()
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    assert all(torch.equal(z[t], x) for t in range(3))


def test_model_close_refused_while_a_plan_replays_it(gpu):
    """The native plan replays the model's raw handle: close() is refused while a live
    plan holds a bound forward of the model, allowed once the plan is closed; a bound
    forward called after close() raises rather than launching on the freed handle."""
    import torch

    from fv3net_amd import workloads as W
    from fv3net_amd.plan import LaunchPlan

    wl = W.make_dense_workload(12, seed=2)
    bound = wl.model.bind(wl.inputs, level_axes=[1, 1])
    plan = LaunchPlan([bound])
    with pytest.raises(RuntimeError, match="LaunchPlan"):
        wl.model.close()
    plan()
    torch.cuda.synchronize()
    plan.close()
    wl.model.close()
    with pytest.raises(RuntimeError, match="closed"):
        bound()
    # a fresh bind after close makes a new handle and runs
    wl.model.bind(wl.inputs, level_axes=[1, 1])()
    torch.cuda.synchronize()
