"""The stepper step's fused per-rank reductions (csrc/reduce.hip step_partials_kernel,
fold_rows_repeat_kernel): each output carries the bits of the launches it replaces
(fv3_area_weighted_row_sums_f64, fv3_level_sums_u8, the repeat copy + fv3_fold_rows),
on one rank's C96 band at world 8 and 4, ragged row counts, and a limiter whose rows are
not 16-byte aligned (the two-launch path)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nrows,row_len,nz,offset", [(72, 96, 79, 0), (144, 96, 79, 0), (18, 12, 79, 0),
                                                    (7, 33, 5, 0), (72, 96, 79, 3)])
def test_step_partials_equal_the_two_launches(gpu, nrows, row_len, nz, offset):
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(nrows + row_len + offset)
    dev = torch.device("cuda", 0)
    area = torch.from_numpy(rng.uniform(1e9, 2e9, (nrows, row_len))).to(dev)
    diags = [torch.from_numpy(rng.normal(0, s, (nrows, row_len))).to(dev) for s in (1e-3, 50.0, 2e-5)]
    ncol = nrows * row_len
    flat = torch.from_numpy((rng.random(nz * ncol + offset) < 0.3).astype(np.uint8)).to(dev)
    lim = flat[offset:].view(nz, ncol)  # offset 3: rows not 16-byte aligned
    part = torch.full((nrows, 6), np.nan, dtype=torch.float64, device=dev)
    lev = torch.full((nz,), np.nan, dtype=torch.float64, device=dev)
    fused = D.bind_step_partials(diags, area, lim, out=part, level_out=lev)
    got_rows, got_lev = fused()
    want_rows = D.area_row_partials(diags, area, out=torch.empty((nrows, 6), dtype=torch.float64, device=dev))
    want_lev = D.level_sums(lim)
    torch.cuda.synchronize()
    assert got_rows.data_ptr() == part.data_ptr() and got_lev.data_ptr() == lev.data_ptr()
    assert torch.equal(part.view(torch.int64), want_rows.view(torch.int64))
    assert torch.equal(lev.view(torch.int64), want_lev.view(torch.int64))
    assert torch.equal(lev, lim.sum(1, dtype=torch.float64))


@pytest.mark.parametrize("nrows,times", [(144, 8), (72, 8), (18, 4), (1, 3), (200, 1)])
def test_fold_rows_repeat_equals_repeat_then_fold(gpu, nrows, times):
    import torch

    from fv3net_amd import distributed as D

    rng = np.random.default_rng(nrows * times)
    rows = torch.from_numpy(rng.normal(0, 1e6, (nrows, 6))).cuda()
    rep = torch.full((times * nrows, 6), np.nan, dtype=torch.float64, device="cuda")
    out = torch.empty(6, dtype=torch.float64, device="cuda")
    b = D.bind_fold_rows_repeat(rows, times, rep=rep, out=out)
    b()
    want = D.fold_rows(rows.repeat(times, 1))
    torch.cuda.synchronize()
    assert torch.equal(rep, rows.repeat(times, 1))
    assert torch.equal(out.view(torch.int64), want.view(torch.int64))
    with pytest.raises(ValueError):
        D.bind_fold_rows_repeat(rows, times, rep=rep[1:])
