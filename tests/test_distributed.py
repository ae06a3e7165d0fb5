"""Multi-rank path: column bands with no data-path exchange, and
the one collective — global means (runtime/metrics.py:18-55) — as an all-gather
of float64 partials summed in fixed rank order.  gloo world_size 2..4 on CPU."""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_helpers as H
from fv3net_amd import distributed as D


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n_rows,world,align", [(576, 8, 1), (576, 3, 1), (2304, 8, 8), (72, 5, 8), (10, 4, 1)])
def test_row_band_partitions_exactly(n_rows, world, align):
    bands = [D.row_band(n_rows, r, world, align) for r in range(world)]
    assert bands[0][0] == 0 and bands[-1][1] == n_rows
    for (a0, a1), (b0, b1) in zip(bands[:-1], bands[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in bands]
    assert all(a % align == 0 for a, _ in bands)
    assert max(sizes) - min(sizes) <= align


def test_row_band_rejects_bad_arguments():
    with pytest.raises(ValueError):
        D.row_band(10, 3, 3)
    with pytest.raises(ValueError):
        D.row_band(10, 0, 2, align=4)


@pytest.mark.parametrize("res,world", [(96, 8), (96, 4), (48, 8), (384, 8), (12, 5)])
def test_column_segments_cover_the_sphere_once(res, world):
    seen = np.zeros((6, res), dtype=int)
    for r in range(world):
        for s in D.column_segments(6, res, r, world):
            assert 0 <= s.y0 < s.y1 <= res
            seen[s.tile, s.y0:s.y1] += 1
    assert (seen == 1).all()


def test_segment_view_is_a_view():
    import torch

    a = torch.arange(2 * 3 * 4 * 5, dtype=torch.float32).reshape(2, 3, 4, 5)
    v = D.segment_view(a, D.Segment(1, 1, 3))
    assert v.shape == (3, 2, 5) and v.data_ptr() == a[1, 0, 1].data_ptr()


def _spawn(fn, world, *args):
    mp.start_processes(fn, args=(world, _port()) + args, nprocs=world, join=True, start_method="spawn")


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_global_average_matches_single_process(tmp_path, world):
    _spawn(H.global_average_worker, world, str(tmp_path), False)
    res = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    rng = np.random.default_rng(0)
    x = rng.normal(280, 20, (6, 12, 12)).astype(np.float32).astype(np.float64)
    area = rng.uniform(0.5, 1.0, (6, 12, 12)).astype(np.float32).astype(np.float64)
    expect = np.array([np.sum(area * x), np.sum(area * x * 2)]) / np.sum(area)
    for r in res:
        assert (r.view(np.uint64) == res[0].view(np.uint64)).all()  # identical bits on every rank
        np.testing.assert_allclose(r, expect, rtol=1e-13)


def test_gloo_partials_summed_in_rank_order(tmp_path):
    _spawn(H.rank_order_worker, 4, str(tmp_path))
    tot = [np.load(tmp_path / f"rank{r}.npy") for r in range(4)]
    expect = ((1e16 + 1.0) + -1e16) + 3.0  # == 3.0 (the 1.0 is absorbed), not 4.0
    for t in tot:
        assert t[0, 0] == expect and t[0, 1] == 4.0


def test_combine_without_process_group_is_identity():
    import torch

    p = torch.tensor([[2.0, 4.0]], dtype=torch.float64)
    assert D.global_average(p)[0] == 0.5


@pytest.mark.gpu
def test_gpu_global_average_two_ranks(gpu, tmp_path):
    """HIP partials on the GPU per rank + gloo all-gather (2 processes on one GPU)."""
    _spawn(H.global_average_worker, 2, str(tmp_path), True)
    res = [np.load(tmp_path / f"rank{r}.npy") for r in range(2)]
    rng = np.random.default_rng(0)
    x = rng.normal(280, 20, (6, 12, 12)).astype(np.float32).astype(np.float64)
    area = rng.uniform(0.5, 1.0, (6, 12, 12)).astype(np.float32).astype(np.float64)
    expect = np.array([np.sum(area * x), np.sum(area * x * 2)]) / np.sum(area)
    assert (res[0].view(np.uint64) == res[1].view(np.uint64)).all()
    np.testing.assert_allclose(res[0], expect, rtol=1e-12)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_row_partials_are_world_size_invariant(tmp_path, world):
    """Row partials gathered in global row order and folded row by row: every rank of
    every world size gets the world-1 bits (distributed.gather_rows + fv3_fold_rows order)."""
    _spawn(H.gather_rows_worker, world, str(tmp_path))
    res = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    rng = np.random.default_rng(1)
    x = rng.normal(280, 20, (72, 12))
    area = rng.uniform(0.5, 1.0, (72, 12))
    rows = H._rows_partials_np(x, area)
    total = H.fold_rows_np(rows)
    expect = np.concatenate([total, rows.reshape(-1)])
    for r in res:
        assert (r.view(np.uint64) == expect.view(np.uint64)).all()
    np.testing.assert_allclose(total, [np.sum(area * x), np.sum(area)], rtol=1e-13)


def test_gather_rows_without_process_group_is_identity():
    import torch

    x = torch.arange(6.0).reshape(3, 2)
    assert D.gather_rows(x) is x


@pytest.mark.gpu
def test_gpu_row_partials_match_restatement(gpu):
    """fv3_area_weighted_row_sums_f64 / fv3_level_row_sums_u8 / fv3_fold_rows vs the
    numpy restatement of their order, bit for bit."""
    import torch

    rng = np.random.default_rng(2)
    x = rng.normal(280, 20, (40, 96))
    area = rng.uniform(0.5, 1.0, (40, 96))
    got = D.area_row_partials([torch.from_numpy(x).cuda()], torch.from_numpy(area).cuda()).cpu().numpy()
    ref = H._rows_partials_np(x, area)
    assert (got[:, 0].view(np.uint64) == ref.view(np.uint64)).all()
    # numpy float64 operands take the float64 kernel too (numpy's promotion), not a
    # float32 rounding of the host arrays
    host = D.area_row_partials([x], area).cpu().numpy()
    assert (host[:, 0].view(np.uint64) == ref.view(np.uint64)).all()
    flag = (rng.uniform(size=(7, 40, 96)) < 0.2).astype(np.uint8)
    lev = D.level_row_partials(torch.from_numpy(flag).cuda()).cpu().numpy()
    assert (lev == flag.sum(axis=2).T).all()
    big = rng.normal(0, 1e6, (700, 5))  # more rows than lanes: lane-strided partial sums
    for rows in (ref, big):
        tot = D.fold_rows(torch.from_numpy(rows).cuda()).cpu().numpy()
        expect = H.fold_rows_np(rows)
        assert (tot.view(np.uint64) == expect.view(np.uint64)).all()


@pytest.mark.gpu
def test_sharded_stepper_two_ranks_bit_identical_to_one(gpu, tmp_path):
    """Config #4 sharded over 2 ranks (2 processes on one GPU, gloo exchange): after two
    steps the global means / limiter profile have the world-1 bits on both ranks, and
    each rank's state band equals the world-1 state's rows."""
    for world in (1, 2):
        (tmp_path / f"w{world}").mkdir()
        _spawn(H.sharded_stepper_worker, world, str(tmp_path / f"w{world}"), 12, 2)
    one = np.load(tmp_path / "w1" / "total0.npy")
    q1 = np.load(tmp_path / "w1" / "q0.npy")
    for r in range(2):
        t = np.load(tmp_path / "w2" / f"total{r}.npy")
        assert (t.view(np.uint64) == one.view(np.uint64)).all()
        r0, r1 = np.load(tmp_path / "w2" / f"rows{r}.npy")
        q = np.load(tmp_path / "w2" / f"q{r}.npy")
        assert (q.view(np.uint64) == q1[:, r0:r1].view(np.uint64)).all()
    assert np.isfinite(one).all() and one[6:].sum() > 0  # the limiter engaged somewhere


@pytest.mark.gpu
def test_sharded_stepper_c96_world4_bit_identical_to_one(gpu, tmp_path):
    """Config #4's own geometry: C96 over 4 ranks, 144 of the 576 (tile, y) rows each (4
    processes on one GPU, gloo exchange).  After two steps the global means / limiter
    profile carry the world-1 bits on every rank, and each rank's state band equals the
    world-1 state's rows."""
    for world in (1, 4):
        (tmp_path / f"w{world}").mkdir()
        _spawn(H.sharded_stepper_worker, world, str(tmp_path / f"w{world}"), 96, 2)
    one = np.load(tmp_path / "w1" / "total0.npy")
    q1 = np.load(tmp_path / "w1" / "q0.npy")
    for r in range(4):
        t = np.load(tmp_path / "w4" / f"total{r}.npy")
        assert (t.view(np.uint64) == one.view(np.uint64)).all(), r
        r0, r1 = np.load(tmp_path / "w4" / f"rows{r}.npy")
        assert r1 - r0 == 144
        q = np.load(tmp_path / "w4" / f"q{r}.npy")
        assert (q.view(np.uint64) == q1[:, r0:r1].view(np.uint64)).all(), r
    assert np.isfinite(one).all() and one[6:].sum() > 0


@pytest.mark.gpu
def test_sharded_stepper_rccl_exchange_matches_gloo(gpu, tmp_path):
    """The RCCL (nccl backend) branch of the per-step exchange (device tensors in the
    all-gather) on the box's one GPU (world 1: RCCL runs one rank per device): the same
    bits as the gloo exchange."""
    for be in ("gloo", "nccl"):
        (tmp_path / be).mkdir()
        _spawn(H.sharded_stepper_worker, 1, str(tmp_path / be), 12, 2, be)
    a = np.load(tmp_path / "gloo" / "total0.npy")
    b = np.load(tmp_path / "nccl" / "total0.npy")
    assert (a.view(np.uint64) == b.view(np.uint64)).all()
    qa = np.load(tmp_path / "gloo" / "q0.npy")
    qb = np.load(tmp_path / "nccl" / "q0.npy")
    assert (qa.view(np.uint64) == qb.view(np.uint64)).all()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_count_sums_are_exact(tmp_path, world):
    """The limiter-profile exchange: per-rank integer counts (float64), one all-reduce;
    exact in any order, so equal to the serial sum on every rank."""
    _spawn(H.count_sums_worker, world, str(tmp_path))
    counts = np.random.default_rng(7).integers(0, 2 ** 40, (world, 79)).astype(np.float64)
    expect = counts.sum(axis=0)
    for r in range(world):
        assert (np.load(tmp_path / f"rank{r}.npy") == expect).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "bf16x6"])
def test_sharded_predict_mappm_bit_identical_across_world_sizes(gpu, tmp_path, precision):
    """north_star's predict + mappm sharded as 8(e) lays it out (row bands of one global
    state, no data-path exchange): at world 2 and 3 (gloo, processes sharing the GPU)
    each rank's band of tendencies and remapped tendencies equals the world-1 columns
    bit for bit (C24 stands in for C384: the same code with 144 rows)."""
    res = 24
    for world in (1, 2, 3):
        (tmp_path / f"w{world}").mkdir()
        _spawn(H.predict_mappm_worker, world, str(tmp_path / f"w{world}"), res, 2, precision)
    one = np.load(tmp_path / "w1" / "out0.npy")
    assert np.isfinite(one).all()
    for world in (2, 3):
        cols = 0
        for r in range(world):
            r0, r1 = np.load(tmp_path / f"w{world}" / f"rows{r}.npy")
            got = np.load(tmp_path / f"w{world}" / f"out{r}.npy")
            assert (got.view(np.uint32) == one[:, :, r0 * res:r1 * res].view(np.uint32)).all(), (world, r)
            cols += got.shape[-1]
        assert cols == one.shape[-1]
