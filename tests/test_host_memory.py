"""The host boundary's page-locked arena (csrc/host_memory.cpp, fv3net_amd/transfer.py).

Round 4's registered host path faulted (profiles/gpu_tests_reversed_r04z5.log), and a
page-exclusive, refcounted registration of the caller's arrays still faulted a later
pageable copy (profiles/r05b_gpu_tests.log).  The library now page-locks
only memory it allocates: arena blocks (hipHostMalloc) handed out as numpy arrays and
reused after the caller drops them.  These tests pin that down: blocks reused and
released, copies from / to arena and plain memory bit-exact, and the round-4 fault's call
sequence repeated on the new path.
"""
import numpy as np
import pytest

PAGE = 4096


def test_arena_switch(monkeypatch):
    """FV3_HOST_ARENA=0: plain numpy arrays, no library call (works without a GPU)."""
    from fv3net_amd import transfer

    monkeypatch.delenv("FV3_HOST_ARENA", raising=False)
    assert transfer.arena_enabled() and "arena" in transfer.host_path()
    monkeypatch.setenv("FV3_HOST_ARENA", "0")
    assert not transfer.arena_enabled() and "pageable" in transfer.host_path()
    a = transfer.empty_host((3, 4), np.float64)
    assert a.shape == (3, 4) and a.dtype == np.float64 and not transfer.is_arena(a)


@pytest.mark.gpu
def test_host_copy_arena_and_pageable_bit_exact(gpu):
    """fv3_host_copy over windows of an arena array (asynchronous DMA) and of a plain numpy
    array (the runtime's pageable copy), both directions: bytes unchanged, nothing outside
    the window touched."""
    import torch

    from fv3net_amd import transfer

    rng = np.random.default_rng(5)
    n = (1 << 20) + 333
    src_plain = rng.integers(0, 256, n, dtype=np.uint8)
    src_arena = transfer.empty_host((n,), np.uint8)
    src_arena[:] = src_plain
    cuts = [0, 1, 4095, 4096, 5000, n // 2, n - 4097, n - 1, n]
    windows = [(lo, hi) for lo in cuts for hi in cuts if hi > lo]
    dev = torch.zeros(n, dtype=torch.uint8, device="cuda")
    back_plain = np.zeros(n, np.uint8)
    back_arena = transfer.empty_host((n,), np.uint8)
    for src in (src_plain, src_arena):
        for lo, hi in windows:
            dev.zero_()
            transfer.host_copy(dev[lo:hi], src[lo:hi])
            back_arena[:] = 0
            back_plain[:] = 0
            transfer.host_copy(back_arena[lo:hi], dev[lo:hi])
            transfer.host_copy(back_plain[lo:hi], dev[lo:hi])
            torch.cuda.synchronize()
            for back in (back_arena, back_plain):
                assert np.array_equal(back[lo:hi], src_plain[lo:hi]), (lo, hi)
                assert not back[:lo].any() and not back[hi:].any(), (lo, hi)


@pytest.mark.gpu
def test_copy_band_arena_and_pageable(gpu):
    """fv3_copy_2d for bands of columns of a [level][column] array, arena and plain host
    memory, both directions: every band bit-exact, the other columns untouched."""
    import torch

    from fv3net_amd import transfer

    rng = np.random.default_rng(9)
    a = rng.normal(size=(79, 3001)).astype(np.float32)
    a_arena = transfer.empty_host(a.shape, np.float32)
    a_arena[:] = a
    d = torch.zeros((79, 3001), dtype=torch.float32, device="cuda")
    for src in (a, a_arena):
        for back in (transfer.empty_host((79, 3001), np.float32), np.empty((79, 3001), np.float32)):
            for c0, c1 in ((0, 3001), (0, 1), (3000, 3001), (17, 1500), (1500, 3001), (999, 1000)):
                d.zero_()
                back[:] = np.nan
                transfer.copy_band(d[:, c0:c1], src[:, c0:c1])
                transfer.copy_band(back[:, c0:c1], d[:, c0:c1])
                torch.cuda.synchronize()
                assert np.array_equal(back[:, c0:c1], a[:, c0:c1]), (c0, c1)
                assert np.isnan(back[:, :c0]).all() and np.isnan(back[:, c1:]).all()


@pytest.mark.gpu
def test_arena_blocks_reused_and_released(gpu):
    import gc

    from fv3net_amd import _native, transfer

    lib = _native.load()
    base = transfer.memory_stats()
    a = transfer.empty_host((1000, 333), np.float32)
    assert transfer.is_arena(a) and transfer.is_arena(a[3:, 5:])
    p = a.ctypes.data
    assert p % PAGE == 0
    n = -(-a.nbytes // PAGE) * PAGE
    assert transfer.memory_stats()["arena_live"] == base["arena_live"] + n
    v = a[10]  # a view keeps the block alive
    del a
    gc.collect()
    assert transfer.memory_stats()["arena_live"] == base["arena_live"] + n
    del v
    gc.collect()
    s = transfer.memory_stats()
    assert s["arena_live"] == base["arena_live"] and s["arena_cached"] >= n
    b = transfer.empty_host((333, 1000), np.float32)  # same page-rounded size: the cached block
    assert b.ctypes.data == p
    del b
    gc.collect()
    assert lib.fv3_host_arena_limit(0) == 0
    assert transfer.memory_stats()["arena_cached"] == 0
    assert lib.fv3_host_arena_limit(8 << 30) == 0
    assert lib.fv3_host_free(12345) == _native.FV3_ERR_INVALID


@pytest.mark.gpu
def test_host_path_sequence_of_the_r04z5_fault(gpu):
    """The call sequence around round 4's fault, many times over, on the default host
    path: a host predict (fresh caller inputs, fresh arena outputs or caller `out` arrays
    that malloc places on the same heap pages call after call), its output uploaded again
    by a pageable torch copy and run through a kernel (TaperConfig.apply's pattern), and
    outputs dropped so arena blocks are reused.  Bits stay equal to the device-resident
    predict and the arena's live bytes return to where they started."""
    import gc

    import torch

    from fv3net_amd import transfer
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    rng = np.random.default_rng(2)
    cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [79, 79], [79, 79], width=128, depth=2)
    T = rng.normal(260, 15, (79, 48, 48))
    q = rng.uniform(0, 0.02, (79, 48, 48))
    m = DenseColumnModel.random(cfg, seed=4, sample_inputs=[T.reshape(79, -1).T, q.reshape(79, -1).T])
    ref = [r.cpu().numpy() for r in m.forward([torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()],
                                               level_axes=[0, 0])]
    gc.collect()
    base = transfer.memory_stats()["arena_live"]
    for it in range(40):
        Tc, qc = T.copy(), q.copy()  # fresh caller arrays, often at the previous ones' addresses
        outs = None if it % 2 else [np.empty(T.shape, np.float32), np.empty(T.shape, np.float32)]
        got = m.forward_host([Tc, qc], [0, 0], out=outs)
        assert transfer.is_arena(got[0]) == (outs is None)
        for g, r in zip(got, ref):
            assert (g.view(np.uint32) == r.view(np.uint32)).all(), it
        up = torch.from_numpy(got[1]).cuda()  # a pageable (or arena) copy of the output's pages
        back = (up * 2).cpu().numpy()
        assert (back == got[1] * 2).all()
        del got, up, back, Tc, qc, outs, g  # g: the comparison loop's last output
        if it % 5 == 0:
            gc.collect()
    gc.collect()
    assert transfer.memory_stats()["arena_live"] == base
    torch.cuda.synchronize()
