"""Host <-> device staging (fv3net_amd/transfer.py): bytes unchanged for every size
(empty, below / at / across the chunk size), dtype and shape; the predictor's numpy
path through it equals its device path."""
import numpy as np
import pytest


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.uint8, np.int64])
@pytest.mark.parametrize("arena", [None, 1 << 13])
def test_round_trip_bit_exact(gpu, dtype, arena):
    """Every host path: staging through arena blocks, pageable copies, and results in arena
    arrays (from 8 KiB here) or plain ones (arena None)."""
    import torch

    from fv3net_amd import transfer

    st = transfer.PinnedStager(torch.device("cuda", 0), chunk_bytes=1 << 16, threads=4, min_staged=1 << 12,
                               min_arena=arena)
    rng = np.random.default_rng(3)
    for n in (0, 1, 1000, (1 << 16) // np.dtype(dtype).itemsize, 3 * (1 << 16) + 17, 1 << 20):
        a = (rng.normal(0, 1e3, n) if np.dtype(dtype).kind == "f" else rng.integers(0, 200, n)).astype(dtype)
        a = a.reshape(-1, 1) if n else a
        t = st.h2d(a)
        assert t.is_cuda and tuple(t.shape) == a.shape
        ref = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        assert torch.equal(t, ref)
        t2 = t * 1 if np.dtype(dtype).kind != "u" else t.clone()  # produced on the current stream
        back = st.d2h(t2)
        assert back.dtype == a.dtype and back.shape == a.shape
        assert (back.view(np.uint8) == a.view(np.uint8)).all()
        out = np.empty_like(a)
        st.d2h(t2, out=out)
        assert (out.view(np.uint8) == a.view(np.uint8)).all()
    with pytest.raises(ValueError):
        st.h2d(np.zeros(10, dtype), out=torch.empty(11, dtype=torch.from_numpy(np.zeros(1, dtype)).dtype,
                                                     device="cuda"))


@pytest.mark.gpu
def test_float64_host_inputs_cast_on_device(gpu):
    """to_device_f32 on float64 numpy: the device cast equals numpy's astype."""
    from fv3net_amd import _device

    a = np.random.default_rng(0).normal(0, 1, (79, 3000)) * 10.0 ** np.random.default_rng(1).integers(-30, 30, (79, 1))
    t = _device.to_device_f32(a)
    assert (t.cpu().numpy().view(np.uint32) == a.astype(np.float32).view(np.uint32)).all()


@pytest.mark.gpu
def test_predict_mappm_host_to_host_matches_device_resident(gpu):
    """north_star's predict + mappm through the host boundary (bench.py's
    predict_mappm_c384_host_to_host leg, here at C24): float64 numpy T/q and float32
    numpy edge pressures in, float32 numpy remapped tendencies out, bit-identical to the
    same state run device-resident."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    rec = bench.predict_mappm_host_to_host(gpu, res=24, steps=1)
    assert rec["bit_identical_to_device_resident"]
    assert rec["host_bytes_per_step"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [16, 4096, 4100, 1 << 20, (1 << 20) + 7])
def test_copy_to_host_kernel(gpu, nbytes):
    """fv3_copy_to_host: a kernel storing device bytes into the library's page-locked host
    memory (16-byte vector stores and a byte tail) gives the bytes, into an arena block;
    a misaligned arena address or a range past the block is refused, and memory outside
    the arena (a plain array) is refused with FV3_ERR_UNSUPPORTED (the caller then uses the
    copy engines)."""
    import torch

    from fv3net_amd import _native, transfer

    lib = _native.load()
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    h = torch.cuda.current_stream().cuda_stream
    arena = transfer.empty_host((max(nbytes, 1 << 16),), np.uint8)
    arena[:] = 0
    assert transfer.is_arena(arena)
    assert lib.fv3_copy_to_host(arena.ctypes.data, src.data_ptr(), nbytes, h) == 0
    torch.cuda.synchronize()
    assert np.array_equal(arena[:nbytes], src.cpu().numpy()) and not arena[nbytes:].any()
    assert lib.fv3_copy_to_host(arena[1:].ctypes.data, src.data_ptr(), nbytes, h) == _native.FV3_ERR_UNSUPPORTED
    torch.cuda.synchronize()
    plain = np.zeros(nbytes, np.uint8)
    assert lib.fv3_copy_to_host(plain.ctypes.data, src.data_ptr(), nbytes, 0) == _native.FV3_ERR_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_copy_band_pitched_both_ways(gpu, dtype):
    """transfer.copy_band: a band of columns of a [level][column] numpy array to the same
    band of a device array and back (one pitched copy each), other columns untouched;
    mismatched shapes and non-contiguous levels refused."""
    import torch

    from fv3net_amd import transfer

    rng = np.random.default_rng(3)
    a = rng.normal(size=(79, 3000)).astype(dtype)
    d = torch.zeros((79, 3000), dtype=torch.from_numpy(a[:0]).dtype, device="cuda")
    back = np.full_like(a, -1)
    transfer.copy_band(d[:, 512:1536], a[:, 512:1536])
    transfer.copy_band(back[:, 512:1536], d[:, 512:1536])
    assert np.array_equal(d[:, 512:1536].cpu().numpy(), a[:, 512:1536])
    assert (d[:, :512] == 0).all() and (d[:, 1536:] == 0).all()
    assert np.array_equal(back[:, 512:1536], a[:, 512:1536]) and (back[:, :512] == -1).all()
    small = np.ascontiguousarray(a[:3, :5])  # pageable memory: a synchronous copy
    transfer.copy_band(d[:3, :5], small)
    torch.cuda.synchronize()
    assert np.array_equal(d[:3, :5].cpu().numpy(), small)
    with pytest.raises(ValueError):
        transfer.copy_band(d[:, :10], a[:, :11])
    with pytest.raises(ValueError):
        transfer.copy_band(d[:, ::2], a[:, ::2])


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [4096, 1 << 20])
def test_h2d_from_memory_pinned_elsewhere_complete_on_return(gpu, nbytes):
    """A caller's array in memory page-locked by someone else (torch pin_memory): the copy
    is a real asynchronous DMA there, so h2d must wait for it before returning; the
    caller overwrites the array at once and the device must still hold the old bytes."""
    import torch

    from fv3net_amd import transfer

    n = nbytes // 4
    pinned = torch.empty(n, dtype=torch.float32).pin_memory()
    a = pinned.numpy()
    rng = np.random.default_rng(nbytes)
    for _ in range(5):
        vals = rng.normal(0, 1, n).astype(np.float32)
        a[:] = vals
        # a long kernel ahead of the copy on the same stream keeps the DMA pending
        big = torch.randn(4096, 4096, device="cuda")
        _ = big @ big
        t = transfer.h2d(a)
        a[:] = -1.0  # the caller reuses its buffer right after the call
        assert np.array_equal(t.cpu().numpy(), vals)


@pytest.mark.gpu
def test_arena_cap_falls_back_to_pageable(gpu):
    """Past the arena's live + cached cap, empty_host hands out pageable arrays."""
    import gc

    from fv3net_amd import transfer

    gc.collect()
    live = transfer.memory_stats()["arena_live"]
    try:
        transfer.set_arena_limits(total_bytes=live + (4 << 20))
        small = transfer.empty_host((1 << 20,), np.float32)  # 4 MiB: fits
        assert transfer.is_arena(small)
        big = transfer.empty_host((2 << 20,), np.float32)  # 8 MiB more: past the cap
        assert not transfer.is_arena(big) and big.shape == (2 << 20,)
        del small
        gc.collect()
    finally:
        transfer.set_arena_limits(cached_bytes=2 << 30, total_bytes=32 << 30)
