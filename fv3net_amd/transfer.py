"""Host <-> device copies of numpy arrays: the library's page-locked arena, pinned staging,
or the runtime's pageable copies.

The reference predicts on host arrays: ``PureKerasModel.predict`` stacks an xarray
Dataset into numpy and returns numpy-backed outputs
(external/fv3fit/fv3fit/keras/_models/shared/pure_keras.py:98-118), and the prognostic
run hands the predictor host state every step.  On this path each call crosses PCIe
twice.

* Arrays handed back to the caller come from the library's page-locked arena
  (``empty_host``, ``fv3_host_alloc``): DMA targets with no registration per call, their
  pages reused (already faulted in) once the caller drops them.
* Caller arrays are never page-locked (csrc/host_memory.cpp, DESIGN.md §3.7: round 4's
  per-call registration of the caller's pages faulted later pageable copies).  They take
  the runtime's pageable copy (56 GB/s for a C384 field, profiles/r05e_host_ab.json); an
  arena array (``empty_host``) as input is DMA'd directly.  ``PinnedStager`` can also
  stage through arena blocks (the host memcpy, threads splitting each chunk, overlapping
  the DMA of the previous chunk) for a caller that sets ``min_staged``.

Plumbing only: bytes are moved unchanged (float64 stays float64; the kernels that read
float64 in place, or a device cast, do any conversion).
"""
import concurrent.futures
import ctypes
import os
import threading

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

_CHUNK = 16 << 20  # bytes per staging block
_MIN_ARENA = 64 << 10  # d2h results from here on land in the arena
_MIN_SPLIT = 1 << 20  # host copies below this run on the calling thread


def arena_enabled() -> bool:
    """Whether host results go to the library's page-locked arena (default on;
    ``FV3_HOST_ARENA=0``: plain numpy arrays and pageable copies)."""
    return os.environ.get("FV3_HOST_ARENA", "1") != "0"


def host_path() -> str:
    """What the host boundary does now, for the bench records."""
    if arena_enabled():
        return ("arena: outputs DMA'd into the library's page-locked arena (reused across calls); inputs staged "
                "through arena blocks (64 MiB and more) or pageable copies; no caller memory is page-locked")
    return "pageable: FV3_HOST_ARENA=0, outputs in plain numpy arrays, pageable or staged copies"


class _ArenaBlock:
    """Owner of one ``fv3_host_alloc`` block, exported to numpy through the array
    interface: the numpy array (and every view of it) keeps this object alive, and the
    block returns to the library's cache when the last one is dropped."""

    __slots__ = ("ptr", "__array_interface__", "__weakref__")

    def __init__(self, ptr: int, shape, dtype: np.dtype):
        self.ptr = ptr
        self.__array_interface__ = {"data": (ptr, False), "shape": tuple(shape), "typestr": dtype.str,
                                    "strides": None, "version": 3}

    def __del__(self):
        try:
            _lib().fv3_host_free(self.ptr)
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def _lib():
    from . import _native

    return _native.load()


def empty_host(shape, dtype=np.float32) -> np.ndarray:
    """An uninitialised C-contiguous numpy array in page-locked memory owned by the
    library (``fv3_host_alloc``): the copy engines DMA into it asynchronously with no
    registration per call, and its pages are reused (already faulted in) by a later array
    of the same size once this one is dropped.  Plain ``np.empty`` when the arena is off
    (``FV3_HOST_ARENA=0``) or cannot allocate."""
    dtype = np.dtype(dtype)
    shape = tuple(int(n) for n in (shape if isinstance(shape, (tuple, list)) else (shape,)))
    nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    if nbytes == 0 or not arena_enabled():
        return np.empty(shape, dtype)
    p = ctypes.c_void_p()
    if _lib().fv3_host_alloc(nbytes, ctypes.byref(p)) != 0 or not p.value:
        return np.empty(shape, dtype)
    return np.asarray(_ArenaBlock(p.value, shape, dtype))


def is_arena(a) -> bool:
    """Whether ``a`` (or the array it views) lives in an ``empty_host`` block."""
    while isinstance(a, np.ndarray):
        a = a.base
    return isinstance(a, _ArenaBlock)


def set_arena_limits(cached_bytes=None, total_bytes=None) -> None:
    """Bound the library's page-locked memory: ``cached_bytes`` kept for reuse after the
    caller drops arrays (default 2 GiB), ``total_bytes`` live + cached at most (default
    32 GiB).  Arrays the caller keeps (outputs held across steps) stay page-locked; past
    the total, ``empty_host`` hands out pageable ``np.empty`` arrays instead."""
    from . import _native

    if cached_bytes is not None:
        _native.check(_lib().fv3_host_arena_limit(int(cached_bytes)), "host_arena_limit")
    if total_bytes is not None:
        _native.check(_lib().fv3_host_arena_cap(int(total_bytes)), "host_arena_cap")


def memory_stats() -> dict:
    """The arena's counters: live / cached bytes and blocks (fv3_host_memory_stats)."""
    st = (ctypes.c_uint64 * 3)()
    _lib().fv3_host_memory_stats(st)
    return {"arena_live": st[0], "arena_cached": st[1], "blocks": st[2]}


def host_copy(dst, src, stream=None) -> None:
    """One copy between a C-contiguous numpy array and a contiguous CUDA tensor of the same
    byte size (either direction) on ``stream`` (torch stream, raw handle or None: the
    current stream), ``fv3_host_copy``: asynchronous DMA when the host array is arena
    memory (keep it alive and unchanged until the stream is done), else the runtime's
    pageable copy, complete on return."""
    from . import _device, _native

    h2d = isinstance(src, np.ndarray)
    host, dev = (src, dst) if h2d else (dst, src)
    if not (isinstance(host, np.ndarray) and torch.is_tensor(dev) and dev.is_cuda):
        raise ValueError("host_copy: one numpy array and one CUDA tensor")
    if not (host.flags.c_contiguous and dev.is_contiguous()) or host.nbytes != dev.numel() * dev.element_size():
        raise ValueError("host_copy: contiguous operands of the same byte size")
    if host.nbytes == 0:
        return
    h = stream if isinstance(stream, int) else _device.stream_handle(stream, [dev])
    if h2d:
        st = _lib().fv3_host_copy(dev.data_ptr(), host.ctypes.data, host.nbytes, 1, h)
    else:
        st = _lib().fv3_host_copy(host.ctypes.data, dev.data_ptr(), host.nbytes, 2, h)
    _native.check(st, "host_copy")


class PinnedStager:
    """Two staging blocks of the arena, one copy stream, a small thread pool for the host
    memcpy.  One instance per device (``stager()``); calls are serialised."""

    def __init__(self, device, chunk_bytes: int = _CHUNK, threads: int = 0, min_staged: int = None,
                 min_arena: int = _MIN_ARENA):
        self.device = torch.device(device)
        self.chunk = int(chunk_bytes)
        # d2h results of this size and more land in the arena (None: never)
        self.min_arena = min_arena
        # the runtime's own pageable copy is the default at every size: with no caller
        # memory registered it measured at least as fast as staging (profiles/
        # r05e_host_ab.json: one C384 float64 field, 560 MB, 9.9 ms pageable = 56 GB/s
        # against 10.6-14.9 ms staged; one rank's two (79, 48, 48) fields 0.079 ms against
        # 0.11-0.22 ms).  Staging stays for a caller that asks for it (min_staged).
        self.min_staged = (1 << 62) if min_staged is None else int(min_staged)
        self._host = [None, None]  # the staging blocks, allocated on first use
        self._done = [None, None]  # event after the last DMA that used block i
        self._stream = torch.cuda.Stream(device=self.device)
        n = threads or min(8, os.cpu_count() or 1)
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=n) if n > 1 else None
        self._nthreads = n
        self._lock = threading.Lock()

    def _block(self, b: int) -> np.ndarray:
        if self._host[b] is None:
            self._host[b] = empty_host((self.chunk,), np.uint8)
        return self._host[b]

    def _memcpy(self, dst: np.ndarray, src: np.ndarray) -> None:
        """dst[:] = src for two uint8 vectors, split over the pool when large."""
        n = src.size
        if self._pool is None or n < 2 * _MIN_SPLIT:
            np.copyto(dst, src)
            return
        parts = min(self._nthreads, n // _MIN_SPLIT)
        step = -(-n // parts)
        futs = [self._pool.submit(np.copyto, dst[i:i + step], src[i:i + step]) for i in range(0, n, step)]
        for f in futs:
            f.result()

    def h2d(self, arr, out=None, stream=None):
        """numpy array -> CUDA tensor of the same dtype and shape (``out`` if given: a
        contiguous CUDA tensor of the same dtype and size), ordered on ``stream`` (default
        the current one).  The caller may reuse ``arr`` as soon as this returns."""
        a = np.ascontiguousarray(arr)
        if out is None:
            out = torch.empty(a.shape, dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device=self.device)
        if not (out.is_cuda and out.is_contiguous() and out.numel() * out.element_size() == a.nbytes):
            raise ValueError("h2d: out must be a contiguous CUDA tensor of the array's size")
        nbytes = a.nbytes
        if nbytes == 0:
            return out
        cur = stream if stream is not None else torch.cuda.current_stream(self.device)
        if is_arena(a):  # page-locked already: one DMA
            host_copy(out.view(-1), a.reshape(-1), cur.cuda_stream)
            cur.synchronize()
            return out
        if nbytes < self.min_staged:
            host_copy(out.view(-1), a.reshape(-1), cur.cuda_stream)  # the runtime's pageable copy
            return out
        src = a.reshape(-1).view(np.uint8)
        dst = out.view(-1).view(torch.uint8)
        with self._lock:
            self._stream.wait_stream(cur)  # `out` may have been allocated / used on cur
            for i, off in enumerate(range(0, nbytes, self.chunk)):
                b = i & 1
                if self._done[b] is not None:
                    self._done[b].synchronize()  # the DMA reading this block is finished
                n = min(self.chunk, nbytes - off)
                blk = self._block(b)
                self._memcpy(blk[:n], src[off:off + n])
                host_copy(dst[off:off + n], blk[:n], self._stream.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(self._stream)
                self._done[b] = ev
            cur.wait_stream(self._stream)
        out.record_stream(self._stream)
        return out

    def d2h(self, t, out=None) -> np.ndarray:
        """CUDA tensor -> numpy array of the same dtype and shape (``out`` if given; else an
        arena array from ``min_arena`` bytes on).  Complete on return."""
        t = t.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        if out is None:
            dt = torch.empty(0, dtype=t.dtype).numpy().dtype
            nb = t.numel() * t.element_size()
            out = (empty_host(tuple(t.shape), dt) if self.min_arena is not None and nb >= self.min_arena
                   else np.empty(tuple(t.shape), dtype=dt))
        if not (out.flags.c_contiguous and out.nbytes == t.numel() * t.element_size()):
            raise ValueError("d2h: out must be a C-contiguous array of the tensor's size")
        nbytes = out.nbytes
        if nbytes == 0:
            return out
        cur = torch.cuda.current_stream(self.device)
        if is_arena(out) or nbytes < self.min_staged:  # one DMA, or the runtime's pageable copy
            host_copy(out.reshape(-1), t.view(-1), cur.cuda_stream)
            cur.synchronize()
            return out
        src = t.view(-1).view(torch.uint8)
        dst = out.reshape(-1).view(np.uint8)
        offs = list(range(0, nbytes, self.chunk))
        with self._lock:
            self._stream.wait_stream(cur)  # the producer of `t` ran on cur

            def issue(i):
                b = i & 1
                if self._done[b] is not None:
                    self._done[b].synchronize()
                n = min(self.chunk, nbytes - offs[i])
                host_copy(self._block(b)[:n], src[offs[i]:offs[i] + n], self._stream.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(self._stream)
                self._done[b] = ev

            issue(0)
            for i in range(len(offs)):
                if i + 1 < len(offs):
                    issue(i + 1)  # the next chunk's DMA runs while this one is copied out
                b = i & 1
                self._done[b].synchronize()
                n = min(self.chunk, nbytes - offs[i])
                self._memcpy(dst[offs[i]:offs[i] + n], self._host[b][:n])
        t.record_stream(self._stream)
        return out


_stagers = {}
_stagers_lock = threading.Lock()


def stager(device=None) -> PinnedStager:
    """The process-wide stager of ``device`` (default: the current CUDA device)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    with _stagers_lock:
        s = _stagers.get(key)
        if s is None:
            s = PinnedStager(torch.device("cuda", key))
            _stagers[key] = s
        return s


def h2d(arr, out=None, device=None, stream=None):
    return stager(device if device is not None else (out.device if out is not None else None)).h2d(arr, out, stream)


def d2h(t, out=None):
    return stager(t.device).d2h(t, out)


def copy_fence(stream, idle):
    """After a block's pageable host-to-device copies on ``stream``: make ``stream`` wait
    for an event recorded on ``idle`` (a stream with no work).  The wait orders nothing,
    but with it the runtime's pageable in-copies run at full rate while the previous
    block's out-copies (arena DMA on another stream) drain; without it the two
    directions shared the link as if in sequence.  Measured on the pipelined C384 call
    (two float64 fields in, two float32 out, six tile blocks; tools/host_ab.py,
    profiles/r05l_h2h_overlap.json): 32.55 -> 24.46 ms, the host's time inside the
    in-copy calls 30.2 -> 22.0 ms; the same wait on the out-copy stream, a second kernel
    or fresh streams changed nothing."""
    ev = torch.cuda.Event()
    ev.record(idle)
    stream.wait_event(ev)


def copy_band(dst, src, stream=None):
    """One pitched copy (fv3_copy_2d) between a numpy array view and a CUDA tensor view of
    the same shape whose first axis (levels) is a fixed pitch apart and whose remaining
    axes are contiguous within each level: e.g. ``a[:, c0:c1]`` of a [level][column]
    array, a band of columns.  Host to device when ``src`` is numpy, else device to host;
    enqueued on ``stream`` (a torch stream, a raw handle, or None for the current one; a
    torch stream other than the current one first waits for the current one, a raw handle
    does not).  Asynchronous when
    the host array is arena memory (``empty_host``), else the runtime's pageable copy."""
    from . import _device, _native

    host, dev = (src, dst) if isinstance(src, np.ndarray) else (dst, src)
    if not (isinstance(host, np.ndarray) and torch.is_tensor(dev) and dev.is_cuda):
        raise ValueError("copy_band: one numpy array and one CUDA tensor")
    if tuple(host.shape) != tuple(dev.shape) or host.itemsize != dev.element_size() or host.ndim < 1:
        raise ValueError(f"copy_band: shapes / dtypes differ ({host.shape} {host.dtype}, {tuple(dev.shape)} {dev.dtype})")
    if not (host[0].flags.c_contiguous and dev[0].is_contiguous()):
        raise ValueError("copy_band: each level's elements must be contiguous")
    width = host[0].nbytes
    h_pitch = host.strides[0] if host.shape[0] > 1 else width
    d_pitch = dev.stride(0) * dev.element_size() if dev.shape[0] > 1 else width
    lib = _native.load()
    h = stream if isinstance(stream, int) else _device.stream_handle(stream, [dev])
    if host is src:
        st = lib.fv3_copy_2d(dev.data_ptr(), d_pitch, host.ctypes.data, h_pitch, width, host.shape[0], 1, h)
    else:
        st = lib.fv3_copy_2d(host.ctypes.data, h_pitch, dev.data_ptr(), d_pitch, width, host.shape[0], 2, h)
    _native.check(st, "copy_band")
