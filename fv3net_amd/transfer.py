"""Host <-> device copies of numpy arrays through pinned, double-buffered staging.

The reference predicts on host arrays: ``PureKerasModel.predict`` stacks an xarray
Dataset into numpy and returns numpy-backed outputs
(external/fv3fit/fv3fit/keras/_models/shared/pure_keras.py:98-118), and the prognostic
run hands the predictor host state every step.  On this path each call crosses PCIe
twice.  A copy from pageable numpy memory goes through the driver's own bounce buffer
one piece at a time; here the host side of the copy (numpy <-> pinned buffer, threads
splitting each chunk) runs while the DMA of the previous chunk is in flight on a copy
stream, so both directions run at the host-memcpy or PCIe rate, whichever is lower.

Arrays of 64 KiB and more are instead page-locked in place for the copy (HostPages,
fv3_host_register): the copy engines DMA straight from / to the caller's memory with no
host memcpy at all; the staging path remains for memory that cannot be registered.

Plumbing only: bytes are moved unchanged (float64 stays float64; the kernels that read
float64 in place, or a device cast, do any conversion).
"""
import concurrent.futures
import os
import threading
from typing import Optional

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

_CHUNK = 16 << 20  # bytes per staging buffer
_MIN_REGISTER = 64 << 10  # arrays from here on are page-locked for their copy (HostPages)
_MIN_SPLIT = 1 << 20  # host copies below this run on the calling thread


def register_enabled() -> bool:
    """Whether HostPages page-locks the caller's arrays (``FV3_HOST_REGISTER=1``).

    Off by default since the round-4 closing runs.  Two full GPU-test runs that exercised
    the registered host path hit an illegal-address fault. One was in the usual test
    order, before HostPages synchronised the device on exit. The other was with the test
    files reversed: an H2D copy of an output array just after its pages were released.
    Neither was reproduced in isolation, and the cause is not established (DESIGN.md
    §3.7). With the switch off, host arrays cross through the pinned staging buffers or
    as pageable copies, as in round 3.  The registered path stays available and tested."""
    return os.environ.get("FV3_HOST_REGISTER", "0") == "1"


class PinnedStager:
    """Two pinned staging buffers, one copy stream, a small thread pool for the host
    memcpy.  One instance per device (``stager()``); calls are serialised."""

    def __init__(self, device, chunk_bytes: int = _CHUNK, threads: int = 0, min_staged: int = None,
                 min_register: Optional[int] = _MIN_REGISTER):
        self.device = torch.device(device)
        # arrays of this size and more are page-locked for their copy (None: never)
        self.min_register = min_register
        self.chunk = int(chunk_bytes)
        # below 4 chunks the driver's own pageable copy is faster (measured on the box:
        # a C48 float64 field, 8.7 MB, 22 GB/s pageable vs 19 staged; a C384 one, 560 MB,
        # 11 vs 46 GB/s)
        self.min_staged = 4 * self.chunk if min_staged is None else int(min_staged)
        self._bufs = [torch.empty(self.chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self._host = [b.numpy() for b in self._bufs]
        self._done = [None, None]  # event after the last DMA that used buffer i
        self._stream = torch.cuda.Stream(device=self.device)
        n = threads or min(8, os.cpu_count() or 1)
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=n) if n > 1 else None
        self._nthreads = n
        self._lock = threading.Lock()

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

    def h2d(self, arr, out=None):
        """numpy array -> CUDA tensor of the same dtype and shape (``out`` if given:
        a contiguous CUDA tensor of the same dtype and size)."""
        a = np.ascontiguousarray(arr)
        if out is None:
            out = torch.empty(a.shape, dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device=self.device)
        if not (out.is_cuda and out.is_contiguous() and out.numel() * out.element_size() == a.nbytes):
            raise ValueError("h2d: out must be a contiguous CUDA tensor of the array's size")
        nbytes = a.nbytes
        if nbytes == 0:
            return out
        if self.min_register is not None and nbytes >= self.min_register:
            # DMA straight from the caller's pages, registered for the copy: a C384 float64
            # field in + a float32 one out, 18.4 ms staged -> 14.7 ms (tools/h2h_register.py)
            with HostPages([a], self.min_register) as pages:
                if pages.registered:
                    out.view(-1).copy_(torch.from_numpy(a.reshape(-1)), non_blocking=True)
                    return out  # leaving the block waits for the copy, then releases the pages
        if nbytes < self.min_staged:
            out.view(-1).copy_(torch.from_numpy(a.reshape(-1)))
            return out
        src = a.reshape(-1).view(np.uint8)
        dst = out.view(-1).view(torch.uint8)
        cur = torch.cuda.current_stream(self.device)
        with self._lock:
            self._stream.wait_stream(cur)  # `out` may have been allocated / used on cur
            for i, off in enumerate(range(0, nbytes, self.chunk)):
                b = i & 1
                if self._done[b] is not None:
                    self._done[b].synchronize()  # the DMA reading this buffer is finished
                n = min(self.chunk, nbytes - off)
                self._memcpy(self._host[b][:n], src[off:off + n])
                with torch.cuda.stream(self._stream):
                    dst[off:off + n].copy_(self._bufs[b][:n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                    self._done[b] = ev
            cur.wait_stream(self._stream)
        out.record_stream(self._stream)
        return out

    def d2h(self, t, out=None) -> np.ndarray:
        """CUDA tensor -> numpy array of the same dtype and shape (``out`` if given)."""
        t = t.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        if out is None:
            out = np.empty(tuple(t.shape), dtype=torch.empty(0, dtype=t.dtype).numpy().dtype)
        if not (out.flags.c_contiguous and out.nbytes == t.numel() * t.element_size()):
            raise ValueError("d2h: out must be a C-contiguous array of the tensor's size")
        nbytes = out.nbytes
        if nbytes == 0:
            return out
        if self.min_register is not None and nbytes >= self.min_register:
            with HostPages([out], self.min_register) as pages:
                if pages.registered:
                    torch.from_numpy(out.reshape(-1)).copy_(t.view(-1), non_blocking=True)
                    return out
        if nbytes < self.min_staged:
            np.copyto(out.reshape(-1), t.view(-1).cpu().numpy())
            return out
        src = t.view(-1).view(torch.uint8)
        dst = out.reshape(-1).view(np.uint8)
        cur = torch.cuda.current_stream(self.device)
        offs = list(range(0, nbytes, self.chunk))
        with self._lock:
            self._stream.wait_stream(cur)  # the producer of `t` ran on cur

            def issue(i):
                b = i & 1
                if self._done[b] is not None:
                    self._done[b].synchronize()
                n = min(self.chunk, nbytes - offs[i])
                with torch.cuda.stream(self._stream):
                    self._bufs[b][:n].copy_(src[offs[i]:offs[i] + n], non_blocking=True)
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


class HostPages:
    """``with HostPages(arrays) as p:`` page-locks the arrays' own memory
    (fv3_host_register) so that copies on the current stream DMA straight from / to it,
    with no bounce buffer and no host memcpy; ``p.add(more)`` registers more arrays in
    the block.  On exit the device is synchronised (every copy issued in the block, on
    any stream, is complete) and what was registered here is released.  Arrays below
    ``min_bytes`` (sharing pages with other allocations) and arrays whose pages cannot
    be registered are left as they are: copies from them are pageable copies, which
    the runtime completes before returning."""

    def __init__(self, arrays=(), min_bytes: int = 64 << 10, enable: Optional[bool] = None):
        from . import _native

        self._lib = _native.load()
        self.min_bytes = int(min_bytes)
        # None: the process-wide switch (register_enabled); False: register nothing
        self.enable = register_enabled() if enable is None else bool(enable)
        self._registered = []
        self._pending = list(arrays)

    @property
    def registered(self) -> int:
        """How many arrays this block registered."""
        return len(self._registered)

    def is_registered(self, a) -> bool:
        """Whether this block page-locked ``a``'s memory."""
        return isinstance(a, np.ndarray) and a.ctypes.data in self._registered

    def add(self, arrays):
        if not self.enable:
            return
        for a in arrays:
            if not (isinstance(a, np.ndarray) and a.flags.c_contiguous) or a.nbytes < self.min_bytes:
                continue
            if any(a.ctypes.data == p for p in self._registered):
                continue
            if self._lib.fv3_host_register(a.ctypes.data, a.nbytes) == 0:
                self._registered.append(a.ctypes.data)

    def __enter__(self):
        self.add(self._pending)
        self._pending = []
        return self

    def __exit__(self, *exc):
        try:
            # the whole device, not only the current stream: a copy or kernel that a
            # caller put on a side stream must not touch the pages after they are released
            if self._registered:
                torch.cuda.synchronize()
            else:
                torch.cuda.current_stream().synchronize()
        finally:
            for p in self._registered:
                self._lib.fv3_host_unregister(p)
            self._registered = []
        return False


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


def h2d(arr, out=None, device=None):
    return stager(device if device is not None else (out.device if out is not None else None)).h2d(arr, out)


def d2h(t, out=None):
    return stager(t.device).d2h(t, out)


def copy_band(dst, src, stream=None):
    """One pitched copy (fv3_copy_2d) between a numpy array view and a CUDA tensor view of
    the same shape whose first axis (levels) is a fixed pitch apart and whose remaining
    axes are contiguous within each level: e.g. ``a[:, c0:c1]`` of a [level][column]
    array, a band of columns.  Host to device when ``src`` is numpy, else device to host;
    enqueued on ``stream`` (a torch stream or None for the current one).  The host memory
    should be page-locked (``HostPages``) for the copy to be asynchronous."""
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
    h = _device.stream_handle(stream, [dev])
    if host is src:
        st = lib.fv3_copy_2d(dev.data_ptr(), d_pitch, host.ctypes.data, h_pitch, width, host.shape[0], 1, h)
    else:
        st = lib.fv3_copy_2d(host.ctypes.data, h_pitch, dev.data_ptr(), d_pitch, width, host.shape[0], 2, h)
    _native.check(st, "copy_band")
