"""Device-memory plumbing (PyTorch-ROCm is used only for allocation, streams and
``torch.distributed``; all arithmetic happens in the HIP library)."""
import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

from . import _native


def require_gpu():
    if torch is None or not torch.cuda.is_available():
        raise _native.NativeLibraryError(
            "fv3net_amd needs an MI355X (torch.cuda unavailable); there is no CPU fallback"
        )
    _native.load()


def stream_handle(stream=None, keep=()) -> int:
    """The hipStream_t of ``stream`` (default: the current stream).  A launch on another
    stream is ordered after the current stream's work so far, where the caller's inputs
    (or their device copies) were produced, and every tensor in ``keep`` (the temporaries
    and outputs the kernel touches, allocated on the current stream) stays allocated
    until the side stream's work is done (``record_stream``): without it the caching
    allocator could hand a returned-and-dropped buffer to new current-stream work while
    the side-stream kernel still reads or writes it."""
    if stream is None:
        return int(torch.cuda.current_stream().cuda_stream)
    cur = torch.cuda.current_stream()
    if stream != cur:
        stream.wait_stream(cur)
        keep_for(stream, keep)
    return int(stream.cuda_stream)


def keep_for(stream, tensors):
    """Tensors allocated on the current stream but used on ``stream`` stay allocated
    until that stream's work is done."""
    if stream is not None:
        for t in tensors:
            if torch.is_tensor(t) and t.is_cuda:
                t.record_stream(stream)


def to_device_f32(x, device=None, contiguous: bool = True):
    """numpy / torch -> float32 CUDA tensor (copy only when needed).  With
    ``contiguous=False`` a float32 CUDA view is returned as is (strides kept)."""
    require_gpu()
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev, dtype=torch.float32)
    else:
        a = np.asarray(x)
        if a.dtype in (np.float32, np.float64):
            # pinned, double-buffered H2D of the array's own bytes; a float64 host array
            # is cast on the device (round to nearest, as numpy's astype)
            from . import transfer

            t = transfer.h2d(a, device=dev)
            if t.dtype != torch.float32:
                t = t.to(torch.float32)
        else:
            t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32))).to(dev)
    return t.contiguous() if contiguous else t


def column_view(x, level_axis: int, keep_f64: bool = False):
    """(tensor, fv3_layout, ncol, nz) for ``x`` with levels on ``level_axis``: strided
    CUDA views the layout can express are used in place, anything else is copied to a
    contiguous device tensor first.  float32 unless ``keep_f64`` and ``x`` is a float64
    CUDA tensor (kernels that read float64 in place)."""
    if keep_f64 and torch.is_tensor(x) and x.is_cuda and x.dtype == torch.float64:
        t = x
    else:
        t = to_device_f32(x, contiguous=False)
    try:
        lay, ncol, nz = level_layout(t, level_axis)
    except ValueError:
        t = t.contiguous()
        lay, ncol, nz = level_layout(t, level_axis)
    return t, lay, ncol, nz


def ptr(t) -> int:
    return int(t.data_ptr())


def level_layout(t, level_axis: int):
    """fv3_layout for a tensor whose columns are every axis but ``level_axis``: axes
    before it are 'blocks' (e.g. tile), axes after it the horizontal plane (e.g. y, x).
    Views are fine as long as the plane is contiguous and the block axes flatten to a
    single stride, e.g. a (tile, z, y, x) array, its (z, rows, x) row band, or a
    tile slice; the level stride may be anything."""
    shape = tuple(int(n) for n in t.shape)
    st = tuple(int(x) for x in t.stride())
    nz = shape[level_axis]
    inner = shape[level_axis + 1:]
    plane = int(np.prod(inner, dtype=np.int64)) if inner else 1
    if t.numel() == 0:  # nothing to address: any layout will do
        nblk = int(np.prod(shape[:level_axis], dtype=np.int64)) if level_axis > 0 else 1
        p = max(plane, 1)
        return _native.layout(p, p, max(nz, 1) * p), nblk * plane, nz
    expect = 1
    for n, x in zip(reversed(inner), reversed(st[level_axis + 1:])):
        if n != 1 and x != expect:
            raise ValueError(f"the horizontal plane of a {shape} tensor with strides {st} is not contiguous")
        expect *= n
    blocks = [(n, x) for n, x in zip(shape[:level_axis], st[:level_axis]) if n != 1]
    nblk = int(np.prod([n for n, _ in blocks], dtype=np.int64)) if blocks else 1
    blk_stride = blocks[-1][1] if blocks else nz * plane
    for (n0, x0), (n1, x1) in zip(blocks[:-1], blocks[1:]):
        if x0 != x1 * n1:
            raise ValueError(f"the block axes of a {shape} tensor with strides {st} do not flatten")
    ld = st[level_axis] if nz > 1 else plane
    return _native.layout(plane, ld, blk_stride), nblk * plane, nz


class BoundLaunch:
    """One C-ABI launch marshalled once over fixed device buffers, re-issued per call
    with only the stream handle added: ``fn(*args, stream)``.  ``keep``: the tensors it
    touches (kept alive, and ordered on a side stream like stream_handle does);
    ``result``: what a call returns (its buffers are rewritten each time)."""

    def __init__(self, fn, args, keep, what: str, result=None):
        self.fn, self.args, self.keep, self.what, self.result = fn, tuple(args), list(keep), what, result

    def __call__(self, stream=None):
        h = stream if isinstance(stream, int) else stream_handle(stream, self.keep)
        st = self.fn(*self.args, h)
        if st:
            _native.check(st, self.what)
        return self.result
