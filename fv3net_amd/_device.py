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


def stream_handle(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return int(s.cuda_stream)


def to_device_f32(x, device=None):
    """numpy / torch -> contiguous float32 CUDA tensor (copy only when needed)."""
    require_gpu()
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev, dtype=torch.float32)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float32))).to(dev)
    return t.contiguous()


def ptr(t) -> int:
    return int(t.data_ptr())


def level_layout(t, level_axis: int):
    """fv3_layout for a contiguous tensor whose columns are every axis but
    ``level_axis``: axes before it are 'blocks' (e.g. tile), axes after it are the
    horizontal plane (e.g. y, x)."""
    shape = tuple(t.shape)
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    plane = int(np.prod(shape[level_axis + 1:], dtype=np.int64)) if level_axis + 1 < len(shape) else 1
    nz = int(shape[level_axis])
    nblk = int(np.prod(shape[:level_axis], dtype=np.int64)) if level_axis > 0 else 1
    ncol = nblk * plane
    return _native.layout(plane, plane, nz * plane), ncol, nz
