"""Multi-GPU: column sharding and the path's one collective (global means).

Columns are independent on this path (mappm loops columns independently,
mappm.f90:58-124; the dense model has n_halo = 0, dense.py:228), so ranks own
disjoint column bands and the data path has no exchange at all.  The only
collective in the reference's per-step loop is the global average of 2-D
diagnostics (workflows/prognostic_c48_run/runtime/metrics.py:18-24:
``comm.reduce((area * x).sum())`` and ``comm.reduce(area.sum())``), done here as
one all-gather of float64 per-rank partials [n_diag, 2] summed in fixed rank order,
so every rank gets the same bits whatever the backend's reduction tree.

One process per GPU; backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" in
the CPU tests.
"""
import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _device, _native

try:
    import torch
    import torch.distributed as dist
except ImportError:  # pragma: no cover
    torch = None
    dist = None


@dataclass(frozen=True)
class Segment:
    """Rows [y0, y1) of one tile: a contiguous run of (y, x) columns per level."""
    tile: int
    y0: int
    y1: int


def row_band(n_rows: int, rank: int, world: int, align: int = 1) -> Tuple[int, int]:
    """Contiguous band [start, stop) of ``n_rows`` rows for ``rank`` of ``world``;
    boundaries are multiples of ``align`` (e.g. the coarsening factor, so a coarse
    cell never straddles two ranks).  Bands differ in size by at most ``align``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if align < 1 or n_rows % align:
        raise ValueError(f"{n_rows} rows are not divisible by align={align}")
    units = n_rows // align
    lo = rank * units // world
    hi = (rank + 1) * units // world
    return lo * align, hi * align


def column_segments(ntile: int, ny: int, rank: int, world: int, align: int = 1) -> List[Segment]:
    """The rank's band of the flattened (tile, y) rows, split at tile
    boundaries: at most ceil(band / ny) + 1 segments, each an in-place view of a
    (tile, z, y, x) array."""
    if ny % align:
        raise ValueError(f"ny={ny} is not divisible by align={align}")
    start, stop = row_band(ntile * ny, rank, world, align)
    segs = []
    r = start
    while r < stop:
        t, y = divmod(r, ny)
        y1 = min(ny, y + (stop - r))
        segs.append(Segment(t, y, y1))
        r += y1 - y
    return segs


def segment_view(arr, seg: Segment):
    """(tile, z, y, x) -> the (z, rows, x) view of one segment (no copy)."""
    return arr[seg.tile, :, seg.y0:seg.y1]


def _area_partials_setup(diags, area, out=None):
    _device.require_gpu()
    wide = any(_is_f64(t) for t in [area, *diags])
    if wide:
        conv = lambda t: _f64_on_device(t, torch.device("cuda", torch.cuda.current_device()))  # noqa: E731
    else:
        conv = lambda t: _device.to_device_f32(t).contiguous()  # noqa: E731
    area = conv(area)
    xs = [conv(d) for d in diags]
    for d in xs:
        if d.shape != area.shape:
            raise ValueError(f"diagnostic shape {tuple(d.shape)} != area shape {tuple(area.shape)}")
    if out is None:
        out = torch.empty((len(xs), 2), dtype=torch.float64, device=area.device)
    elif not (out.dtype == torch.float64 and tuple(out.shape) == (len(xs), 2) and out.is_contiguous()):
        raise ValueError(f"out must be a contiguous [{len(xs)}, 2] float64 tensor")
    tab = (ctypes.c_void_p * max(len(xs), 1))(*[d.data_ptr() for d in xs])
    lib = _native.load()
    fn = lib.fv3_area_weighted_sums_f64 if wide else lib.fv3_area_weighted_sums
    return fn, (tab, len(xs), area.data_ptr(), area.numel(), out.data_ptr()), [area, out] + xs, out, len(xs)


def area_weighted_partials(diags: Sequence, area, stream=None):
    """Device float64 partials [n_diag, 2] = (sum(area * x_d), sum(area)) over this
    rank's columns, computed by the deterministic two-stage HIP reduction
    (csrc/reduce.hip).  ``diags``: CUDA tensors shaped like ``area``.  As numpy's
    ``area * ds`` promotes, any float64 operand puts the whole reduction on the float64
    kernel (float32 operands widened exactly); all-float32 inputs use the float32 one."""
    fn, args, keep, out, n = _area_partials_setup(diags, area)
    if not n:
        return out
    st = fn(*args, _device.stream_handle(stream, keep))
    _native.check(st, "area_weighted_sums")
    return out


def bind_area_weighted_partials(diags: Sequence, area, out=None) -> "_device.BoundLaunch":
    """area_weighted_partials over fixed buffers, marshalled once (the per-step reduction
    of the stepper's diagnostics); each call rewrites and returns ``out``."""
    fn, args, keep, out, n = _area_partials_setup(diags, area, out)
    if not n:
        raise ValueError("no diagnostics to reduce")
    return _device.BoundLaunch(fn, args, keep, "area_weighted_sums", out)


def _backend_device(group=None):
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def combine_partials(partials, group=None):
    """All-gather float64 partials [n_diag, 2] and sum them in rank order 0..N-1.
    Returns the global [n_diag, 2] sums (identical bits on every rank)."""
    p = torch.as_tensor(partials, dtype=torch.float64)
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return p.clone()
    dev = _backend_device(group)
    world = dist.get_world_size(group)
    local = p.to(dev).contiguous()
    gathered = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(gathered, local, group=group)
    total = gathered[0].clone()
    for g in gathered[1:]:  # fixed order: bitwise reproducible on every rank
        total += g
    return total.to(p.device)


def global_average(partials, group=None) -> np.ndarray:
    """metrics.py:18-24 global_average for n_diag diagnostics at once: global
    sum(area*x) / sum(area).  Unlike the reference (which returns -1 off rank 0)
    every rank gets the value."""
    total = combine_partials(partials, group).cpu().numpy()
    return total[:, 0] / total[:, 1]


def _is_2d(v, area_shape) -> bool:
    dims = getattr(v, "dims", None)
    if dims is not None and not callable(dims):
        return set(dims) == {"x", "y"}
    return tuple(v.shape) == tuple(area_shape)


def _data(v):
    d = getattr(v, "data", v)
    return d if (torch is not None and isinstance(d, torch.Tensor)) else getattr(v, "values", d)


def globally_average_2d_diagnostics(diagnostics: dict, exclude: Sequence[str] = None, group=None) -> dict:
    """metrics.py:33-43: the global area-weighted mean of every (x, y) diagnostic not
    in ``exclude`` (area from ``diagnostics["area"]``, itself included, as in the
    reference) — one HIP reduction for all of them plus one all-gather."""
    exclude = set(exclude or ())
    area = _data(diagnostics["area"])
    names = [k for k, v in diagnostics.items() if k not in exclude and _is_2d(v, np.shape(area))]
    if not names:
        return {}
    means = global_average(area_weighted_partials([_data(diagnostics[k]) for k in names], area), group)
    return {k: float(m) for k, m in zip(names, means)}


def _level_sums_setup(field, out=None):
    _device.require_gpu()
    lib = _native.load()
    dev = torch.device("cuda", torch.cuda.current_device())
    src = field if torch.is_tensor(field) else torch.from_numpy(np.ascontiguousarray(field))
    if src.dtype in (torch.float64, torch.uint8):  # read in the field's own dtype (no f32 rounding)
        t = src.to(dev)
        fn = lib.fv3_level_sums_f64 if t.dtype == torch.float64 else lib.fv3_level_sums_u8
    else:  # float32, or integer/bool flags that float32 holds exactly
        t = _device.to_device_f32(src)
        fn = lib.fv3_level_sums
    try:
        lay, ncol, nz = _device.level_layout(t, 0)
    except ValueError:
        t = t.contiguous()
        lay, ncol, nz = _device.level_layout(t, 0)
    if out is None:
        out = torch.empty(nz, dtype=torch.float64, device=t.device)
    elif not (out.dtype == torch.float64 and out.numel() == nz and out.is_contiguous()):
        raise ValueError(f"out must be a contiguous float64 tensor of {nz} values")
    return fn, (t.data_ptr(), lay, ncol, nz, out.data_ptr()), [t, out], out


def level_sums(field, stream=None):
    """Device float64 per-level horizontal sums of a (z, ...) field (deterministic
    fixed-tree HIP reduction): the per-rank part of metrics.py:27-32."""
    fn, args, keep, out = _level_sums_setup(field)
    st = fn(*args, _device.stream_handle(stream, keep))
    _native.check(st, "level_sums")
    return out


def bind_level_sums(field, out=None) -> "_device.BoundLaunch":
    """level_sums of a fixed device field into a fixed ``out`` (e.g. a slice of a wider
    result buffer), marshalled once."""
    fn, args, keep, out = _level_sums_setup(field, out)
    return _device.BoundLaunch(fn, args, keep, "level_sums", out)


def globally_sum_3d_diagnostics(diagnostics: dict, include: Sequence[str], group=None) -> dict:
    """metrics.py:46-55: ``{name}_global_sum`` = per-level sums over x, y and all
    ranks of each included (z, y, x) diagnostic (rank partials summed in rank order)."""
    sums = {}
    for k, v in diagnostics.items():
        dims = getattr(v, "dims", None)
        if k in include and dims is not None and set(dims) == {"x", "y", "z"}:
            data = _data(v)
            if tuple(dims) != ("z", "y", "x"):
                data = data.permute(*[dims.index(d) for d in ("z", "y", "x")]) if hasattr(data, "permute") \
                    else np.transpose(data, [dims.index(d) for d in ("z", "y", "x")])
            part = level_sums(data)[:, None]
            total = combine_partials(part, group)[:, 0]
            sums[f"{k}_global_sum"] = [float(x) for x in total.cpu().numpy()]
    return sums


# --------------------------------------------------------------------------------
# World-size-invariant global sums: partials per grid ROW, gathered in global row
# order and folded row by row (csrc/reduce.hip).  A rank owns a contiguous band of the
# flattened (tile, y) rows (row_band), so the gathered rows are the global rows in
# order and the folded sums carry the same bits for 1, 2, 4 or 8 ranks.
# --------------------------------------------------------------------------------
def _is_f64(t) -> bool:
    """float64 operand, torch or numpy (numpy's promotion decides the arithmetic)."""
    if torch.is_tensor(t):
        return t.dtype == torch.float64
    return np.asarray(t).dtype == np.float64


def _f64_on_device(t, dev):
    if not torch.is_tensor(t):
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(t)))
    return t.to(dev, torch.float64).contiguous()


def _area_row_setup(diags, area, out=None):
    _device.require_gpu()
    wide = any(_is_f64(t) for t in [area, *diags])
    dev = torch.device("cuda", torch.cuda.current_device())
    conv = (lambda t: _f64_on_device(t, dev)) if wide else \
        (lambda t: _device.to_device_f32(t).contiguous())  # noqa: E731
    area = conv(area)
    xs = [conv(d) for d in diags]
    if area.dim() < 1:
        raise ValueError("area must have a row axis")
    row_len = int(area.shape[-1])
    nrows = area.numel() // max(row_len, 1)
    for d in xs:
        if d.shape != area.shape:
            raise ValueError(f"diagnostic shape {tuple(d.shape)} != area shape {tuple(area.shape)}")
    if out is None:
        out = torch.empty((nrows, len(xs), 2), dtype=torch.float64, device=dev)
    elif not (out.dtype == torch.float64 and out.dim() == 2 and out.shape[0] == nrows and out.stride(1) == 1
              and out.shape[1] >= 2 * len(xs)):
        raise ValueError(f"out must be a row-major [{nrows}, >= {2 * len(xs)}] float64 buffer")
    tab = (ctypes.c_void_p * max(len(xs), 1))(*[d.data_ptr() for d in xs])
    lib = _native.load()
    fn = lib.fv3_area_weighted_row_sums_f64 if wide else lib.fv3_area_weighted_row_sums
    ld = out.stride(0) if out.dim() == 2 else 2 * len(xs)
    args = (tab, len(xs), area.data_ptr(), nrows, row_len, out.data_ptr(), ld)
    return fn, args, [area, out] + xs, out, bool(xs) and nrows > 0


def area_row_partials(diags: Sequence, area, stream=None, out=None):
    """Device float64 [nrows, n_diag, 2]: per row of (rows, row_len) fields,
    (sum area*x_d, sum area).  float64 if any operand is (numpy's promotion).  ``out``:
    a [nrows, W >= 2 n_diag] float64 buffer whose leading columns receive them."""
    fn, args, keep, out, work = _area_row_setup(diags, area, out)
    if not work:
        return out
    st = fn(*args, _device.stream_handle(stream, keep))
    _native.check(st, "area_weighted_row_sums")
    return out


def bind_area_row_partials(diags: Sequence, area, out=None) -> "_device.BoundLaunch":
    """area_row_partials over fixed buffers, marshalled once; each call rewrites ``out``."""
    fn, args, keep, out, work = _area_row_setup(diags, area, out)
    if not work:
        raise ValueError("no rows or diagnostics to reduce")
    return _device.BoundLaunch(fn, args, keep, "area_weighted_row_sums", out)


def bind_step_partials(diags: Sequence, area, limiter, out=None, level_out=None) -> "_device.BoundLaunch":
    """One launch for a stepper step's per-rank reductions (fv3_step_partials_f64): the
    area-weighted row partials of float64 ``diags`` over ``area`` (as
    bind_area_row_partials, into ``out``) and the per-level counts of the uint8
    ``limiter`` flags (as bind_level_sums, into ``level_out``), each with the bits of its
    own launch.  The result is ``(out, level_out)``."""
    rfn, rargs, rkeep, out, work = _area_row_setup(diags, area, out)
    if not work:
        raise ValueError("no rows or diagnostics to reduce")
    if rfn.__name__ != "fv3_area_weighted_row_sums_f64":
        raise ValueError("bind_step_partials: float64 diagnostics or area")
    lfn, largs, lkeep, level_out = _level_sums_setup(limiter, level_out)
    if lfn.__name__ != "fv3_level_sums_u8":
        raise ValueError("bind_step_partials: uint8 limiter flags")
    lib = _native.load()
    args = rargs + (largs[0], largs[1], largs[2], largs[3], largs[4])
    return _device.BoundLaunch(lib.fv3_step_partials_f64, args, rkeep + lkeep, "step_partials", (out, level_out))


def bind_fold_rows_repeat(rows, times: int, rep=None, out=None) -> "_device.BoundLaunch":
    """The stubbed exchange and its fold in one launch (fv3_fold_rows_repeat): ``rep``
    receives ``times`` copies of ``rows`` (the bytes an all-gather over ``times`` ranks
    moves), ``out`` the fold over them (bind_fold_rows of ``rep``, the same bits)."""
    if not (torch.is_tensor(rows) and rows.is_cuda and rows.dtype == torch.float64 and rows.is_contiguous()
            and rows.dim() == 2):
        raise ValueError("bind_fold_rows_repeat needs a contiguous [nrows, width] float64 CUDA buffer")
    nrows, width = (int(n) for n in rows.shape)
    if rep is None:
        rep = torch.empty((times * nrows, width), dtype=torch.float64, device=rows.device)
    if not (rep.dtype == torch.float64 and rep.is_contiguous() and tuple(rep.shape) == (times * nrows, width)):
        raise ValueError(f"rep must be a contiguous [{times * nrows}, {width}] float64 buffer")
    if out is None:
        out = torch.empty(width, dtype=torch.float64, device=rows.device)
    if not (out.dtype == torch.float64 and out.is_contiguous() and out.numel() == width):
        raise ValueError(f"out must be {width} contiguous float64 values")
    lib = _native.load()
    return _device.BoundLaunch(lib.fv3_fold_rows_repeat, (rows.data_ptr(), nrows, width, int(times), rep.data_ptr(),
                                                          out.data_ptr()), [rows, rep, out], "fold_rows_repeat", out)


def level_row_partials(field, stream=None, out=None):
    """Device float64 [nrows, nz] per-row level sums of a (nz, rows, row_len) field
    (uint8 flags such as specific_humidity_limiter_active, or float64) read in place.
    ``out``: a [nrows, >= nz] float64 view (e.g. columns of a wider buffer)."""
    _device.require_gpu()
    t = field if torch.is_tensor(field) else torch.from_numpy(np.ascontiguousarray(field))
    t = t.to(torch.device("cuda", torch.cuda.current_device()))
    if t.dtype not in (torch.uint8, torch.float64):
        t = t.to(torch.float64)
    if t.dim() != 3:
        raise ValueError("field must be (z, rows, row_len)")
    if not (t.stride(2) == 1 and t.stride(1) == t.shape[2]):
        t = t.contiguous()
    nz, nrows, row_len = (int(n) for n in t.shape)
    if out is None:
        out = torch.empty((nrows, nz), dtype=torch.float64, device=t.device)
    elif not (out.dtype == torch.float64 and out.dim() == 2 and out.shape[0] == nrows and out.stride(1) == 1
              and out.shape[1] >= nz):
        raise ValueError(f"out must be a row-major [{nrows}, >= {nz}] float64 view")
    lib = _native.load()
    fn = lib.fv3_level_row_sums_u8 if t.dtype == torch.uint8 else lib.fv3_level_row_sums_f64
    st = fn(t.data_ptr(), nz, nrows, row_len, int(t.stride(0)) if nz > 1 else nrows * row_len, out.data_ptr(),
            int(out.stride(0)), _device.stream_handle(stream, [t, out]))
    _native.check(st, "level_row_sums")
    return out


def _distributed() -> bool:
    return dist is not None and dist.is_available() and dist.is_initialized()


def row_counts(nrows: int, group=None) -> List[int]:
    """Every rank's row count (one small all-gather; fixed for a run, so callers keep it)."""
    if not _distributed():
        return [int(nrows)]
    dev = _backend_device(group)
    n = torch.tensor([int(nrows)], dtype=torch.int64, device=dev)
    counts = [torch.empty_like(n) for _ in range(dist.get_world_size(group))]
    dist.all_gather(counts, n, group=group)
    return [int(c.item()) for c in counts]


def gather_rows(local, group=None, counts: Optional[Sequence[int]] = None):
    """All ranks' [nrows_r, W] row partials concatenated in rank order (= global row
    order for row bands): one all-gather of the rows padded to the largest band
    (``counts`` from row_counts, gathered here when not given).  Without a process
    group: ``local`` itself."""
    if not _distributed():
        return local
    dev = _backend_device(group)
    world = dist.get_world_size(group)
    x = local.to(dev).contiguous()
    counts = list(counts) if counts is not None else row_counts(x.shape[0], group)
    if len(counts) != world or counts[dist.get_rank(group)] != x.shape[0]:
        raise ValueError(f"row counts {counts} do not match this rank's {x.shape[0]} rows")
    cap = max(counts)
    pad = torch.zeros((cap,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
    pad[: x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


def _fold_setup(rows, out=None):
    _device.require_gpu()
    r = rows.to(torch.device("cuda", torch.cuda.current_device()), torch.float64).contiguous()
    nrows = int(r.shape[0])
    width = int(r[0].numel()) if nrows else int(np.prod(r.shape[1:], dtype=np.int64))
    if out is None:
        out = torch.empty(tuple(r.shape[1:]), dtype=torch.float64, device=r.device)
    elif not (out.dtype == torch.float64 and out.numel() == width and out.is_contiguous()):
        raise ValueError(f"out must be a contiguous float64 tensor of {width} values")
    return _native.load().fv3_fold_rows, (r.data_ptr(), nrows, width, out.data_ptr()), [r, out], out


def fold_rows(rows, stream=None):
    """Device float64 sums over the rows of [nrows, ...] partials, in row order (HIP)."""
    fn, args, keep, out = _fold_setup(rows)
    st = fn(*args, _device.stream_handle(stream, keep))
    _native.check(st, "fold_rows")
    return out


def bind_fold_rows(rows, out=None) -> "_device.BoundLaunch":
    """fold_rows of a fixed [nrows, ...] float64 device buffer into ``out``, marshalled once."""
    if not (torch.is_tensor(rows) and rows.is_cuda and rows.dtype == torch.float64 and rows.is_contiguous()):
        raise ValueError("bind_fold_rows needs a contiguous float64 CUDA buffer (read in place every call)")
    fn, args, keep, out = _fold_setup(rows, out)
    return _device.BoundLaunch(fn, args, keep, "fold_rows", out)


def global_row_sums(local_rows, group=None, counts: Optional[Sequence[int]] = None):
    """fold_rows(gather_rows(local_rows)): the same bits on every rank and for every
    world size."""
    return fold_rows(gather_rows(local_rows, group, counts))


def global_count_sums(local_counts, group=None):
    """Global sums of integer-valued float64 counts (e.g. the per-level number of
    columns where the humidity limiter fired, metrics.py:27-32 on a 0/1 field): one
    all-reduce.  Integers below 2**53 add exactly in float64 in any order, so unlike
    the float partials they need no row granularity to be world-size invariant."""
    x = torch.as_tensor(local_counts, dtype=torch.float64)
    if not _distributed():
        return x.clone()
    dev = _backend_device(group)
    y = x.to(dev).contiguous().clone()
    dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
    return y.to(x.device)
