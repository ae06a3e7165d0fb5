"""Vertical interpolation of columns to new levels on the device (csrc/interpolate.hip).

Mirrors (paths under /root/reference):
* ``interpolate_2d``   mappm.interpolate_2d (external/mappm/mappm/interpolate_2d.f90:1-27):
  rows are columns, float64 in and out, fill_value where no level brackets.
* ``interpolate_1d``   vcm.interpolate_1d (external/vcm/vcm/interpolate.py:100-145): output
  levels per column (``xp`` with the level axis) go through interpolate_2d; one set of
  levels for every column (1-D ``xp``) through metpy.interpolate.interpolate_1d's
  algorithm (:148-173).
* ``pressure_at_midpoint_log``  vcm/calc/thermo/vertically_dependent.py:153-178.
* ``interpolate_to_pressure_levels``  vcm/interpolate.py:77-97.

Arrays carry their level axis at ``axis`` (default 0: the stacked [z, column] layout,
used in place); every other axis is a column axis.  Results are CUDA tensors; the
interpolated values are float64 (the reference's dtype: f2py real*8, and numpy's
promotion against float64 levels).  No CPU fallback.
"""
import ctypes

import numpy as np

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

# vcm/interpolate.py:30-68 (ERA-Interim levels), Pa
PRESSURE_GRID = np.array([
    300.0, 500.0, 700.0, 1000.0, 2000.0, 3000.0, 5000.0, 7000.0, 10000.0, 12500.0, 15000.0, 17500.0,
    20000.0, 22500.0, 25000.0, 30000.0, 35000.0, 40000.0, 45000.0, 50000.0, 55000.0, 60000.0, 65000.0,
    70000.0, 75000.0, 77500.0, 80000.0, 82500.0, 85000.0, 87500.0, 90000.0, 92500.0, 95000.0, 97500.0,
    100000.0,
])
TOA_PRESSURE = 300.0


def _dev(x, dtype=None):
    """CUDA tensor (float32/float64 kept unless ``dtype`` is given)."""
    _device.require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev)
    else:
        a = np.asarray(x)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    if dtype is not None:
        t = t.to(dtype)
    elif t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    return t


def _levels_first(t, axis):
    """(nlev, ncol) contiguous view/copy with the level axis first, and the column shape."""
    t = t.movedim(axis % t.dim(), 0)
    cols = tuple(t.shape[1:])
    return t.reshape(t.shape[0], -1).contiguous(), cols


def interpolate_2d(xp, x, y, fill_value=np.nan, stream=None):
    """mappm.interpolate_2d(xp, x, y, fill_value): xp (m, n_out), x and y (m, n_in) ->
    (m, n_out) float64.  For each output level the LAST bracketing interval wins, as in
    the Fortran (no early exit)."""
    xp, x, y = (_dev(a, torch.float64) for a in (xp, x, y))
    if x.dim() != 2 or y.shape != x.shape or xp.dim() != 2 or xp.shape[0] != x.shape[0]:
        raise ValueError(f"interpolate_2d: xp (m, n_out), x and y (m, n_in); got {tuple(xp.shape)}, "
                         f"{tuple(x.shape)}, {tuple(y.shape)}")
    out = _interp_columns(xp.t().contiguous(), x.t().contiguous(), y.t().contiguous(), fill_value, stream)
    return out.t()


def _interp_columns(xp, x, y, fill_value, stream):
    """level-major (n, ncol) float64 tensors -> (n_out, ncol) float64."""
    n_in, ncol = x.shape
    n_out = xp.shape[0]
    out = torch.empty((n_out, ncol), dtype=torch.float64, device=x.device)
    st = _native.load().fv3_interpolate_2d(xp.data_ptr(), ncol, x.data_ptr(), ncol, y.data_ptr(), ncol,
                                            out.data_ptr(), ncol, ncol, n_in, n_out, float(fill_value),
                                            _device.stream_handle(stream, [xp, x, y, out]))
    _native.check(st, "interpolate_2d")
    return out


def _interp_levels(levels, xp, var, fill_value, stream):
    """metpy algorithm for 1-D ``levels``; xp/var level-major (n_in, ncol)."""
    lv = np.asarray(levels, dtype=np.float64).reshape(-1)
    order = np.argsort(lv, kind="stable")
    srt = np.ascontiguousarray(lv[order])
    reverse = int(lv.size > 0 and lv[0] > lv[-1])
    n_in, ncol = xp.shape
    out = torch.empty((lv.size, ncol), dtype=torch.float64, device=xp.device)
    dl = torch.from_numpy(srt).to(xp.device)
    dtypes = int(xp.dtype == torch.float64) | (int(var.dtype == torch.float64) << 1)
    st = _native.load().fv3_interpolate_levels(xp.data_ptr(), ncol, var.data_ptr(), ncol, dtypes, dl.data_ptr(),
                                                lv.size, reverse, out.data_ptr(), ncol, ncol, n_in,
                                                float(fill_value), _device.stream_handle(stream, [xp, var, dl, out]))
    _native.check(st, "interpolate_levels")
    return out


def interpolate_1d(xp, x, field, axis: int = 0, fill_value=np.nan, stream=None):
    """vcm.interpolate_1d: ``field`` and its coordinate ``x`` (levels on ``axis``)
    interpolated to ``xp`` — 1-D output levels shared by all columns, or per-column
    levels shaped like ``field`` with n_out levels on ``axis``.  ``x`` must increase
    along the axis, as the reference requires (interpolate.py:108): for shared levels
    the kernel does not re-sort columns the way metpy's argsort would."""
    x = _dev(x)
    field = _dev(field)
    if tuple(x.shape) != tuple(field.shape):
        raise ValueError(f"x {tuple(x.shape)} and field {tuple(field.shape)} must have the same shape")
    xl, cols = _levels_first(x, axis)
    fl, _ = _levels_first(field, axis)
    if np.ndim(xp) == 1 and not (isinstance(xp, torch.Tensor) and xp.dim() != 1):
        lv = xp.detach().cpu().numpy() if isinstance(xp, torch.Tensor) else np.asarray(xp)
        out = _interp_levels(lv, xl, fl, fill_value, stream)
    else:
        xpt = _dev(xp, torch.float64)
        xpl, xcols = _levels_first(xpt, axis)
        if xcols != cols:
            raise ValueError(f"xp columns {xcols} do not match the field's {cols}")
        out = _interp_columns(xpl, xl.to(torch.float64), fl.to(torch.float64), fill_value, stream)
    return out.reshape((out.shape[0],) + cols).movedim(0, axis % field.dim())


def pressure_at_midpoint_log(delp, axis: int = 0, toa_pressure: float = TOA_PRESSURE, stream=None):
    """delp / diff(log(cumsum([toa, delp]))) in delp's dtype (Simmons & Burridge 1981)."""
    d = _dev(delp)
    dl, cols = _levels_first(d, axis)
    nz, ncol = dl.shape
    out = torch.empty_like(dl)
    st = _native.load().fv3_pressure_midpoint_log(dl.data_ptr(), int(dl.dtype == torch.float64), ncol,
                                                   out.data_ptr(), ncol, ncol, nz, float(toa_pressure),
                                                   _device.stream_handle(stream, [dl, out]))
    _native.check(st, "pressure_midpoint_log")
    return out.reshape((nz,) + cols).movedim(0, axis % d.dim())


def interpolate_to_pressure_levels(field, delp, levels=PRESSURE_GRID, axis: int = 0, stream=None):
    """vcm.interpolate_to_pressure_levels: ``field`` on model levels -> ``levels`` (Pa),
    float64, NaN below the lowest / above the highest model midpoint."""
    p = pressure_at_midpoint_log(delp, axis=axis, stream=stream)
    return interpolate_1d(levels, p, field, axis=axis, stream=stream)
