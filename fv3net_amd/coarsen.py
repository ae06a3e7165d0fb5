"""Pressure-level coarse-graining (vcm.cubedsphere) on MI355X.

``coarsen_on_pressure`` fuses, for the masked area-weighted variables of
``coarsen_restarts_on_pressure`` (external/vcm/vcm/cubedsphere/coarsen_restarts.py:411-516,
840-887), the whole ``regrid_to_area_weighted_pressure`` (regridz.py:25-55) ->
``weighted_block_average`` (coarsen.py:183-218) chain into one HIP kernel
(csrc/coarsen.hip).  ``regrid_vertical`` mirrors regridz.py:164-279 on device.
"""
import ctypes
from typing import Dict, Mapping, Sequence

import numpy as np

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

TOA_PRESSURE = 300.0  # external/vcm/vcm/calc/thermo/constants.py:17


def coarsen_on_pressure(delp, area, fields: Mapping[str, object], factor: int, iv: int = 1, kord: int = 1,
                        ptop: float = TOA_PRESSURE, stream=None, coarse_delp_f64: bool = False,
                        exact: bool = False):
    """delp and fields (tile, z, y, x), area (tile, y, x) -> dict of coarse fields
    (tile, z, y/f, x/f) and the area-weighted coarse delp (float32, or float64 when
    ``coarse_delp_f64`` and delp is float64: the restart-precision
    weighted_block_average(delp, area) of coarsen_restarts.py:480-486).  Device tensors
    in and out.  ``exact`` selects the remap's arithmetic as in ``mappm_device``
    (default: the 1e-5 rel contract for finite inputs; True: bit-exact to the reference
    and oracle/coarsen.py, NaNs included)."""
    _device.require_gpu()
    delp64 = (isinstance(delp, np.ndarray) and delp.dtype == np.float64) or (
        torch is not None and isinstance(delp, torch.Tensor) and delp.dtype == torch.float64)
    if delp64:  # keep restart precision: pressures are cumulated in float64 on device
        delp = (torch.as_tensor(delp) if not isinstance(delp, torch.Tensor) else delp).to(
            device=torch.device("cuda", torch.cuda.current_device()), dtype=torch.float64).contiguous()
    else:
        delp = _device.to_device_f32(delp)
    area = _device.to_device_f32(area)
    if delp.dim() != 4 or area.dim() != 3:
        raise ValueError("delp must be (tile, z, y, x) and area (tile, y, x)")
    nt, km, ny, nx = delp.shape
    if tuple(area.shape) != (nt, ny, nx):
        raise ValueError(f"area shape {tuple(area.shape)} does not match delp {tuple(delp.shape)}")
    names = list(fields)
    tens = []
    for n in names:
        t = _device.to_device_f32(fields[n])
        if tuple(t.shape) != tuple(delp.shape):
            raise ValueError(f"{n} shape {tuple(t.shape)} != delp shape {tuple(delp.shape)}")
        tens.append(t)
    if ny % factor or nx % factor:
        raise ValueError(f"grid {ny}x{nx} is not divisible by the coarsening factor {factor}")
    cshape = (nt, km, ny // factor, nx // factor)
    outs = [torch.empty(cshape, dtype=torch.float32, device=delp.device) for _ in names]
    want64 = delp64 and coarse_delp_f64
    delp_c = torch.empty(cshape, dtype=torch.float64 if want64 else torch.float32, device=delp.device)
    fptr = (ctypes.c_void_p * max(1, len(tens)))(*[t.data_ptr() for t in tens])
    optr = (ctypes.c_void_p * max(1, len(outs)))(*[t.data_ptr() for t in outs])
    lib = _native.load()
    fn = lib.fv3_regrid_coarsen_f64d if want64 else (lib.fv3_regrid_coarsen_f64 if delp64 else lib.fv3_regrid_coarsen)
    st = fn(delp.data_ptr(), area.data_ptr(), fptr, optr, len(tens), delp_c.data_ptr(), nt, km, ny, nx,
            int(factor), int(iv), int(kord), float(ptop), _native.arith(exact),
            _device.stream_handle(stream, [delp, area, delp_c] + tens + outs))
    _native.check(st, "regrid_coarsen")
    return dict(zip(names, outs)), delp_c


def _delp_on_device(delp):
    delp64 = (isinstance(delp, np.ndarray) and delp.dtype == np.float64) or (
        torch is not None and isinstance(delp, torch.Tensor) and delp.dtype == torch.float64)
    if delp64:  # keep restart precision: pressures are cumulated in float64 on device
        delp = (torch.as_tensor(delp) if not isinstance(delp, torch.Tensor) else delp).to(
            device=torch.device("cuda", torch.cuda.current_device()), dtype=torch.float64).contiguous()
    else:
        delp = _device.to_device_f32(delp)
    return delp, delp64


def coarsen_edges_on_pressure(delp, spacing, fields: Mapping[str, object], factor: int, edge: str = "x",
                              iv: int = 1, kord: int = 1, ptop: float = TOA_PRESSURE, stream=None,
                              exact: bool = False):
    """D-grid winds on coarse pressure levels: regrid_to_edge_weighted_pressure
    (regridz.py:58-112) followed by the masked edge_weighted_block_average of
    coarsen_restarts.py:493-509, fused (csrc/coarsen.hip, regrid_coarsen_edge_kernel).

    delp (6, z, n, n) cell centers; edge "x": spacing dx (6, n+1, n) and fields u
    (6, z, n+1, n) -> (6, z, n/f+1, n/f); edge "y": spacing dy (6, n, n+1) and fields
    v (6, z, n, n+1) -> (6, z, n/f, n/f+1).  Device tensors in and out; ``exact`` as in
    ``coarsen_on_pressure``."""
    _device.require_gpu()
    if edge not in ("x", "y"):
        raise ValueError(f"'edge' most be either 'x' or 'y'; got {edge}.")  # coarsen.py:253
    delp, delp64 = _delp_on_device(delp)
    spacing = _device.to_device_f32(spacing)
    if delp.dim() != 4 or spacing.dim() != 3:
        raise ValueError("delp must be (tile, z, y, x) and the edge spacing (tile, y, x)")
    nt, km, ny, nx = delp.shape
    eshape = (nt, ny + 1, nx) if edge == "x" else (nt, ny, nx + 1)
    if tuple(spacing.shape) != eshape:
        raise ValueError(f"edge {edge!r} spacing must be {eshape}, got {tuple(spacing.shape)}")
    names = list(fields)
    tens = []
    for n in names:
        t = _device.to_device_f32(fields[n])
        if tuple(t.shape) != (nt, km) + eshape[1:]:
            raise ValueError(f"{n} shape {tuple(t.shape)} != {(nt, km) + eshape[1:]}")
        tens.append(t)
    if ny % factor or nx % factor:
        raise ValueError(f"grid {ny}x{nx} is not divisible by the coarsening factor {factor}")
    nc = nx // factor
    cshape = (nt, km, nc + 1, nc) if edge == "x" else (nt, km, nc, nc + 1)
    outs = [torch.empty(cshape, dtype=torch.float32, device=delp.device) for _ in names]
    fptr = (ctypes.c_void_p * max(1, len(tens)))(*[t.data_ptr() for t in tens])
    optr = (ctypes.c_void_p * max(1, len(outs)))(*[t.data_ptr() for t in outs])
    lib = _native.load()
    fn = lib.fv3_regrid_coarsen_edge_f64 if delp64 else lib.fv3_regrid_coarsen_edge
    st = fn(delp.data_ptr(), spacing.data_ptr(), fptr, optr, len(tens), nt, km, ny, nx, int(factor),
            0 if edge == "x" else 1, int(iv), int(kord), float(ptop), _native.arith(exact),
            _device.stream_handle(stream, [delp, spacing] + tens + outs))
    _native.check(st, "regrid_coarsen_edge")
    return dict(zip(names, outs))


def regrid_vertical(p_in, f_in, p_out, iv: int = 1, kord: int = 1, z_axis: int = -1, exact: bool = False):
    """Device regrid_vertical (regridz.py:164-279) on arrays whose vertical axis is
    ``z_axis`` (default last, as the reference transposes to); float32 result with
    the input's axis order.  Raises the reference's ValueErrors.  ``exact`` as in
    ``mappm_device``."""
    from .mappm import mappm_device

    p_in, f_in, p_out = (_device.to_device_f32(a) for a in (p_in, f_in, p_out))
    ax = z_axis % p_in.dim()
    if f_in.shape[ax] != p_in.shape[ax] - 1:
        raise ValueError("f_in must have a vertical dimension one shorter than p_in")
    cols = lambda t: t.movedim(ax, 0).reshape(t.shape[ax], -1)
    if cols(p_in).shape[1] != cols(f_in).shape[1] or cols(p_out).shape[1] != cols(f_in).shape[1]:
        raise ValueError("All dimensions except vertical must be same size for p_in, f_in and p_out")
    q2 = mappm_device(cols(p_in).contiguous(), cols(f_in).contiguous(), cols(p_out).contiguous(), iv, kord,
                      exact=exact)
    shape = list(f_in.movedim(ax, 0).shape)
    shape[0] = q2.shape[0]
    return q2.reshape(shape).movedim(0, ax).contiguous()
