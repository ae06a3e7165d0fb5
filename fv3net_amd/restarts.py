"""Restart coarse-graining on pressure levels (vcm.cubedsphere) on MI355X.

``coarsen_restarts_on_pressure`` mirrors
external/vcm/vcm/cubedsphere/coarsen_restarts.py:152-225 for the fv_core, fv_tracer and
fv_srf_wnd categories, with every arithmetic stage in HIP:

* masked area-weighted pressure-level fields (W, T, [ua, va] of fv_core, every tracer of
  fv_tracer; :411-458, 488-494, 840-887): ONE fused ``fv3_regrid_coarsen_f64d`` pass over
  the shared delp, which also returns the area-weighted coarse delp in float64;
* D-grid winds u (dx) and v (dy) (:460-478, 496-512): ``fv3_regrid_coarsen_edge_f64``;
* plain area-weighted phis, DZ (:439, 480-486) and u_srf, v_srf (:890-913):
  ``fv3_weighted_block_average[_f64]``;
* _impose_hydrostatic_balance (:916-938): ``fv3_hydrostatic_balance`` replaces DZ and phis.

Inputs are mappings of arrays (numpy or torch) with the restart files' dims:
(tile, Time, z, y, x) / (tile, Time, y, x) as in the reference's regression data, or the
same without the Time axis.  ``grid_spec`` holds area (tile, y, x), dx (tile, y+1, x) and
dy (tile, y, x+1).  Outputs are device tensors with the input's dims; dtypes follow the
reference: float32 for the pressure-level fields (mappm output), float64 for delp, DZ,
phis and the surface winds (float64 restart data).

sfc_data (the 'complex' surface method: categorical modes, vegetation/soil rules) is not
on the hot path and raises NotImplementedError.
"""
import ctypes
from typing import Dict, Mapping

import numpy as np

from . import _device, _native
from .coarsen import TOA_PRESSURE, coarsen_edges_on_pressure, coarsen_on_pressure

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

# coarsen_restarts.py:56-66
FRACTION_TRACERS = ["cld_amt"]
NON_FRACTION_TRACERS = ["sphum", "liq_wat", "rainwat", "ice_wat", "snowwat", "graupel", "o3mr", "sgs_tke"]


def _dev(x, dtype=None):
    """numpy / torch -> contiguous CUDA tensor, float64 kept as float64 unless ``dtype``."""
    dev = torch.device("cuda", torch.cuda.current_device())
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if dtype is None:
        dtype = torch.float64 if t.dtype == torch.float64 else torch.float32
    return t.to(device=dev, dtype=dtype).contiguous()


def weighted_block_average(fields: Mapping[str, object], weights, factor: int, stream=None) -> Dict[str, object]:
    """sum(obj * weights) / sum(weights) over factor x factor blocks of the last two axes
    (cubedsphere/coarsen.py:183-218) for each field, in the field's dtype (float64 kept),
    weights (tile, y, x) float32.  Fields are (tile, y, x) or (tile, z, y, x)."""
    _device.require_gpu()
    w = _device.to_device_f32(weights)
    if w.dim() != 3:
        raise ValueError(f"weights must be (tile, y, x), got shape {tuple(w.shape)}")
    nt, ny, nx = w.shape
    if ny % factor or nx % factor:
        raise ValueError(f"grid {ny}x{nx} is not divisible by the coarsening factor {factor}")
    out = {}
    groups = {}
    for name, x in fields.items():
        t = _dev(x)
        if t.dim() not in (3, 4) or t.shape[0] != nt or tuple(t.shape[-2:]) != (ny, nx):
            raise ValueError(f"{name} shape {tuple(t.shape)} does not match weights {tuple(w.shape)}")
        nz = 1 if t.dim() == 3 else t.shape[1]
        res = torch.empty(t.shape[:-2] + (ny // factor, nx // factor), dtype=t.dtype, device=t.device)
        out[name] = res
        groups.setdefault((t.dtype, nz), []).append((t, res))
    lib = _native.load()
    for (dt, nz), items in groups.items():
        fn = lib.fv3_weighted_block_average_f64 if dt == torch.float64 else lib.fv3_weighted_block_average
        for i in range(0, len(items), 16):
            chunk = items[i:i + 16]
            fp = (ctypes.c_void_p * len(chunk))(*[a.data_ptr() for a, _ in chunk])
            op = (ctypes.c_void_p * len(chunk))(*[r.data_ptr() for _, r in chunk])
            st = fn(fp, op, len(chunk), w.data_ptr(), nt, nz, ny, nx, int(factor),
                    _device.stream_handle(stream, [w] + [a for a, _ in chunk] + [r for _, r in chunk]))
            _native.check(st, "weighted_block_average")
    return out


def impose_hydrostatic_balance(temperature, sphum, delp, dz, phis, ptop: float = TOA_PRESSURE, stream=None):
    """_impose_hydrostatic_balance (coarsen_restarts.py:916-938) on (tile, z, y, x)
    coarse fields: returns (hydrostatic DZ, adjusted phis), float64."""
    _device.require_gpu()
    T, q = _device.to_device_f32(temperature), _device.to_device_f32(sphum)
    delp, dz, phis = _dev(delp, torch.float64), _dev(dz, torch.float64), _dev(phis, torch.float64)
    if T.dim() != 4 or not (T.shape == q.shape == delp.shape == dz.shape):
        raise ValueError("temperature, sphum, delp and DZ must share one (tile, z, y, x) shape")
    nt, km, ny, nx = T.shape
    if tuple(phis.shape) != (nt, ny, nx):
        raise ValueError(f"phis must be (tile, y, x) = {(nt, ny, nx)}, got {tuple(phis.shape)}")
    dz_out = torch.empty_like(dz)
    phis_out = torch.empty_like(phis)
    st = _native.load().fv3_hydrostatic_balance(T.data_ptr(), q.data_ptr(), delp.data_ptr(), dz.data_ptr(),
                                                 phis.data_ptr(), dz_out.data_ptr(), phis_out.data_ptr(), nt, km,
                                                 ny, nx, float(ptop),
                                                 _device.stream_handle(stream, [T, q, delp, dz, phis, dz_out, phis_out]))
    _native.check(st, "hydrostatic_balance")
    return dz_out, phis_out


def coarsen_restarts_on_pressure(coarsening_factor: int, grid_spec: Mapping[str, object],
                                 restarts: Mapping[str, Mapping[str, object]], coarsen_agrid_winds: bool = False,
                                 iv: int = 1, kord: int = 1, stream=None,
                                 exact: bool = False) -> Dict[str, Dict[str, object]]:
    """coarsen_restarts_on_pressure (coarsen_restarts.py:152-225) for fv_core.res,
    fv_tracer.res and (if given) fv_srf_wnd.res.  Returns {category: {name: tensor}}.
    ``exact`` selects the pressure remap's arithmetic (``coarsen.coarsen_on_pressure``)."""
    _device.require_gpu()
    if "sfc_data" in restarts:
        raise NotImplementedError("sfc_data ('complex' surface coarsening) is outside this build's scope; "
                                  "coarsen it with vcm and pass the other categories here")
    core, tracer = restarts["fv_core.res"], restarts["fv_tracer.res"]
    f = int(coarsening_factor)
    has_time = len(tuple(np.shape(core["delp"]) if not torch.is_tensor(core["delp"]) else core["delp"].shape)) == 5
    strip = (lambda a: a[:, 0]) if has_time else (lambda a: a)
    back = (lambda t: t.unsqueeze(1)) if has_time else (lambda t: t)
    masked = ["W", "T"]
    if coarsen_agrid_winds:
        if not ("ua" in core and "va" in core):
            raise ValueError("If 'coarsen_agrid_winds' is active, 'ua' and 'va' "
                             "must be present in the 'fv_core.res' restart files.")
        masked += ["ua", "va"]
    area = grid_spec["area"]
    delp = _dev(strip(core["delp"]))
    # one fused pass: masked core fields and every tracer share delp and area
    fused = {("c", n): strip(core[n]) for n in masked}
    # only the listed tracers are coarsened and returned, cld_amt first (xr.merge order of
    # _coarse_grain_fv_tracer_on_pressure, coarsen_restarts.py:859-887); a missing one is
    # the reference's KeyError on ds_regridded[...]
    tracer_names = FRACTION_TRACERS + NON_FRACTION_TRACERS
    missing = [n for n in tracer_names if n not in tracer]
    if missing:
        raise KeyError(f"fv_tracer.res lacks {missing}")
    fused.update({("t", n): strip(tracer[n]) for n in tracer_names})
    keys = list(fused)
    names = [f"{c}:{n}" for c, n in keys]
    res, delp_c = coarsen_on_pressure(delp, area, dict(zip(names, (fused[k] for k in keys))), f, iv, kord,
                                      stream=stream, coarse_delp_f64=True, exact=exact)
    out_core = {n: res[f"c:{n}"] for n in masked}
    out_tracer = {n: res[f"t:{n}"] for n in tracer_names}
    out_core["delp"] = delp_c
    out_core["u"] = coarsen_edges_on_pressure(delp, grid_spec["dx"], {"u": strip(core["u"])}, f, "x", iv, kord,
                                              stream=stream, exact=exact)["u"]
    out_core["v"] = coarsen_edges_on_pressure(delp, grid_spec["dy"], {"v": strip(core["v"])}, f, "y", iv, kord,
                                              stream=stream, exact=exact)["v"]
    plain = weighted_block_average({"phis": strip(core["phis"]), "DZ": strip(core["DZ"])}, area, f, stream)
    out_core["DZ"], out_core["phis"] = impose_hydrostatic_balance(out_core["T"], out_tracer["sphum"], delp_c,
                                                                  plain["DZ"], plain["phis"], stream=stream)
    result = {"fv_core.res": out_core, "fv_tracer.res": out_tracer}
    if "fv_srf_wnd.res" in restarts:
        srf = restarts["fv_srf_wnd.res"]
        result["fv_srf_wnd.res"] = weighted_block_average({n: strip(srf[n]) for n in ("u_srf", "v_srf")}, area, f,
                                                          stream)
    return {cat: {n: back(t) for n, t in d.items()} for cat, d in result.items()}
