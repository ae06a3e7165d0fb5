"""ORACLE (test infrastructure only): numpy restatement of the pressure-level
coarse-graining path of vcm.cubedsphere, with the reference's dtype flow.

Reference (paths under /root/reference/external/vcm/vcm):
* weighted_block_average     cubedsphere/coarsen.py:183-218  sum(obj*w)/sum(w) over f x f
                                                              (xarray coarsen().sum(): NaN-skipping)
* block_upsample_like        cubedsphere/coarsen.py:900-938 (+ _upsample_staggered_or_unstaggered :843-866)
* pressure_at_interface      calc/thermo/vertically_dependent.py:41-66  cumsum([300 Pa, delp])
* regrid_vertical            cubedsphere/regridz.py:164-279  -> mappm(p_in, f_in, p_out, 1, ncol, iv, kord, 0)
                             (f2py casts every argument to real*4; result float32)
* _mask_weights              cubedsphere/regridz.py:150-161  weights where phalf_c[1:] < phalf_f[-1]
* regrid_to_area_weighted_pressure + the masked weighted average of
  coarsen_restarts.py:_coarse_grain_fv_core_on_pressure (:411-516) and
  _coarse_grain_fv_tracer_on_pressure (:840-887)

Arrays are (tile, z, y, x) for 3-D fields and (tile, y, x) for area.
"""
import numpy as np

from .mappm import oracle_mappm

TOA_PRESSURE = 300.0  # vcm/calc/thermo/constants.py:17


def weighted_block_average(obj, weights, f):
    """sum(obj*weights)/sum(weights) over f x f blocks of the last two axes, in the
    arrays' own (numpy-promoted) dtype, NaN-skipping sums like xarray's coarsen().sum()."""
    num = obj * weights
    *lead, ny, nx = num.shape
    num = np.nansum(num.reshape(*lead, ny // f, f, nx // f, f), axis=(-3, -1))
    *wl, wy, wx = weights.shape
    den = np.nansum(weights.reshape(*wl, wy // f, f, wx // f, f), axis=(-3, -1))
    return num / den


def block_upsample(obj, f):
    return np.repeat(np.repeat(obj, f, axis=-2), f, axis=-1)


def pressure_at_interface(delp, axis=1, toa=TOA_PRESSURE):
    shape = list(delp.shape)
    shape[axis] = 1
    top = np.full(shape, toa, dtype=delp.dtype)
    return np.cumsum(np.concatenate([top, delp], axis=axis), axis=axis)


def regrid_vertical(p_in, f_in, p_out, iv=1, kord=1):
    """(tile, z, y, x) arrays; the f2py call sees (ncol, nz) float32."""
    nt, nzp, ny, nx = p_in.shape
    to_cols = lambda a: np.ascontiguousarray(a.transpose(1, 0, 2, 3).reshape(a.shape[1], -1), dtype=np.float32)
    q2 = oracle_mappm(to_cols(p_in), to_cols(f_in), to_cols(p_out), iv, kord)
    return q2.reshape(q2.shape[0], nt, ny, nx).transpose(1, 0, 2, 3)


def mask_weights(weights, phalf_coarse_on_fine, phalf_fine):
    """area (tile, y, x) -> (tile, z, y, x): weights where phalf_c[k+1] < phalf_f[-1]."""
    cond = phalf_coarse_on_fine[:, 1:] < phalf_fine[:, -1:]
    return np.where(cond, weights[:, None], np.zeros((), dtype=weights.dtype)).astype(weights.dtype)


def coarsen_on_pressure(delp, area, fields, factor, iv=1, kord=1):
    """Masked area-weighted pressure-level coarse-graining of ``fields`` (list of
    (tile, z, y, x)); returns (coarse fields, area-weighted coarse delp)."""
    delp_c = weighted_block_average(delp, area[:, None], factor)
    delp_c_on_f = block_upsample(delp_c, factor)
    phalf_c_on_f = pressure_at_interface(delp_c_on_f)
    phalf_f = pressure_at_interface(delp)
    masked = mask_weights(area, phalf_c_on_f, phalf_f)
    out = []
    for fld in fields:
        regridded = regrid_vertical(phalf_f, fld, phalf_c_on_f, iv, kord)
        out.append(weighted_block_average(regridded, masked, factor))
    return out, delp_c


def synth_uniform(lo, hi, shape, dtype):
    """external/synth Range.generate_array (synth/core.py:63-67): seed 0 per chunk."""
    np.random.seed(0)
    return np.random.uniform(low=lo, high=hi, size=shape).astype(dtype)
