"""ORACLE (test infrastructure only): numpy restatement of vertical interpolation to
new levels.

Reference (paths under /root/reference):
* interpolate_2d          external/mappm/mappm/interpolate_2d.f90:1-27 (real*8; f2py
                          casts every argument to float64), called as
                          mappm.interpolate_2d(xp, x, y, fill_value=np.nan) by
                          external/vcm/vcm/interpolate.py:176-180 with rows = columns
* metpy_interpolate_1d    metpy.interpolate.interpolate_1d (MetPy is not vendored and not
                          installed here; its published algorithm: argsort the column
                          coordinate, searchsorted(..., 'left'), linear interpolation
                          var[below] + (var[above] - var[below]) * ((x - xp[below]) /
                          (xp[above] - xp[below])), fill outside) as called by
                          vcm/interpolate.py:148-173.  Pinned only by the reference's
                          KATs in external/vcm/tests/test_interpolate.py:73-107, 135-147.
* pressure_at_midpoint_log  external/vcm/vcm/calc/thermo/vertically_dependent.py:153-178
"""
import numpy as np

TOA_PRESSURE = 300.0


def interpolate_2d(xp, x, y, fill_value=np.nan):
    """(m, n_out) from xp (m, n_out), x and y (m, n_in), in float64.  The Fortran loops
    over every interval with no early exit: later matches overwrite earlier ones."""
    xp, x, y = (np.asarray(a, dtype=np.float64) for a in (xp, x, y))
    m, n_in = x.shape
    out = np.full(xp.shape, fill_value, dtype=np.float64)
    for k in range(n_in - 1):
        x0, x1 = x[:, k:k + 1], x[:, k + 1:k + 2]
        y0, y1 = y[:, k:k + 1], y[:, k + 1:k + 2]
        inside = (x0 <= xp) & (xp < x1)
        with np.errstate(divide="ignore", invalid="ignore"):
            w = (xp - x0) / (x1 - x0)
            lin = y0 * (1 - w) + y1 * w
        out = np.where(inside, lin, np.where(x0 == xp, y0, np.where(x1 == xp, y1, out)))
    return out


def metpy_interpolate_1d(levels, xp, var, axis=0, fill_value=np.nan):
    """metpy.interpolate.interpolate_1d(levels, xp, var, axis=axis) for 1-D levels."""
    levels = np.asanyarray(levels).reshape(-1)
    xp = np.asarray(xp)
    var = np.asarray(var)
    xp = np.moveaxis(xp, axis, -1)
    var = np.moveaxis(var, axis, -1)
    sort_args = np.argsort(xp, axis=-1, kind="stable")
    xp = np.take_along_axis(xp, sort_args, -1)
    var = np.take_along_axis(var, sort_args, -1)
    sort_x = np.argsort(levels, kind="stable")
    x_array = levels[sort_x]
    n = xp.shape[-1]
    minv = np.stack([np.searchsorted(row, x_array) for row in xp.reshape(-1, n)]).reshape(xp.shape[:-1] + (-1,))
    minv2 = minv.copy()
    minv2[minv == n] = n - 1
    minv2[minv == 0] = 1
    above = minv2
    below = minv2 - 1
    xb = np.take_along_axis(xp, below, -1)
    xa = np.take_along_axis(xp, above, -1)
    vb = np.take_along_axis(var, below, -1)
    va = np.take_along_axis(var, above, -1)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = vb + (va - vb) * ((x_array - xb) / (xa - xb))
    out[minv == n] = fill_value
    out[x_array < xb] = fill_value
    if levels[0] > levels[-1]:
        out = out[..., ::-1]
    return np.moveaxis(out, -1, axis)


def pressure_at_midpoint_log(delp, axis=0, toa=TOA_PRESSURE):
    delp = np.moveaxis(np.asarray(delp), axis, 0)
    top = np.full((1,) + delp.shape[1:], toa, dtype=delp.dtype)
    pi = np.cumsum(np.concatenate([top, delp], axis=0), axis=0)
    dlogp = np.diff(np.log(pi), axis=0)
    return np.moveaxis(delp / dlogp, 0, axis)
