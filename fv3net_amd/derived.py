"""fv3fit's DerivedModel and TransformedPredictor, mirrored over this package's registry,
with the vcm.DerivedMapping / vcm.DataTransform catalogue entries a dQ1/dQ2 model feeds
computed by HIP kernels (csrc/derived.hip).

Reference (paths under /root/reference/external):
* ``DerivedModel``         ("derived_model")            fv3fit/fv3fit/_shared/models.py:110-220
* ``TransformedPredictor`` ("output_transformed_model") fv3fit/fv3fit/_shared/models.py:279-337
* ``DerivedMapping``       vcm/vcm/derived_mapping.py:8-111 (registry, find_all_required_inputs),
                           entries :123-127, 264-410
* ``DataTransform`` / ``ChainedDataTransform``          vcm/vcm/data_transform.py:15-370

Every DerivedMapping entry of derived_mapping.py is computed on the device, the D-grid wind
rotation (dQu / dQv / eastward_wind / northward_wind, rotate.py:9-56 with coarsen.py:54-75's
edge centring, one fused kernel) and the solar zenith angle (_zenith_angle.py: the
per-time factors on the host, the per-point cosine on the device) included.  Every
DataTransform of the registry is mirrored.  Arithmetic keeps numpy's dtype flow
(bit-identical to oracle/derived.py; the zenith angle's sin / cos and the wind norm's
summation order to rounding); device tensors stay on the device, host arrays come back
as host arrays.
"""
import ctypes
import dataclasses
import os
from typing import Hashable, Iterable, List, Mapping, MutableMapping, Optional, Sequence

import numpy as np
import yaml

from . import _device, _native
from . import dataset as dsmod
from .predictor import Predictor, load, register
from .predictor import dump as dump_predictor

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

Z = "z"
DELP = "pressure_thickness_of_atmospheric_layer"
DSW_TOA = "total_sky_downward_shortwave_flux_at_top_of_atmosphere"
DSW_SFC = "total_sky_downward_shortwave_flux_at_surface"
DLW_SFC = "total_sky_downward_longwave_flux_at_surface"
ULW_SFC = "total_sky_upward_longwave_flux_at_surface"
ULW_TOA = "total_sky_upward_longwave_flux_at_top_of_atmosphere"
USW_SFC = "total_sky_upward_shortwave_flux_at_surface"
USW_TOA = "total_sky_upward_shortwave_flux_at_top_of_atmosphere"
COL_T_NUDGE = "storage_of_internal_energy_path_due_to_fine_res_temperature_nudging"
LHF = "latent_heat_flux"
SHF = "sensible_heat_flux"

# vcm/calc/thermo/constants.py, calc/clouds.py
_RDGAS = 287.05
_CP = 1004
_LV0 = 2.5e6
_H_LIQ, _H_VAP = 4185.5, 1846
_T_FREEZE = 273.15
_DEFAULT_SURFACE_TEMPERATURE = _T_FREEZE + 15
_KG_M2S_TO_MM_DAY = (1e3 * 86400) / 997.0
CLIMIT1, CLIMIT2 = 1.0e-3, 5.0e-2

EW_ADD, EW_SUB, EW_IADD, EW_SCALE, EW_DIV_SCALAR, EW_MSE, EW_TEMP_TEND = 1, 2, 3, 4, 5, 6, 7
EW_INCLOUD_TO_GRIDCELL, EW_GRIDCELL_TO_INCLOUD, EW_MUL, EW_ONE_MINUS_MUL, EW_ISCLOSE_ONEHOT = 8, 9, 10, 11, 12
EW_SIGN_PARALLEL, EW_PROJECT = 13, 14
COL_MASS_INTEGRAL, COL_TENDENCY_TO_FLUX, COL_IMPLIED_SURFACE_FLUX, COL_FLUX_TO_TENDENCY = 1, 2, 3, 4


def _lv(t: float) -> float:
    """latent_heat_vaporization of a Python float (local.py:25-28)."""
    return _LV0 + (_H_LIQ - _H_VAP) * (t - _T_FREEZE)


# ------------------------------------------------------------------ device operands
class _Ctx:
    """Host/device bookkeeping of one predict call: results come back as host arrays
    when every operand was a host array."""

    def __init__(self):
        self.host = True

    def dev(self, data):
        if torch.is_tensor(data):
            self.host = self.host and not data.is_cuda
            t = data if data.is_cuda else data.cuda()
        else:
            t = torch.from_numpy(np.ascontiguousarray(np.asarray(data))).cuda()
        if t.dtype not in (torch.float32, torch.float64):
            t = t.to(torch.float64)
        return t

    def back(self, t):
        return t.cpu().numpy() if self.host else t


def _f64(t) -> int:
    return int(t.dtype == torch.float64)


def _promote(*ts):
    return torch.float64 if any(t is not None and t.dtype == torch.float64 for t in ts) else torch.float32


def _aligned(da: "dsmod.DataArray", dims: Sequence[Hashable], ctx: _Ctx):
    """``da``'s data as a contiguous device tensor in ``dims`` order (xarray aligns binary
    operands by dim name)."""
    if set(da.dims) != set(dims):
        raise NotImplementedError(f"operands with dims {tuple(da.dims)} and {tuple(dims)}: broadcasting is not "
                                  "supported by the derived-variable kernels")
    if tuple(da.dims) != tuple(dims):
        da = da.transpose(*dims)
    return ctx.dev(da.data).contiguous()


def _ew(op, operands, out_dtype, params=(), shape=None):
    """fv3_derived_elementwise over contiguous tensors (None: zeros_like of a dtype given as
    ('zeros', dtype))."""
    ptrs, flags = [], []
    ref = None
    for o in operands:
        if isinstance(o, tuple):
            ptrs.append(None)
            flags.append(int(o[1] == torch.float64))
        else:
            ptrs.append(o.data_ptr())
            flags.append(_f64(o))
            ref = o if ref is None else ref
    shape = tuple(ref.shape) if shape is None else shape
    for o in operands:
        if not isinstance(o, tuple) and tuple(o.shape) != shape:
            raise ValueError(f"operand shape {tuple(o.shape)} != {shape}")
    out = torch.empty(shape, dtype=out_dtype, device=ref.device)
    n = len(operands)
    parr = (ctypes.c_double * max(1, len(params)))(*params)
    st = _native.load().fv3_derived_elementwise(
        op, (ctypes.c_void_p * n)(*ptrs), (ctypes.c_int * n)(*flags), n, out.data_ptr(), _f64(out), out.numel(),
        parr, len(params), _device.stream_handle(None))
    _native.check(st, "derived_elementwise")
    return out


def _field(t, ncol):
    if t is None:
        return _native.Field(None, 0, _native.layout(max(ncol, 1), max(ncol, 1), 0))
    if isinstance(t, tuple):  # ('zeros', dtype): zeros_like of that dtype
        return _native.Field(None, int(t[1] == torch.float64), _native.layout(max(ncol, 1), max(ncol, 1), 0))
    return _native.Field(t.data_ptr(), _f64(t), _native.layout(max(ncol, 1), max(ncol, 1), 0))


def _cols(op, inputs, outputs, ncol, nz, params):
    fin = (_native.Field * len(inputs))(*[_field(t, ncol) for t in inputs])
    fout = (_native.Field * len(outputs))(*[_field(t, ncol) for t in outputs])
    parr = (ctypes.c_double * max(1, len(params)))(*params)
    st = _native.load().fv3_derived_columns(op, fin, len(inputs), fout, len(outputs), ncol, nz, parr, len(params),
                                            _device.stream_handle(None))
    _native.check(st, "derived_columns")


def _zfirst(dims):
    if Z not in dims:
        raise ValueError(f"expected a vertical dimension {Z!r} in {tuple(dims)}")
    return (Z,) + tuple(d for d in dims if d != Z)


def _column_operands(x: "dsmod.DataArray", ctx: _Ctx):
    """([z][col] contiguous tensor of x, its dims in z-first order, horizontal dims, ncol,
    nz, pairwise): numpy sums a reduction over the contiguous last axis pairwise."""
    dims = _zfirst(x.dims)
    t = _aligned(x, dims, ctx)
    nz = int(t.shape[0])
    ncol = int(t.numel() // max(nz, 1))
    return t.reshape(nz, ncol), dims, dims[1:], ncol, nz, int(x.dims[-1] == Z and len(x.dims) > 1)


def _da(data, dims, like: Optional["dsmod.DataArray"] = None, attrs=None):
    coords = {d: like.coords[d] for d in dims if like is not None and d in like.coords}
    return dsmod.DataArray(data, dims, coords, attrs if attrs is not None else {})


# ------------------------------------------------------------- array-level operations
def mass_integrate(x: "dsmod.DataArray", delp: "dsmod.DataArray", scale: float = None, in_sign: float = 1.0,
                   negate: bool = False, ctx: _Ctx = None, attrs=None) -> "dsmod.DataArray":
    """[-] scale * (in_sign * x * delp / g).sum("z") (vertically_dependent.py:18-22,
    279-325): NaN-skipping, in numpy's order (sequential over a leading or middle z,
    pairwise when z is the contiguous last axis)."""
    ctx = ctx or _Ctx()
    _device.require_gpu()
    xt, dims, hdims, ncol, nz, pairwise = _column_operands(x, ctx)
    dt = _aligned(delp, dims, ctx).reshape(nz, ncol)
    out = torch.empty(ncol, dtype=_promote(xt, dt), device=xt.device)
    _cols(COL_MASS_INTEGRAL, [xt, dt], [out], ncol, nz,
          [in_sign, float("nan") if scale is None else float(scale), float(bool(negate)), float(pairwise)])
    shape = tuple(x.sizes[d] for d in hdims)
    return _da(ctx.back(out.reshape(shape)), hdims, x, attrs)


def _broadcast(das: Sequence, ctx: _Ctx):
    """xarray's broadcasting of elementwise operands: the result has the first operand's
    dims followed by every other operand's new dims; each operand becomes a contiguous
    device tensor of the result's shape."""
    dims: List[Hashable] = []
    sizes = {}
    for da in das:
        for d, n in da.sizes.items():
            if d not in dims:
                dims.append(d)
                sizes[d] = n
            elif sizes[d] != n:
                raise ValueError(f"conflicting sizes for dimension {d!r}: {n} vs {sizes[d]}")
    shape = tuple(sizes[d] for d in dims)
    out = []
    for da in das:
        t = ctx.dev(da.data)
        own = [d for d in dims if d in da.dims]
        t = t.permute(*[da.dims.index(d) for d in own]) if list(da.dims) != own else t
        t = t.reshape(tuple(sizes[d] if d in da.dims else 1 for d in dims)).expand(shape).contiguous()
        out.append(t)
    return out, tuple(dims), shape


def _ew_da(op, das: Sequence, params=(), ctx: _Ctx = None, out_dtype=None, attrs=None, zeros_like=None):
    """Elementwise op over DataArrays broadcast like xarray's binary operations.
    ``zeros_like``: index of an operand replaced by zeros_like(that DataArray)."""
    ctx = ctx or _Ctx()
    _device.require_gpu()
    ts, dims, shape = _broadcast(das, ctx)
    ops = [("zeros", _dtype_of(das[j])) if zeros_like is not None and j == zeros_like else t
           for j, t in enumerate(ts)]
    if out_dtype is None:
        out_dtype = _promote(*[o if not isinstance(o, tuple) else torch.empty(0, dtype=o[1]) for o in ops])
    out = _ew(op, ops, out_dtype, params, shape=shape)
    return _da(ctx.back(out), dims, das[0], attrs)


def _torch_dtype(data):
    if torch.is_tensor(data):
        return torch.float64 if data.dtype == torch.float64 else (torch.float32 if data.dtype == torch.float32
                                                                   else torch.float64)
    dt = np.asarray(data).dtype
    return torch.float32 if dt == np.float32 else torch.float64


def _dtype_of(da) -> "torch.dtype":
    return _torch_dtype(da.data)


# ------------------------------------------------------------------- DerivedMapping
class DerivedMapping(Mapping):
    """vcm.DerivedMapping (derived_mapping.py:8-111) over a Dataset of this package."""

    VARIABLES: MutableMapping[Hashable, object] = {}
    REQUIRED_INPUTS: MutableMapping[Hashable, Iterable[Hashable]] = {}
    USE_NONDERIVED_IF_EXISTS: List[Hashable] = []

    def __init__(self, mapper):
        self._mapper = mapper

    @classmethod
    def register(cls, name: Hashable, required_inputs: Iterable[Hashable] = None,
                 use_nonderived_if_exists: bool = False):
        def decorator(func):
            cls.VARIABLES[name] = func
            if required_inputs:
                cls.REQUIRED_INPUTS[name] = required_inputs
            if use_nonderived_if_exists is True:
                cls.USE_NONDERIVED_IF_EXISTS.append(name)
            return func

        return decorator

    def __getitem__(self, key: Hashable):
        if key in self.VARIABLES:
            if key in self.USE_NONDERIVED_IF_EXISTS:
                try:
                    return self._mapper[key]
                except KeyError:
                    return self.VARIABLES[key](self)
            return self.VARIABLES[key](self)
        return self._mapper[key]

    def keys(self):
        return set(self._mapper) | set(self.VARIABLES)

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def dataset(self, keys: Iterable[Hashable]) -> "dsmod.Dataset":
        return dsmod.Dataset({key: self[key] for key in keys})

    @classmethod
    def find_all_required_inputs(cls, derived_variables: Iterable[Hashable]) -> List[Hashable]:
        """derived_mapping.py:84-111 (set order as the reference's list(set(...)))."""
        def _recurse(vars_, deps):
            with_deps = [v for v in vars_ if v in cls.REQUIRED_INPUTS]
            if not with_deps:
                return
            new = []
            for v in with_deps:
                new += cls.REQUIRED_INPUTS[v]
            deps += new
            _recurse(new, deps)

        deps: List[Hashable] = []
        _recurse(derived_variables, deps)
        nonderived = list(set(d for d in deps if d not in cls.VARIABLES))
        maybe = list(set(d for d in deps if d in cls.USE_NONDERIVED_IF_EXISTS))
        return nonderived + maybe


# --------------------------------------------------- D-grid wind rotation (rotate.py)
EDGE_TO_CENTER_DIMS = {"x_interface": "x", "y_interface": "y"}  # rotate.py:7
ROTATION_COEFFS = ("eastward_wind_u_coeff", "eastward_wind_v_coeff", "northward_wind_u_coeff",
                   "northward_wind_v_coeff")


def _strided(t, dims, out_dims, rename=None):
    """fv3_strided of device tensor ``t`` (dims ``dims``) over a result with ``out_dims``:
    its element stride per result dim (a dim renamed by ``rename`` {own: result} maps to
    the result's), 0 where ``t`` lacks the dim."""
    rename = rename or {}
    own = {rename.get(d, d): k for k, d in enumerate(dims)}
    st = [int(t.stride(own[d])) if d in own else 0 for d in out_dims]
    return _native.Strided(t.data_ptr(), _f64(t), (ctypes.c_int64 * _native.MAX_DIMS)(*st))


def _staggered_dim(da):
    """coarsen.py:54-75's choice: the first of x_interface, y_interface that the array has."""
    for dim in EDGE_TO_CENTER_DIMS:
        if dim in da.dims:
            return dim
    raise ValueError("Variable to shift to center must be centered on one horizontal axis and edge-valued on the "
                     "other.")


def center_and_rotate_xy_winds(wind_rotation_matrix, x_component, y_component, ctx: _Ctx = None):
    """vcm/cubedsphere/rotate.py:9-56 (with coarsen.py:54-75's centering): D-grid x/y winds
    to A-grid (eastward, northward), one fused HIP kernel (fv3_center_rotate_winds):
    0.5 * (e[j + 1] + e[j]) on each component's staggered dim, then the 2x2 rotation by the
    grid's coefficients broadcast by dim name, in numpy's dtype flow.  Returns DataArrays
    in the centred x component's dims (northward in the centred y component's)."""
    ctx = ctx or _Ctx()
    _device.require_gpu()
    coeffs = [wind_rotation_matrix[name] for name in ROTATION_COEFFS]
    sx, sy = _staggered_dim(x_component), _staggered_dim(y_component)
    cx = tuple(EDGE_TO_CENTER_DIMS[d] if d == sx else d for d in x_component.dims)
    cy = tuple(EDGE_TO_CENTER_DIMS[d] if d == sy else d for d in y_component.dims)
    if len(set(cx)) != len(cx) or len(set(cy)) != len(cy):
        raise ValueError(f"centring {x_component.dims} / {y_component.dims} repeats a dimension")
    if set(cx) != set(cy):
        raise ValueError(f"centred winds have different dims: {cx} vs {cy}")
    sizes = {}
    for da, stag, cd in ((x_component, sx, cx), (y_component, sy, cy)):
        for d, c in zip(da.dims, cd):
            n = da.sizes[d] - 1 if d == stag else da.sizes[d]
            if sizes.setdefault(c, n) != n:
                raise ValueError(f"conflicting sizes for dimension {c!r}: {n} vs {sizes[c]}")
    for c in coeffs:
        for d, n in c.sizes.items():
            if d not in sizes:
                raise ValueError(f"rotation coefficient dims {c.dims} not among the winds' {cx}")
            if sizes[d] != n:
                raise ValueError(f"conflicting sizes for dimension {d!r}: {n} vs {sizes[d]}")
    if len(cx) > _native.MAX_DIMS:
        raise NotImplementedError(f"more than {_native.MAX_DIMS} dims")
    shape = tuple(sizes[d] for d in cx)
    xt, yt = ctx.dev(x_component.data), ctx.dev(y_component.data)
    ct = [ctx.dev(c.data) for c in coeffs]
    ops_x = _strided(xt, x_component.dims, cx, {sx: EDGE_TO_CENTER_DIMS[sx]})
    ops_y = _strided(yt, y_component.dims, cx, {sy: EDGE_TO_CENTER_DIMS[sy]})
    ops_c = (_native.Strided * 4)(*[_strided(t, c.dims, cx) for t, c in zip(ct, coeffs)])
    wx, wy = xt.dtype == torch.float64, yt.dtype == torch.float64
    f64 = [t.dtype == torch.float64 for t in ct]
    e_dt = torch.float64 if (f64[0] or wx or f64[1] or wy) else torch.float32
    n_dt = torch.float64 if (f64[2] or wx or f64[3] or wy) else torch.float32
    east = torch.empty(shape, dtype=e_dt, device=xt.device)
    north = torch.empty(shape, dtype=n_dt, device=xt.device)
    # every offset the kernel forms stays inside the operands (checked here: no launch
    # with a stride that could leave an array)
    for t, da, stag in ((xt, x_component, sx), (yt, y_component, sy)):
        if t.shape[da.dims.index(stag)] < 1 or tuple(t.shape) != tuple(da.shape):
            raise ValueError("wind data and dims disagree")
    shp = (ctypes.c_int64 * len(shape))(*shape)
    st = _native.load().fv3_center_rotate_winds(
        len(shape), shp, ops_x, int(xt.stride(x_component.dims.index(sx))), ops_y,
        int(yt.stride(y_component.dims.index(sy))), ops_c, east.data_ptr(), int(e_dt == torch.float64),
        north.data_ptr(), int(n_dt == torch.float64), _device.stream_handle(None))
    _native.check(st, "center_rotate_winds")
    # coords: the rotation matrix's x / y (rotate.py:27-30), the winds' other coords
    coords = {d: x_component.coords[d] for d in cx if d in x_component.coords and d not in ("x", "y")}
    for c in coeffs:
        for d in ("x", "y"):
            if d in c.coords:
                coords.setdefault(d, c.coords[d])
    e_da = _da(ctx.back(east), cx, None, {})
    e_da.coords.update({d: v for d, v in coords.items() if d in cx})
    n_dev = north if cy == cx else north.permute(*[cx.index(d) for d in cy]).contiguous()
    n_da = _da(ctx.back(n_dev), cy, None, {})
    n_da.coords.update({d: v for d, v in coords.items() if d in cy})
    return e_da, n_da


def _rotate(self, x, y):
    """derived_mapping.py:129-140."""
    wind_rotation_matrix = self.dataset(list(ROTATION_COEFFS))
    return center_and_rotate_xy_winds(wind_rotation_matrix, self[x], self[y])


@DerivedMapping.register("dQu", required_inputs=["dQxwind", "dQywind"], use_nonderived_if_exists=True)
def _dqu(self):
    return _rotate(self, "dQxwind", "dQywind")[0]


@DerivedMapping.register("dQv", required_inputs=["dQxwind", "dQywind"], use_nonderived_if_exists=True)
def _dqv(self):
    return _rotate(self, "dQxwind", "dQywind")[1]


@DerivedMapping.register("eastward_wind", use_nonderived_if_exists=True)
def _eastward_wind(self):
    return _rotate(self, "x_wind", "y_wind")[0]


@DerivedMapping.register("northward_wind", use_nonderived_if_exists=True)
def _northward_wind(self):
    return _rotate(self, "x_wind", "y_wind")[1]


@DerivedMapping.register("dQu_parallel_to_eastward_wind", required_inputs=["eastward_wind", "dQu"])
def _dqu_parallel(self):
    # sign(eastward_wind / dQu) * abs(dQu) (derived_mapping.py:163-167)
    return _ew_da(EW_SIGN_PARALLEL, [self["eastward_wind"], self["dQu"]])


@DerivedMapping.register("dQv_parallel_to_northward_wind", required_inputs=["northward_wind", "dQv"])
def _dqv_parallel(self):
    return _ew_da(EW_SIGN_PARALLEL, [self["northward_wind"], self["dQv"]])


@DerivedMapping.register("horizontal_wind_tendency_parallel_to_horizontal_wind",
                         required_inputs=["eastward_wind", "dQu", "northward_wind", "dQv"])
def _horizontal_parallel(self):
    """derived_mapping.py:177-187: (E dQu + N dQv) / np.linalg.norm((E, N)), the norm of
    BOTH whole arrays (one scalar: np.linalg.norm of the stacked pair, no axis)."""
    E, dqu, N, dqv = self["eastward_wind"], self["dQu"], self["northward_wind"], self["dQv"]
    ctx = _Ctx()
    norm, norm64 = wind_norm(E, N, ctx)
    return _ew_da(EW_PROJECT, [E, dqu, N, dqv], [norm, float(norm64)], ctx=ctx)


def wind_norm(E, N, ctx: _Ctx = None):
    """np.linalg.norm((E, N)) for two arrays of one shape: sqrt of the sum of squares of
    every element, in promote(E, N) (a float32 pair gives a float32 norm).  The squares are
    summed in float64 on the device (fv3_sum_squares, a fixed order): BLAS's dot order is
    its own, so the norm agrees with numpy's to rounding, not bitwise.  Returns (norm as a
    Python float, is_float64)."""
    ctx = ctx or _Ctx()
    _device.require_gpu()
    if tuple(E.shape) != tuple(N.shape):
        raise ValueError(f"setting an array element with a sequence: shapes {tuple(E.shape)} and {tuple(N.shape)}")
    et, nt = ctx.dev(E.data).contiguous(), ctx.dev(N.data).contiguous()
    w = et.dtype == torch.float64 or nt.dtype == torch.float64
    out = torch.empty(1, dtype=torch.float64, device=et.device)
    st = _native.load().fv3_sum_squares((ctypes.c_void_p * 2)(et.data_ptr(), nt.data_ptr()),
                                        (ctypes.c_int * 2)(_f64(et), _f64(nt)), 2, et.numel(), out.data_ptr(),
                                        _device.stream_handle(None))
    _native.check(st, "sum_squares")
    s = float(out.cpu().item())
    return (float(np.sqrt(np.float64(s))) if w else float(np.sqrt(np.float32(s)))), w


# ------------------------------------------------ solar zenith angle (_zenith_angle.py)
RAD_PER_DEG = np.pi / 180.0


def _days_from_2000(times) -> np.ndarray:
    """_zenith_angle.py:96-112 for an array of datetime.datetime or Julian-calendar times
    (cftime.DatetimeJulian; cftime is absent here: emulation.JulianTime): days since
    2000-01-01 12:00 of the same calendar, float64 (microseconds / 86400e6)."""
    import datetime

    from .emulation import JulianTime

    flat = np.asarray(times, dtype=object).ravel()
    date_type = type(flat[0])
    if date_type not in (datetime.datetime, JulianTime):
        raise ValueError(f"model_time has an invalid date type. It must be either datetime.datetime or "
                         f"cftime.DatetimeJulian. Got {date_type}.")
    epoch = date_type(2000, 1, 1, 12, 0)
    us = np.array([(t - epoch) // datetime.timedelta(microseconds=1) for t in flat], dtype=np.int64)
    return us.astype(np.float64) / np.float64(86400000000)


def solar_terms(times) -> np.ndarray:
    """The time-dependent factors of _zenith_angle.py:115-244 per time value, float64
    [4][n]: Greenwich mean sidereal time, the sun's right ascension, and the sine and
    cosine of its declination.  A few numbers per time value, on the host in numpy (the
    reference's own expressions); the per-point part runs in fv3_cos_zenith."""
    days = _days_from_2000(times)
    jc = days / 36525.0
    theta = 67310.54841 + jc * (876600 * 3600 + 8640184.812866 + jc * (0.093104 - jc * 6.2 * 10e-6))
    gmst = np.deg2rad(theta / 240.0) % (2 * np.pi)
    mean_anomaly = np.deg2rad(357.52910 + 35999.05030 * jc - 0.0001559 * jc * jc - 0.00000048 * jc * jc * jc)
    mean_longitude = np.deg2rad(280.46645 + 36000.76983 * jc + 0.0003032 * (jc ** 2))
    d_l = np.deg2rad((1.914600 - 0.004817 * jc - 0.000014 * (jc ** 2)) * np.sin(mean_anomaly)
                     + (0.019993 - 0.000101 * jc) * np.sin(2 * mean_anomaly) + 0.000290 * np.sin(3 * mean_anomaly))
    eclon = mean_longitude + d_l
    eps = np.deg2rad(23.0 + 26.0 / 60 + 21.406 / 3600.0
                     - (46.836769 * jc - 0.0001831 * (jc ** 2) + 0.00200340 * (jc ** 3) - 0.576e-6 * (jc ** 4)
                        - 4.34e-8 * (jc ** 5)) / 3600.0)
    x = np.cos(eclon)
    y = np.cos(eps) * np.sin(eclon)
    z = np.sin(eps) * np.sin(eclon)
    r = np.sqrt(1.0 - z * z)
    dec = np.arctan2(z, r)
    ra = 2 * np.arctan2(y, (x + r))
    return np.stack([gmst, ra, np.sin(dec), np.cos(dec)]).astype(np.float64)


def _is_rad(da) -> bool:
    return isinstance(da, dsmod.DataArray) and "rad" in str(da.attrs.get("units", "")).lower()


def cos_zenith_angle(time, lon, lat, ctx: _Ctx = None):
    """vcm.cos_zenith_angle (_zenith_angle.py:54-93): float64 cosine of the solar zenith
    angle at ``time`` (UTC: a datetime.datetime / Julian-calendar time, an array of them,
    or a DataArray of them) for ``lon`` / ``lat`` in degrees (DataArrays whose units name
    radians are converted, as _ensure_units_of_degrees).  DataArray inputs broadcast by
    dim name like xr.apply_ufunc (the result's dims: time's, then lon's, then lat's new
    ones) and give a DataArray named "cos_zenith_angle"; numpy inputs broadcast like
    numpy.  The time factors come from the host (solar_terms), each point from
    fv3_cos_zenith on the device."""
    ctx = ctx or _Ctx()
    _device.require_gpu()
    as_da = isinstance(lon, dsmod.DataArray)
    if as_da:
        tda = time if isinstance(time, dsmod.DataArray) else None
        parts = ([tda] if tda is not None else []) + [lon, lat]
        dims: List[Hashable] = []
        sizes = {}
        for da in parts:
            for d, n in da.sizes.items():
                if d not in dims:
                    dims.append(d)
                    sizes[d] = n
                elif sizes[d] != n:
                    raise ValueError(f"conflicting sizes for dimension {d!r}: {n} vs {sizes[d]}")
        shape = tuple(sizes[d] for d in dims)
        tvals = np.asarray(tda.values if tda is not None else time, dtype=object)
        tdims = tuple(tda.dims) if tda is not None else ()
        lt, at = ctx.dev(lon.data), ctx.dev(lat.data)
        lon_op, lat_op = _strided(lt, lon.dims, dims), _strided(at, lat.dims, dims)
        tcont = np.ascontiguousarray(tvals)
        tst = {d: tcont.strides[k] // tcont.itemsize for k, d in enumerate(tdims)}
        tstride = [int(tst.get(d, 0)) for d in dims]
    else:
        larr, aarr = np.asarray(lon), np.asarray(lat)
        if larr.dtype not in (np.float32, np.float64):
            larr = larr.astype(np.float64)
        if aarr.dtype not in (np.float32, np.float64):
            aarr = aarr.astype(np.float64)
        tvals = np.asarray(time, dtype=object)
        shape = np.broadcast_shapes(tvals.shape, larr.shape, aarr.shape)
        dims = list(range(len(shape))) or [0]
        shape = shape or (1,)

        def bstrides(a):
            a = np.ascontiguousarray(a)
            pad = len(shape) - a.ndim
            return [0 if k < pad or a.shape[k - pad] == 1 else a.strides[k - pad] // a.itemsize
                    for k in range(len(shape))], a

        ls, larr = bstrides(larr)
        as_, aarr = bstrides(aarr)
        tstride, tcont = bstrides(tvals)
        lt = torch.from_numpy(larr).cuda()
        at = torch.from_numpy(aarr).cuda()
        lon_op = _native.Strided(lt.data_ptr(), _f64(lt), (ctypes.c_int64 * _native.MAX_DIMS)(*ls))
        lat_op = _native.Strided(at.data_ptr(), _f64(at), (ctypes.c_int64 * _native.MAX_DIMS)(*as_))
    if len(shape) > _native.MAX_DIMS:
        raise NotImplementedError(f"more than {_native.MAX_DIMS} dims")
    terms = torch.from_numpy(np.ascontiguousarray(solar_terms(tcont))).cuda()
    nt = int(terms.shape[1])
    out = torch.empty(shape, dtype=torch.float64, device=lt.device)
    st = _native.load().fv3_cos_zenith(
        len(shape), (ctypes.c_int64 * len(shape))(*shape), lon_op, int(_is_rad(lon)), lat_op, int(_is_rad(lat)),
        (ctypes.c_int64 * len(shape))(*tstride), terms.data_ptr(), nt, out.data_ptr(), _device.stream_handle(None))
    _native.check(st, "cos_zenith")
    if not as_da:
        res = out.cpu().numpy().reshape(
            np.broadcast_shapes(np.asarray(time, dtype=object).shape, np.shape(lon), np.shape(lat)))
        return res[()]  # scalar inputs: a numpy float64 scalar, as _star_cos_zenith returns
    coords = {}
    for da in parts:
        for d, v in da.coords.items():
            coords.setdefault(d, v)
    return dsmod.DataArray(ctx.back(out), dims, coords, {"units": ""}, "cos_zenith_angle")


@DerivedMapping.register("cos_zenith_angle", required_inputs=["time", "lon", "lat"])
def _cos_zenith(self):
    return cos_zenith_angle(self["time"], self["lon"], self["lat"])


ALBEDO = "surface_diffused_shortwave_albedo"
DSW_OVERRIDE = "override_for_time_adjusted_total_sky_downward_shortwave_flux_at_surface"
SW_TRANSMISSIVITY = "shortwave_transmissivity_of_atmospheric_column"


@DerivedMapping.register("net_shortwave_sfc_flux_derived", required_inputs=[ALBEDO, DSW_OVERRIDE])
def _net_sw_derived(self):
    # (1 - albedo) * downward flux (derived_mapping.py:194-211)
    return _ew_da(EW_ONE_MINUS_MUL, [self[ALBEDO], self[DSW_OVERRIDE]])


@DerivedMapping.register("downward_shortwave_sfc_flux_via_transmissivity", required_inputs=[DSW_TOA, SW_TRANSMISSIVITY])
def _down_sw_transmissivity(self):
    return _ew_da(EW_MUL, [self[SW_TRANSMISSIVITY], self[DSW_TOA]])


@DerivedMapping.register("net_shortwave_sfc_flux_via_transmissivity",
                         required_inputs=[ALBEDO, "downward_shortwave_sfc_flux_via_transmissivity"])
def _net_sw_transmissivity(self):
    return _ew_da(EW_ONE_MINUS_MUL, [self[ALBEDO], self["downward_shortwave_sfc_flux_via_transmissivity"]])


def _one_hot(value):
    def f(self):
        # xr.where(vcm.xarray_utils.isclose(mask, value), 1.0, 0.0): float64
        return _ew_da(EW_ISCLOSE_ONEHOT, [self["land_sea_mask"]], [float(value), 1e-05, 1e-08],
                      out_dtype=torch.float64)
    return f


DerivedMapping.register("is_land", required_inputs=["land_sea_mask"])(_one_hot(1))
DerivedMapping.register("is_sea", required_inputs=["land_sea_mask"])(_one_hot(0))
DerivedMapping.register("is_sea_ice", required_inputs=["land_sea_mask"])(_one_hot(2))


@DerivedMapping.register("evaporation", required_inputs=[LHF])
def _evaporation(self):
    return latent_heat_flux_to_evaporation(self[LHF])


@DerivedMapping.register("Q1", required_inputs=["pQ1"], use_nonderived_if_exists=True)
def _q1(self):
    return _q_total(self, "1")


@DerivedMapping.register("Q2", required_inputs=["pQ2"], use_nonderived_if_exists=True)
def _q2(self):
    return _q_total(self, "2")


def _q_total(self, i):
    """derived_mapping.py:264-277: dQ + pQ (pQ from the data, else zeros_like(delp))."""
    if f"dQ{i}" not in self.keys():
        return self[f"pQ{i}"]
    dq = self[f"dQ{i}"]
    try:
        return _ew_da(EW_ADD, [dq, self._mapper[f"pQ{i}"]])
    except KeyError:  # pQ = xr.zeros_like(delp): dQ + 0 in promote(dQ, delp)
        return _ew_da(EW_ADD, [dq, self._mapper[DELP]], zeros_like=1)


@DerivedMapping.register("pQ1", required_inputs=[DELP], use_nonderived_if_exists=True)
def _pq1(self):
    return _zeros_like(self[DELP])


@DerivedMapping.register("pQ2", required_inputs=[DELP], use_nonderived_if_exists=True)
def _pq2(self):
    return _zeros_like(self[DELP])


def _zeros_like(da):
    data = torch.zeros_like(da.data) if torch.is_tensor(da.data) else np.zeros_like(np.asarray(da.data))
    return dsmod.DataArray(data, da.dims, da.coords, da.attrs)


@DerivedMapping.register("internal_energy", required_inputs=["air_temperature"])
def _internal_energy(self):
    return _ew_da(EW_SCALE, [self._mapper["air_temperature"]], [_CP - _RDGAS],
                  attrs={"long_name": "internal energy", "units": "J/kg"})


def _col_heating(self, name):
    return mass_integrate(self._mapper[name], self._mapper[DELP], scale=_CP - _RDGAS,
                          attrs={"long_name": "column integrated heating", "units": "W/m**2"})


def _col_moistening(self, name):
    # -minus_column_integrated_moistening: -(K * mass_integrate(dQ2 * -1, delp))
    return mass_integrate(self._mapper[name], self._mapper[DELP], scale=_KG_M2S_TO_MM_DAY, in_sign=-1.0, negate=True,
                          attrs={"long_name": "column integrated moistening", "units": "mm/day"})


@DerivedMapping.register("column_integrated_dQ1", required_inputs=["dQ1", DELP])
def _ci_dq1(self):
    return _col_heating(self, "dQ1")


@DerivedMapping.register("column_integrated_dQ2", required_inputs=["dQ2", DELP])
def _ci_dq2(self):
    return _col_moistening(self, "dQ2")


@DerivedMapping.register("column_integrated_Q1", required_inputs=["Q1", DELP])
def _ci_q1(self):
    return _col_heating(self, "Q1")


@DerivedMapping.register("column_integrated_Q2", required_inputs=["Q2", DELP])
def _ci_q2(self):
    return _col_moistening(self, "Q2")


@DerivedMapping.register("water_vapor_path", required_inputs=["specific_humidity", DELP],
                         use_nonderived_if_exists=True)
def _wvp(self):
    return mass_integrate(self._mapper["specific_humidity"], self._mapper[DELP],
                          attrs={"long_name": "column integrated water vapor", "units": "mm"})


@DerivedMapping.register("upward_heat_flux_at_surface", required_inputs=[USW_SFC, ULW_SFC, SHF])
def _upward_heat_flux(self):
    return _ew_da(EW_ADD, [self[USW_SFC], self[ULW_SFC], self[SHF]],
                  attrs={"long_name": "Upward heat (sensible+radiative) flux at surface", "units": "W/m**2"})


@DerivedMapping.register("incloud_water_mixing_ratio", required_inputs=["cloud_amount", "cloud_water_mixing_ratio"])
def _incloud_water(self):
    return gridcell_to_incloud_condensate(self["cloud_amount"], self["cloud_water_mixing_ratio"],
                                          attrs={"long_name": "in-cloud water mixing ratio", "units": "kg/kg"})


@DerivedMapping.register("incloud_ice_mixing_ratio", required_inputs=["cloud_amount", "cloud_ice_mixing_ratio"])
def _incloud_ice(self):
    return gridcell_to_incloud_condensate(self["cloud_amount"], self["cloud_ice_mixing_ratio"],
                                          attrs={"long_name": "in-cloud ice mixing ratio", "units": "kg/kg"})


def latent_heat_flux_to_evaporation(lhf, surface_temperature: float = _DEFAULT_SURFACE_TEMPERATURE, ctx=None):
    """local.py:69-82 (a Python-float surface temperature)."""
    return _ew_da(EW_DIV_SCALAR, [lhf], [_lv(surface_temperature)], ctx=ctx)


def gridcell_to_incloud_condensate(cf, condensate, climit1=CLIMIT1, climit2=CLIMIT2, attrs=None):
    return _ew_da(EW_GRIDCELL_TO_INCLOUD, [cf, condensate], [climit1, climit2], attrs=attrs)


def incloud_to_gridcell_condensate(cf, incloud, climit1=CLIMIT1, climit2=CLIMIT2, attrs=None):
    return _ew_da(EW_INCLOUD_TO_GRIDCELL, [cf, incloud], [climit1, climit2], attrs=attrs)


# ----------------------------------------------------------------- data transforms
def _tapered(src):
    def f(ds, cutoff: int, rate: float):
        from .composite import TaperConfig

        out = TaperConfig(cutoff=cutoff, rate=rate, taper_dim=Z).apply(ds[src])
        ds[f"tapered_{src}"] = out
        return ds
    return f


def _mse(ds, temperature_dependent=False):
    ops = [ds["Q1"], ds["Q2"]] + ([ds["air_temperature"]] if temperature_dependent else [])
    ds["Qm"] = _ew_da(EW_MSE, ops, attrs={"units": "W/kg", "long_name": "tendency of moist static energy"})
    return ds


def _q1_from_qm(ds, temperature_dependent=False):
    ops = [ds["Qm"], ds["Q2"]] + ([ds["air_temperature"]] if temperature_dependent else [])
    ds["Q1"] = _ew_da(EW_TEMP_TEND, ops, attrs={"units": "K/s", "long_name": "tendency of air temperature"})
    return ds


def _q_from_dq_pq(i):
    def f(ds):
        ds[f"Q{i}"] = _ew_da(EW_ADD, [ds[f"dQ{i}"], ds[f"pQ{i}"]])
        return ds
    return f


def _toa_net(ds, include_temperature_nudging):
    toa = _ew_da(EW_SUB, [ds[DSW_TOA], ds[USW_TOA], ds[ULW_TOA]])
    if include_temperature_nudging:  # toa_net_flux += nudging: in place, toa's dtype
        toa = _ew_da(EW_IADD, [toa, ds[COL_T_NUDGE]], out_dtype=_dtype_of(toa))
    return toa


def _surface_up(ds):
    return _ew_da(EW_ADD, [ds[LHF], ds[SHF], ds[USW_SFC], ds[ULW_SFC]])


def _tendency_to_flux(tendency, toa, surface_up, delp, rectify, toa_zeros_like=None):
    """flux_form.py:7-42 -> (interface-flux DataArray, downward surface flux)."""
    ctx = _Ctx()
    xt, dims, hdims, ncol, nz, _ = _column_operands(tendency, ctx)
    dt = _aligned(delp, dims, ctx).reshape(nz, ncol)
    up = _aligned(surface_up, hdims, ctx).reshape(ncol)
    tt = ("zeros", _dtype_of(toa_zeros_like)) if toa is None else _aligned(toa, hdims, ctx).reshape(ncol)
    pdt = _promote(xt, dt)
    flux = torch.empty((nz, ncol), dtype=pdt, device=xt.device)
    down = torch.empty(ncol, dtype=_promote(xt, dt, up), device=xt.device)
    _cols(COL_TENDENCY_TO_FLUX, [xt, dt, tt, up], [flux, down], ncol, nz, [float(bool(rectify))])
    hshape = tuple(tendency.sizes[d] for d in hdims)
    fshape = (nz,) + hshape
    # the result keeps the tendency's own dim order (z-first here, transposed back)
    return (_da(ctx.back(flux.reshape(fshape)), dims, tendency).transpose(*tendency.dims),
            _da(ctx.back(down.reshape(hshape)), hdims, tendency))


def _implied_surface_flux(tendency, toa, surface_up, delp, rectify, toa_zeros_like=None):
    """flux_form.py:45-73."""
    ctx = _Ctx()
    xt, dims, hdims, ncol, nz, pairwise = _column_operands(tendency, ctx)
    dt = _aligned(delp, dims, ctx).reshape(nz, ncol)
    up = _aligned(surface_up, hdims, ctx).reshape(ncol)
    if toa is None:
        tt, tdt = ("zeros", _dtype_of(toa_zeros_like)), _dtype_of(toa_zeros_like)
    else:
        tt = _aligned(toa, hdims, ctx).reshape(ncol)
        tdt = tt.dtype
    down = torch.empty(ncol, dtype=_promote(xt, dt, up, torch.empty(0, dtype=tdt)), device=xt.device)
    _cols(COL_IMPLIED_SURFACE_FLUX, [xt, dt, tt, up], [down], ncol, nz, [float(bool(rectify)), float(pairwise)])
    hshape = tuple(tendency.sizes[d] for d in hdims)
    return _da(ctx.back(down.reshape(hshape)), hdims, tendency)


def _flux_to_tendency(net_flux, surface_down, surface_up, delp):
    """flux_form.py:76-100."""
    ctx = _Ctx()
    ft, dims, hdims, ncol, nz, _ = _column_operands(net_flux, ctx)
    dt = _aligned(delp, dims, ctx).reshape(nz, ncol)
    dn = _aligned(surface_down, hdims, ctx).reshape(ncol)
    up = _aligned(surface_up, hdims, ctx).reshape(ncol)
    out = torch.empty((nz, ncol), dtype=_promote(ft, dn, up, dt), device=ft.device)
    _cols(COL_FLUX_TO_TENDENCY, [ft, dt, dn, up], [out], ncol, nz, [])
    out = _da(ctx.back(out.reshape((nz,) + tuple(net_flux.sizes[d] for d in hdims))), dims, net_flux)
    return out.transpose(*net_flux.dims)


def _qm_flux_from_qm(ds, rectify_downward_radiative_flux=True, include_temperature_nudging=True):
    flux, down = _tendency_to_flux(ds["Qm"], _toa_net(ds, include_temperature_nudging), _surface_up(ds), ds[DELP],
                                   rectify_downward_radiative_flux)
    down.attrs.update(units="W/m**2", long_name="Implied downward radiative flux from <Qm> budget closure")
    flux.attrs.update(units="W/m**2", long_name="Net flux of MSE")
    ds["Qm_flux"] = flux
    ds["implied_downward_radiative_flux_at_surface"] = down
    return ds


def _q2_flux_from_q2(ds, rectify_surface_precipitation_rate=True):
    flux, down = _tendency_to_flux(ds["Q2"], None, latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP],
                                   rectify_surface_precipitation_rate, toa_zeros_like=ds[LHF])
    down.attrs.update(units="kg/s/m**2", long_name="Implied surface precipitation rate computed as E-<Q2>")
    flux.attrs.update(units="kg/s/m**2", long_name="Net flux of moisture")
    ds["Q2_flux"] = flux
    ds["implied_surface_precipitation_rate"] = down
    return ds


def _qm_from_qm_flux(ds):
    qm = _flux_to_tendency(ds["Qm_flux"], ds["implied_downward_radiative_flux_at_surface"], _surface_up(ds), ds[DELP])
    qm.attrs.update(units="W/kg")
    ds["Qm"] = qm
    return ds


def _q2_from_q2_flux(ds):
    q2 = _flux_to_tendency(ds["Q2_flux"], ds["implied_surface_precipitation_rate"],
                           latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP])
    q2.attrs.update(units="kg/kg/s")
    ds["Q2"] = q2
    return ds


def _implied_radiative(ds, rectify=True, include_temperature_nudging=True):
    down = _implied_surface_flux(ds["Qm"], _toa_net(ds, include_temperature_nudging), _surface_up(ds), ds[DELP],
                                 rectify)
    down.attrs.update(units="W/m**2", long_name="Implied downward radiative flux from <Qm> budget closure")
    ds["implied_downward_radiative_flux_at_surface"] = down
    return ds


def _implied_precip(ds, rectify=True):
    down = _implied_surface_flux(ds["Q2"], None, latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP], rectify,
                                 toa_zeros_like=ds[LHF])
    down.attrs.update(units="kg/s/m**2", long_name="Implied surface precipitation rate computed as E-<Q2>")
    ds["implied_surface_precipitation_rate"] = down
    return ds


def _cloud_from_incloud(kind):
    def f(ds):
        out = incloud_to_gridcell_condensate(ds["cloud_amount"], ds[f"incloud_{kind}_mixing_ratio"])
        out.attrs.update(long_name=f"cloud {kind} mixing ratio", units="kg/kg")
        ds[f"cloud_{kind}_mixing_ratio"] = out
        return ds
    return f


_QM_FLUX_INPUTS = ["Qm", DELP, DLW_SFC, DSW_SFC, DSW_TOA, ULW_SFC, ULW_TOA, USW_SFC, USW_TOA, LHF, SHF, COL_T_NUDGE]


@dataclasses.dataclass
class _Entry:
    func: object
    inputs: Sequence[str]
    outputs: Sequence[str]


# data_transform.py:65-323, in registration order
DATA_TRANSFORM_REGISTRY: Mapping[str, _Entry] = {
    "tapered_dQ1": _Entry(_tapered("dQ1"), ["dQ1"], ["tapered_dQ1"]),
    "tapered_dQ2": _Entry(_tapered("dQ2"), ["dQ2"], ["tapered_dQ2"]),
    "Qm_from_Q1_Q2": _Entry(lambda ds: _mse(ds), ["Q1", "Q2"], ["Qm"]),
    "Q1_from_Qm_Q2": _Entry(lambda ds: _q1_from_qm(ds), ["Qm", "Q2"], ["Q1"]),
    "Qm_from_Q1_Q2_temperature_dependent": _Entry(lambda ds: _mse(ds, True), ["Q1", "Q2", "air_temperature"], ["Qm"]),
    "Q1_from_Qm_Q2_temperature_dependent": _Entry(lambda ds: _q1_from_qm(ds, True), ["Qm", "Q2", "air_temperature"],
                                                  ["Q1"]),
    "Q1_from_dQ1_pQ1": _Entry(_q_from_dq_pq("1"), ["dQ1", "pQ1"], ["Q1"]),
    "Q2_from_dQ2_pQ2": _Entry(_q_from_dq_pq("2"), ["dQ2", "pQ2"], ["Q2"]),
    "Qm_flux_from_Qm_tendency": _Entry(_qm_flux_from_qm, _QM_FLUX_INPUTS,
                                       ["Qm_flux", "implied_downward_radiative_flux_at_surface"]),
    "Q2_flux_from_Q2_tendency": _Entry(_q2_flux_from_q2, ["Q2", DELP, LHF],
                                       ["Q2_flux", "implied_surface_precipitation_rate"]),
    "Qm_tendency_from_Qm_flux": _Entry(_qm_from_qm_flux, ["Qm_flux", "implied_downward_radiative_flux_at_surface",
                                                          DELP, ULW_SFC, USW_SFC, LHF, SHF], ["Qm"]),
    "Q2_tendency_from_Q2_flux": _Entry(_q2_from_q2_flux, ["Q2_flux", "implied_surface_precipitation_rate", DELP,
                                                          LHF], ["Q2"]),
    "implied_downward_radiative_flux_at_surface": _Entry(_implied_radiative, _QM_FLUX_INPUTS,
                                                         ["implied_downward_radiative_flux_at_surface"]),
    "implied_surface_precipitation_rate": _Entry(_implied_precip, ["Q2", DELP, LHF],
                                                 ["implied_surface_precipitation_rate"]),
    "cloud_water_mixing_ratio_from_incloud": _Entry(_cloud_from_incloud("water"),
                                                    ["cloud_amount", "incloud_water_mixing_ratio"],
                                                    ["cloud_water_mixing_ratio"]),
    "cloud_ice_mixing_ratio_from_incloud": _Entry(_cloud_from_incloud("ice"), ["cloud_amount",
                                                                               "incloud_ice_mixing_ratio"],
                                                  ["cloud_ice_mixing_ratio"]),
}


@dataclasses.dataclass
class DataTransform:
    """data_transform.py:326-342."""
    name: str
    kwargs: dict = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        if self.name not in DATA_TRANSFORM_REGISTRY:
            raise ValueError(f"unknown DataTransform {self.name!r}")

    def apply(self, ds):
        return DATA_TRANSFORM_REGISTRY[self.name].func(ds, **self.kwargs)

    @property
    def input_variables(self) -> Sequence[str]:
        return DATA_TRANSFORM_REGISTRY[self.name].inputs

    @property
    def output_variables(self) -> Sequence[str]:
        return DATA_TRANSFORM_REGISTRY[self.name].outputs


@dataclasses.dataclass
class ChainedDataTransform:
    """data_transform.py:345-370."""
    transforms: Sequence[DataTransform]

    def apply(self, ds):
        for transform in self.transforms:
            ds = transform.apply(ds)
        return ds

    @property
    def input_variables(self) -> Sequence[str]:
        inputs = set()
        for transform in self.transforms[::-1]:
            inputs.update(transform.input_variables)
            for output in transform.output_variables:
                inputs.discard(output)
        return sorted(inputs)

    @property
    def output_variables(self) -> Sequence[str]:
        outputs = set()
        for transform in self.transforms:
            outputs.update(transform.output_variables)
        return sorted(outputs)


# ------------------------------------------------------------------------ composites
def _merge(datasets, override=False):
    """xr.merge (compat "no_conflicts"; "override": the first one wins)."""
    from .stepper import merge

    if not override:
        return merge(datasets)
    out = dsmod.Dataset()
    for ds in datasets:
        for name in ds:
            if name not in out:
                da = ds[name]
                out[name] = dsmod.DataArray(da.data, da.dims, da.coords, da.attrs)
    return out


@register("derived_model")
class DerivedModel(Predictor):
    """models.py:110-220: the base model's prediction plus derived variables of it."""

    _CONFIG_FILENAME = "derived_model.yaml"
    _BASE_MODEL_SUBDIR = "base_model_data"

    def __init__(self, model: Predictor, derived_output_variables: Sequence[Hashable]):
        if isinstance(model, DerivedModel):  # combine instead of wrapping twice
            self.base_model: Predictor = model.base_model
            self._derived_output_variables = list(model._derived_output_variables) + list(derived_output_variables)
        else:
            self.base_model = model
            self._derived_output_variables = list(derived_output_variables)
        self._additional_input_variables = self.get_additional_inputs()
        full_inputs = sorted(set(list(model.input_variables) + list(self._additional_input_variables)))
        full_outputs = sorted(set(list(model.output_variables) + list(derived_output_variables)))
        self._check_derived_predictions_supported()
        super().__init__(full_inputs, full_outputs)

    def get_additional_inputs(self):
        deps = DerivedMapping.find_all_required_inputs(self._derived_output_variables)
        return [i for i in deps if i not in self.base_model.output_variables]

    def predict(self, X):
        self._check_additional_inputs_present(X)
        base_prediction = self.base_model.predict(X)
        required = dsmod.Dataset({k: X[k] for k in self._additional_input_variables})
        mapping = DerivedMapping(_merge([required, base_prediction]))
        derived_prediction = mapping.dataset(self._derived_output_variables)
        return _merge([base_prediction, derived_prediction])

    def dump(self, path: str):
        base_model_path = os.path.join(path, self._BASE_MODEL_SUBDIR)
        options = {"derived_output_variables": list(self._derived_output_variables), "model": base_model_path}
        dump_predictor(self.base_model, base_model_path)
        with open(os.path.join(path, self._CONFIG_FILENAME), "w") as f:
            yaml.safe_dump(options, f)

    @classmethod
    def load(cls, path: str) -> "DerivedModel":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        return cls(load(config["model"]), config["derived_output_variables"])

    def _check_additional_inputs_present(self, X):
        missing = np.setdiff1d(self._additional_input_variables, list(X.data_vars))
        if len(missing) > 0:
            raise KeyError(f"Missing additional inputs {missing} in input dataset needed to compute derived "
                           "prediction variables. Make sure these are present in the data and included in the "
                           "DerivedModel config under additional_input_variables.")

    def _check_derived_predictions_supported(self):
        invalid = np.setdiff1d(self._derived_output_variables, list(DerivedMapping.VARIABLES))
        if len(invalid) > 0:
            raise ValueError(f"Invalid variables {invalid} provided in init arg derived_output_variables. "
                             "Variables in this arg must be available as derived variables in vcm.DerivedMapping.")


@register("output_transformed_model")
class TransformedPredictor(Predictor):
    """models.py:279-337: the base model's prediction plus data transforms of it."""

    _CONFIG_FILENAME = "output_transformed_model.yaml"
    _BASE_MODEL_SUBDIR = "base_model_data"

    def __init__(self, base_model: Predictor, transforms: Sequence[DataTransform]):
        self.base_model = base_model
        self.transforms = transforms
        self.output_transform = ChainedDataTransform(self.transforms)
        inputs = set(base_model.input_variables) | set(self.output_transform.input_variables)
        outputs = set(base_model.output_variables) | set(self.output_transform.output_variables)
        for name in set(base_model.output_variables):
            inputs.discard(name)
        super().__init__(sorted(inputs), sorted(outputs))

    def predict(self, X):
        prediction = self.base_model.predict(X)
        transform_inputs = _merge([prediction, X], override=True)  # xr.merge(compat="override")
        transformed = self.output_transform.apply(transform_inputs)
        outputs = dsmod.Dataset({k: transformed[k] for k in self.output_transform.output_variables})
        return _merge([prediction, outputs])

    def dump(self, path: str):
        base_model_path = os.path.join(path, self._BASE_MODEL_SUBDIR)
        options = {"base_model": base_model_path,
                   "transforms": [dataclasses.asdict(x) for x in self.transforms]}
        dump_predictor(self.base_model, base_model_path)
        with open(os.path.join(path, self._CONFIG_FILENAME), "w") as f:
            yaml.safe_dump(options, f)

    @classmethod
    def load(cls, path: str) -> "TransformedPredictor":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        base_model = load(os.path.join(path, cls._BASE_MODEL_SUBDIR))
        transforms = [DataTransform(x["name"], dict(x.get("kwargs") or {})) for x in config["transforms"]]
        return cls(base_model, transforms)
