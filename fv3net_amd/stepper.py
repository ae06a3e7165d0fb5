"""The ML stepper around the predictor: adapters, limiter, diagnostics and tendency
application.

Mirrors (paths under /root/reference/workflows/prognostic_c48_run/runtime):
* ``RenamingAdapter`` / ``MultiModelAdapter`` / ``open_model`` / ``predict`` /
  ``MachineLearningConfig``                        steppers/machine_learning.py:24-211
* ``PureMLStepper.__call__`` / ``get_diagnostics``  steppers/machine_learning.py:214-315
* the tendency / state-update split                names.py:31-65
* compute_diagnostics + compute_ml_momentum_diagnostics  diagnostics/compute.py:77-161
* the loop's fillna / add_tendency / precipitation_sum   loop.py:103-145, 202-219, 604-628
* the per-step global metrics                      main.py:55-60, metrics.py:18-55

Every arithmetic stage runs in HIP: the dQ1/dQ2 limiter + diagnostics + apply in one
fused kernel (``fv3_ml_epilogue_ex``, csrc/stepper.hip), the other tendencies (dQu, dQv,
dQp) in one column pass each (``fv3_tendency_columns``).  State variables are device
tensors (float64 like the FV3 state, or float32) or DataArrays over them; the model's
tendencies are float32 (Keras output).
"""
import dataclasses
from typing import Dict, Hashable, Iterable, Mapping, Optional, Sequence, Set, Tuple

from . import _device, _native
from . import dataset as dsmod

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

# names.py
TEMP = "air_temperature"
SPHUM = "specific_humidity"
DELP = "pressure_thickness_of_atmospheric_layer"
TOTAL_PRECIP = "total_precipitation"
TOTAL_PRECIP_RATE = "total_precipitation_rate"
EASTWARD_WIND_TENDENCY = "dQu"
NORTHWARD_WIND_TENDENCY = "dQv"
TENDENCY_TO_STATE_NAME = {"dQ1": TEMP, "dQ2": SPHUM, "dQu": "eastward_wind", "dQv": "northward_wind",
                          "dQx_wind": "x_wind", "dQy_wind": "y_wind", "dQp": DELP}
A_GRID_WIND_TENDENCIES = {EASTWARD_WIND_TENDENCY, NORTHWARD_WIND_TENDENCY}
TENDENCY_NAMES = set(TENDENCY_TO_STATE_NAME) | A_GRID_WIND_TENDENCIES

COLUMN_DIAGNOSTICS = (
    "column_integrated_dQ1_change_non_neg_sphum_constraint",
    "column_integrated_dQ2_change_non_neg_sphum_constraint",
    "net_moistening_due_to_{label}",
    "column_heating_due_to_{label}",
    "dQ1_filled_frac",
    "dQ2_filled_frac",
    TOTAL_PRECIP,
)


def is_state_update_variable(key, state) -> bool:
    """names.py:54-61."""
    return (key in state.keys() and key not in TENDENCY_NAMES) or key == TOTAL_PRECIP_RATE


def is_tendency_variable(key) -> bool:
    """names.py:64-65."""
    return key in TENDENCY_NAMES


# ------------------------------------------------------------------------ kernels
def _epilogue_setup(dq1, dq2, sphum, delp, temperature, dt, physics_precip, mse_conserving, hydrostatic, label,
                    in_place, level_axis, has_dq1, has_dq2, column=None):
    """Validate and marshal one fv3_ml_epilogue_ex call: (args without the stream,
    tensors the launch touches, the output dict).  ``column``: a [7, ncol] buffer of the
    state dtype for the column diagnostics (allocated here when None); its last row may
    be ``physics_precip`` itself (the kernel reads a column's precipitation before
    writing the new total to the same element)."""
    _device.require_gpu()
    state_dtype = sphum.dtype if isinstance(sphum, torch.Tensor) else torch.float64
    if state_dtype not in (torch.float32, torch.float64):
        raise ValueError("state arrays must be float32 or float64")
    dev = torch.device("cuda", torch.cuda.current_device())

    def st(x):
        t = torch.as_tensor(x).to(device=dev, dtype=state_dtype)
        return t if t.is_contiguous() else t.contiguous()

    sphum_in, temperature_in = sphum, temperature
    sphum, delp, temperature = st(sphum), st(delp), st(temperature)
    if in_place and (sphum is not sphum_in or temperature is not temperature_in):
        # the kernel would update a copy and leave the caller's state unchanged
        raise ValueError("ml_epilogue(in_place=True) needs the specific humidity and air temperature as "
                         "contiguous CUDA tensors of one dtype (float32 or float64)")
    dq1 = _device.to_device_f32(dq1)
    dq2 = _device.to_device_f32(dq2)
    for name, t in (("dQ1", dq1), ("dQ2", dq2), (DELP, delp), (TEMP, temperature)):
        if tuple(t.shape) != tuple(sphum.shape):
            raise ValueError(f"{name} shape {tuple(t.shape)} != specific humidity shape {tuple(sphum.shape)}")
    lay, ncol, nz = _device.level_layout(sphum, level_axis)  # e.g. (z, y, x) or (tile, z, y, x)
    col_shape = tuple(s for i, s in enumerate(sphum.shape) if i != level_axis)
    out = {
        "dQ1": torch.empty_like(sphum),
        "dQ2": torch.empty_like(sphum),
        "specific_humidity_limiter_active": torch.empty(sphum.shape, dtype=torch.uint8, device=dev),
        TEMP: temperature if in_place else torch.empty_like(temperature),
        SPHUM: sphum if in_place else torch.empty_like(sphum),
    }
    if column is None:
        column = torch.empty((7, ncol), dtype=state_dtype, device=dev)
    elif not (column.dtype == state_dtype and tuple(column.shape) == (7, ncol) and column.is_contiguous()
              and column.device == dev):
        raise ValueError(f"column must be a contiguous [7, {ncol}] {state_dtype} CUDA tensor")
    precip = None
    if physics_precip is not None:
        precip = st(physics_precip).reshape(-1)
        if precip.numel() != ncol:
            raise ValueError("physics precipitation must have one value per column")
    io = _native.EpilogueIO(dq1.data_ptr(), dq2.data_ptr(), sphum.data_ptr(), delp.data_ptr(),
                            temperature.data_ptr(), precip.data_ptr() if precip is not None else None,
                            out["dQ1"].data_ptr(), out["dQ2"].data_ptr(),
                            out["specific_humidity_limiter_active"].data_ptr(), out[TEMP].data_ptr(),
                            out[SPHUM].data_ptr(), column.data_ptr(), ncol)
    flags = (_native.EPI_HAS_DQ1 if has_dq1 else 0) | (_native.EPI_HAS_DQ2 if has_dq2 else 0)
    args = (ctypes_byref(io), lay, ncol, nz, int(state_dtype == torch.float64), float(dt), int(bool(mse_conserving)),
            int(bool(hydrostatic)), flags)
    keep = [dq1, dq2, sphum, delp, temperature, precip, column] + list(out.values())
    for i, name in enumerate(COLUMN_DIAGNOSTICS):
        if name == TOTAL_PRECIP and precip is None:
            continue
        out[name.format(label=label)] = column[i].reshape(col_shape)
    return (io, args), keep, out


def ml_epilogue(dq1, dq2, sphum, delp, temperature, dt: float, physics_precip=None,
                mse_conserving: bool = True, hydrostatic: bool = False, label: str = "machine_learning",
                in_place: bool = False, level_axis: int = 0, stream=None, has_dq1: bool = True,
                has_dq2: bool = True) -> Dict[str, object]:
    """Limiter + diagnostics + apply for one (dQ1, dQ2) prediction, one kernel.

    ``level_axis`` is the vertical axis of every 3-D array (axes before it are
    blocks such as tiles).  Returns device tensors: limited ``dQ1``/``dQ2`` (pre-fillna, as the stepper
    returns them), ``specific_humidity_limiter_active`` (uint8), the updated
    ``air_temperature``/``specific_humidity`` (written into the inputs when
    ``in_place``), the column diagnostics of COLUMN_DIAGNOSTICS and, with
    ``physics_precip``, the new ``total_precipitation``.  ``has_dq1``/``has_dq2`` False:
    the model lacks that tendency, pass zeros (machine_learning.py:258-259); its state
    variable is left as it is and its column diagnostic is zero.
    """
    (_, args), keep, out = _epilogue_setup(dq1, dq2, sphum, delp, temperature, dt, physics_precip, mse_conserving,
                                           hydrostatic, label, in_place, level_axis, has_dq1, has_dq2)
    st_ = _native.load().fv3_ml_epilogue_ex(*args, _device.stream_handle(stream, keep))
    _native.check(st_, "ml_epilogue")
    return out


class BoundEpilogue:
    """``ml_epilogue`` validated and marshalled once over fixed device buffers, then one
    C-ABI call per timestep (the prognostic loop applies the same state buffers every
    step; the per-call Python of ``ml_epilogue`` costs more than the kernel on one rank's
    band).  ``column``: as ``_epilogue_setup``; passing a buffer whose last row is the
    state's precipitation accumulates the total in place.  Calling returns the same
    output dict every time (its tensors are rewritten)."""

    def __init__(self, dq1, dq2, sphum, delp, temperature, dt: float, physics_precip=None,
                 mse_conserving: bool = True, hydrostatic: bool = False, label: str = "machine_learning",
                 in_place: bool = True, level_axis: int = 0, has_dq1: bool = True, has_dq2: bool = True,
                 column=None):
        (self._io, self._args), self._keep, self.out = _epilogue_setup(
            dq1, dq2, sphum, delp, temperature, dt, physics_precip, mse_conserving, hydrostatic, label, in_place,
            level_axis, has_dq1, has_dq2, column)
        self._fn = _native.load().fv3_ml_epilogue_ex

    def __call__(self, stream=None) -> Dict[str, object]:
        """``stream``: a torch stream, a raw hipStream_t handle (int), or None (current)."""
        h = stream if isinstance(stream, int) else _device.stream_handle(stream, self._keep)
        st_ = self._fn(*self._args, h)
        if st_:
            _native.check(st_, "ml_epilogue")
        return self.out


def tendency_columns(tendency, delp, dt: float, mode: str, level_axis: int = 0, stream=None) -> Dict[str, object]:
    """One column pass over a non-(dQ1, dQ2) tendency (csrc/stepper.hip
    ``fv3_tendency_columns``).  ``mode`` "wind" (dQu / dQv): ``integral`` =
    mass_integrate(dQ, delp) (compute.py:145-146), ``filled`` = fillna(dQ) as float64
    (loop.py:126-145), ``filled_frac``.  ``mode`` "mass" (dQp): ``integral`` =
    mass_integrate(ones_like(dQp), dQp) (float32, compute.py:107-115), ``state`` = delp +
    fillna(dQp) dt (add_tendency), ``filled_frac``."""
    _device.require_gpu()
    state_dtype = delp.dtype if isinstance(delp, torch.Tensor) else torch.float64
    dev = torch.device("cuda", torch.cuda.current_device())
    delp = torch.as_tensor(delp).to(device=dev, dtype=state_dtype).contiguous()
    t = _device.to_device_f32(tendency)
    if tuple(t.shape) != tuple(delp.shape):
        raise ValueError(f"tendency shape {tuple(t.shape)} != delp shape {tuple(delp.shape)}")
    lay, ncol, nz = _device.level_layout(delp, level_axis)
    col_shape = tuple(s for i, s in enumerate(delp.shape) if i != level_axis)
    out = {"filled_frac": torch.empty(ncol, dtype=state_dtype, device=dev)}
    if mode == "wind":
        m = _native.TEND_WIND
        out["integral"] = torch.empty(ncol, dtype=state_dtype, device=dev)
        out["filled"] = torch.empty(delp.shape, dtype=torch.float64, device=dev)
        filled, state_out = out["filled"].data_ptr(), None
    elif mode == "mass":
        m = _native.TEND_MASS
        out["integral"] = torch.empty(ncol, dtype=torch.float32, device=dev)
        out["state"] = torch.empty_like(delp)
        filled, state_out = None, out["state"].data_ptr()
    else:
        raise ValueError(f"mode must be 'wind' or 'mass', got {mode!r}")
    st_ = _native.load().fv3_tendency_columns(t.data_ptr(), delp.data_ptr(), filled, state_out,
                                              out["integral"].data_ptr(), out["filled_frac"].data_ptr(), lay, ncol,
                                              nz, int(state_dtype == torch.float64), m, float(dt),
                                              _device.stream_handle(stream, [t, delp] + list(out.values())))
    _native.check(st_, "tendency_columns")
    out["integral"] = out["integral"].reshape(col_shape)
    out["filled_frac"] = out["filled_frac"].reshape(col_shape)
    return out


def ctypes_byref(obj):
    import ctypes

    return ctypes.byref(obj)


# ----------------------------------------------------------------------- adapters
def _invert_dict(d: Mapping) -> Mapping:
    return dict(zip(d.values(), d.keys()))


def _rename(ds, rename: Mapping):
    """RenamingAdapter._rename (machine_learning.py:123-131): dims, then data vars."""
    if dsmod.is_xarray(ds):
        dims = {k: rename[k] for k in set(ds.dims) & set(rename)}
        redimed = ds.rename_dims(dims)
        names = {k: rename[k] for k in set(ds.data_vars) & set(rename)}
        return redimed.rename(names)
    out = dsmod.Dataset(attrs=ds.attrs)
    for name in ds:
        da = ds[name]
        dims = tuple(rename.get(d, d) for d in da.dims)
        coords = {rename.get(k, k): v for k, v in da.coords.items()}
        out[rename.get(name, name)] = dsmod.DataArray(da.data, dims, coords, da.attrs)
    return out


class RenamingAdapter:
    """machine_learning.py:106-147: rename the model's inputs and outputs."""

    def __init__(self, model, rename_in: Mapping, rename_out: Optional[Mapping] = None):
        self.model = model
        self.rename_in = rename_in
        self.rename_out = {} if rename_out is None else rename_out

    def _rename_inputs(self, ds):
        return _rename(ds, self.rename_in)

    def _rename_outputs(self, ds):
        return _rename(ds, _invert_dict(self.rename_out))

    @property
    def input_variables(self) -> Set[str]:
        invert_rename_in = _invert_dict(self.rename_in)
        return {invert_rename_in.get(var, var) for var in self.model.input_variables}

    def predict(self, arg):
        return self._rename_outputs(self.model.predict(self._rename_inputs(arg)))


def _same(a, b) -> bool:
    if torch is not None and torch.is_tensor(a) and torch.is_tensor(b):
        return a.shape == b.shape and bool(torch.equal(a, b))
    import numpy as np

    return np.array_equal(dsmod._to_numpy(a), dsmod._to_numpy(b), equal_nan=True)


def merge(datasets: Sequence):
    """xr.merge of prediction datasets (compat 'no_conflicts' for identically-shaped
    variables: a name predicted by two models must agree, else ValueError)."""
    out = dsmod.Dataset()
    for ds in datasets:
        for name in ds:
            da = ds[name]
            if name in out:
                old = out[name]
                if tuple(old.dims) != tuple(da.dims) or not _same(old.data, da.data):
                    raise ValueError(f"conflicting values for variable {name!r} on objects to be combined")
                continue
            out[name] = dsmod.DataArray(da.data, da.dims, da.coords, da.attrs)
    return out


class MultiModelAdapter:
    """machine_learning.py:150-179: predict with every model, merge, scale."""

    def __init__(self, models: Iterable[RenamingAdapter], scaling: Optional[Mapping[str, float]] = None):
        self.models = models
        self._scaling: Mapping[str, float] = {} if scaling is None else scaling

    @property
    def input_variables(self) -> Set[str]:
        return {var for model in self.models for var in model.input_variables}

    def predict(self, arg):
        ds = merge([model.predict(arg) for model in self.models])
        for var, scale in self._scaling.items():
            da = ds[var]
            # ds[var] *= scale: a float32 prediction times a Python float stays float32
            ds[var] = dsmod.DataArray(da.data * scale, da.dims, da.coords, da.attrs)
        return ds


@dataclasses.dataclass
class MachineLearningConfig:
    """machine_learning.py:24-64."""
    model: Sequence[str] = dataclasses.field(default_factory=list)
    diagnostic_ml: bool = False
    input_standard_names: Mapping[Hashable, Hashable] = dataclasses.field(default_factory=dict)
    output_standard_names: Mapping[Hashable, Hashable] = dataclasses.field(default_factory=dict)
    use_mse_conserving_humidity_limiter: bool = True
    scaling: Mapping[str, float] = dataclasses.field(default_factory=dict)


def open_model(config: MachineLearningConfig) -> MultiModelAdapter:
    """machine_learning.py:182-190, loading through this package's name-file registry."""
    from .predictor import load

    models = [RenamingAdapter(load(path), config.input_standard_names, config.output_standard_names)
              for path in config.model]
    return MultiModelAdapter(models, scaling=config.scaling)


def predict(model, state: Mapping, dims: Sequence[Hashable] = ("z", "y", "x")) -> Dict[Hashable, object]:
    """machine_learning.py:206-211.  State values may be DataArrays or bare arrays
    (labelled with ``dims``)."""
    ds = dsmod.Dataset({key: _as_dataarray(state[key], dims) for key in model.input_variables})
    output = model.predict(ds)
    return {key: output[key] for key in output.data_vars}


def _as_dataarray(x, dims):
    if hasattr(x, "dims") and not callable(getattr(x, "dims")):
        return x if isinstance(x, dsmod.DataArray) else dsmod.DataArray(_values(x), x.dims)
    d = tuple(dims)
    if len(d) != len(x.shape):  # a 2-D (y, x) field of a (z, y, x) state
        d = tuple(n for n in d if n != "z")
    return dsmod.DataArray(x, d)


# ----------------------------------------------------------------------- stepper
class PureMLStepper:
    """machine_learning.py:214-315.  ``__call__`` predicts, splits the prediction into
    tendencies / state updates / diagnostics, limits dQ1/dQ2 and diagnoses; ``apply`` is
    the loop's fillna + add_tendency + precipitation_sum (loop.py:604-628) for the same
    step; ``global_metrics`` the per-step statistics of main.py:55-60."""

    def __init__(self, model, timestep: float, hydrostatic: bool = False, mse_conserving_limiter: bool = True,
                 label: str = "machine_learning", dims: Sequence[Hashable] = ("z", "y", "x")):
        self.model = model
        self.timestep = float(timestep)
        self.hydrostatic = hydrostatic
        self.mse_conserving_limiter = mse_conserving_limiter
        self.label = label
        self.dims = tuple(dims)  # dims of bare-array state variables
        self._last: Optional[Dict[str, object]] = None

    def _state_dims(self, state) -> Tuple[Hashable, ...]:
        v = state[SPHUM]
        dims = getattr(v, "dims", None)
        return tuple(dims) if dims is not None and not callable(dims) else self.dims

    def __call__(self, time, state: Mapping) -> Tuple[Dict, Dict, Dict]:
        """-> (tendency, diagnostics, state_updates) like PureMLStepper.__call__."""
        dims = self._state_dims(state)
        lev = dims.index("z")
        wrap = lambda t: dsmod.DataArray(t, dims)  # noqa: E731
        wrap2 = lambda t: dsmod.DataArray(t, tuple(d for d in dims if d != "z"))  # noqa: E731
        sphum, delp, temp = _values(state[SPHUM]), _values(state[DELP]), _values(state[TEMP])
        prediction = predict(self.model, state, dims)
        tendency, state_updates, diagnostics = {}, {}, {}
        for key, value in prediction.items():
            if is_state_update_variable(key, state):
                state_updates[key] = value
            elif is_tendency_variable(key):
                tendency[key] = value
            else:
                diagnostics[key] = value
        for name in state_updates:
            diagnostics[name] = state_updates[name]

        def tend(name):
            v = tendency[name]
            d = tuple(v.dims)
            data = _values(v)
            if d != dims:  # the predictor returns the input's dim order; normalise to the state's
                data = data.permute(*[d.index(n) for n in dims]) if hasattr(data, "permute") else data
            return data

        has1, has2 = "dQ1" in tendency, "dQ2" in tendency
        zeros = None if (has1 and has2) else torch.zeros(tuple(sphum.shape), dtype=torch.float32,
                                                          device=torch.device("cuda", torch.cuda.current_device()))
        res = ml_epilogue(tend("dQ1") if has1 else zeros, tend("dQ2") if has2 else zeros, sphum, delp, temp,
                          self.timestep, _values(state[TOTAL_PRECIP]) if TOTAL_PRECIP in state else None,
                          self.mse_conserving_limiter, self.hydrostatic, self.label, level_axis=lev,
                          has_dq1=has1, has_dq2=has2)
        if has1:
            diagnostics["column_integrated_dQ1_change_non_neg_sphum_constraint"] = wrap2(
                res["column_integrated_dQ1_change_non_neg_sphum_constraint"])
            tendency["dQ1"] = wrap(res["dQ1"])
        if has2:
            diagnostics["column_integrated_dQ2_change_non_neg_sphum_constraint"] = wrap2(
                res["column_integrated_dQ2_change_non_neg_sphum_constraint"])
            tendency["dQ2"] = wrap(res["dQ2"])
        diagnostics["specific_humidity_limiter_active"] = wrap(res["specific_humidity_limiter_active"])
        extra = {}
        for name in list(tendency):
            if name in A_GRID_WIND_TENDENCIES:
                extra[name] = tendency_columns(tend(name), delp, self.timestep, "wind", lev)
                tendency[name] = wrap(_device.to_device_f32(tend(name)))
            elif name == "dQp":
                extra[name] = tendency_columns(tend(name), delp, self.timestep, "mass", lev)
                tendency[name] = wrap(_device.to_device_f32(tend(name)))
            elif name not in ("dQ1", "dQ2"):
                raise NotImplementedError(f"tendency {name!r} (D-grid winds) is applied by the fv3gfs wrapper; "
                                          "not supported by this stepper")
        self._last = {"res": res, "extra": extra, "has": (has1, has2), "dims": dims, "state": state}
        return tendency, diagnostics, state_updates

    def get_diagnostics(self, state, tendency) -> Tuple[Dict, object]:
        """compute_diagnostics + compute_ml_momentum_diagnostics (compute.py:77-161) of
        the last step -> (diags, net moistening)."""
        last = self._require()
        res, extra, (has1, has2), dims = last["res"], last["extra"], last["has"], last["dims"]
        delp = _values(state[DELP])
        dev = delp.device
        cdims = tuple(d for d in dims if d != "z")
        col_shape = res[f"net_moistening_due_to_{self.label}"].shape
        wrap2 = lambda t: dsmod.DataArray(t, cdims)  # noqa: E731
        zeros3 = lambda: torch.zeros(tuple(delp.shape), dtype=delp.dtype, device=dev)  # noqa: E731
        net = res[f"net_moistening_due_to_{self.label}"]
        diags = {f"net_moistening_due_to_{self.label}": wrap2(net),
                 f"column_heating_due_to_{self.label}": wrap2(res[f"column_heating_due_to_{self.label}"])}
        if "dQp" in extra:
            diags[f"net_mass_tendency_due_to_{self.label}"] = wrap2(extra["dQp"]["integral"])
        diags["dQ1"] = tendency["dQ1"] if "dQ1" in tendency else dsmod.DataArray(zeros3(), dims)
        diags["dQ2"] = tendency["dQ2"] if "dQ2" in tendency else dsmod.DataArray(zeros3(), dims)
        for w in ("dQu", "dQv"):
            if w in extra:
                diags[w] = tendency[w]
                diags[f"column_integrated_{w}_stress"] = wrap2(extra[w]["integral"])
            else:
                diags[w] = dsmod.DataArray(zeros3(), dims)
                diags[f"column_integrated_{w}_stress"] = wrap2(torch.zeros(col_shape, dtype=delp.dtype, device=dev))
        for name in (TEMP, SPHUM, DELP):
            diags[name] = state[name]
        return diags, diags[f"net_moistening_due_to_{self.label}"]

    def apply(self) -> Tuple[Dict, Dict]:
        """-> (updated state, filled fractions): fillna + add_tendency of every
        predicted tendency, precipitation_sum (loop.py:604-628).  A-grid wind
        tendencies come back as the float64 filled ``dQu``/``dQv`` the loop hands to the
        wrapper's A->D-grid transform (loop.py:126-182)."""
        last = self._require()
        res, extra, (has1, has2) = last["res"], last["extra"], last["has"]
        updated, fracs = {}, {}
        if has1:
            updated[TEMP] = res[TEMP]
            fracs["dQ1_filled_frac"] = res["dQ1_filled_frac"]
        if has2:
            updated[SPHUM] = res[SPHUM]
            fracs["dQ2_filled_frac"] = res["dQ2_filled_frac"]
        for name, e in extra.items():
            fracs[f"{name}_filled_frac"] = e["filled_frac"]
            if name == "dQp":
                updated[DELP] = e["state"]
            else:
                updated[name] = e["filled"]
        if TOTAL_PRECIP in res:
            updated[TOTAL_PRECIP] = res[TOTAL_PRECIP]
        return updated, fracs

    def global_metrics(self, diagnostics: Mapping, area, group=None) -> Tuple[Dict, Dict]:
        """main.py:55-60 for this rank's diagnostics: (global area-weighted means of every
        2-D diagnostic, ``specific_humidity_limiter_active_global_sum`` per level), one
        deterministic HIP reduction each and an all-gather of the rank partials."""
        from .distributed import globally_average_2d_diagnostics, globally_sum_3d_diagnostics

        dims = self._require()["dims"]
        cdims = tuple(d for d in dims if d != "z")
        two_d = {k: v for k, v in diagnostics.items() if set(getattr(v, "dims", ())) == {"x", "y"}}
        two_d["area"] = area if hasattr(area, "dims") else dsmod.DataArray(area, cdims)
        averages = globally_average_2d_diagnostics(two_d, group=group)
        profiles = globally_sum_3d_diagnostics(diagnostics, ["specific_humidity_limiter_active"], group=group)
        return averages, profiles

    def _require(self):
        if self._last is None:
            raise RuntimeError("call the stepper first")
        return self._last


def _values(x):
    d = getattr(x, "data", x)
    return d if isinstance(d, torch.Tensor) else getattr(x, "values", x)
