"""The ML stepper around the predictor: limiter, diagnostics and tendency application.

Mirrors ``PureMLStepper`` (workflows/prognostic_c48_run/runtime/steppers/
machine_learning.py:239-315) and the part of the prognostic loop that applies its
output (runtime/loop.py:103-219, diagnostics/compute.py:21-39, 77-106), with the
whole post-prediction epilogue fused into one HIP kernel (csrc/stepper.hip).

State variables are [z, ...] device tensors (float64 like the FV3 state, or float32);
the model's dQ1/dQ2 are float32 (Keras output).
"""
from typing import Dict, Mapping, Optional, Tuple

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

SPHUM = "specific_humidity"
DELP = "pressure_thickness_of_atmospheric_layer"
TEMP = "air_temperature"
TOTAL_PRECIP = "total_precipitation"

COLUMN_DIAGNOSTICS = (
    "column_integrated_dQ1_change_non_neg_sphum_constraint",
    "column_integrated_dQ2_change_non_neg_sphum_constraint",
    "net_moistening_due_to_{label}",
    "column_heating_due_to_{label}",
    "dQ1_filled_frac",
    "dQ2_filled_frac",
    TOTAL_PRECIP,
)


def ml_epilogue(dq1, dq2, sphum, delp, temperature, dt: float, physics_precip=None,
                mse_conserving: bool = True, hydrostatic: bool = False, label: str = "machine_learning",
                in_place: bool = False, level_axis: int = 0, stream=None) -> Dict[str, object]:
    """Limiter + diagnostics + apply for one (dQ1, dQ2) prediction, one kernel.

    ``level_axis`` is the vertical axis of every 3-D array (axes before it are
    blocks such as tiles).  Returns device tensors: limited ``dQ1``/``dQ2`` (pre-fillna, as the stepper
    returns them), ``specific_humidity_limiter_active`` (uint8), the updated
    ``air_temperature``/``specific_humidity`` (written into the inputs when
    ``in_place``), the column diagnostics of COLUMN_DIAGNOSTICS and, with
    ``physics_precip``, the new ``total_precipitation``.
    """
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
    column = torch.empty((7, ncol), dtype=state_dtype, device=dev)
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
    st_ = _native.load().fv3_ml_epilogue(ctypes_byref(io), lay, ncol, nz, int(state_dtype == torch.float64),
                                         float(dt), int(bool(mse_conserving)), int(bool(hydrostatic)),
                                         _device.stream_handle(stream))
    _native.check(st_, "ml_epilogue")
    for i, name in enumerate(COLUMN_DIAGNOSTICS):
        if name == TOTAL_PRECIP and precip is None:
            continue
        out[name.format(label=label)] = column[i].reshape(col_shape)
    return out


def ctypes_byref(obj):
    import ctypes

    return ctypes.byref(obj)


class PureMLStepper:
    """machine_learning.py:198-315: predict, limit, diagnose; ``apply`` is the loop's
    fillna + add_tendency + precipitation_sum (loop.py:575-632) for the same step."""

    def __init__(self, model, timestep: float, hydrostatic: bool = False, mse_conserving_limiter: bool = True,
                 label: str = "machine_learning"):
        self.model = model
        self.timestep = float(timestep)
        self.hydrostatic = hydrostatic
        self.mse_conserving_limiter = mse_conserving_limiter
        self.label = label
        self._last: Optional[Dict[str, object]] = None

    def __call__(self, time, state: Mapping) -> Tuple[Dict, Dict, Dict]:
        """-> (tendency, diagnostics, state_updates) like PureMLStepper.__call__."""
        from .dataset import Dataset, DataArray

        inputs = Dataset({k: state[k] if hasattr(state[k], "dims") else DataArray(state[k], ("z", "y", "x"))
                          for k in self.model.input_variables})
        prediction = self.model.predict(inputs)
        dq1 = _values(prediction["dQ1"])
        dq2 = _values(prediction["dQ2"])
        res = ml_epilogue(dq1, dq2, _values(state[SPHUM]), _values(state[DELP]), _values(state[TEMP]),
                          self.timestep, _values(state[TOTAL_PRECIP]) if TOTAL_PRECIP in state else None,
                          self.mse_conserving_limiter, self.hydrostatic, self.label)
        self._last = res
        tendency = {"dQ1": res["dQ1"], "dQ2": res["dQ2"]}
        diagnostics = {k: res[k] for k in ("column_integrated_dQ1_change_non_neg_sphum_constraint",
                                           "column_integrated_dQ2_change_non_neg_sphum_constraint",
                                           "specific_humidity_limiter_active")}
        return tendency, diagnostics, {}

    def get_diagnostics(self, state, tendency) -> Tuple[Dict, object]:
        """compute_diagnostics (diagnostics/compute.py:77-106) of the last step."""
        res = self._require()
        net = res[f"net_moistening_due_to_{self.label}"]
        diags = {f"net_moistening_due_to_{self.label}": net,
                 f"column_heating_due_to_{self.label}": res[f"column_heating_due_to_{self.label}"]}
        return diags, net

    def apply(self) -> Tuple[Dict, Dict]:
        """-> (updated state, filled fractions): add_tendency of the NaN-filled
        tendencies and precipitation_sum (loop.py:620-632)."""
        res = self._require()
        updated = {TEMP: res[TEMP], SPHUM: res[SPHUM]}
        if TOTAL_PRECIP in res:
            updated[TOTAL_PRECIP] = res[TOTAL_PRECIP]
        return updated, {"dQ1_filled_frac": res["dQ1_filled_frac"], "dQ2_filled_frac": res["dQ2_filled_frac"]}

    def _require(self):
        if self._last is None:
            raise RuntimeError("call the stepper first")
        return self._last


def _values(x):
    d = getattr(x, "data", x)
    return d if isinstance(d, torch.Tensor) else getattr(x, "values", x)
