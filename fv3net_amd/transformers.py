"""The prognostic run's second Predictor caller: the online transformer Adapter
(workflows/prognostic_c48_run/runtime/transformers/fv3fit.py:17-109).

``Adapter`` loads its models through this package's registry (any registered predictor,
the build's ``mi355x-dense`` included, or a composite nesting it), predicts through
``MultiModelAdapter`` like the reference, and runs everything after the prediction in
one HIP kernel (``fv3_adapter_apply``, csrc/composite.hip): the tendency sum over the
outputs mapped to each state variable, the MSE-conserving non-negative-humidity limiter
(steppers/machine_learning.py:77-99) and ``state + tendency * timestep`` for every
tendency target, in the state's dtype with numpy's promotion order.
"""
import dataclasses
from collections import defaultdict
from typing import Dict, Hashable, Iterable, Mapping, MutableMapping, Sequence

import numpy as np

from . import _device, _native
from . import dataset as dsmod
from .stepper import SPHUM, TEMP, MultiModelAdapter

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

__all__ = ["Config", "Adapter"]


@dataclasses.dataclass
class Config:
    """transformers/fv3fit.py:17-50: model paths, output -> state name maps for
    tendency and state predictions, the humidity limiter and the online switch."""
    url: Sequence[str]
    tendency_predictions: Mapping[str, str] = dataclasses.field(default_factory=dict)
    state_predictions: Mapping[str, str] = dataclasses.field(default_factory=dict)
    limit_negative_humidity: bool = True
    online: bool = True

    def __post_init__(self):
        state_targets = list(self.state_predictions.values())
        tendency_targets = list(self.tendency_predictions.values())
        if len(set(state_targets)) < len(state_targets):
            raise ValueError("Cannot have multiple state predictions for same variable.")
        if len(set(state_targets).intersection(tendency_targets)) > 0:
            raise ValueError("A variable cannot be updated by tendency and state predictions.")


def _dims(x):
    d = getattr(x, "dims", None)
    return tuple(d) if d is not None and not callable(d) else None


def _data(x):
    return getattr(x, "data", x)


def _prediction_on_device(x, dev):
    """A prediction as a contiguous device array in its own dtype when that is float64
    (a TaperedModel / float64 ensemble returns float64) and float32 otherwise."""
    t = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if t.dtype == torch.float64:
        return t.to(dev).contiguous()
    return _device.to_device_f32(t)


class Adapter:
    """transformers/fv3fit.py:53-109 (``predict`` / ``apply`` / ``partial_fit`` /
    ``input_variables``); ``models`` may be given directly instead of loaded from
    ``config.url``."""

    def __init__(self, config: Config, timestep: float, models: Iterable = None):
        from .predictor import load

        self.config = config
        self.timestep = timestep
        models = list(models) if models is not None else [load(url) for url in config.url]
        self.model = MultiModelAdapter(models)
        self.tendency_names: Dict[Hashable, list] = defaultdict(list)
        for k, v in config.tendency_predictions.items():
            self.tendency_names[v].append(k)
        self.state_names = {v: k for k, v in config.state_predictions.items()}

    @property
    def input_variables(self) -> Iterable[Hashable]:
        return list(set(self.model.input_variables) | set(self.tendency_names))

    def predict(self, inputs: Mapping) -> Dict[Hashable, object]:
        """The state updates: ``state_predictions`` as predicted, every tendency target
        as ``inputs[name] + tendency * timestep`` (limited first when configured), with
        the input's dims and attrs (keep_attrs)."""
        ds = dsmod.Dataset({k: v if isinstance(v, dsmod.DataArray) else dsmod.DataArray(_data(v), _dims(v))
                            for k, v in inputs.items() if _dims(v) is not None})
        prediction = self.model.predict(ds)
        state_updates: MutableMapping[Hashable, object] = {k: prediction[v] for k, v in self.state_names.items()}
        if self.config.limit_negative_humidity and SPHUM not in self.tendency_names:
            raise NotImplementedError("Cannot limit specific humidity tendencies if specific humidity "
                                      "updates not being predicted.")
        if not self.tendency_names:
            return dict(state_updates)
        state_updates.update(self._apply_tendencies(prediction, inputs))
        return dict(state_updates)

    def _apply_tendencies(self, prediction, inputs) -> Dict[Hashable, object]:
        _device.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        names = list(self.tendency_names)
        limit = bool(self.config.limit_negative_humidity)
        if limit:  # the humidity target first, then temperature: both in the kernel's limiter launch
            names.sort(key=lambda n: (n != SPHUM, n != TEMP))
        states, hosts, keep = {}, {}, []
        for name in names:
            x = _data(inputs[name])
            hosts[name] = not (torch.is_tensor(x) and x.is_cuda)
            t = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
            t = t.to(dev)
            if t.dtype not in (torch.float32, torch.float64):
                t = t.to(torch.float64)
            states[name] = t.contiguous()
        shapes = {tuple(t.shape) for t in states.values()}
        if len(shapes) != 1:
            raise ValueError(f"tendency targets must share one shape, got {sorted(shapes)}")
        dtypes = {t.dtype for t in states.values()}
        if len(dtypes) != 1:
            raise ValueError(f"tendency targets must share one dtype, got {sorted(map(str, dtypes))}")
        state_f64 = int(dtypes.pop() == torch.float64)
        targets = (_native.AdapterTarget * len(names))()
        outs = {}
        for g, name in enumerate(names):
            st = states[name]
            sdims = _dims(inputs[name])
            items = self.tendency_names[name]
            if not 1 <= len(items) <= _native.ADAPTER_MAX_PREDS:
                raise NotImplementedError(f"{name}: 1..{_native.ADAPTER_MAX_PREDS} predictions per target")
            for p, item in enumerate(items):
                da = prediction[item]  # KeyError if the model does not predict it
                if sdims is not None and tuple(da.dims) != sdims:
                    da = da.transpose(*sdims)  # xarray aligns the sum by dim name
                pt = _prediction_on_device(_data(da), dev)  # float64 predictions stay float64
                if tuple(pt.shape) != tuple(st.shape):
                    raise ValueError(f"prediction {item} shape {tuple(pt.shape)} != state {name} "
                                     f"{tuple(st.shape)}")
                keep.append(pt)
                targets[g].preds[p] = pt.data_ptr()
                if pt.dtype == torch.float64:
                    targets[g].pred_f64 |= 1 << p
            targets[g].n_preds = len(items)
            targets[g].state = st.data_ptr()
        if len(names) > _native.ADAPTER_MAX_TARGETS:
            raise NotImplementedError(f"at most {_native.ADAPTER_MAX_TARGETS} tendency targets")
        q_index = names.index(SPHUM) if limit else -1
        t_index = names.index(TEMP) if (limit and TEMP in names) else -1
        for g, name in enumerate(names):
            # numpy's result dtype of state + tendency * dt (the limited tendencies promoted
            # with the humidity state and tendency, as xr.where and the MSE terms do)
            wide = state_f64 or targets[g].pred_f64 != 0
            if limit and g in (q_index, t_index):
                wide = wide or targets[q_index].pred_f64 != 0
            out = torch.empty(states[name].shape, dtype=torch.float64 if wide else torch.float32, device=dev)
            outs[name] = out
            targets[g].out = out.data_ptr()
            targets[g].out_f64 = int(wide)
        n = next(iter(states.values())).numel()
        status = _native.load().fv3_adapter_apply(targets, len(names), n, state_f64, float(self.timestep), int(limit),
                                                  q_index, t_index, _device.stream_handle(None))
        _native.check(status, "adapter_apply")
        result = {}
        for name in names:
            src = inputs[name]
            data = outs[name].cpu().numpy() if hosts[name] else outs[name]
            sdims = _dims(src)
            result[name] = dsmod.DataArray(data, sdims, getattr(src, "coords", None), getattr(src, "attrs", None),
                                           name) if sdims is not None else data
        return result

    def apply(self, prediction: Mapping, state: MutableMapping):
        if self.config.online:
            state.update(prediction)

    def partial_fit(self, inputs, state):
        pass
