"""fv3fit's Predictor plugin API, mirrored, with an MI355X DenseModel predictor.

Reference (paths under /root/reference/external/fv3fit/fv3fit):
* ``Predictor`` ABC                     _shared/predictor.py:44-95
* name-file registry register/load/dump _shared/io.py:17-100
* ``stack`` / ``match_prediction_to_input_coords``  _shared/stacking.py:12-52
* ``vcm.safe.stack_once`` broadcast guard           external/vcm/vcm/safe.py:23-44
* ``PureKerasModel.predict``                        keras/_models/shared/pure_keras.py:98-118
* ``ConstantOutputPredictor``                       testing.py:30-117

Contract kept: ``predict`` never mutates its input and returns
new arrays; output dims follow the input's first-seen dim order; outputs are
float32 (the Keras model's dtype); KeyError for a missing input variable,
ValueError for a disallowed broadcast, TypeError for unknown constructor kwargs,
ValueError for a duplicate registry name.

The device path needs no stack copy: the kernel reads each variable's
[level][column] layout in place (any column order gives the same per-column
result, written back at the same column), which is exactly stack -> predict ->
unstack -> transpose-to-input-order.
"""
import abc
import os
import warnings
from typing import Dict, Hashable, Iterable, Mapping, MutableMapping, Optional, Sequence, Type

import numpy as np
import yaml

from . import dataset as dsmod

SAMPLE_DIM_NAME = "_fv3fit_sample"
DATASET_DIM_NAME = "dataset"
Z_DIM_NAMES = ["z", "pfull"]

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


# ---------------------------------------------------------------------------- ABC
class Predictor(abc.ABC):
    """Abstract predictor (predictor.py:44-95)."""

    def __init__(self, input_variables: Iterable[Hashable], output_variables: Iterable[Hashable], **kwargs):
        super().__init__()
        if len(kwargs.keys()) > 0:
            raise TypeError(f"received unexpected keyword arguments: {tuple(kwargs.keys())}")
        self.input_variables = input_variables
        self.output_variables = output_variables

    @abc.abstractmethod
    def predict(self, X):
        """Predict an output dataset from an input dataset."""

    @abc.abstractmethod
    def dump(self, path: str) -> None:
        """Serialize to a directory."""

    @classmethod
    @abc.abstractmethod
    def load(cls, path: str) -> "Predictor":
        """Load a serialized model from a directory."""


# ---------------------------------------------------------------------- registry
_NAME_PATH = "name"
_NAME_ENCODING = "UTF-8"


class _Register:
    """Name-file registry (io.py:17-100) on the local filesystem."""

    def __init__(self) -> None:
        self._model_types: MutableMapping[str, type] = {}

    def __call__(self, name: str):
        if name in self._model_types:
            raise ValueError(f"{name} is already registered by {self._model_types[name]}.")

        def deco(cls):
            self._model_types[name] = cls
            return cls

        return deco

    def get_name(self, obj) -> str:
        return_name, name_cls = None, None
        for name, cls in self._model_types.items():
            if isinstance(obj, cls) and (name_cls is None or issubclass(cls, name_cls)):
                return_name, name_cls = name, cls
        if return_name is None:
            raise ValueError(f"{type(obj)} is not registered. Consider decorating with "
                             '@fv3net_amd.predictor.register("name")')
        return return_name

    def load(self, path: str):
        from . import composite, derived, novelty, pytorch_predictor  # noqa: F401  register the composites, "pytorch_predictor"

        name_file = os.path.join(path, _NAME_PATH)
        if not os.path.exists(name_file):
            warnings.warn(f"Model type is not located at {name_file}. Trying all known models one-by-one.",
                          UserWarning)
            for name, cls in self._model_types.items():
                try:
                    return cls.load(path)
                except Exception:  # noqa
                    pass
            raise KeyError(_NAME_PATH)
        with open(name_file, "rb") as f:
            name = f.read().decode(_NAME_ENCODING).strip()
        return self._model_types[name].load(path)

    def dump(self, obj, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, _NAME_PATH), "wb") as f:
            f.write(self.get_name(obj).encode(_NAME_ENCODING))
        obj.dump(path)


register = _Register()
dump = register.dump
load = register.load


# ---------------------------------------------------------------- stack semantics
def _validate_stack_dims(ds, dims, allowed_broadcast_dims=()):
    """vcm.safe._validate_stack_dims (safe.py:23-33)."""
    for variable in ds:
        var_dims = ds[variable].dims
        broadcast_dims = set(dims) - (set(var_dims) | set(allowed_broadcast_dims))
        if len(broadcast_dims) > 0:
            raise ValueError(f"{variable} will be broadcast to include unallowed dimensions "
                             f"{broadcast_dims}. This could greatly increase the size of dataset.")


def stack(ds, unstacked_dims: Optional[Sequence[str]] = None):
    """fv3fit ``stack`` (stacking.py:12-27) for fv3net_amd.Dataset: stack every dim
    except ``unstacked_dims`` into ``_fv3fit_sample`` (C order over the SORTED dims,
    xarray 0.19), unstacked dims sorted after it."""
    if dsmod.is_xarray(ds):
        raise TypeError("use fv3fit's own stack() on xarray objects")
    unstacked_dims = list(unstacked_dims or [])
    all_dims = list(dsmod.dataset_dims(ds))
    stack_dims = [d for d in all_dims if d not in unstacked_dims]
    unstacked = sorted(d for d in all_dims if d in unstacked_dims)
    out = dsmod.Dataset()
    if len(stack_dims) == 0:
        for name in ds:
            da = ds[name]
            order = [d for d in unstacked if d in da.dims]
            data = da.transpose(*order).values[None, ...]
            out[name] = dsmod.DataArray(data, [SAMPLE_DIM_NAME] + order)
        return out
    _validate_stack_dims(ds, stack_dims, allowed_broadcast_dims=list(unstacked) + ["time", "dataset"])
    sizes = ds.dims
    n = int(np.prod([sizes[d] for d in stack_dims]))
    for name in ds:
        da = ds[name]
        order = [d for d in stack_dims] + [d for d in unstacked if d in da.dims]
        values = da.values
        # broadcast allowed missing stack dims (time/dataset/unstacked), then order
        present = [d for d in order if d in da.dims]
        arr = np.transpose(values, [da.dims.index(d) for d in present])
        shape = [sizes[d] if d in da.dims else 1 for d in order]
        arr = np.broadcast_to(arr.reshape(shape), [sizes[d] for d in order])
        out_dims = [SAMPLE_DIM_NAME] + [d for d in unstacked if d in da.dims]
        out[name] = dsmod.DataArray(np.ascontiguousarray(arr).reshape([n] + [sizes[d] for d in out_dims[1:]]),
                                    out_dims)
    out.coords[SAMPLE_DIM_NAME + "_dims"] = np.array(stack_dims)
    return out


def unstack(stacked, template_dims: Mapping[Hashable, int], stack_dims: Sequence[Hashable]):
    """Inverse of ``stack`` for a [sample, ...] dataset (xarray .unstack appends the
    stacked dims after the remaining ones, pure_keras.py:79-96)."""
    out = dsmod.Dataset()
    for name in stacked:
        da = stacked[name]
        rest = list(da.dims[1:])
        data = da.values.reshape([template_dims[d] for d in stack_dims] + list(da.shape[1:]))
        data = np.moveaxis(data, list(range(len(stack_dims))), list(range(len(rest), len(rest) + len(stack_dims))))
        out[name] = dsmod.DataArray(data, rest + list(stack_dims))
    return out


def match_prediction_to_input_coords(input_ds, prediction):
    """stacking.py:40-52: drop coords not in the input, transpose to the input's
    first-seen dim order."""
    order = dsmod.infer_dimension_order(input_ds)
    out = dsmod.Dataset()
    for name in prediction:
        da = prediction[name]
        dims = [d for d in order if d in da.dims] + [d for d in da.dims if d not in order]
        coords = {d: input_ds.coords[d] for d in dims if d in getattr(input_ds, "coords", {})}
        t = da.transpose(*dims)
        out[name] = dsmod.DataArray(t.data, t.dims, coords)
    return out


# --------------------------------------------------------------- dense predictor
def _level_dim(dims, unstacked_dims):
    lv = [d for d in dims if d in unstacked_dims]
    if len(lv) > 1:
        raise ValueError(f"variable has several unstacked dims {lv}; one level dim is supported")
    return lv[0] if lv else None


@register("mi355x-dense")
class DenseColumnPredictor(Predictor):
    """fv3fit DenseModel (``PureKerasModel`` with ``unstacked_dims=("z",)``, n_halo 0)
    predicting on MI355X through the fused HIP kernel.

    ``input_sources``: for a model whose input features are derived from the dataset's
    variables in the graph -- the microphysics emulator's dict model (``all-keras-dict``,
    ``PureKerasDictPredictor``, pure_keras.py:181-258) takes raw variables and logs some
    of them inside (transforms.py:111-129) -- the dataset variable each model feature
    reads (``cfg.input_variables`` order; the kernel applies the feature's LogTransform).
    The predictor's ``input_variables`` are then those variables, each once, in order."""

    _CONFIG_FILENAME = "config.yaml"
    _MODEL_DIR = "dense"

    def __init__(self, input_variables, output_variables, model, unstacked_dims: Sequence[str] = ("z",),
                 n_halo: int = 0, input_sources: Optional[Sequence[str]] = None):
        super().__init__(input_variables, output_variables)
        if n_halo != 0:
            raise NotImplementedError("halo models (n_halo > 0) are out of scope (SURVEY.md §8(e))")
        self.input_variables = list(input_variables)
        self.output_variables = list(output_variables)
        self.model = model
        self._unstacked_dims = tuple(unstacked_dims)
        self._n_halo = n_halo
        cfg = model.config
        features = list(cfg.input_variables)
        self._sources = list(input_sources) if input_sources is not None else features
        if len(self._sources) != len(features):
            raise ValueError(f"{len(self._sources)} input sources for {len(features)} model inputs")
        if list(dict.fromkeys(self._sources)) != self.input_variables or \
                list(cfg.output_variables) != self.output_variables:
            raise ValueError("model variables do not match the predictor's")

    # -- predict ----------------------------------------------------------------
    def predict(self, X):
        xr_in = dsmod.is_xarray(X)
        plan = None
        if not xr_in and isinstance(X, dsmod.Dataset):
            # the call's layout decisions depend only on the variables' names, dims, shapes
            # and array kinds: a prognostic run passes the same layout every step
            sig = tuple((k, v.dims, v.data.shape, type(v.data), getattr(v.data, "dtype", None))
                        for k, v in X.data_vars.items())
            cache = self.__dict__.setdefault("_plans", {})
            plan = cache.get(sig)
            if plan is None:
                plan = self._plan(X)
                if len(cache) > 16:
                    cache.clear()
                cache[sig] = plan
        else:
            plan = self._plan(X)
        in_specs, out_specs, host, src_is_torch = plan
        own = isinstance(X, dsmod.Dataset)
        tensors, axes = [], []
        for name, axis, perm, lead in in_specs:
            data = X.data_vars[name].data if own else dsmod.variable_data(X, name)
            is_torch = torch is not None and isinstance(data, torch.Tensor)
            if perm is not None:
                data = data.permute(*perm) if is_torch else np.transpose(np.asarray(data), perm)
            elif not is_torch:
                data = np.asarray(data)
            if lead:
                data = data[None, ...]
            tensors.append(_as_contig(data))
            axes.append(axis)
        if host:
            outs = self._host_forward(tensors, axes)  # numpy in, numpy out
        else:
            outs = self.model.forward(tensors, level_axes=axes)
        result = {}
        for (name, reshape, tgt, perm), t in zip(out_specs, outs):
            if reshape is not None:  # scalar_singleton_dim squeeze (pure_keras.py:85-90)
                t = t.reshape(reshape)
            if isinstance(t, np.ndarray):
                t = t if perm is None else np.ascontiguousarray(np.transpose(t, perm))
            else:
                t = (t if perm is None else t.permute(*perm)).contiguous()
            result[name] = (tgt, t)
        return _make_output(X, result, xr_in, src_is_torch)

    def _plan(self, X):
        """Validate X against the model and fix the call's layout: per input (name, the
        level axis the kernel reads, the permutation to [level] + column order or None,
        a level axis to add for a 2-D input), per output (name, the squeeze shape of a
        one-level output, the output dims in the input's order, the permutation there or
        None), whether the call is numpy in / numpy out, whether X holds torch data."""
        cfg = self.model.config
        all_dims = list(dsmod.dataset_dims(X))
        stack_dims = [d for d in all_dims if d not in self._unstacked_dims]
        # stack_once broadcast guard (safe.py:36-44) over the model inputs
        sub = {name: X[name] for name in self.input_variables}  # KeyError if missing
        for name, da in sub.items():
            missing = set(stack_dims) - set(da.dims) - {"time", "dataset"}
            if missing:
                raise ValueError(f"{name} will be broadcast to include unallowed dimensions {missing}. "
                                 "This could greatly increase the size of dataset.")
        # one common column order: the first input's horizontal dims
        first = sub[self._sources[0]]
        col_dims = [d for d in first.dims if d not in self._unstacked_dims]
        col_shape = [dict(zip(first.dims, first.shape))[d] for d in col_dims]
        in_specs, axes, host = [], [], True
        for v, name in enumerate(self._sources):  # per model feature: the variable it reads
            da = sub[name]
            lv = _level_dim(da.dims, self._unstacked_dims)
            if set(d for d in da.dims if d != lv) != set(col_dims):
                raise ValueError(f"{name} dims {da.dims} do not share the horizontal dims {col_dims}")
            data = dsmod.variable_data(X, name)
            host = host and not (torch is not None and isinstance(data, torch.Tensor)) and \
                np.asarray(data).dtype in (np.float32, np.float64)
            if lv and [d for d in da.dims if d != lv] == col_dims:
                # horizontal dims already in column order: the kernel reads the array in
                # place with the level axis where it is, e.g. (tile, z, y, x)
                in_specs.append((name, da.dims.index(lv), None, False))
                axes.append(da.dims.index(lv))
                continue
            order = ([lv] if lv else []) + col_dims
            perm = [da.dims.index(d) for d in order]
            in_specs.append((name, 0, perm if perm != list(range(len(perm))) else None, not lv))
            axes.append(0)
        # back to the input's dim order (match_prediction_to_input_coords)
        order = dsmod.infer_dimension_order(X)
        out_specs = []
        ax0 = axes[0]  # the outputs carry their level axis where the first input had it
        for o, name in enumerate(self.output_variables):
            dims = list(col_dims)
            reshape = None
            if cfg.out_nz[o] == 1:
                reshape = tuple(col_shape)
            else:
                dims.insert(ax0, self._unstacked_dims[0])
            tgt = [d for d in order if d in dims] + [d for d in dims if d not in order]
            perm = [dims.index(d) for d in tgt]
            out_specs.append((name, reshape, tgt, perm if perm != list(range(len(perm))) else None))
        src_is_torch = any(torch is not None and isinstance(dsmod.variable_data(X, n), torch.Tensor) for n in X)
        return in_specs, out_specs, host, src_is_torch

    def _host_forward(self, arrays, axes):
        """Host arrays in, host float32 arrays out, for the drop-in call on numpy data
        (pure_keras.py:98-118 predicts on host arrays): ``DenseColumnModel.forward_host``
        (device buffers of the inputs' own dtype cached per shape, outputs in the library's
        page-locked arena, tile blocks pipelined over two streams)."""
        return self.model.forward_host(arrays, axes)

    # -- persistence ------------------------------------------------------------
    def dump(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        self.model.dump(os.path.join(path, self._MODEL_DIR))
        with open(os.path.join(path, self._CONFIG_FILENAME), "w") as f:
            config = {"input_variables": list(self.input_variables),
                      "output_variables": list(self.output_variables),
                      "unstacked_dims": list(self._unstacked_dims), "n_halo": self._n_halo}
            if self._sources != list(self.model.config.input_variables):
                config["input_sources"] = list(self._sources)
            if getattr(self.model, "precision", "f32") != "f32":
                config["precision"] = self.model.precision
            yaml.safe_dump(config, f)

    @classmethod
    def load(cls, path: str) -> "DenseColumnPredictor":
        from .dense import DenseColumnModel

        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        model = DenseColumnModel.load(os.path.join(path, cls._MODEL_DIR))
        if config.get("precision"):
            model.precision = config["precision"]
        return cls(config["input_variables"], config["output_variables"], model,
                   unstacked_dims=config.get("unstacked_dims") or ("z",), n_halo=config.get("n_halo", 0),
                   input_sources=config.get("input_sources"))


def _as_contig(t):
    if torch is not None and isinstance(t, torch.Tensor):
        return t.contiguous()
    return np.ascontiguousarray(t)


def _to_host(t) -> np.ndarray:
    """A device output back to numpy (pinned, double-buffered D2H), or a host tensor's view."""
    if t.is_cuda:
        from .transfer import d2h

        return d2h(t)
    return t.detach().numpy()


def _make_output(X, result: Dict, xr_in: bool, src_is_torch: Optional[bool] = None):
    """Build the output dataset of the input's kind; coords copied from the input."""
    coords = getattr(X, "coords", {})
    if xr_in:
        import xarray as xr  # noqa: F401  (only when the caller passed xarray)

        data_vars = {}
        for name, (dims, t) in result.items():
            arr = _to_host(t) if hasattr(t, "detach") else np.asarray(t)
            data_vars[name] = xr.DataArray(arr, dims=dims, coords={d: coords[d] for d in dims if d in coords})
        return xr.Dataset(data_vars)
    out = dsmod.Dataset()
    if src_is_torch is None:
        src_is_torch = any(torch is not None and isinstance(dsmod.variable_data(X, n), torch.Tensor) for n in X)
    for name, (dims, t) in result.items():
        data = t
        if not src_is_torch and hasattr(t, "detach"):
            data = _to_host(t)
        out[name] = dsmod.DataArray(data, dims, {d: coords[d] for d in dims if d in coords})
    return out


# ------------------------------------------------------------ constant predictor
@register("constant-output")
class ConstantOutputPredictor(Predictor):
    """testing.py:30-117: scalar or per-level constant outputs, stacked over Z_DIM_NAMES.
    (No arithmetic: the smallest full-contract predictor, for boundary tests.)"""

    def __init__(self, input_variables, output_variables):
        super().__init__(input_variables=input_variables, output_variables=output_variables)
        self._outputs: Dict[Hashable, object] = {}

    def set_outputs(self, **outputs):
        self._outputs.update(outputs)

    def predict(self, X):
        sub = dsmod.Dataset({name: X[name] for name in self.input_variables})
        stacked = stack(sub, unstacked_dims=Z_DIM_NAMES)
        stack_dims = list(stacked.coords.get(SAMPLE_DIM_NAME + "_dims", []))
        n = stacked[self.input_variables[0]].shape[0] if len(stacked) else 1
        pred = dsmod.Dataset()
        for name in self.output_variables:
            output = self._outputs.get(name, 0.0)
            if isinstance(output, np.ndarray):
                pred[name] = dsmod.DataArray(np.repeat(output[None, :], n, axis=0), [SAMPLE_DIM_NAME, "z"])
            else:
                pred[name] = dsmod.DataArray(np.full([n], float(output)), [SAMPLE_DIM_NAME])
        sizes = dict(sub.dims)
        return match_prediction_to_input_coords(X, unstack(pred, sizes, stack_dims))

    def dump(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        np.savez(os.path.join(path, "_outputs.npz"), **self._outputs)
        with open(os.path.join(path, "attrs.yaml"), "w") as f:
            yaml.safe_dump({"input_variables": list(self.input_variables),
                            "output_variables": list(self.output_variables)}, f)

    @classmethod
    def load(cls, path: str) -> "ConstantOutputPredictor":
        outputs = dict(np.load(os.path.join(path, "_outputs.npz"), allow_pickle=False))
        with open(os.path.join(path, "attrs.yaml")) as f:
            attrs = yaml.safe_load(f)
        obj = cls(**attrs)
        for key, value in outputs.items():
            if value.ndim == 0:
                outputs[key] = value.item()
        obj.set_outputs(**outputs)
        return obj
