"""fv3fit's composite predictors, mirrored over this package's registry, so the build's
predictor (``mi355x-dense``) nests as a ``base_model`` the way fv3fit's own models do.

Reference: external/fv3fit/fv3fit/_shared/models.py
* ``CombinedOutputModel`` ("combined_output_model")  :19-62  merge of disjoint outputs
* ``TaperedModel``        ("tapered_model")          :65-107 per-output vertical taper
* ``EnsembleModel``       ("ensemble")               :223-276 member mean / median
* ``TaperConfig``                                    _shared/config.py:15-29

Each composite loads its members by recursive ``load`` of the paths in its yaml file
(the name-file registry, predictor.py), exactly as the reference's ``io.load`` does, and
post-processes their outputs on the device: the member reduction and the taper run as
HIP kernels (csrc/composite.hip, ``fv3_member_reduce`` / ``fv3_scale_levels``).  A
composite hands back the kind of data its members produced (device tensors stay on
the device; host arrays come back as host arrays).

``DerivedModel`` ("derived_model") and ``TransformedPredictor``
("output_transformed_model") live in derived.py, over the vcm.DerivedMapping /
vcm.DataTransform catalogues; ``OutOfSampleModel`` ("out_of_sample") with the min-max
novelty detector in novelty.py.
"""
import ctypes
import dataclasses
import os
from typing import Iterable, Mapping, Set

import numpy as np
import yaml

from . import _device, _native
from . import dataset as dsmod
from .predictor import Predictor, load, register

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _on_device(data):
    """(device tensor, came-from-host flag)."""
    if torch.is_tensor(data):
        return (data if data.is_cuda else data.cuda()), not data.is_cuda
    return torch.from_numpy(np.ascontiguousarray(np.asarray(data))).cuda(), True


def _back(t, host: bool):
    return t.cpu().numpy() if host else t


# ------------------------------------------------------------------ combined outputs
@register("combined_output_model")
class CombinedOutputModel(Predictor):
    """models.py:19-62: every member's outputs merged (members must predict disjoint
    variables)."""

    _CONFIG_FILENAME = "combined_output_model.yaml"

    def __init__(self, models: Iterable[Predictor]):
        self._models = tuple(models)
        if len(self._models) == 0:
            raise ValueError("at least one model must be given")
        inputs: Set = set()
        outputs: Set = set()
        for model in self._models:
            common = set(model.output_variables).intersection(outputs)
            if common:
                raise ValueError(f"All models being combined must have different outputs, got {common} "
                                 "multiple times.")
            inputs.update(model.input_variables)
            outputs.update(model.output_variables)
        super().__init__(input_variables=tuple(sorted(inputs)), output_variables=tuple(sorted(outputs)))

    def predict(self, X):
        from .stepper import merge

        return merge([m.predict(X) for m in self._models])

    def dump(self, path):
        raise NotImplementedError("no dump method yet for this class, you can define one manually "
                                  "(a combined_output_model.yaml listing the member paths, and a name file)")

    @classmethod
    def load(cls, path: str) -> "CombinedOutputModel":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        return cls([load(p) for p in config["models"]])


# ------------------------------------------------------------------------- taper
def vertical_tapering_scale_factors(n_levels: int, cutoff: int, rate: float) -> np.ndarray:
    """vcm/calc/calc.py:45-49 (float64 factors: exp((z - cutoff) / rate) below the
    cutoff, 1 from it on).  Host-side: a few dozen constants per output variable."""
    z_arr = np.arange(n_levels)
    scaled = np.exp((z_arr[slice(None, cutoff)] - cutoff) / rate)
    unscaled = np.ones(n_levels - cutoff)
    return np.hstack([scaled, unscaled])


@dataclasses.dataclass
class TaperConfig:
    """_shared/config.py:15-29."""
    cutoff: int
    rate: float
    taper_dim: str = "z"

    def apply(self, data: "dsmod.DataArray") -> "dsmod.DataArray":
        """scaling * data: float64, the taper dim first then the data's other dims (the
        DataArray product's broadcast order), on the device (fv3_scale_levels)."""
        if self.taper_dim not in data.dims:
            raise KeyError(self.taper_dim)
        ax = data.dims.index(self.taper_dim)
        n_levels = data.shape[ax]
        scale = vertical_tapering_scale_factors(n_levels, self.cutoff, self.rate)
        _device.require_gpu()
        x, host = _on_device(data.data)
        if x.dtype not in (torch.float32, torch.float64):
            x = x.to(torch.float64)
        xv, lay, ncol, nz = _device.column_view(x, ax, keep_f64=True)
        s = torch.from_numpy(scale).cuda()
        out = torch.empty((nz, ncol), dtype=torch.float64, device=x.device)
        st = _native.load().fv3_scale_levels(xv.data_ptr(), int(xv.dtype == torch.float64), lay, s.data_ptr(), ncol,
                                              nz, out.data_ptr(), _device.stream_handle(None))
        _native.check(st, "scale_levels")
        dims = (self.taper_dim,) + tuple(d for d in data.dims if d != self.taper_dim)
        shape = tuple(data.sizes[d] for d in dims)
        coords = {d: data.coords[d] for d in dims if d in data.coords}
        return dsmod.DataArray(_back(out.reshape(shape), host), dims, coords, data.attrs, data.name)


@register("tapered_model")
class TaperedModel(Predictor):
    """models.py:65-107: the base model's prediction with some outputs tapered."""

    _CONFIG_FILENAME = "tapered_model.yaml"

    def __init__(self, model, tapering: Mapping[str, TaperConfig]):
        for taper_var in tapering:
            if taper_var not in model.output_variables:
                raise KeyError(f"Tapered variable {taper_var} not in model output variables.")
        self.model = model
        self.tapering = tapering
        super().__init__(input_variables=tuple(sorted(model.input_variables)),
                         output_variables=tuple(sorted(model.output_variables)))

    @classmethod
    def load(cls, path: str) -> "TaperedModel":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        model = load(config["model"])
        tapering = {var: TaperConfig(**c) for var, c in config["tapering"].items()}
        return cls(model, tapering)

    def predict(self, X):
        output = self.model.predict(X)
        for taper_variable, taper_config in self.tapering.items():
            output[taper_variable] = taper_config.apply(output[taper_variable])
        return output

    def dump(self, path):
        raise NotImplementedError("no dump method yet for this class, you can define one manually "
                                  "(a tapered_model.yaml with the model path and tapering, and a name file)")


# ---------------------------------------------------------------------- ensemble
@register("ensemble")
class EnsembleModel(Predictor):
    """models.py:223-276: the members' outputs reduced over the member axis (mean or
    median, NaN-skipping as xarray's float reductions)."""

    _CONFIG_FILENAME = "ensemble_model.yaml"

    def __init__(self, models: Iterable[Predictor], reduction: str):
        self._models = tuple(models)
        if len(self._models) == 0:
            raise ValueError("at least one model must be given")
        if reduction.lower() not in ("mean", "median"):
            raise NotImplementedError(f"Got reduction {reduction}: only mean, median supported")
        if len(self._models) > 32:
            raise NotImplementedError("ensembles of more than 32 members are not supported by fv3_member_reduce")
        self._reduction = reduction
        inputs: Set = set()
        outputs: Set = set()
        first = set(self._models[0].output_variables)
        for model in self._models:
            if set(model.output_variables) != first:
                raise ValueError(f"all models in ensemble must have same outputs, got {first} and "
                                 f"{set(model.output_variables)}")
            inputs.update(model.input_variables)
            outputs.update(model.output_variables)
        super().__init__(input_variables=tuple(sorted(inputs)), output_variables=tuple(sorted(outputs)))

    @staticmethod
    def _reduce(members, reduction: str):
        """Device tensors of one shape -> their nanmean / nanmedian over the members
        (fv3_member_reduce), in the members' promoted float dtype."""
        _device.require_gpu()
        dtype = members[0].dtype
        for t in members[1:]:
            dtype = torch.promote_types(dtype, t.dtype)
        if dtype not in (torch.float32, torch.float64):
            dtype = torch.float64
        members = [t.to(dtype).contiguous() for t in members]
        for t in members[1:]:
            if t.shape != members[0].shape:
                raise ValueError(f"ensemble members disagree in shape: {tuple(t.shape)} vs {tuple(members[0].shape)}")
        op = _native.REDUCE_MEDIAN if reduction == "median" else _native.REDUCE_MEAN
        out = torch.empty_like(members[0])
        ptrs = (ctypes.c_void_p * len(members))(*[t.data_ptr() for t in members])
        st = _native.load().fv3_member_reduce(ptrs, len(members), out.numel(), int(dtype == torch.float64), op,
                                               out.data_ptr(), _device.stream_handle(None))
        _native.check(st, "member_reduce")
        return out

    def predict(self, X):
        outputs = [m.predict(X) for m in self._models]
        result = dsmod.Dataset()
        for name in outputs[0]:
            first = outputs[0][name]
            members, host = [], False
            for ds in outputs:
                da = ds[name]
                if tuple(da.dims) != tuple(first.dims):  # xr.concat aligns by dim name
                    da = da.transpose(*first.dims)
                t, h = _on_device(da.data)
                host = host or h
                members.append(t)
            out = self._reduce(members, self._reduction)
            result[name] = dsmod.DataArray(_back(out, host), first.dims, first.coords, first.attrs)
        return result

    def dump(self, path):
        raise NotImplementedError("no dump method yet for this class, you can define one manually "
                                  "(an ensemble_model.yaml with the member paths and reduction, and a name file)")

    @classmethod
    def load(cls, path: str) -> "EnsembleModel":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        return cls([load(p) for p in config["models"]], config["reduction"])
