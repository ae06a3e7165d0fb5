"""PytorchPredictor artifacts (fv3fit.pytorch) on MI355X: ``scalers.zip`` and a
weights-only column MLP.

Reference (paths under /root/reference/external/fv3fit/fv3fit):
* ``dump_mapping`` / ``load_mapping`` — scalers.zip, one StandardScaler npz per
  variable                                        pytorch/predict.py:40-57
* ``PytorchPredictor`` ("pytorch_predictor")       pytorch/predict.py:60-120, 274-387:
  pack = per input variable (x - mean) / std in float64, rounded to float32 and
  concatenated along the feature axis (2-D variables add one feature) -> the model ->
  unpack = per output variable the next len(mean) features, y * std + mean in float64.

The reference saves the whole ``nn.Module`` with ``torch.save`` (a pickle).  Pickles are
not loaded here: ``weight.pt`` must hold a state dict (``torch.save(model.state_dict())``,
read with ``torch.load(weights_only=True)``) of a column MLP, an ``nn.Sequential`` of
``Linear`` layers with ReLU between them (equal hidden widths).  Such a model runs on the
fused dense kernel: the scalers' float64 normalisation (csrc/scaler.hip) into a
[feature, column] buffer, the MLP with identity normalisation (csrc/dense.hip), the
float64 denormalisation per output variable.
"""
import os
import re
import zipfile
from typing import IO, Dict, Hashable, Iterable, Mapping, Sequence

import numpy as np
import yaml

from . import dataset as dsmod
from .dense import DenseColumnModel, DenseModelConfig
from .normalization import StandardScaler
from .predictor import Predictor, register

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def dump_mapping(mapping: Mapping[str, StandardScaler], f: IO[bytes]) -> None:
    """predict.py:40-47: a zip with one member per variable, each a scaler npz."""
    with zipfile.ZipFile(f, "w") as archive:
        for key, value in mapping.items():
            with archive.open(str(key), "w") as member:
                value.dump(member)


def load_mapping(cls, f: IO[bytes]) -> Dict[str, StandardScaler]:
    """predict.py:50-56."""
    with zipfile.ZipFile(f, "r") as archive:
        return {name: cls.load(archive.open(name, "r")) for name in archive.namelist()}


def _linear_layers(state_dict: Mapping[str, object]):
    """(weight, bias) of the Linear layers of an nn.Sequential state dict, in order."""
    idx = sorted({int(m.group(1)) for k in state_dict for m in [re.fullmatch(r"(?:.*\.)?(\d+)\.weight", k)] if m})
    if not idx:
        raise ValueError("weight.pt: no '<i>.weight' entries (an nn.Sequential of Linear layers is expected)")
    prefix = next(k for k in state_dict if k.endswith(f"{idx[0]}.weight"))[: -len(f"{idx[0]}.weight")]
    layers = []
    for i in idx:
        w = np.asarray(state_dict[f"{prefix}{i}.weight"].cpu().numpy() if hasattr(state_dict[f"{prefix}{i}.weight"], "cpu")
                       else state_dict[f"{prefix}{i}.weight"], dtype=np.float32)
        bkey = f"{prefix}{i}.bias"
        b = state_dict.get(bkey)
        b = np.zeros(w.shape[0], np.float32) if b is None else np.asarray(
            b.cpu().numpy() if hasattr(b, "cpu") else b, dtype=np.float32)
        if w.ndim != 2:
            raise ValueError(f"layer {i}: weight of shape {w.shape} is not a Linear layer")
        layers.append((w, b))
    return layers


class ColumnMLP:
    """A Linear/ReLU column MLP mapped onto the fused dense kernel (identity
    normalisation: the scalers run as their own float64 kernels)."""

    def __init__(self, state_dict: Mapping[str, object], in_features: int, out_features: Sequence[int]):
        layers = _linear_layers(state_dict)
        if len(layers) < 2:
            raise NotImplementedError("a column MLP needs at least one hidden layer")
        widths = {w.shape[0] for w, _ in layers[:-1]}
        if len(widths) != 1:
            raise NotImplementedError(f"hidden layers of different widths {sorted(widths)} are not supported")
        width = widths.pop()
        if layers[0][0].shape[1] != in_features:
            raise ValueError(f"the first Linear takes {layers[0][0].shape[1]} features, the scalers give {in_features}")
        if layers[-1][0].shape[0] != sum(out_features):
            raise ValueError(f"the last Linear gives {layers[-1][0].shape[0]} features, the scalers take "
                             f"{sum(out_features)}")
        self.state_dict = {k: (v.detach().cpu() if torch.is_tensor(v) else torch.as_tensor(np.asarray(v)))
                           for k, v in state_dict.items()}
        names = [f"y{i}" for i in range(len(out_features))]
        cfg = DenseModelConfig(["packed"], names, [in_features], list(out_features), width=width,
                               depth=len(layers), epsilon=0.0)
        w_last, b_last = layers[-1]
        offs = np.cumsum([0] + list(out_features))
        params = dict(
            hidden_kernels=[np.ascontiguousarray(w.T) for w, _ in layers[:-1]],  # torch (out, in) -> (in, out)
            hidden_biases=[b for _, b in layers[:-1]],
            out_kernels=[np.ascontiguousarray(w_last[offs[o]:offs[o + 1]].T) for o in range(len(out_features))],
            out_biases=[b_last[offs[o]:offs[o + 1]] for o in range(len(out_features))],
            in_mean=[np.zeros(in_features, np.float32)], in_sigma=[np.ones(in_features, np.float32)],
            out_mean=[np.zeros(n, np.float32) for n in out_features],
            out_sigma=[np.ones(n, np.float32) for n in out_features],
        )
        self.dense = DenseColumnModel(cfg, params)


@register("pytorch_predictor")
class PytorchColumnPredictor(Predictor):
    """PytorchPredictor (pytorch/predict.py:60-120) for column MLPs, on device."""

    _MODEL_FILENAME = "weight.pt"
    _CONFIG_FILENAME = "config.yaml"
    _SCALERS_FILENAME = "scalers.zip"

    def __init__(self, input_variables: Iterable[Hashable], output_variables: Iterable[Hashable], model: ColumnMLP,
                 scalers: Mapping[str, StandardScaler]):
        super().__init__(input_variables, output_variables)
        self.input_variables = list(input_variables)
        self.output_variables = list(output_variables)
        self.model = model
        self.scalers = dict(scalers)

    @staticmethod
    def n_features(scaler: StandardScaler) -> int:
        """_unpack_tensor (predict.py:386-392): len(mean) features, 1 for a scalar."""
        if scaler.mean is None:
            raise RuntimeError("scaler has not been fit")
        m = np.asarray(scaler.mean)
        return int(m.shape[0]) if m.ndim > 0 and m.shape[0] > 1 else 1

    @classmethod
    def from_state_dict(cls, input_variables, output_variables, state_dict, scalers):
        n_in = sum(cls.n_features(scalers[v]) for v in input_variables)
        n_out = [cls.n_features(scalers[v]) for v in output_variables]
        return cls(input_variables, output_variables, ColumnMLP(state_dict, n_in, n_out), scalers)

    def predict(self, X):
        """(time, tile, x, y[, z]) variables -> outputs on the same columns, dims in the
        reference's unpack order (time, tile, x, y, z) restricted to those present."""
        expected = [d for d in ("time", "tile", "x", "y") if d in dsmod.dataset_dims(X)]
        col_shape = None
        offs = 0
        pieces = []
        for name in self.input_variables:
            da = X[name]
            dims = tuple(da.dims)
            data = dsmod.variable_data(X, name)
            t = data if torch.is_tensor(data) else torch.from_numpy(np.ascontiguousarray(np.asarray(data)))
            order = expected + (["z"] if "z" in dims else [])
            if sorted(dims) != sorted(order):
                raise ValueError(f"received variable {name} with unexpected dimensions {dims}")
            t = t.permute(*[dims.index(d) for d in order])
            shape = tuple(t.shape[:len(expected)])
            if col_shape is None:
                col_shape = shape
            elif shape != col_shape:
                raise ValueError(f"{name}: columns {shape} != {col_shape}")
            pieces.append((name, t))
        ncol = int(np.prod(col_shape)) if col_shape else 1
        n_in = self.model.dense.config.in_nz[0]
        dev = torch.device("cuda", torch.cuda.current_device())
        buf = torch.empty((n_in, ncol), dtype=torch.float32, device=dev)
        for name, t in pieces:
            nf = self.n_features(self.scalers[name])
            scalar = np.ndim(self.scalers[name].mean) == 0
            x = t.reshape(ncol) if scalar else t.reshape(ncol, -1)  # [column(, feature)]
            if (1 if scalar else x.shape[1]) != nf:
                raise ValueError(f"{name} has {x.shape[1]} features, its scaler {nf}")
            # float32((x - mean) / std) written straight into the packed [feature, column] rows
            self.scalers[name].normalize(x.to(dev), out_f32=True, out=buf[offs:offs + nf].T)
            offs += nf
        outs = self.model.dense.forward([buf], level_axes=[0])
        result = {}
        for name, y in zip(self.output_variables, outs):
            nf = self.n_features(self.scalers[name])
            val = self.scalers[name].denormalize(y, feature_axis=0)  # [feature, column] float64
            if nf == 1:  # a 2-D variable (predict.py:391-393)
                data, dims = val.reshape(col_shape), list(expected)
            else:
                data, dims = val.T.reshape(tuple(col_shape) + (nf,)), list(expected) + ["z"]
            result[name] = dsmod.DataArray(data, dims)
        return dsmod.Dataset(result)

    # -- persistence ----------------------------------------------------------------------
    def dump(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        torch.save(self.model.state_dict, os.path.join(path, self._MODEL_FILENAME))
        with open(os.path.join(path, self._SCALERS_FILENAME), "wb") as f:
            dump_mapping(self.scalers, f)
        with open(os.path.join(path, self._CONFIG_FILENAME), "w") as f:
            yaml.safe_dump({"input_variables": list(self.input_variables),
                            "output_variables": list(self.output_variables)}, f)

    @classmethod
    def load(cls, path: str) -> "PytorchColumnPredictor":
        try:
            state = torch.load(os.path.join(path, cls._MODEL_FILENAME), map_location="cpu", weights_only=True)
        except Exception as e:  # a pickled nn.Module is refused by weights_only
            raise ValueError(f"{path}/{cls._MODEL_FILENAME} is not a weights-only state dict ({e}); re-save it "
                             "with torch.save(model.state_dict(), ...) where the model class is importable") from e
        if not isinstance(state, Mapping):
            raise ValueError(f"{path}/{cls._MODEL_FILENAME} holds a {type(state).__name__}, not a state dict")
        with open(os.path.join(path, cls._SCALERS_FILENAME), "rb") as f:
            scalers = load_mapping(StandardScaler, f)
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        return cls.from_state_dict(config["input_variables"], config["output_variables"], state, scalers)
