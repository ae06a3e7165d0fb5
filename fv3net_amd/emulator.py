"""The Zhao-Carr microphysics emulator (BASELINE config #5) on MI355X.

The inference graph of the trained emulator
(projects/microphysics/train/dense.yaml:12-94, built by
external/fv3fit/fv3fit/emulation/models/microphysics.py:100-136 and wrapped by
transformed_model.py:9-37) is one fused dense kernel (csrc/dense.hip):

    inputs sorted by name (architecture.py:27-50), 3 of them LogTransform'ed
    log(max(x, eps)) (transforms.py:111-129) -> NormLayer (x - center) / scale
    (normalization2.py:20-24) -> 2 x Dense(256, relu) (MLPBlock, architecture.py:228-272)
    -> one Dense per output (StandardOutput, :296-333) -> y * scale + center
    (FieldOutput, fields.py:44-66) -> after = before + difference (Difference.backward,
    transforms.py:55-58)

Inputs are read in place from the Fortran state layout [feature, sample] (the
hook's state dict, _emulate/microphysics.py:83-101), which is the kernel's
[level][column] layout: no transposes.

Precision: ``"bf16x3"`` (the default, csrc/dense_b3.hip) runs every product on bf16
MFMA with each f32 operand split into hi + lo (3 MFMAs per product, ~1e-5 against the
float64 graph); ``"bf16x6"`` splits into hi + mid + lo (6 MFMAs per product, f32-level
error); ``"f32"`` runs exact-f32 MFMA (csrc/dense.hip, ~1e-6).  Config #5's contract is
1e-3 rel; the tests hold bf16x3 to 1e-4 and bf16x6 / f32 to 1e-5 per level.
"""
import dataclasses
from typing import Callable, Dict, List, Mapping, Optional

import numpy as np

from .dense import DenseColumnModel, DenseModelConfig, _glorot

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


@dataclasses.dataclass(frozen=True)
class EmulatorFeature:
    name: str
    source: str
    log_eps: Optional[float] = None


@dataclasses.dataclass(frozen=True)
class EmulatorOutput:
    name: str          # the model's output (a direct output or a difference)
    nz: int
    residual_of: Optional[str] = None  # raw input `before` of a Difference transform
    after: Optional[str] = None        # name of `before + difference`


def zhao_carr_features() -> List[EmulatorFeature]:
    """dense.yaml input_variables + tensor_transform log entries, sorted by name
    (combine_inputs concatenates in sorted-key order)."""
    feats = [
        EmulatorFeature("air_temperature_input", "air_temperature_input"),
        EmulatorFeature("specific_humidity_input", "specific_humidity_input"),
        EmulatorFeature("cloud_water_mixing_ratio_input", "cloud_water_mixing_ratio_input"),
        EmulatorFeature("log_cloud_input", "cloud_water_mixing_ratio_input", 1e-10),
        EmulatorFeature("log_humidity_input", "specific_humidity_input", 1e-8),
        EmulatorFeature("pressure_thickness_of_atmospheric_layer", "pressure_thickness_of_atmospheric_layer"),
        EmulatorFeature("air_temperature_after_last_gscond", "air_temperature_after_last_gscond"),
        EmulatorFeature("specific_humidity_after_last_gscond", "specific_humidity_after_last_gscond"),
        EmulatorFeature("log_humidity_after_last_gscond", "specific_humidity_after_last_gscond", 1e-8),
    ]
    return sorted(feats, key=lambda f: f.name)


def zhao_carr_outputs(nz: int = 79) -> List[EmulatorOutput]:
    """dense.yaml direct_out_variables with the Difference transforms that turn them
    into after-states (tensor_transform entries with before/after)."""
    return [
        EmulatorOutput("total_precipitation", 1),
        EmulatorOutput("cloud_precpd_difference", nz, "cloud_water_mixing_ratio_input",
                       "cloud_water_mixing_ratio_after_precpd"),
        EmulatorOutput("temperature_precpd_difference", nz, "air_temperature_input", "air_temperature_after_precpd"),
        EmulatorOutput("humidity_precpd_difference", nz, "specific_humidity_input", "specific_humidity_after_precpd"),
        EmulatorOutput("temperature_gscond_difference", nz, "air_temperature_input", "air_temperature_after_gscond"),
        EmulatorOutput("humidity_gscond_difference", nz, "specific_humidity_input", "specific_humidity_after_gscond"),
    ]


def features_outputs_from_config(train_config: Mapping, out_nz: Mapping[str, int], nz: int = 79):
    """(features, outputs) of a microphysics training configuration
    (fv3fit/train_microphysics.py's ``TrainConfig``, e.g. projects/microphysics/train/
    dense.yaml, read with yaml.safe_load): ``model.input_variables`` sorted by name (the
    order combine_inputs concatenates them, architecture.py:27-50), each a raw variable
    or the ``to`` of a ``tensor_transform`` LogTransform entry (``source``,
    ``transform.epsilon``); ``model.direct_out_variables`` in order, each a direct output
    or the ``to`` of a Difference entry (``before`` / ``after``: the kernel adds the raw
    ``before`` and names the result ``after``).  ``out_nz``: levels per direct output (1
    for a surface field such as total_precipitation; default ``nz``)."""
    transforms = {t["to"]: t for t in (train_config.get("tensor_transform") or [])}
    model = train_config.get("model") or {}
    feats = []
    for name in model.get("input_variables") or []:
        t = transforms.get(name)
        if t is not None and "source" in t:
            eps = float((t.get("transform") or {}).get("epsilon", 1e-30))
            feats.append(EmulatorFeature(name, t["source"], eps))
        elif t is not None:
            raise NotImplementedError(f"input {name!r}: only LogTransform inputs are supported")
        else:
            feats.append(EmulatorFeature(name, name))
    outs = []
    for name in model.get("direct_out_variables") or []:
        t = transforms.get(name)
        n = int(out_nz.get(name, nz))
        if t is not None and "before" in t:
            outs.append(EmulatorOutput(name, n, t["before"], t["after"]))
        elif t is not None:
            raise NotImplementedError(f"output {name!r}: only Difference transforms are supported")
        else:
            outs.append(EmulatorOutput(name, n))
    return sorted(feats, key=lambda f: f.name), outs


def fit_center_per_feature(x) -> np.ndarray:
    """MeanMethod.per_feature (normalization2.py:75-77), float32."""
    x = np.asarray(x)
    return x.astype(np.float64).mean(axis=0).astype(np.float32)


def fit_scale_all(x) -> np.float32:
    """StdDevMethod.all (normalization2.py:62-72): one std over samples and features
    around the per-feature mean."""
    x = np.asarray(x, np.float64)
    return np.float32(np.sqrt(((x - x.mean(axis=0)) ** 2).mean()))


class MicrophysicsEmulator:
    """A dense microphysics emulator on the fused HIP kernel.

    ``__call__(state)``: state maps raw input names to [nz, ncol] (Fortran
    [feature, sample]) arrays; returns the after-states and direct outputs as
    [nz, ncol] / [ncol] float32 device tensors.

    ``precision`` (None keeps the model's): "bf16x3" runs the MLP on bf16 MFMA with a
    3-term split (BASELINE config #5: bf16 MFMA, 1e-3 rel), "f32" on exact f32 MFMA.
    """

    def __init__(self, features: List[EmulatorFeature], outputs: List[EmulatorOutput], model: DenseColumnModel,
                 precision: Optional[str] = None):
        self.features = list(features)
        self.outputs = list(outputs)
        self.model = model
        if precision is not None:
            model.precision = precision

    @property
    def raw_inputs(self) -> List[str]:
        seen = []
        for f in self.features:
            if f.source not in seen:
                seen.append(f.source)
        return seen

    @staticmethod
    def config(features, outputs, nz: int = 79, width: int = 256, depth: int = 2) -> DenseModelConfig:
        out_names = [o.after or o.name for o in outputs]
        return DenseModelConfig(
            input_variables=[f.name for f in features],
            output_variables=out_names,
            in_nz=[nz] * len(features),
            out_nz=[o.nz for o in outputs],
            width=width,
            depth=depth + 1,  # MLPBlock depth = hidden layers; DenseModelConfig counts the output layer
            epsilon=0.0,      # NormLayer: (x - center) / scale
            input_log_eps={f.name: float(f.log_eps) for f in features if f.log_eps},
            output_residuals={(o.after or o.name): next(f.name for f in features if f.source == o.residual_of)
                              for o in outputs if o.residual_of},
        )

    @classmethod
    def random(cls, sample_raw: Mapping[str, np.ndarray], sample_out: Mapping[str, np.ndarray],
               features: Optional[List[EmulatorFeature]] = None, outputs: Optional[List[EmulatorOutput]] = None,
               width: int = 256, depth: int = 2, seed: int = 0,
               precision: str = "bf16x3") -> "MicrophysicsEmulator":
        """Glorot-initialised weights, normalisation fitted like MicrophysicsConfig.build
        on a sample: raw inputs [ncol, nz] per name, model outputs (differences and
        direct outputs) [ncol, nz] per output name."""
        features = features or zhao_carr_features()
        outputs = outputs or zhao_carr_outputs(next(iter(sample_raw.values())).shape[-1])
        nz = next(iter(sample_raw.values())).shape[-1]
        cfg = cls.config(features, outputs, nz, width, depth)
        rng = np.random.default_rng(seed)
        in_mean, in_sigma = [], []
        for f in features:
            x = np.asarray(sample_raw[f.source], np.float32)
            if f.log_eps:
                x = np.log(np.maximum(x, np.float32(f.log_eps)))
            in_mean.append(fit_center_per_feature(x))
            in_sigma.append(np.full(nz, fit_scale_all(x), np.float32))
        out_mean, out_sigma = [], []
        for o in outputs:
            y = np.asarray(sample_out[o.name], np.float32).reshape(-1, o.nz)
            out_mean.append(fit_center_per_feature(y))
            out_sigma.append(np.full(o.nz, fit_scale_all(y), np.float32))
        k_in = nz * len(features)
        hk, hb = [], []
        fan_in = k_in
        for _ in range(depth):
            hk.append(_glorot(rng, fan_in, width))
            hb.append(np.zeros(width, np.float32))
            fan_in = width
        params = dict(hidden_kernels=hk, hidden_biases=hb,
                      out_kernels=[_glorot(rng, width, o.nz) for o in outputs],
                      out_biases=[np.zeros(o.nz, np.float32) for o in outputs],
                      out_mean=out_mean, out_sigma=out_sigma, in_mean=in_mean, in_sigma=in_sigma)
        return cls(features, outputs, DenseColumnModel(cfg, params), precision=precision)

    def predictor(self):
        """This emulator as a registered predictor: the drop-in for the reference's
        ``all-keras-dict`` emulator model (``PureKerasDictPredictor``,
        pure_keras.py:181-258): raw variables in, after-states and direct outputs out,
        ``predict`` on (z, ...) datasets, ``dump`` / ``load`` through the registry
        (``mi355x-dense`` with input sources, its precision kept)."""
        from .predictor import DenseColumnPredictor

        return DenseColumnPredictor(self.raw_inputs, [o.after or o.name for o in self.outputs], self.model,
                                    input_sources=[f.source for f in self.features])

    @classmethod
    def from_predictor(cls, pred) -> "MicrophysicsEmulator":
        """The emulator behind a loaded ``predictor()`` (its outputs named by their
        after-state, the name the kernel writes)."""
        cfg = pred.model.config
        sources = dict(zip(cfg.input_variables, pred._sources))
        feats = [EmulatorFeature(n, sources[n], cfg.input_log_eps.get(n)) for n in cfg.input_variables]
        outs = []
        for name, nz in zip(cfg.output_variables, cfg.out_nz):
            r = cfg.output_residuals.get(name)
            outs.append(EmulatorOutput(name, nz, sources[r], name) if r else EmulatorOutput(name, nz))
        return cls(feats, outs, pred.model)

    def params_by_name(self) -> dict:
        """Weights/normalisations keyed like the oracle (tests)."""
        p = self.model.params
        return {
            "in_center": {f.name: p["in_mean"][i] for i, f in enumerate(self.features)},
            "in_scale": {f.name: p["in_sigma"][i][0] for i, f in enumerate(self.features)},
            "hidden_kernels": p["hidden_kernels"], "hidden_biases": p["hidden_biases"],
            "out_kernels": {o.name: p["out_kernels"][i] for i, o in enumerate(self.outputs)},
            "out_biases": {o.name: p["out_biases"][i] for i, o in enumerate(self.outputs)},
            "out_center": {o.name: p["out_mean"][i] for i, o in enumerate(self.outputs)},
            "out_scale": {o.name: p["out_sigma"][i][0] for i, o in enumerate(self.outputs)},
        }

    def __call__(self, state: Mapping[str, object], out: Optional[Dict[str, object]] = None, stream=None):
        missing = [n for n in self.raw_inputs if n not in state]
        if missing:
            raise KeyError(f"emulator inputs missing from the state: {missing}")
        xs = [state[f.source] for f in self.features]  # the same array feeds a log and a raw feature
        outs = None if out is None else [out[o.after or o.name] for o in self.outputs]
        res = self.model.forward(xs, level_axes=[0] * len(xs), outputs=outs, out_level_axis=0, stream=stream)
        result = {}
        for o, t in zip(self.outputs, res):
            result[o.after or o.name] = t[0] if o.nz == 1 else t
        return result


class MicrophysicsHook:
    """external/emulation/emulation/_emulate/microphysics.py:48-101: apply the emulator
    to the Fortran state dict in place.  Arrays are [feature, sample] (the Fortran
    order) and are used as they are — the reference transposes to [sample, feature]
    for Keras and back."""

    def __init__(self, model: Callable, mask: Optional[Callable] = None):
        self.name = "microphysics emulator"
        self.model = model
        self.mask = mask or (lambda state, emulator: emulator)

    def microphysics(self, state: Dict[str, object]) -> None:
        predictions = self.model(state)
        predictions.update(self.mask(state, predictions))
        state.update(predictions)
