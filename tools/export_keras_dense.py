#!/usr/bin/env python
"""Export a trained fv3fit DenseModel (a PureKerasModel directory: model.tf + config.yaml,
external/fv3fit/fv3fit/keras/_models/shared/pure_keras.py:60-77,120-135) to this package's
``mi355x-dense`` predictor directory (name file + config.yaml + dense/weights.npz +
dense/dense_config.yaml), which ``fv3net_amd.predictor.load`` runs on the fused kernel.

Run it where TensorFlow 2.8 and fv3fit are installed (they are not in this image):

    python tools/export_keras_dense.py MODEL_DIR OUT_DIR [--training-config TRAIN.yaml]

The graph of dense.py:234-305 is read layer by layer:
* StandardNormLayer (fv3fit/emulation/layers/normalization.py:121-139), one per input in
  input order: mean, sigma, epsilon;
* the hidden Dense layers in graph order, then ``dense_network_output_<i>`` per output
  (kernels [fan_in, fan_out], Keras' own layout);
* StandardDenormLayer per output: mean, sigma.
Clip slices and output limits live in the graph as tensor slicing / tf.where ops, so
they come from the training configuration (DenseHyperparameters ``clip_config`` /
``output_limit_config``, dense.py:39-106) when given.

``--dict TRAIN.yaml``: an ``all-keras-dict`` directory instead (``PureKerasDictPredictor``,
pure_keras.py:181-258: ``model.tf`` only), the microphysics emulator that
train_microphysics.py saves (emulation/models/microphysics.py:100-136).  Its structure
comes from the training configuration (inputs, LogTransform and Difference entries:
``fv3net_amd.emulator.features_outputs_from_config``), its numbers from the layers: the
``FieldInput`` norms (``normalized_<input>``), the ``MLPBlock`` Dense layers, the
``StandardOutput`` Dense per output (``standard_output_<name>``) and the ``FieldOutput``
denorms (``denormalized_<output>``, fields.py, architecture.py:228-333).  The result is
an ``mi355x-dense`` directory with input sources (raw variables in, after-states out)
that ``fv3net_amd.predictor.load`` runs on the bf16x3 kernel by default.

``write_predictor`` / ``write_emulator_predictor`` (the parts after the TF read) need no
TensorFlow and are unit-tested on synthetic arrays (tests/test_artifacts.py).
"""
import argparse
import os
import sys
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def write_predictor(out_dir: str, input_variables: Sequence[str], output_variables: Sequence[str],
                    in_nz: Sequence[int], out_nz: Sequence[int], params: Mapping[str, List[np.ndarray]],
                    epsilon: float = 1e-7, clip: Optional[Mapping[str, Tuple[int, int]]] = None,
                    output_limits: Optional[Mapping[str, Tuple[Optional[float], Optional[float]]]] = None):
    """Write the mi355x-dense predictor directory from Keras-layout arrays:
    params = hidden_kernels / hidden_biases / out_kernels / out_biases / in_mean /
    in_sigma (clipped lengths) / out_mean / out_sigma."""
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from fv3net_amd.predictor import DenseColumnPredictor, dump

    hk = [np.asarray(k, np.float32) for k in params["hidden_kernels"]]
    width = int(hk[0].shape[1])
    cfg = DenseModelConfig(list(input_variables), list(output_variables), [int(n) for n in in_nz],
                           [int(n) for n in out_nz], width=width, depth=len(hk) + 1, epsilon=float(epsilon),
                           clip={k: (v[0], v[1]) for k, v in (clip or {}).items()},
                           output_limits={k: (v[0], v[1]) for k, v in (output_limits or {}).items()})
    arrays = {k: [np.asarray(a, np.float32) for a in v] for k, v in params.items()}
    model = DenseColumnModel(cfg, arrays)  # validates every shape
    dump(DenseColumnPredictor(cfg.input_variables, cfg.output_variables, model), out_dir)
    return cfg


def write_emulator_predictor(out_dir: str, train_config: Mapping, out_nz: Mapping[str, int], nz: int,
                             params: Mapping[str, object], precision: str = "bf16x3"):
    """Write an all-keras-dict emulator as an ``mi355x-dense`` directory with input
    sources.  params: ``hidden_kernels`` / ``hidden_biases`` (MLPBlock order),
    ``in_center`` / ``in_scale`` keyed by model input name (NormLayer: (x - center) /
    scale; a scalar scale is broadcast over the levels), ``out_kernels`` /
    ``out_biases`` / ``out_center`` / ``out_scale`` keyed by direct output name."""
    from fv3net_amd.dense import DenseColumnModel
    from fv3net_amd.emulator import MicrophysicsEmulator, features_outputs_from_config
    from fv3net_amd.predictor import dump

    feats, outs = features_outputs_from_config(train_config, out_nz, nz)
    hk = [np.asarray(k, np.float32) for k in params["hidden_kernels"]]
    cfg = MicrophysicsEmulator.config(feats, outs, nz, width=int(hk[0].shape[1]), depth=len(hk))
    vec = lambda a, n: np.broadcast_to(np.asarray(a, np.float32), (n,)).copy()  # noqa: E731
    arrays = dict(
        hidden_kernels=hk, hidden_biases=[np.asarray(b, np.float32) for b in params["hidden_biases"]],
        in_mean=[vec(params["in_center"][f.name], nz) for f in feats],
        in_sigma=[vec(params["in_scale"][f.name], nz) for f in feats],
        out_kernels=[np.asarray(params["out_kernels"][o.name], np.float32) for o in outs],
        out_biases=[np.asarray(params["out_biases"][o.name], np.float32) for o in outs],
        out_mean=[vec(params["out_center"][o.name], o.nz) for o in outs],
        out_sigma=[vec(params["out_scale"][o.name], o.nz) for o in outs])
    emu = MicrophysicsEmulator(feats, outs, DenseColumnModel(cfg, arrays), precision=precision)
    pred = emu.predictor()
    dump(pred, out_dir)
    return pred


def read_keras_dict(model_dir: str, train_config: Mapping):  # pragma: no cover - needs TensorFlow
    """(out_nz, nz, params) of an all-keras-dict emulator, from its layers: the saved
    model is the TransformedModel around the inner Keras model (transformed_model.py:9-37),
    so every layer is searched for among the nested submodules."""
    import tensorflow as tf
    import fv3fit  # noqa: F401  registers the custom layers

    model = tf.keras.models.load_model(os.path.join(model_dir, "model.tf"), compile=False)
    subs = [m for m in model.submodules] + [model]
    kind = lambda k: [m for m in subs if type(m).__name__ == k]  # noqa: E731
    f_in = {m.name[len("processed_"):]: m for m in kind("FieldInput") if m.name.startswith("processed_")}
    f_out = {m.name: m for m in kind("FieldOutput")}
    mlp, std = kind("MLPBlock"), kind("StandardOutput")
    if len(mlp) != 1 or len(std) != 1:
        raise ValueError("expected one MLPBlock and one StandardOutput (the 'dense' architecture)")
    ins = (train_config.get("model") or {}).get("input_variables") or []
    outs = (train_config.get("model") or {}).get("direct_out_variables") or []
    params = {"hidden_kernels": [d.kernel.numpy() for d in mlp[0].dense],
              "hidden_biases": [d.bias.numpy() for d in mlp[0].dense],
              "in_center": {}, "in_scale": {}, "out_kernels": {}, "out_biases": {}, "out_center": {},
              "out_scale": {}}
    nz = None
    for name in ins:
        layer = f_in.get(name)
        if layer is None or layer.normalize is None or layer.selection is not None:
            raise ValueError(f"input {name!r}: a normalised FieldInput without a selection is expected")
        params["in_center"][name] = layer.normalize.center.numpy()
        params["in_scale"][name] = layer.normalize.scale.numpy()
        nz = nz or int(np.size(params["in_center"][name]))
    out_nz = {}
    for name in outs:
        dense = std[0].output_layers[name]
        params["out_kernels"][name], params["out_biases"][name] = dense.kernel.numpy(), dense.bias.numpy()
        norm = f_out[name].normalizer
        params["out_center"][name], params["out_scale"][name] = norm.center.numpy(), norm.scale.numpy()
        out_nz[name] = int(dense.kernel.shape[1])
    return out_nz, nz, params


def _training_limits(path: Optional[str]):
    if not path:
        return {}, {}
    with open(path) as f:
        hp = yaml.safe_load(f) or {}
    clip = {k: (v.get("start"), v.get("stop")) for k, v in (hp.get("clip_config", {}) or {}).get("clip", {}).items()}
    limits = {k: (v.get("min"), v.get("max"))
              for k, v in (hp.get("output_limit_config", {}) or {}).get("limits", {}).items()}
    return clip, limits


def read_keras(model_dir: str):  # pragma: no cover - needs TensorFlow
    import tensorflow as tf
    import fv3fit  # noqa: F401  registers the custom layers

    with open(os.path.join(model_dir, "config.yaml")) as f:
        config = yaml.safe_load(f)
    model = tf.keras.models.load_model(os.path.join(model_dir, "model.tf"), compile=False)
    norms = [l for l in model.layers if type(l).__name__ == "StandardNormLayer"]
    denorms = [l for l in model.layers if type(l).__name__ == "StandardDenormLayer"]
    dense = [l for l in model.layers if isinstance(l, tf.keras.layers.Dense)]
    outs = sorted([l for l in dense if l.name.startswith("dense_network_output_")],
                  key=lambda l: int(l.name.rsplit("_", 1)[1]))
    hidden = [l for l in dense if not l.name.startswith("dense_network_output_")]
    params = {
        "hidden_kernels": [l.kernel.numpy() for l in hidden], "hidden_biases": [l.bias.numpy() for l in hidden],
        "out_kernels": [l.kernel.numpy() for l in outs], "out_biases": [l.bias.numpy() for l in outs],
        "in_mean": [l.mean.numpy() for l in norms], "in_sigma": [l.sigma.numpy() for l in norms],
        "out_mean": [l.mean.numpy() for l in denorms], "out_sigma": [l.sigma.numpy() for l in denorms],
    }
    in_nz = [int(t.shape[-1]) for t in model.inputs]
    out_nz = [int(t.shape[-1]) for t in model.outputs]
    return config["input_variables"], config["output_variables"], in_nz, out_nz, params, float(norms[0].epsilon)


def main(argv=None):  # pragma: no cover - needs TensorFlow
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("model_dir")
    p.add_argument("out_dir")
    p.add_argument("--training-config", default=None)
    p.add_argument("--dict", default=None, metavar="TRAIN.yaml",
                   help="an all-keras-dict emulator directory, with its training configuration")
    a = p.parse_args(argv)
    if a.dict:
        with open(a.dict) as f:
            train_config = yaml.safe_load(f)
        out_nz, nz, params = read_keras_dict(a.model_dir, train_config)
        pred = write_emulator_predictor(a.out_dir, train_config, out_nz, nz, params)
        print(f"wrote {a.out_dir}: {pred.input_variables} -> {pred.output_variables}")
        return
    ins, outs, in_nz, out_nz, params, eps = read_keras(a.model_dir)
    clip, limits = _training_limits(a.training_config)
    cfg = write_predictor(a.out_dir, ins, outs, in_nz, out_nz, params, eps, clip, limits)
    print(f"wrote {a.out_dir}: {cfg.input_variables} -> {cfg.output_variables}, width {cfg.width}, "
          f"depth {cfg.depth}")


if __name__ == "__main__":
    main()
