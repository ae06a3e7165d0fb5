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

``write_predictor`` (the part after the TF read) needs no TensorFlow and is unit-tested
on synthetic arrays (tests/test_artifacts.py).
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
    a = p.parse_args(argv)
    ins, outs, in_nz, out_nz, params, eps = read_keras(a.model_dir)
    clip, limits = _training_limits(a.training_config)
    cfg = write_predictor(a.out_dir, ins, outs, in_nz, out_nz, params, eps, clip, limits)
    print(f"wrote {a.out_dir}: {cfg.input_variables} -> {cfg.output_variables}, width {cfg.width}, "
          f"depth {cfg.depth}")


if __name__ == "__main__":
    main()
