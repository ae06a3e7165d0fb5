"""ORACLE (test infrastructure only): numpy restatement of the fv3fit DenseModel
predict graph and of the normalisation layers' fitting rules.

Reference (paths under /root/reference/external/fv3fit/fv3fit):
* graph: keras/_models/dense.py:234-305
    input clip             keras/_models/shared/clip.py:65-83 (clip_sequence)
    StandardNormLayer      emulation/layers/normalization.py:121-139  (x - mean) / (sigma + eps)
    concat                 keras/_models/shared/utils.py:65-86
    hidden Dense(relu)     keras/_models/shared/dense_network.py:59-76 (depth-1 layers)
    per-output Dense       dense.py:259-264
    StandardDenormLayer    normalization.py:142-149   y * sigma + mean
    OutputLimit            keras/_models/shared/output_limit.py:29-47
    zero mask              clip.py:33-46 (ClipConfig.zero_mask_clipped_layer)
* fitting: PerFeatureMean/PerFeatureStd (normalization.py:63-94): mean and
  POPULATION std over the sample axis, float32.

The Keras model runs in float32; ``dense_predict(..., dtype=np.float64)`` is the
high-precision reference the GPU kernel is checked against (tolerance written in
the tests), ``dtype=np.float32`` follows Keras' own precision.
"""
from typing import Dict, List, Sequence

import numpy as np


def fit_norm(array: np.ndarray):
    """mean and population std over all but the last axis, float32
    (PerFeatureMean._fit_mean / PerFeatureStd._fit_sigma)."""
    a = np.asarray(array, dtype=np.float32)
    axes = tuple(range(a.ndim - 1))
    return a.mean(axis=axes).astype(np.float32), a.std(axis=axes).astype(np.float32)


def standard_norm(x, mean, sigma, epsilon=1e-7, dtype=np.float32):
    """StandardNormLayer.call: (tensor - mean) / (sigma + epsilon)."""
    x = np.asarray(x, dtype)
    denom = (np.asarray(sigma, np.float32) + np.float32(epsilon)).astype(dtype)
    return (x - np.asarray(mean, dtype)) / denom


def standard_denorm(y, mean, sigma, dtype=np.float32):
    """StandardDenormLayer.call: tensor * sigma + mean."""
    return np.asarray(y, dtype) * np.asarray(sigma, dtype) + np.asarray(mean, dtype)


def output_limit(x, lo=None, hi=None):
    """OutputLimit._limit_activation (output_limit.py:29-47), NaN passes through."""
    out = np.array(x, copy=True)
    orig = np.asarray(x)
    if lo is not None:
        out = np.where(orig < lo, np.asarray(lo, out.dtype), out)
    if hi is not None:
        out = np.where(orig >= hi, np.asarray(hi, out.dtype), out)
    return out


def dense_predict(
    inputs: Sequence[np.ndarray],
    params: Dict,
    dtype=np.float64,
) -> List[np.ndarray]:
    """Predict with the DenseModel graph.

    ``inputs[v]``: ``[N, nz_v]`` sample-major arrays (what PureKerasModel.predict
    hands to Keras, pure_keras.py:111).  ``params`` keys:
      in_clip [(start, stop) per input], in_mean/in_sigma [per input, kept levels],
      epsilon, hidden_kernels [list of (fan_in, width)], hidden_biases,
      out_kernels [(width, nz_out) per output], out_biases, out_mean/out_sigma
      [per output], out_min/out_max [per output array or None], out_mask [per output or None].
    Returns ``[N, nz_out]`` arrays.
    """
    normed = []
    for v, x in enumerate(inputs):
        x = np.asarray(x)
        if x.ndim == 1:
            x = x[:, None]
        z0, z1 = params["in_clip"][v]
        normed.append(standard_norm(x[:, z0:z1], params["in_mean"][v], params["in_sigma"][v],
                                    params["epsilon"], dtype))
    h = np.concatenate(normed, axis=1)
    for w, b in zip(params["hidden_kernels"], params["hidden_biases"]):
        h = np.maximum(h @ np.asarray(w, dtype) + np.asarray(b, dtype), 0)
    outs = []
    for o, (w, b) in enumerate(zip(params["out_kernels"], params["out_biases"])):
        y = h @ np.asarray(w, dtype) + np.asarray(b, dtype)
        y = standard_denorm(y, params["out_mean"][o], params["out_sigma"][o], dtype)
        lo = params.get("out_min", [None] * len(params["out_kernels"]))[o]
        hi = params.get("out_max", [None] * len(params["out_kernels"]))[o]
        if lo is not None or hi is not None:
            y = output_limit(y, lo, hi)
        mask = params.get("out_mask", [None] * len(params["out_kernels"]))[o]
        if mask is not None:
            y = y * np.asarray(mask, dtype)
        outs.append(y)
    return outs


def predict_flops_per_column(k_in: int, width: int, n_hidden: int, k_out: int) -> int:
    """2*(k_in*w + (n_hidden-1)*w*w + w*k_out): the GEMM chain of dense.py:234-305."""
    return 2 * (k_in * width + (n_hidden - 1) * width * width + width * k_out)
