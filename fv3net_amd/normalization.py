"""Normalisation parameter objects (host-side containers; the arithmetic that
uses them on the hot path runs inside the HIP kernels).

* ``fit_mean_std`` — PerFeatureMean / PerFeatureStd fitting
  (external/fv3fit/fv3fit/emulation/layers/normalization.py:63-94): mean and
  population std over the sample axes, float32.
* ``StandardScaler`` — external/fv3fit/fv3fit/_shared/scaler.py:36-100: float64
  mean, std = np.std + std_epsilon (1e-12), npz dump/load, RuntimeError when
  used unfitted.  ``as_norm_layer()`` hands (mean, std) to a dense model as a
  StandardNormLayer with epsilon 0, i.e. (x - mean) / std.
"""
from typing import IO, Optional

import numpy as np


def fit_mean_std(array):
    a = np.asarray(array, dtype=np.float32)
    axes = tuple(range(a.ndim - 1))
    return a.mean(axis=axes).astype(np.float32), a.std(axis=axes).astype(np.float32)


class StandardScaler:
    kind: str = "standard"

    def __init__(self, std_epsilon: np.float64 = 1e-12, n_sample_dims: int = 1):
        self.mean: Optional[np.ndarray] = None
        self.std: Optional[np.ndarray] = None
        self.std_epsilon = std_epsilon
        self._n_sample_dims = n_sample_dims

    def fit(self, data: np.ndarray):
        axes = tuple(range(self._n_sample_dims))
        self.mean = np.mean(data, axis=axes).astype(np.float64)
        self.std = np.std(data, axis=axes).astype(np.float64) + self.std_epsilon

    def _require(self, what):
        if self.mean is None or self.std is None:
            raise RuntimeError(f"StandardScaler.fit must be called before {what}.")

    def normalize(self, data):
        self._require("normalize")
        return (data - self.mean) / self.std

    def denormalize(self, data):
        self._require("denormalize")
        return data * self.std + self.mean

    def as_norm_layer(self):
        """(mean, sigma, epsilon) for a StandardNorm stage computing (x-mean)/std."""
        self._require("as_norm_layer")
        return self.mean.astype(np.float32), self.std.astype(np.float32), 0.0

    def __eq__(self, other) -> bool:
        if not isinstance(other, StandardScaler):
            return False
        return (np.all(self.mean == other.mean) and np.all(self.std == other.std)
                and self.std_epsilon == other.std_epsilon
                and self._n_sample_dims == other._n_sample_dims)

    def dump(self, f: IO[bytes]):
        data = {}
        if self.mean is not None:
            data["mean"] = self.mean
        if self.std is not None:
            data["std"] = self.std
        return np.savez(f, **data)

    @classmethod
    def load(cls, f: IO[bytes]):
        data = np.load(f, allow_pickle=False)
        scaler = cls()
        scaler.mean = data.get("mean")
        scaler.std = data.get("std")
        return scaler
