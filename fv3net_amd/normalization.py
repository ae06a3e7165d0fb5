"""Normalisation objects around the column models.

* ``fit_mean_std`` — PerFeatureMean / PerFeatureStd fitting
  (external/fv3fit/fv3fit/emulation/layers/normalization.py:63-94): mean and population
  std over the sample axes, float32 (training-time statistics of a synthetic or
  exported model; not on the hot path).
* ``StandardScaler`` — the fv3fit scaler (external/fv3fit/fv3fit/_shared/scaler.py:36-100)
  with the same file format (an npz holding ``mean`` and ``std``) and semantics:
  float64 statistics, std = population std + ``std_epsilon`` (1e-12), RuntimeError when
  used unfitted.  ``fit`` runs on the host (training); ``normalize`` / ``denormalize``
  run on the GPU (csrc/scaler.hip, float64 arithmetic identical to numpy's), and hand
  back the kind of array they were given (float64).
"""
from typing import IO, Optional

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def fit_mean_std(array):
    a = np.asarray(array, dtype=np.float32)
    axes = tuple(range(a.ndim - 1))
    return a.mean(axis=axes).astype(np.float32), a.std(axis=axes).astype(np.float32)


class StandardScaler:
    """(x - mean) / std and y * std + mean per feature, in float64."""

    kind: str = "standard"

    def __init__(self, std_epsilon: np.float64 = 1e-12, n_sample_dims: int = 1):
        self.std_epsilon = std_epsilon
        self._n_sample_dims = n_sample_dims
        self.mean: Optional[np.ndarray] = None
        self.std: Optional[np.ndarray] = None
        self._device_stats = {}

    # -- statistics ---------------------------------------------------------------------
    def fit(self, data: np.ndarray):
        """Population mean / std over the leading ``n_sample_dims`` axes (host)."""
        x = np.asarray(data)
        sample_axes = tuple(range(self._n_sample_dims))
        self.mean = np.asarray(np.mean(x, axis=sample_axes), dtype=np.float64)
        self.std = np.asarray(np.std(x, axis=sample_axes), dtype=np.float64) + self.std_epsilon
        self._device_stats = {}

    def _stats(self, what: str):
        if self.mean is None or self.std is None:
            raise RuntimeError(f"StandardScaler.fit must be called before {what}.")
        return np.asarray(self.mean, np.float64), np.asarray(self.std, np.float64)

    def _on_device(self, dev):
        """Device copies of mean / std, keyed on their current values: the reference's
        load assigns the attributes directly (scaler.py:86-100), and a reassigned or
        edited statistic must never be served from a stale copy (a few hundred bytes
        compared per call)."""
        m, s = self._stats("use")
        key = (m.shape, s.shape, m.tobytes(), s.tobytes())
        hit = self._device_stats.get(str(dev))
        if hit is None or hit[0] != key:
            hit = (key, torch.as_tensor(np.ascontiguousarray(m.ravel()), device=dev),
                   torch.as_tensor(np.ascontiguousarray(s.ravel()), device=dev))
            self._device_stats[str(dev)] = hit
        return hit[1], hit[2]

    # -- device arithmetic ----------------------------------------------------------------
    def _apply(self, data, forward: bool, feature_axis: Optional[int], out_f32: bool = False, out=None):
        from . import _device, _native

        mean, _ = self._stats("normalize" if forward else "denormalize")
        _device.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        is_torch = torch.is_tensor(data)
        src = data if is_torch else torch.from_numpy(np.ascontiguousarray(np.asarray(data)))
        nfeat = int(mean.size)
        if feature_axis is None:  # the reference's layout: sample axes first, features last
            lead = src.shape[:src.dim() - mean.ndim] if mean.ndim else src.shape
            if mean.ndim and tuple(src.shape[src.dim() - mean.ndim:]) != tuple(mean.shape):
                raise ValueError(f"data shape {tuple(src.shape)} does not end in the scaler's {mean.shape}")
            x = src.reshape(tuple(lead) + (nfeat,) if mean.ndim else tuple(lead) + (1,))
            axis = x.dim() - 1
        else:
            x = src
            axis = feature_axis % x.dim()
            if nfeat != 1 and x.shape[axis] != nfeat:
                raise ValueError(f"axis {feature_axis} holds {x.shape[axis]} features, the scaler {nfeat}")
        if x.dtype not in (torch.float32, torch.float64):
            x = x.to(torch.float64)
        x = x.to(dev)
        in64 = x.dtype == torch.float64
        x, lay, ncol, nz = _device.column_view(x, axis, keep_f64=True)
        odt = torch.float32 if (forward and out_f32) else torch.float64
        if out is None:
            res = torch.empty(x.shape, dtype=odt, device=dev)
        else:  # a caller's view (e.g. rows of a packed [feature, column] buffer)
            res = out
            if not (torch.is_tensor(out) and out.is_cuda and out.dtype == odt and tuple(out.shape) == tuple(x.shape)):
                raise ValueError(f"out must be a {odt} CUDA tensor of shape {tuple(x.shape)}")
        olay, _, _ = _device.level_layout(res, axis)
        m, s = self._on_device(dev)
        lib = _native.load()
        sh = _device.stream_handle(None)
        if forward:
            fn = lib.fv3_standard_normalize if out_f32 else lib.fv3_standard_normalize_f64
            st = fn(x.data_ptr(), int(in64), lay, m.data_ptr(), s.data_ptr(), m.numel(), res.data_ptr(), olay, ncol,
                    nz, sh)
        else:
            fn = lib.fv3_standard_denormalize_f64 if in64 else lib.fv3_standard_denormalize
            st = fn(x.data_ptr(), lay, m.data_ptr(), s.data_ptr(), m.numel(), res.data_ptr(), olay, ncol, nz, sh)
        _native.check(st, "standard_normalize" if forward else "standard_denormalize")
        if out is not None:
            return out
        res = res.reshape(src.shape)
        return res if is_torch else res.cpu().numpy()

    def normalize(self, data, feature_axis: Optional[int] = None, out_f32: bool = False, out=None):
        """(data - mean) / std in float64 (scaler.py:65-68).  ``out_f32``: rounded to
        float32 in the same pass, as the PytorchPredictor packs (predict.py:371-375).
        Features on the trailing axes like the reference, or on ``feature_axis`` (e.g. 0
        for a [level, column] state read in place).  ``out``: a device view to write
        (shaped like the data with the features flattened)."""
        return self._apply(data, True, feature_axis, out_f32, out)

    def denormalize(self, data, feature_axis: Optional[int] = None):
        """data * std + mean in float64 (scaler.py:70-73; the model's float32 output is
        promoted, predict.py:378-399)."""
        return self._apply(data, False, feature_axis)

    def as_norm_layer(self):
        """(mean, sigma, epsilon) for a StandardNorm stage computing (x-mean)/std."""
        m, s = self._stats("as_norm_layer")
        return m.astype(np.float32), s.astype(np.float32), 0.0

    # -- persistence (the reference's npz) --------------------------------------------------
    def __eq__(self, other) -> bool:
        if not isinstance(other, StandardScaler):
            return False
        same = lambda a, b: (a is None and b is None) or (a is not None and b is not None and  # noqa: E731
                                                         np.array_equal(a, b))
        return (same(self.mean, other.mean) and same(self.std, other.std) and
                self.std_epsilon == other.std_epsilon and self._n_sample_dims == other._n_sample_dims)

    def dump(self, f: IO[bytes]):
        arrays = {name: value for name, value in (("mean", self.mean), ("std", self.std)) if value is not None}
        np.savez(f, **arrays)

    @classmethod
    def load(cls, f: IO[bytes]) -> "StandardScaler":
        with np.load(f, allow_pickle=False) as z:
            scaler = cls()
            scaler.mean = z["mean"] if "mean" in z.files else None
            scaler.std = z["std"] if "std" in z.files else None
        return scaler
