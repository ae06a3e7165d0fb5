"""fv3fit's out-of-sample composite over this package's registry: a novelty detector
scores every column, a taper turns the scores into a factor per column, and the base
model's outputs are multiplied by it, so the build's predictor (``mi355x-dense``) nests
as the ``base_model`` the way fv3fit's own models do.

Reference (paths under /root/reference/external/fv3fit/fv3fit):
* ``NoveltyDetector`` (``predict_novelties``)            _shared/novelty_detector.py:7-45
* ``MinMaxNoveltyDetector`` ("minmax")                   sklearn/_min_max_novelty_detector.py:41-160
* ``OutOfSampleModel`` ("out_of_sample")                 _shared/models.py:340-439
* ``taper_mask`` / ``taper_ramp`` / ``taper_decay``      _shared/taper_function.py:6-49
* ``ConstantOutputNoveltyDetector`` ("constant-output-novelty")  testing.py:120-150

The per-column work runs on the device: the min-max score (csrc/novelty.hip,
``fv3_minmax_scores``: the packed features scaled as MinMaxScaler.transform does, max /
min over the features) and the taper fused with the multiplication of every base
output (``fv3_taper_columns``), both in numpy's dtype flow (the mask taper is int64, so
a float32 output times it is float64, as in the reference).

Model files: the reference pickles its fitted sklearn MinMaxScaler (``minmax.pkl``,
joblib).  Pickles are not loaded here; the detector reads ``minmax.npz`` (the scaler's
arrays, ``numpy.load`` without pickle) next to the same ``metadata.bin``.
``tools/export_minmax.py``, run where the reference's model is trusted, writes it.
"""
import ctypes
import os
from typing import Callable, Hashable, Iterable, Mapping, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import _device, _native
from . import dataset as dsmod
from .predictor import Z_DIM_NAMES, Predictor, load, match_prediction_to_input_coords, register

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _tensor(data):
    """A CUDA tensor of a DataArray's data (float64 kept, other dtypes as float32)."""
    t = data if torch.is_tensor(data) else torch.from_numpy(np.ascontiguousarray(np.asarray(data)))
    if not t.is_cuda:
        t = t.cuda()
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64 if t.dtype in (torch.int64, torch.int32) else torch.float32)
    return t


def _is_host(data) -> bool:
    return not (torch.is_tensor(data) and data.is_cuda)


def _sample_dims(das: Sequence["dsmod.DataArray"], order: Sequence[Hashable]) -> Tuple[Hashable, ...]:
    dims = set()
    for da in das:
        dims.update(d for d in da.dims if d not in Z_DIM_NAMES)
    return tuple(d for d in order if d in dims) + tuple(sorted((d for d in dims if d not in order), key=str))


def _columns(da: "dsmod.DataArray", sample_dims: Sequence[Hashable]):
    """(tensor, fv3_layout, nz) of ``da`` as [level][column] with the columns in
    ``sample_dims`` order (a 2-D variable: one level)."""
    z = [d for d in da.dims if d in Z_DIM_NAMES]
    if len(z) > 1:
        raise ValueError(f"{da.name}: more than one vertical dimension {z}")
    if set(d for d in da.dims if d not in Z_DIM_NAMES) != set(sample_dims):
        raise ValueError(f"{da.name}: dims {da.dims} do not cover the sample dims {tuple(sample_dims)}")
    t = _tensor(da.data)
    order = list(z) + list(sample_dims)
    t = t.permute(*[da.dims.index(d) for d in order])
    if not z:
        t = t.unsqueeze(0)
    t, lay, ncol, nz = _device.column_view(t, 0, keep_f64=True)
    return t, lay, ncol, nz


# ------------------------------------------------------------------------ tapers
class _Taper:
    """A taper of taper_function.py on the device: callable on scores like the
    reference's (DataArray in, DataArray of taper values out), and fused with the
    multiplication of the base outputs in ``OutOfSampleModel.predict``."""

    def __init__(self, mode: int, p0: float, p1: float, name: str):
        self.mode, self.p0, self.p1, self.name = mode, float(p0), float(p1), name

    def run(self, scores: "dsmod.DataArray", fields: Sequence["dsmod.DataArray"] = ()):
        """(taper values, tapered fields) for ``scores`` (dims = the sample dims) and base
        outputs whose non-vertical dims are those sample dims."""
        _device.require_gpu()
        s = _tensor(scores.data).contiguous()
        host = _is_host(scores.data)
        sample_dims = tuple(scores.dims)
        tv = torch.empty(s.shape, dtype=torch.int64 if self.mode == _native.TAPER_MASK else s.dtype, device=s.device)
        keep, descs, outs = [s, tv], [], []
        for da in fields:
            t, lay, ncol, nz = _columns(da, sample_dims)
            f64 = t.dtype == torch.float64 or self.mode == _native.TAPER_MASK or s.dtype == torch.float64
            z = [d for d in da.dims if d in Z_DIM_NAMES]
            out = torch.empty((nz,) + tuple(s.shape), dtype=torch.float64 if f64 else torch.float32, device=s.device)
            olay, _, _ = _device.level_layout(out.view(nz, -1), 0)
            descs.append(_native.TaperField(t.data_ptr(), lay, int(t.dtype == torch.float64), out.data_ptr(), olay, nz))
            keep += [t, out]
            dims = (z[0],) + sample_dims if z else sample_dims
            res = out if z else out[0]
            res_da = dsmod.DataArray(res, dims, da.coords, da.attrs, da.name).transpose(*da.dims)
            outs.append((res_da, _is_host(da.data)))
        arr = (_native.TaperField * max(1, len(descs)))(*descs)
        st = _native.load().fv3_taper_columns(s.data_ptr(), int(s.dtype == torch.float64), s.numel(), self.mode,
                                              self.p0, self.p1, tv.data_ptr(), arr, len(descs),
                                              _device.stream_handle(None, keep))
        _native.check(st, "taper_columns")
        values = dsmod.DataArray(tv.cpu().numpy() if host else tv, sample_dims, scores.coords)
        tapered = [dsmod.DataArray(d.values if h else d.data.contiguous(), d.dims, d.coords, d.attrs, d.name)
                   for d, h in outs]
        return values, tapered

    def __call__(self, novelty_score):
        if not isinstance(novelty_score, dsmod.DataArray):  # an xarray DataArray or an array
            data = np.asarray(getattr(novelty_score, "values", novelty_score))
            dims = tuple(getattr(novelty_score, "dims", [f"dim_{i}" for i in range(data.ndim)]))
            novelty_score = dsmod.DataArray(data, dims)
        return self.run(novelty_score)[0]


def taper_mask(cutoff: float = 0, **kwargs) -> _Taper:
    """taper_function.py:6-13: 0 where the score exceeds ``cutoff``, else 1 (int64)."""
    return _Taper(_native.TAPER_MASK, cutoff, 0.0, "taper_mask")


def taper_ramp(ramp_min: float = 0, ramp_max: float = 1, **kwargs) -> _Taper:
    """taper_function.py:16-24: (ramp_max - score) / (ramp_max - ramp_min) clipped to [0, 1]."""
    return _Taper(_native.TAPER_RAMP, ramp_min, ramp_max, "taper_ramp")


def taper_decay(threshold: float = 0, rate: float = 0.5, **kwargs) -> _Taper:
    """taper_function.py:27-35: min(rate ** (score - threshold), 1)."""
    return _Taper(_native.TAPER_DECAY, threshold, rate, "taper_decay")


_TAPERS = {"taper_mask": taper_mask, "taper_ramp": taper_ramp, "taper_decay": taper_decay}


def get_taper_function(name: str = "taper_mask", config: Optional[Mapping] = None) -> _Taper:
    """taper_function.py:38-49 (the configuration's keys a taper does not take are
    ignored, as the reference's **kwargs does)."""
    try:
        return _TAPERS[name](**dict(config or {}))
    except KeyError:
        raise ValueError("Incorrect tapering name")


# --------------------------------------------------------------- novelty detectors
class NoveltyDetector(Predictor):
    """novelty_detector.py:7-45: ``predict`` returns per-column ``novelty_score`` and
    ``centered_score``; ``predict_novelties`` adds ``is_novelty`` (score > cutoff)."""

    _NOVELTY_OUTPUT_VAR = "is_novelty"
    _SCORE_OUTPUT_VAR = "novelty_score"
    _CENTERED_SCORE_OUTPUT_VAR = "centered_score"

    def __init__(self, input_variables: Iterable[Hashable]):
        super().__init__(input_variables, [self._NOVELTY_OUTPUT_VAR, self._SCORE_OUTPUT_VAR,
                                           self._CENTERED_SCORE_OUTPUT_VAR])

    def predict_novelties(self, X, cutoff: float = 0):
        diagnostics = self.predict(X)
        centered = diagnostics[self._CENTERED_SCORE_OUTPUT_VAR]
        data = centered.data
        # xr.where(centered > cutoff, 1, 0): int64
        flag = (data > cutoff).to(torch.int64) if torch.is_tensor(data) else (np.asarray(data) > cutoff).astype(np.int64)
        diagnostics[self._NOVELTY_OUTPUT_VAR] = dsmod.DataArray(flag, centered.dims, centered.coords)
        return diagnostics[self._CENTERED_SCORE_OUTPUT_VAR], diagnostics


@register("minmax")
class MinMaxNoveltyDetector(NoveltyDetector):
    """_min_max_novelty_detector.py:41-160: a column is novel when any packed feature
    lies outside the training range; score = how far past [0, 1] the min-max-scaled
    features reach.  ``scale`` / ``min`` are the fitted MinMaxScaler's ``scale_`` /
    ``min_`` (their dtype kept: fv3fit fits on float32)."""

    _ARRAYS_NAME = "minmax.npz"
    _PICKLE_NAME = "minmax.pkl"
    _METADATA_NAME = "metadata.bin"

    def __init__(self, input_variables: Sequence[Hashable], scale, min_, clip: Optional[Mapping] = None,
                 data_min=None, data_max=None):
        super().__init__(list(input_variables))
        self.scale = np.ascontiguousarray(scale)
        self.min = np.ascontiguousarray(min_)
        if self.scale.shape != self.min.shape or self.scale.ndim != 1:
            raise ValueError("scale and min must be 1-D arrays of one length")
        self.clip = {k: dict(v) for k, v in (clip or {}).items()}
        self.data_min, self.data_max = data_min, data_max

    @classmethod
    def fit(cls, X: np.ndarray, input_variables: Sequence[Hashable], clip: Optional[Mapping] = None,
            feature_range=(0, 1)) -> "MinMaxNoveltyDetector":
        """MinMaxScaler.fit on a packed [sample, feature] array (the reference fits on the
        float32 packing of its training batches): data_min / data_max per feature, scale_ =
        (hi - lo) / range (zero ranges as 1), min_ = lo - data_min * scale_, in X's dtype."""
        X = np.asarray(X)
        dmin, dmax = np.nanmin(X, axis=0), np.nanmax(X, axis=0)
        rng = dmax - dmin
        rng = np.where(rng < 10 * np.finfo(rng.dtype).eps, np.ones_like(rng), rng)  # _handle_zeros_in_scale
        scale = (feature_range[1] - feature_range[0]) / rng
        min_ = feature_range[0] - dmin * scale
        return cls(input_variables, scale, min_, clip, dmin, dmax)

    def _clip_range(self, name, nz: int) -> Tuple[int, int]:
        c = self.clip.get(name)
        if not c:
            return 0, nz
        start, stop, _ = slice(c.get("start"), c.get("stop")).indices(nz)
        return start, max(start, stop)

    def predict(self, X):
        _device.require_gpu()
        names = list(self.input_variables)
        missing = [n for n in names if n not in X]
        if missing:
            raise KeyError(missing[0])
        das = [X[n] for n in names]
        sample_dims = _sample_dims(das, dsmod.infer_dimension_order(X))
        descs, keep, x64, nfeat, ncol = [], [], False, 0, None
        for name, da in zip(names, das):
            t, lay, nc, nz = _columns(da, sample_dims)
            z0, z1 = self._clip_range(name, nz)
            if ncol is not None and nc != ncol:
                raise ValueError(f"{name}: {nc} columns, expected {ncol}")
            ncol = nc
            descs.append(_native.NovVar(t.data_ptr(), lay, int(t.dtype == torch.float64), z0, z1 - z0))
            keep.append(t)
            x64 = x64 or t.dtype == torch.float64
            nfeat += z1 - z0
        if nfeat != self.scale.size:
            raise ValueError(f"X has {nfeat} features, but MinMaxScaler is expecting {self.scale.size} features "
                             "as input.")
        if len(descs) > _native.NOV_MAX_VARS:
            raise NotImplementedError(f"more than {_native.NOV_MAX_VARS} input variables")
        sc = torch.from_numpy(self.scale).cuda()
        mn = torch.from_numpy(self.min.astype(self.scale.dtype)).cuda()
        sizes = dict(zip([d for da in das for d in da.dims], [s for da in das for s in da.shape]))
        shape = tuple(sizes[d] for d in sample_dims)
        score = torch.empty(shape, dtype=torch.float64 if x64 else torch.float32, device=sc.device)
        arr = (_native.NovVar * len(descs))(*descs)
        st = _native.load().fv3_minmax_scores(arr, len(descs), sc.data_ptr(), mn.data_ptr(),
                                              int(sc.dtype == torch.float64), int(x64), int(ncol or 0),
                                              score.data_ptr(), _device.stream_handle(None, keep + [sc, mn, score]))
        _native.check(st, "minmax_scores")
        host = all(_is_host(da.data) for da in das)
        data = score.cpu().numpy() if host else score
        out = dsmod.Dataset()
        out[self._SCORE_OUTPUT_VAR] = dsmod.DataArray(data, sample_dims)
        out[self._CENTERED_SCORE_OUTPUT_VAR] = dsmod.DataArray(data, sample_dims)
        return match_prediction_to_input_coords(X, out)

    def dump(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        arrays = {"scale_": self.scale, "min_": self.min}
        if self.data_min is not None:
            arrays.update(data_min_=np.asarray(self.data_min), data_max_=np.asarray(self.data_max))
        np.savez(os.path.join(path, self._ARRAYS_NAME), **arrays)
        metadata = {"input_variables": list(self.input_variables), "packer_config": {"clip": self.clip}}
        with open(os.path.join(path, self._METADATA_NAME), "w") as f:
            yaml.safe_dump(metadata, f)

    @classmethod
    def load(cls, path: str) -> "MinMaxNoveltyDetector":
        arrays_path = os.path.join(path, cls._ARRAYS_NAME)
        if not os.path.exists(arrays_path):
            if os.path.exists(os.path.join(path, cls._PICKLE_NAME)):
                raise ValueError(f"{path} holds the reference's pickled scaler ({cls._PICKLE_NAME}), which is not "
                                 f"loaded here; convert it with tools/export_minmax.py where the model is trusted")
            raise FileNotFoundError(arrays_path)
        with np.load(arrays_path, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
        with open(os.path.join(path, cls._METADATA_NAME)) as f:
            metadata = yaml.safe_load(f)
        clip = (metadata.get("packer_config") or {}).get("clip", {})
        return cls(metadata["input_variables"], arrays["scale_"], arrays["min_"], clip, arrays.get("data_min_"),
                   arrays.get("data_max_"))


@register("constant-output-novelty")
class ConstantOutputNoveltyDetector(NoveltyDetector):
    """testing.py:120-150: scores of zero for every column (the first input's non-vertical
    dims and dtype: zeros_like(first input).max(z))."""

    def predict(self, data):
        first = data[next(iter(self.input_variables))]
        keep = [d for d in first.dims if d not in Z_DIM_NAMES]
        shape = tuple(first.sizes[d] for d in keep)
        src = first.data
        if torch.is_tensor(src):
            zeros = torch.zeros(shape, dtype=src.dtype, device=src.device)
        else:
            zeros = np.zeros(shape, dtype=np.asarray(src).dtype)
        out = dsmod.Dataset()
        out[self._SCORE_OUTPUT_VAR] = dsmod.DataArray(zeros, keep, first.coords)
        out[self._CENTERED_SCORE_OUTPUT_VAR] = dsmod.DataArray(zeros, keep, first.coords)
        return out

    def dump(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "attrs.yaml"), "w") as f:
            yaml.safe_dump({"input_variables": list(self.input_variables)}, f)

    @classmethod
    def load(cls, path: str) -> "ConstantOutputNoveltyDetector":
        with open(os.path.join(path, "attrs.yaml")) as f:
            return cls(**yaml.safe_load(f))


# ------------------------------------------------------------ out-of-sample model
@register("out_of_sample")
class OutOfSampleModel(Predictor):
    """models.py:340-439: the base model's outputs times taper(novelty scores), merged
    with the detector's diagnostics and the taper values."""

    _TAPER_VALUES_OUTPUT_VAR = "taper_values"
    _CONFIG_FILENAME = "out_of_sample_model.yaml"

    def __init__(self, base_model: Predictor, novelty_detector: NoveltyDetector, cutoff: float = 0,
                 taper: Optional[Callable] = None):
        self.base_model = base_model
        self.novelty_detector = novelty_detector
        self.cutoff = cutoff
        self.taper = taper or get_taper_function("taper_mask", {"cutoff": cutoff})
        input_variables = tuple(sorted(set(base_model.input_variables) | set(novelty_detector.input_variables)))
        output_variables = tuple(sorted(set(base_model.output_variables) | set(novelty_detector.output_variables)
                                        | {self._TAPER_VALUES_OUTPUT_VAR}))
        super().__init__(input_variables=input_variables, output_variables=output_variables)

    def predict(self, X):
        from .stepper import merge

        base_predict = self.base_model.predict(X)
        centered_scores, diagnostics = self.novelty_detector.predict_novelties(X, cutoff=self.cutoff)
        outputs = [base_predict[v] for v in self.base_model.output_variables]
        if isinstance(self.taper, _Taper):  # the taper and every product in one launch
            taper_values, tapered = self.taper.run(centered_scores, outputs)
        else:  # a caller's own taper callable: its values, the products on the device
            taper_values = self.taper(centered_scores)
            tapered = [_multiply(o, taper_values) for o in outputs]
        diagnostics[self._TAPER_VALUES_OUTPUT_VAR] = taper_values
        tapered_predict = dsmod.Dataset()
        for name, da in zip(self.base_model.output_variables, tapered):
            tapered_predict[name] = da
        return merge([tapered_predict, diagnostics])

    def dump(self, path):
        raise NotImplementedError("no dump method yet for this class, you can define one manually using "
                                  "instructions at http://vulcanclimatemodeling.com/docs/fv3fit/composite-models.html")

    @classmethod
    def load(cls, path: str) -> "OutOfSampleModel":
        with open(os.path.join(path, cls._CONFIG_FILENAME)) as f:
            config = yaml.safe_load(f)
        base_model = load(config["base_model_path"])
        novelty_detector = load(config["novelty_detector_path"])
        cutoff = config.get("cutoff", 0)
        if not isinstance(novelty_detector, NoveltyDetector):
            raise AssertionError(f"{config['novelty_detector_path']} is not a novelty detector")
        default_tapering_config = {
            "name": "taper_mask",
            "cutoff": cutoff,
            "ramp_min": cutoff,
            "ramp_max": 1 if cutoff == 0 else max(cutoff * 2, cutoff / 2),
            "threshold": cutoff,
        }
        tapering_config = {**default_tapering_config, **config.get("tapering_function", {})}
        taper = get_taper_function(tapering_config["name"], tapering_config)
        return cls(base_model, novelty_detector, cutoff=cutoff, taper=taper)


def _multiply(output: "dsmod.DataArray", taper_values) -> "dsmod.DataArray":
    """output * taper for a caller-supplied taper: broadcast by dim name (torch on the
    device, numpy's promotion rules)."""
    tv = taper_values if isinstance(taper_values, dsmod.DataArray) else dsmod.DataArray(
        np.asarray(getattr(taper_values, "values", taper_values)), getattr(taper_values, "dims", ()))
    o = _tensor(output.data) if not _is_host(output.data) else torch.from_numpy(np.asarray(output.data))
    t = _tensor(tv.data) if not _is_host(output.data) else torch.from_numpy(np.asarray(tv.data))
    shape = [output.sizes[d] if d in tv.dims else 1 for d in output.dims]
    t = t.permute(*[tv.dims.index(d) for d in output.dims if d in tv.dims]).reshape(shape)
    res = o * t
    return dsmod.DataArray(res.numpy() if _is_host(output.data) else res, output.dims, output.coords, output.attrs,
                           output.name)
