"""The microphysics emulator hook's classifier head and masks (external/emulation) on MI355X.

Mirrors (paths under /root/reference/external/emulation/emulation):
* ``RangeMask`` / ``LevelMask`` / ``compose_masks``            masks.py:9-70
* the Zhao-Carr masks and conservation fixers                  zhao_carr.py:57-371
* ``ModelWithClassifier`` / ``combine_classifier_and_regressor`` models.py:14-85
* ``ModelConfig`` mask options and their order (``_build_masks``) config.py:78-221

Arrays are the hook's Fortran-layout [feature, sample] device tensors (float32 or
float64, contiguous); every arithmetic stage is a HIP kernel of csrc/emulation.hip, and
LevelMask's level copies are device copies.  A mask takes (state, emulator) and returns
the updated emulator dict, as in the reference.

dtype: the kernels compute in one dtype per call, numpy's for same-dtype operands; a
float32 emulator output meeting a float64 state is promoted to float64 first (numpy
promotes at the first mixed operation instead; identical whenever state and emulator
share a dtype, e.g. the all-float32 and all-float64 hooks).  The ``online_schedule``
TimeMask is mirrored by ``IntervalSchedule`` / ``TimeMask`` below on a Julian-calendar
model time (cftime is absent; config.py:78-175).  Not mirrored: the Keras tensor
transforms around a loaded TF model (the MicrophysicsEmulator graph has its own).
"""
import dataclasses
import datetime
from typing import Callable, Dict, Iterable, Mapping, Optional, Sequence, Union

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

FortranState = Dict[str, object]
Mask = Callable[[FortranState, FortranState], FortranState]

# fv3fit/emulation/transforms/zhao_carr.py:24-36: class names, sorted (the one-hot order)
POSITIVE_TENDENCY = "positive_tendency"
ZERO_TENDENCY = "zero_tendency"
ZERO_CLOUD = "zero_cloud"
NEGATIVE_TENDENCY = "negative_tendency"
NONTRIVIAL_TENDENCY = "nontrivial_tendency"
CLASS_NAMES = sorted({POSITIVE_TENDENCY, ZERO_TENDENCY, ZERO_CLOUD, NEGATIVE_TENDENCY})


class Input:
    cloud_water = "cloud_water_mixing_ratio_input"
    humidity = "specific_humidity_input"
    temperature = "air_temperature_input"
    delp = "pressure_thickness_of_atmospheric_layer"


class GscondOutput:
    cloud_water = "cloud_water_mixing_ratio_after_gscond"
    humidity = "specific_humidity_after_gscond"
    temperature = "air_temperature_after_gscond"


class PrecpdOutput:
    cloud_water = "cloud_water_mixing_ratio_after_precpd"
    humidity = "specific_humidity_after_precpd"
    temperature = "air_temperature_after_precpd"
    precip = "total_precipitation"


def _dev(x, dtype=None):
    dev = torch.device("cuda", torch.cuda.current_device())
    t = x if torch.is_tensor(x) else torch.as_tensor(x)
    if dtype is None:
        dtype = torch.float64 if t.dtype == torch.float64 else torch.float32
    return t.to(device=dev, dtype=dtype).contiguous()


def _common(*xs):
    """Device tensors of one float dtype (float64 if any is), contiguous."""
    _device.require_gpu()
    dt = torch.float64 if any(torch.is_tensor(x) and x.dtype == torch.float64 or
                              (not torch.is_tensor(x) and getattr(x, "dtype", None) == "float64") for x in xs) \
        else torch.float32
    ts = [_dev(x, dt) for x in xs]
    for t in ts[1:]:
        if t.shape != ts[0].shape:
            raise ValueError(f"shape mismatch: {tuple(t.shape)} vs {tuple(ts[0].shape)}")
    return ts, int(dt == torch.float64)


def _s():
    return _device.stream_handle(None)


# ---------------------------------------------------------------------------- masks.py
def compose_masks(funcs: Iterable[Mask]) -> Mask:
    """masks.py:9-20: masks applied in order."""
    func_list = list(funcs)

    def composed(state, emulator):
        out = emulator
        for func in func_list:
            out = func(state, out)
        return out

    return composed


# ------------------------------------------------------------ _emulate/microphysics.py
@dataclasses.dataclass(frozen=True)
class JulianTime:
    """A date on the Julian calendar (what cftime.DatetimeJulian holds for the schedule,
    _time.py:6-13; cftime is not a dependency here): subtraction gives the exact
    ``datetime.timedelta`` between two such dates."""
    year: int
    month: int
    day: int
    hour: int = 0
    minute: int = 0
    second: int = 0

    def _seconds(self) -> int:
        a = (14 - self.month) // 12
        y = self.year + 4800 - a
        m = self.month + 12 * a - 3
        jdn = self.day + (153 * m + 2) // 5 + 365 * y + y // 4 - 32083  # Julian-calendar day number
        return ((jdn * 24 + self.hour) * 60 + self.minute) * 60 + self.second

    def __sub__(self, other: "JulianTime") -> datetime.timedelta:
        return datetime.timedelta(seconds=self._seconds() - other._seconds())


def translate_time(time) -> JulianTime:
    """_time.py:6-13: the Fortran model_time array; index 3 is skipped, as there."""
    return JulianTime(int(time[0]), int(time[1]), int(time[2]), int(time[4]), int(time[5]))


@dataclasses.dataclass
class IntervalSchedule:
    """_emulate/microphysics.py:23-34: 1.0 in the first half of every ``period`` after
    ``initial_time``, else 0.0."""
    period: datetime.timedelta
    initial_time: JulianTime

    def __call__(self, time: JulianTime) -> float:
        fraction_of_interval = ((time - self.initial_time) / self.period) % 1
        return 1.0 if fraction_of_interval < 0.5 else 0.0


class TimeMask:
    """_emulate/microphysics.py:37-47: ``state * alpha + emulator * (1 - alpha)`` for the
    keys both hold, alpha = ``schedule(model time)``; arrays blend on the device
    (fv3_time_blend, numpy's dtype flow), Python numbers as Python does."""

    def __init__(self, schedule: Callable):
        self.schedule = schedule

    def __call__(self, state, emulator):
        alpha = float(self.schedule(translate_time(state["model_time"])))
        out = {}
        for key in set(state) & set(emulator):
            a, b = state[key], emulator[key]
            if isinstance(a, (int, float)) and isinstance(b, (int, float)):
                out[key] = a * alpha + b * (1 - alpha)
                continue
            ta, tb = _dev(a), _dev(b)
            if ta.numel() != tb.numel():
                raise ValueError(f"TimeMask: {key} sizes differ: {tuple(ta.shape)} vs {tuple(tb.shape)}")
            a64, b64 = ta.dtype == torch.float64, tb.dtype == torch.float64
            res = torch.empty(ta.shape, dtype=torch.float64 if (a64 or b64) else torch.float32, device=ta.device)
            st = _native.load().fv3_time_blend(ta.data_ptr(), int(a64), tb.data_ptr(), int(b64), res.data_ptr(),
                                               res.numel(), alpha, _s())
            _native.check(st, "time_blend")
            out[key] = res
        return out


class RangeMask:
    """masks.py:23-39."""

    def __init__(self, key: str, min: Optional[float] = None, max: Optional[float] = None):
        self.min, self.max, self.key = min, max, key

    def __call__(self, state, emulator):
        (x,), f64 = _common(emulator[self.key])
        out = torch.empty_like(x)
        st = _native.load().fv3_range_mask(x.data_ptr(), out.data_ptr(), x.numel(),
                                           float(self.min if self.min is not None else 0.0),
                                           float(self.max if self.max is not None else 0.0),
                                           int(self.min is not None), int(self.max is not None), f64, _s())
        _native.check(st, "range_mask")
        return {**emulator, self.key: out}


class LevelMask:
    """masks.py:42-70: levels [start:stop) of the emulator field taken from the Fortran
    state (fill_value None), from ``state[fill_value]`` (str) or a constant (float)."""

    def __init__(self, key: str, start: Optional[int], stop: Optional[int],
                 fill_value: Union[float, str, None] = None):
        self.key, self.start, self.stop, self.fill_value = key, start, stop, fill_value

    def __call__(self, state, emulator):
        field = _dev(emulator[self.key]).clone()
        sl = slice(self.start, self.stop)
        if self.fill_value is None:
            field[sl] = _dev(state[self.key], field.dtype)[sl]
        elif isinstance(self.fill_value, str):
            field[sl] = _dev(state[self.fill_value], field.dtype)[sl]
        elif isinstance(self.fill_value, float):
            field[sl] = self.fill_value
        return {**emulator, self.key: field}


# ------------------------------------------------------------------------ zhao_carr.py
def classify_output(logit_classes, one_hot_axis: int = 0) -> Dict[str, object]:
    """_get_classify_output (zhao_carr.py:214-219): uint8 one-hot per class name (sorted)
    and ``nontrivial_tendency``.  The class axis must be the leading axis (the hook's
    [class, feature, sample] layout) or, for one_hot_axis=-1, the trailing one."""
    (x,), f64 = _common(logit_classes)
    if one_hot_axis not in (0, -1, x.dim() - 1):
        raise ValueError("the class axis must be the first or the last")
    if one_hot_axis != 0 and x.dim() > 1:
        x = x.movedim(-1, 0).contiguous()
    n_class = x.shape[0]
    if n_class != len(CLASS_NAMES):
        raise ValueError(f"expected {len(CLASS_NAMES)} class logits, got {n_class}")
    inner = x[0].numel()
    masks = torch.empty((n_class + 1,) + tuple(x.shape[1:]), dtype=torch.uint8, device=x.device)
    st = _native.load().fv3_classify_one_hot(x.data_ptr(), n_class, inner, masks.data_ptr(),
                                             CLASS_NAMES.index(POSITIVE_TENDENCY),
                                             CLASS_NAMES.index(NEGATIVE_TENDENCY), f64, _s())
    _native.check(st, "classify_one_hot")
    out = {name: masks[i] for i, name in enumerate(CLASS_NAMES)}
    out[NONTRIVIAL_TENDENCY] = masks[n_class]
    return out


def infer_gscond_cloud_from_conservation(state, emulator):
    """zhao_carr.py:72-76."""
    (qc, qv, qvg), f64 = _common(state[Input.cloud_water], state[Input.humidity], emulator[GscondOutput.humidity])
    out = torch.empty_like(qc)
    st = _native.load().fv3_zc_infer_gscond_cloud(qc.data_ptr(), qv.data_ptr(), qvg.data_ptr(), out.data_ptr(),
                                                   qc.numel(), f64, _s())
    _native.check(st, "zc_infer_gscond_cloud")
    return {**emulator, GscondOutput.cloud_water: out}


def _apply_squash(struct, output_state, cloud_squash: float):
    out = {**output_state}
    if struct.cloud_water in output_state:
        (c, h), f64 = _common(output_state[struct.cloud_water], output_state[struct.humidity])
        co, ho = torch.empty_like(c), torch.empty_like(h)
        st = _native.load().fv3_zc_squash(c.data_ptr(), h.data_ptr(), float(cloud_squash), co.data_ptr(),
                                          ho.data_ptr(), c.numel(), f64, _s())
        _native.check(st, "zc_squash")
        out[struct.cloud_water], out[struct.humidity] = co, ho
    return out


def squash_gscond(state, emulator, cloud_squash):
    """zhao_carr.py:79-80."""
    return _apply_squash(GscondOutput, emulator, cloud_squash)


def squash_precpd(state, emulator, cloud_squash):
    """zhao_carr.py:83-84."""
    return _apply_squash(PrecpdOutput, emulator, cloud_squash)


def _gscond_update(mode, state, emulator, fortran=None, klass=None, ice=None):
    (qc, qv, t, emu), f64 = _common(state[Input.cloud_water], state[Input.humidity], state[Input.temperature],
                                    emulator[GscondOutput.cloud_water])
    dt = qc.dtype
    fq = _dev(fortran, dt) if fortran is not None else None
    outs = [torch.empty_like(qc) for _ in range(3)]
    st = _native.load().fv3_zc_gscond_update(
        mode, qc.data_ptr(), qv.data_ptr(), t.data_ptr(), fq.data_ptr() if fq is not None else None, emu.data_ptr(),
        klass.data_ptr() if klass is not None else None, ice.data_ptr() if ice is not None else None,
        outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), qc.numel(), f64, _s())
    _native.check(st, "zc_gscond_update")
    return {**emulator, GscondOutput.cloud_water: outs[0], GscondOutput.humidity: outs[1],
            GscondOutput.temperature: outs[2]}


def _mask_u8(m, like):
    m = m if torch.is_tensor(m) else torch.as_tensor(m)
    m = m.to(device=like.device, dtype=torch.uint8).contiguous()
    if m.shape != like.shape:
        raise ValueError(f"class mask shape {tuple(m.shape)} != field shape {tuple(like.shape)}")
    return m


def mask_where_fortran_cloud_identical(state, emulator):
    """zhao_carr.py:174-180."""
    return _gscond_update(_native.ZC_CLOUD_IDENTICAL, state, emulator, fortran=state[GscondOutput.cloud_water])


def mask_where_fortran_cloud_vanishes_gscond(state, emulator):
    """zhao_carr.py:164-171."""
    return _gscond_update(_native.ZC_CLOUD_VANISHES, state, emulator, fortran=state[GscondOutput.cloud_water])


def mask_zero_cloud_classifier(state, emulator):
    """zhao_carr.py:222-228."""
    like = _dev(emulator[GscondOutput.cloud_water])
    m = _mask_u8(classify_output(emulator["gscond_classes"])[ZERO_CLOUD], like)
    return _gscond_update(_native.ZC_CLOUD_CLASS_ZERO, state, emulator, klass=m)


def mask_zero_tend_classifier(state, emulator):
    """zhao_carr.py:231-237."""
    like = _dev(emulator[GscondOutput.cloud_water])
    m = _mask_u8(classify_output(emulator["gscond_classes"])[ZERO_TENDENCY], like)
    return _gscond_update(_native.ZC_CLOUD_CLASS_NOTEND, state, emulator, klass=m)


def mask_zero_cloud_classifier_precpd(state, emulator):
    """zhao_carr.py:240-247: the precpd cloud zeroed where the class is zero_cloud (no
    conservation update)."""
    (emu,), f64 = _common(emulator[PrecpdOutput.cloud_water])
    m = _mask_u8(classify_output(emulator["precpd_classes"])[ZERO_CLOUD], emu)
    out = torch.empty_like(emu)
    st = _native.load().fv3_zc_zero_where(m.data_ptr(), emu.data_ptr(), out.data_ptr(), emu.numel(), f64, _s())
    _native.check(st, "zc_zero_where")
    return {**emulator, PrecpdOutput.cloud_water: out}


def enforce_conservative_gscond(state, emulator):
    """zhao_carr.py:250-252."""
    return _gscond_update(_native.ZC_CLOUD_EMULATOR, state, emulator)


def ice_water_flag(temperature_celsius_source, cloud, offset: float = 273.16):
    """ice_water_flag (zhao_carr.py:108-133) of ``temperature - offset`` (the caller's
    ``state[T] - 273.16``), over the last axis of 2-D arrays."""
    (t, c), f64 = _common(temperature_celsius_source, cloud)
    if t.dim() != 2:
        raise ValueError("ice_water_flag expects 2-D arrays")
    iw = torch.empty_like(t)
    st = _native.load().fv3_zc_ice_water_flag(t.data_ptr(), c.data_ptr(), float(offset), iw.data_ptr(),
                                               t.shape[0], t.shape[1], f64, _s())
    _native.check(st, "zc_ice_water_flag")
    return iw


def enforce_conservative_phase_dependent(state, emulator):
    """zhao_carr.py:255-259."""
    iw = ice_water_flag(state[Input.temperature], state[Input.cloud_water])
    return _gscond_update(_native.ZC_PHASE_DEPENDENT, state, emulator, ice=iw.to(torch.uint8))


def enforce_conservative_precpd(state, emulator):
    """zhao_carr.py:313-352 (precip float64, as the reference's np.zeros accumulator)."""
    (qcg, qvg, tg, qce, qve, dp), f64 = _common(
        state[GscondOutput.cloud_water], state[GscondOutput.humidity], state[GscondOutput.temperature],
        emulator[PrecpdOutput.cloud_water], emulator[PrecpdOutput.humidity], state[Input.delp])
    if qcg.dim() != 2:
        raise ValueError("expected 2-D [feature, sample] arrays")
    nz, ncol = qcg.shape
    outs = [torch.empty_like(qcg) for _ in range(3)]
    precip = torch.empty(ncol, dtype=torch.float64, device=qcg.device)
    st = _native.load().fv3_zc_precpd_conservative(qcg.data_ptr(), qvg.data_ptr(), tg.data_ptr(), qce.data_ptr(),
                                                    qve.data_ptr(), dp.data_ptr(), outs[0].data_ptr(),
                                                    outs[1].data_ptr(), outs[2].data_ptr(), precip.data_ptr(), nz,
                                                    ncol, f64, _s())
    _native.check(st, "zc_precpd_conservative")
    return {**emulator, PrecpdOutput.cloud_water: outs[0], PrecpdOutput.humidity: outs[1],
            PrecpdOutput.temperature: outs[2], PrecpdOutput.precip: precip}


def conservative_precip_simple(state, emulator):
    """zhao_carr.py:355-371 (sum over the feature axis)."""
    (qvg, qcg, qve, qce, dp), f64 = _common(state[GscondOutput.humidity], state[GscondOutput.cloud_water],
                                            emulator[PrecpdOutput.humidity], emulator[PrecpdOutput.cloud_water],
                                            state[Input.delp])
    nz, ncol = qvg.shape
    precip = torch.empty(ncol, dtype=qvg.dtype, device=qvg.device)
    st = _native.load().fv3_zc_precip_simple(qvg.data_ptr(), qcg.data_ptr(), qve.data_ptr(), qce.data_ptr(),
                                              dp.data_ptr(), precip.data_ptr(), nz, ncol, f64, _s())
    _native.check(st, "zc_precip_simple")
    return {**emulator, PrecpdOutput.precip: precip}


# --------------------------------------------------------------------------- models.py
class ModelWithClassifier:
    """models.py:14-53 on the hook's [feature, sample] state: the classifier's
    ``class_key`` logits (a [class, feature, sample] output, classes in sorted-name order)
    decoded to one-hot masks, merged into the regressor's inputs and into its outputs."""

    def __init__(self, model: Callable, classifier: Optional[Callable] = None, class_key: str = "gscond_classes",
                 batch_size: int = 1024, inputs_to_ignore: Sequence[str] = ("rank", "model_time")):
        self.model = model
        self.classifier = classifier
        self._class_key = class_key
        self._batch_size = batch_size  # the kernels take every column at once
        self.inputs_to_ignore = inputs_to_ignore

    def __call__(self, state: FortranState) -> FortranState:
        state = {k: v for k, v in state.items() if k not in self.inputs_to_ignore}
        if self.classifier is not None:
            classifier_outputs = dict(self.classifier(state))
            classifier_outputs.update(classify_output(classifier_outputs[self._class_key], one_hot_axis=0))
        else:
            classifier_outputs = {}
        inputs = {**classifier_outputs, **state}
        model_outputs = dict(self.model(inputs))
        model_outputs.update(classifier_outputs)
        return model_outputs


def combine_classifier_and_regressor(classifier, regressor, batch_size: int = 1024) -> ModelWithClassifier:
    """models.py:71-85: the regressor's legacy *_output names renamed to the after-precpd
    names."""
    translation = {"air_temperature_output": PrecpdOutput.temperature,
                   "specific_humidity_output": PrecpdOutput.humidity,
                   "cloud_water_mixing_ratio_output": PrecpdOutput.cloud_water}

    def renamed(x):
        return {translation.get(k, k): v for k, v in regressor(x).items()}

    return ModelWithClassifier(renamed, classifier, batch_size=batch_size)


class ClassifierModel:
    """A dense classifier on the fused kernel: the DenseColumnModel's one output of
    n_class * nz features is the [class][level] logits, returned as a
    [class, feature, sample] tensor under ``class_key``."""

    def __init__(self, model, class_key: str = "gscond_classes", n_class: int = len(CLASS_NAMES)):
        self.model = model
        self.class_key = class_key
        self.n_class = n_class
        if len(model.config.output_variables) != 1:
            raise ValueError("a classifier model has one output (the class logits)")

    def __call__(self, state):
        xs = [state[name] for name in self.model.config.input_variables]
        (logits,) = self.model.forward(xs, level_axes=[0] * len(xs), out_level_axis=0)
        return {self.class_key: logits.reshape(self.n_class, -1, logits.shape[-1])}


# --------------------------------------------------------------------------- config.py
@dataclasses.dataclass
class Range:
    min: Optional[float] = None
    max: Optional[float] = None


@dataclasses.dataclass
class LevelSlice:
    start: Optional[int] = None
    stop: Optional[int] = None
    fill_value: Union[float, str, None] = None


@dataclasses.dataclass
class MaskConfig:
    """The mask options of ModelConfig (config.py:78-163), built in its order
    (``_build_masks``, config.py:178-221)."""
    ranges: Mapping[str, Range] = dataclasses.field(default_factory=dict)
    mask_emulator_levels: Mapping[str, LevelSlice] = dataclasses.field(default_factory=dict)
    cloud_squash: Optional[float] = None
    gscond_cloud_conservative: bool = False
    mask_gscond_identical_cloud: bool = False
    mask_gscond_zero_cloud: bool = False
    enforce_conservative: bool = False
    enforce_conservative_phase_dependent: bool = False
    mask_gscond_zero_cloud_classifier: bool = False
    mask_gscond_no_tend_classifier: bool = False
    mask_precpd_zero_cloud_classifier: bool = False
    enforce_strict_precpd_conservative: bool = False
    simple_precip_conservative: bool = False
    online_schedule: Optional[Callable] = None  # e.g. IntervalSchedule: TimeMask first

    def __post_init__(self):
        if self.enforce_conservative and self.enforce_conservative_phase_dependent:
            raise ValueError("These options are mutually exclusive.")
        if self.enforce_strict_precpd_conservative and self.simple_precip_conservative:
            raise ValueError("Conservative precip flags should not both be true.")

    def build_mask(self) -> Mask:
        return compose_masks(self.build_masks())

    def build_masks(self) -> Iterable[Mask]:
        if self.online_schedule:
            yield TimeMask(self.online_schedule)
        for key, r in self.ranges.items():
            yield RangeMask(key, min=r.min, max=r.max)
        if self.gscond_cloud_conservative:
            yield infer_gscond_cloud_from_conservation
        if self.cloud_squash is not None:
            yield lambda x, y: squash_gscond(x, y, self.cloud_squash)
            yield lambda x, y: squash_precpd(x, y, self.cloud_squash)
        if self.mask_gscond_identical_cloud:
            yield mask_where_fortran_cloud_identical
        if self.mask_gscond_zero_cloud:
            yield mask_where_fortran_cloud_vanishes_gscond
        if self.mask_gscond_no_tend_classifier:
            yield mask_zero_tend_classifier
        if self.mask_gscond_zero_cloud_classifier:
            yield mask_zero_cloud_classifier
        if self.mask_precpd_zero_cloud_classifier:
            yield mask_zero_cloud_classifier_precpd
        if self.enforce_conservative:
            yield enforce_conservative_gscond
        elif self.enforce_conservative_phase_dependent:
            yield enforce_conservative_phase_dependent
        if self.simple_precip_conservative:
            yield conservative_precip_simple
        elif self.enforce_strict_precpd_conservative:
            yield enforce_conservative_precpd
        for key, sl in self.mask_emulator_levels.items():
            yield LevelMask(key, start=sl.start, stop=sl.stop, fill_value=sl.fill_value)
