"""Column-wise DenseModel (fv3fit ``dense``) on MI355X.

Mirrors the predict graph of ``external/fv3fit/fv3fit/keras/_models/dense.py:234-305``
(clip -> StandardNorm -> concat -> Dense(width, relu) x (depth-1) -> Dense(nz) per
output -> StandardDenorm -> OutputLimit -> zero mask) with one fused HIP kernel
(``csrc/dense.hip``) behind ``fv3_dense_create`` / ``fv3_dense_forward``.

Weights are held in Keras' own layout (kernel ``[fan_in, fan_out]``, bias
``[fan_out]``), so a trained Keras/TF model converts with a plain weight dump
(see INTEGRATION.md); the model directory format is npz + yaml.
"""
import ctypes
import dataclasses
import os
import weakref
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


@dataclasses.dataclass
class DenseModelConfig:
    """Shape/configuration of a DenseModel (DenseHyperparameters, dense.py:39-106)."""

    input_variables: List[str]
    output_variables: List[str]
    in_nz: List[int]
    out_nz: List[int]
    width: int = 256  # DenseNetworkConfig.width
    depth: int = 3  # DenseNetworkConfig.depth: depth-1 hidden layers (dense_network.py:59-76)
    epsilon: float = 1e-7  # StandardNormLayer epsilon
    clip: Dict[str, Tuple[int, int]] = dataclasses.field(default_factory=dict)  # ClipConfig
    output_limits: Dict[str, Tuple[Optional[float], Optional[float]]] = dataclasses.field(
        default_factory=dict
    )  # OutputLimitConfig
    # microphysics-emulator graph (fv3fit/emulation/transforms/transforms.py):
    # input name -> eps of a LogTransform log(max(x, eps)) applied before normalisation
    input_log_eps: Dict[str, float] = dataclasses.field(default_factory=dict)
    # output name -> input name whose raw values are added after de-normalisation
    # (Difference.backward: after = before + to)
    output_residuals: Dict[str, str] = dataclasses.field(default_factory=dict)

    @property
    def n_hidden(self) -> int:
        return self.depth - 1

    def in_clip(self) -> List[Tuple[int, int]]:
        out = []
        for name, nz in zip(self.input_variables, self.in_nz):
            s, e = self.clip.get(name, (0, nz))
            out.append((0 if s is None else int(s), nz if e is None else int(e)))
        return out

    @property
    def k_in(self) -> int:
        return sum(e - s for s, e in self.in_clip())

    @property
    def k_out(self) -> int:
        return sum(self.out_nz)

    def flops_per_column(self) -> int:
        w = self.width
        return 2 * (self.k_in * w + (self.n_hidden - 1) * w * w + w * self.k_out)

    def to_dict(self):
        d = dataclasses.asdict(self)
        d["clip"] = {k: list(v) for k, v in self.clip.items()}
        d["output_limits"] = {k: list(v) for k, v in self.output_limits.items()}
        return d

    @classmethod
    def from_dict(cls, d):
        d = dict(d)
        d["clip"] = {k: tuple(v) for k, v in d.get("clip", {}).items()}
        d["output_limits"] = {k: tuple(v) for k, v in d.get("output_limits", {}).items()}
        return cls(**d)


def _glorot(rng, fan_in, fan_out):
    lim = np.sqrt(6.0 / (fan_in + fan_out))  # keras glorot_uniform (Dense default)
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(np.float32)


PRECISIONS = {"f32": _native.DENSE_F32, "bf16x3": _native.DENSE_BF16X3, "bf16x6": _native.DENSE_BF16X6}


class DenseColumnModel:
    """Weights + normalisation of a DenseModel, plus its device handle.

    ``precision`` selects the fused kernel's arithmetic: ``"f32"`` (exact f32 products on
    v_mfma_f32_16x16x4_f32, the Keras precision) or ``"bf16x3"`` (each f32 operand split
    into bf16 hi + lo, three bf16 MFMAs per product; ~1e-5 rel, BASELINE config #5's
    bf16-MFMA path) or ``"bf16x6"`` (hi + mid + lo, six bf16 MFMAs per product: f32-level
    error on bf16 MFMA, csrc/dense_b3.hip)."""

    def __init__(self, config: DenseModelConfig, params: Mapping[str, object], precision: str = "f32"):
        self.config = config
        self.params = dict(params)
        self._handles: Dict[int, int] = {}
        self._plans = weakref.WeakSet()  # LaunchPlans holding a bound forward of this model
        self.precision = precision
        self._validate()

    @property
    def precision(self) -> str:
        return self._precision

    @precision.setter
    def precision(self, value: str):
        if value not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {value!r}")
        self._precision = value

    # ---- construction ----------------------------------------------------------
    @classmethod
    def random(
        cls,
        config: DenseModelConfig,
        seed: int = 1,
        sample_inputs: Optional[Sequence[np.ndarray]] = None,
        sample_outputs: Optional[Sequence[np.ndarray]] = None,
        bias_scale: float = 0.0,
    ) -> "DenseColumnModel":
        """Glorot-uniform kernels (Keras default), biases ``bias_scale * N(0,1)``
        (Keras: zeros), normalisation fitted on samples like build_model does
        (dense.py:279-289, normalization.py:63-94: mean, population std, f32)."""
        from . import normalization

        rng = np.random.default_rng(seed)
        w = config.width
        k_in = config.k_in
        hk, hb = [], []
        fan = k_in
        for _ in range(config.n_hidden):
            hk.append(_glorot(rng, fan, w))
            hb.append((bias_scale * rng.normal(size=w)).astype(np.float32))
            fan = w
        ok, ob = [], []
        for nz in config.out_nz:
            ok.append(_glorot(rng, w, nz))
            ob.append((bias_scale * rng.normal(size=nz)).astype(np.float32))
        clips = config.in_clip()
        in_mean, in_sigma = [], []
        for v, nz in enumerate(config.in_nz):
            s, e = clips[v]
            if sample_inputs is not None:
                m, sd = normalization.fit_mean_std(np.asarray(sample_inputs[v]).reshape(-1, nz)[:, s:e])
            else:
                m, sd = np.zeros(e - s, np.float32), np.ones(e - s, np.float32)
            in_mean.append(m)
            in_sigma.append(sd)
        out_mean, out_sigma = [], []
        for o, nz in enumerate(config.out_nz):
            if sample_outputs is not None:
                m, sd = normalization.fit_mean_std(np.asarray(sample_outputs[o]).reshape(-1, nz))
            else:
                m, sd = np.zeros(nz, np.float32), np.ones(nz, np.float32)
            out_mean.append(m)
            out_sigma.append(sd)
        params = dict(hidden_kernels=hk, hidden_biases=hb, out_kernels=ok, out_biases=ob,
                      in_mean=in_mean, in_sigma=in_sigma, out_mean=out_mean, out_sigma=out_sigma)
        return cls(config, params)

    def _validate(self):
        c, p = self.config, self.params
        if len(c.input_variables) != len(c.in_nz) or len(c.output_variables) != len(c.out_nz):
            raise ValueError("variables and level counts disagree")
        if len(p["hidden_kernels"]) != c.n_hidden or len(p["hidden_biases"]) != c.n_hidden:
            raise ValueError(f"expected {c.n_hidden} hidden layers")
        fan = c.k_in
        for k, b in zip(p["hidden_kernels"], p["hidden_biases"]):
            if tuple(np.shape(k)) != (fan, c.width) or tuple(np.shape(b)) != (c.width,):
                raise ValueError(f"hidden kernel shape {np.shape(k)} != {(fan, c.width)}")
            fan = c.width
        for o, nz in enumerate(c.out_nz):
            if tuple(np.shape(p["out_kernels"][o])) != (c.width, nz):
                raise ValueError(f"output kernel {o} shape {np.shape(p['out_kernels'][o])}")

    def oracle_params(self) -> dict:
        """Parameters in the layout of oracle.dense.dense_predict (tests only)."""
        c = self.config
        d = dict(self.params)
        d["in_clip"] = c.in_clip()
        d["epsilon"] = c.epsilon
        d["out_min"] = [c.output_limits.get(n, (None, None))[0] for n in c.output_variables]
        d["out_max"] = [c.output_limits.get(n, (None, None))[1] for n in c.output_variables]
        d["out_mask"] = [self._out_mask(o) for o in range(len(c.output_variables))]
        return d

    def _out_mask(self, o) -> Optional[np.ndarray]:
        name, nz = self.config.output_variables[o], self.config.out_nz[o]
        if name not in self.config.clip:
            return None
        s, e = self.config.clip[name]
        s = 0 if s is None else s
        e = nz if e is None else e
        return np.hstack([np.zeros(s), np.ones(e - s), np.zeros(nz - e)]).astype(np.float32)

    # ---- device handle ---------------------------------------------------------
    def handle(self) -> int:
        _device.require_gpu()
        dev = torch.cuda.current_device()
        if dev in self._handles:
            return self._handles[dev]
        c, p = self.config, self.params
        keep = []  # keep ctypes buffers alive during create

        def farr(a):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float32).ravel())
            keep.append(a)
            return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))

        def iarr(a):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.int32).ravel())
            keep.append(a)
            return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))

        def parr(arrs):
            ptrs = (ctypes.POINTER(ctypes.c_float) * len(arrs))(*[farr(a) for a in arrs])
            keep.append(ptrs)
            return ctypes.cast(ptrs, ctypes.POINTER(ctypes.POINTER(ctypes.c_float)))

        k_out = c.k_out
        out_min = np.full(k_out, -np.inf, np.float32)
        out_max = np.full(k_out, np.inf, np.float32)
        out_mask = np.ones(k_out, np.float32)
        off = 0
        for o, (name, nz) in enumerate(zip(c.output_variables, c.out_nz)):
            lo, hi = c.output_limits.get(name, (None, None))
            if lo is not None:
                out_min[off:off + nz] = lo
            if hi is not None:
                out_max[off:off + nz] = hi
            m = self._out_mask(o)
            if m is not None:
                out_mask[off:off + nz] = m
            off += nz
        log_eps = [float(c.input_log_eps.get(n, 0.0)) for n in c.input_variables]
        residual = [c.input_variables.index(c.output_residuals[n]) if n in c.output_residuals else -1
                    for n in c.output_variables]
        desc = _native.DenseDesc(
            n_in=len(c.input_variables), in_nz=iarr(c.in_nz), in_clip=iarr(np.array(c.in_clip()).ravel()),
            in_mean=farr(np.concatenate([np.ravel(m) for m in p["in_mean"]])),
            in_sigma=farr(np.concatenate([np.ravel(s) for s in p["in_sigma"]])),
            epsilon=float(c.epsilon), width=int(c.width), n_hidden=int(c.n_hidden),
            hidden_kernel=parr(p["hidden_kernels"]), hidden_bias=parr(p["hidden_biases"]),
            n_out=len(c.output_variables), out_nz=iarr(c.out_nz),
            out_kernel=parr(p["out_kernels"]), out_bias=parr(p["out_biases"]),
            out_mean=farr(np.concatenate([np.ravel(m) for m in p["out_mean"]])),
            out_sigma=farr(np.concatenate([np.ravel(s) for s in p["out_sigma"]])),
            out_min=farr(out_min), out_max=farr(out_max), out_mask=farr(out_mask),
            in_log_eps=farr(log_eps), out_residual=iarr(residual),
        )
        h = ctypes.c_void_p()
        lib = _native.load()
        _native.check(lib.fv3_dense_create(ctypes.byref(desc), ctypes.byref(h)), "dense_create")
        self._handles[dev] = h.value
        return h.value

    def close(self):
        """Free the native model handles.  Refused while a live LaunchPlan holds a bound
        forward of this model (the native plan replays the raw handle); a BoundForward
        called after close() raises instead of launching on the freed handle."""
        if not self._handles:
            return
        if any(p._h for p in list(self._plans)):
            raise RuntimeError("DenseColumnModel.close: a LaunchPlan still replays a bound forward of this "
                               "model; close the plan first")
        lib = _native.load()
        for h in self._handles.values():
            lib.fv3_dense_destroy(h)
        self._handles.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- forward -----------------------------------------------------------------
    def forward(self, inputs: Sequence, level_axes: Optional[Sequence[int]] = None,
                outputs: Optional[Sequence] = None, out_level_axis: int = 0, stream=None,
                precision: Optional[str] = None):
        """Predict on device.  ``inputs[v]``: CUDA tensor whose axis ``level_axes[v]``
        (default 0) holds that variable's levels and whose other axes are columns
        (any leading axes are blocks, e.g. tiles).  A 2-D input may omit the level
        axis (pass ``None``).  Returns output tensors shaped like the first input
        with the level axis sized ``out_nz``; pass ``outputs`` to write in place."""
        c = self.config
        if len(inputs) != len(c.input_variables):
            raise ValueError(f"expected {len(c.input_variables)} inputs")
        level_axes = list(level_axes) if level_axes is not None else [0] * len(inputs)
        prec = precision or self.precision
        outputs_arg = outputs
        # a float64 state (the stepper's) is read in place and cast in the kernel's staging
        in64 = (prec == "f32" and len(inputs) > 0 and all(ax is not None for ax in level_axes)
                and all(torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float64 for t in inputs))
        ts, lays = [], []
        ncol = None
        copied = []  # inputs the kernel reads through a copy (not the caller's buffer)
        for v, (t, ax) in enumerate(zip(inputs, level_axes)):
            orig = t
            if ax is None:
                t = _device.to_device_f32(t, contiguous=False).unsqueeze(0)
                ax = 0
            t, lay, n, nz = _device.column_view(t, ax, keep_f64=in64)  # strided views read in place
            if nz != c.in_nz[v]:
                raise ValueError(f"input {c.input_variables[v]} has {nz} levels, model expects {c.in_nz[v]}")
            if ncol is not None and n != ncol:
                raise ValueError("inputs disagree on the number of columns")
            ncol = n
            if not (torch.is_tensor(orig) and orig.is_cuda and t.data_ptr() == orig.data_ptr()):
                copied.append(c.input_variables[v])
            ts.append(t)
            lays.append(lay)
        ref = ts[0]
        ax0 = level_axes[0] if level_axes[0] is not None else 0
        if outputs is None:
            outputs = []
            for nz in c.out_nz:
                shape = list(ref.shape)
                shape[ax0] = nz
                outputs.append(torch.empty(shape, dtype=torch.float32, device=ref.device))
            out_axes = [ax0] * len(c.out_nz)
        else:
            out_axes = [out_level_axis] * len(outputs)
        olays = []
        for o, (t, ax) in enumerate(zip(outputs, out_axes)):
            lay, n, nz = _device.level_layout(t, ax)
            if nz != c.out_nz[o] or n != ncol:
                raise ValueError(f"output {o} has shape {tuple(t.shape)}")
            olays.append(lay)
        if any(l.ncol_blk != lays[0].ncol_blk for l in lays + olays):
            raise ValueError("all inputs/outputs must share the horizontal layout")
        bound = BoundForward(self, ts, lays, outputs, olays, ncol, prec, in64=in64)
        self._last_copied = copied
        self._last_cast_copy = False
        try:
            bound(stream)
        except NotImplementedError:
            if not in64:
                raise
            self._last_cast_copy = True  # the bound call below reads a float32 copy
            # models the float64 kernel does not cover (residual outputs, narrow widths):
            # cast first, as before
            return self.forward([t.to(torch.float32) for t in inputs], level_axes, outputs_arg, out_level_axis,
                                stream, precision)
        return outputs

    def bind(self, inputs: Sequence, level_axes: Optional[Sequence[int]] = None,
             outputs: Optional[Sequence] = None, out_level_axis: int = 0,
             precision: Optional[str] = None) -> "BoundForward":
        """Validate once and return a callable that re-launches the fused kernel on the
        same device buffers with no per-call argument marshalling (the prognostic loop
        calls predict on the same state arrays every timestep)."""
        self.forward(inputs, level_axes, outputs, out_level_axis, precision=precision)
        if getattr(self, "_last_cast_copy", False):
            raise NotImplementedError("this model reads float64 inputs through a float32 copy made per call "
                                      "(no 8-wave kernel or residual outputs): call forward() each step, "
                                      "or bind float32 buffers")
        if self._last_copied:
            # a bound call on a snapshot would never see the caller's in-place updates
            raise ValueError(f"bind: inputs {self._last_copied} are read through a copy (host/numpy, another "
                             "dtype than the kernel reads, or a layout the kernel cannot address); bind "
                             "device buffers the kernel reads in place, or call forward() each step")
        return self._last_bound

    # ---- host arrays in, host arrays out (the drop-in call on numpy data) ----------
    # one group per block from here on; two halves of the block axis from
    # _pipeline_two_min_bytes() on; one call below (profiles/r05y_pipeline_groups.log,
    # float64 (6, 79, n, n) T/q: C48 16 MiB one call 0.584 / two halves 0.62 / per tile
    # 0.90 ms; C96 66 MiB 2.09 / 1.94 / 2.03; C192 266 MiB 8.08 / 7.09 / 6.44)
    _PIPELINE_MIN_BYTES = 128 << 20

    @staticmethod
    def _pipeline_two_min_bytes() -> int:
        """Inputs from this size on (below _PIPELINE_MIN_BYTES) run as two pipelined
        halves of the block axis; FV3_HOST_TWO_GROUPS_MIB under FV3_VARIANTS=1 for A/B."""
        v = _native.variant("FV3_HOST_TWO_GROUPS_MIB")
        return (int(v) << 20) if v else (48 << 20)

    def forward_host(self, arrays: Sequence, level_axes: Optional[Sequence[int]] = None,
                     precision: Optional[str] = None, out: Optional[Sequence[np.ndarray]] = None) -> List[np.ndarray]:
        """numpy inputs -> numpy float32 outputs (pure_keras.py:98-118 predicts on host
        arrays).  The inputs cross as the runtime's pageable copies (caller memory is never
        page-locked) and land in device buffers of their own dtype (a float64 state is read in place
        by the kernel), cached per shape with the bound kernel.

        Inputs with a common leading block axis (tiles: ``(tile, z, y, x)``, level axis
        > 0) of ``_PIPELINE_MIN_BYTES`` and more run pipelined over the blocks on two
        streams (from ``_pipeline_two_min_bytes()`` on, over two halves of the block axis):
        group g + 1's host-to-device copies and group g's device-to-host copies overlap
        (PCIe is full duplex: in and out at once).  The
        same kernels on the same columns, so the outputs are bit-identical to one call.
        ``out``: float32 numpy arrays to write, else arrays in the library's page-locked
        arena (``transfer.empty_host``: DMA targets with no registration per call, their
        pages reused once the caller drops them)."""
        from . import transfer

        arrays = [np.ascontiguousarray(a) for a in arrays]
        axes = list(level_axes) if level_axes is not None else [0] * len(arrays)
        n0 = arrays[0].shape[0] if arrays[0].ndim else 0
        nbytes = sum(a.nbytes for a in arrays)
        tiled = n0 >= 2 and all(a.ndim >= 2 and a.shape[0] == n0 and ax is not None and ax > 0
                                for a, ax in zip(arrays, axes))
        # pipeline groups of blocks: one block each from _PIPELINE_MIN_BYTES on, two halves
        # from _PIPELINE_TWO_MIN_BYTES on (per-group host work ~60 us: fewer, larger groups
        # for the mid sizes), else one call
        groups = None
        if tiled and nbytes >= self._PIPELINE_MIN_BYTES:
            groups = tuple((t, t + 1) for t in range(n0))
        elif tiled and nbytes >= self._pipeline_two_min_bytes():
            groups = ((0, n0 // 2), (n0 // 2, n0))
        blocks = groups is not None
        key = (tuple((a.shape, a.dtype.str, ax) for a, ax in zip(arrays, axes)), precision, groups)
        ent = getattr(self, "_host_call", None)
        if ent is None or ent[0] != key or ent[1][0].device.index != torch.cuda.current_device():
            _device.require_gpu()
            dev = torch.device("cuda", torch.cuda.current_device())
            bufs = [torch.empty(a.shape, dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device=dev) for a in arrays]
            if blocks:
                sub_axes = [ax - 1 for ax in axes]
                runs = [self._bind_or_forward([b[g0] for b in bufs], sub_axes, precision) if g1 == g0 + 1 else
                        self._bind_or_forward([b[g0:g1] for b in bufs], axes, precision) for g0, g1 in groups]
                # (an idle stream for transfer.copy_fence, the out-copy stream)
                streams = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
            else:
                runs = [self._bind_or_forward(bufs, axes, precision)]
                streams = None
            ent = (key, bufs, runs, streams)
            self._host_call = ent
        _, bufs, runs, streams = ent

        st = transfer.stager(bufs[0].device)
        cur = torch.cuda.current_stream()
        hcur = cur.cuda_stream
        if streams is None:
            for a, b in zip(arrays, bufs):
                st.h2d(a, out=b, stream=cur)
            outs = runs[0]()
            host = _host_outputs(out, [tuple(o.shape) for o in outs])
            for h, o in zip(host, outs):
                transfer.host_copy(h, o, hcur)  # arena outputs: DMA; caller arrays: pageable
            cur.synchronize()
            return host
        _, s_out = streams
        s_out.wait_stream(cur)  # after whatever the caller queued on these buffers
        host = None
        lib = _native.load()
        kernel_out = _native.variant("FV3_D2H_KERNEL") == "1"
        self._last_kernel_out = False
        try:
            for gi, (g0, g1) in enumerate(groups):
                t = slice(g0, g1) if g1 > g0 + 1 else g0
                # group gi's inputs: the runtime's pageable copies, on the compute stream (the
                # host waits for them while s_out copies group gi - 1's outputs).  On a side
                # stream of their own the two directions ran nearly in sequence: C384 30.3 ms
                # against 22.2 ms (profiles/r05g_host_ab.json, pipe_in_*)
                for a, b in zip(arrays, bufs):
                    st.h2d(a[t], out=b[t], stream=cur)
                transfer.copy_fence(cur, streams[0])
                outs = runs[gi](cur)
                if host is None:
                    host = _host_outputs(out, [(n0,) + (tuple(o.shape[1:]) if g1 > g0 + 1 else tuple(o.shape))
                                               for o in outs])
                    # FV3_D2H_KERNEL=1: out-copies as a kernel storing into the arena's pages
                    # on the compute stream (fv3_copy_to_host), the copy engines keeping the
                    # in-copies; default: the copy engines both ways
                    kernel_out = kernel_out and all(transfer.is_arena(h) for h in host)
                done = False
                if kernel_out:
                    done = all(lib.fv3_copy_to_host(h[t].ctypes.data, o.data_ptr(), o.numel() * 4, hcur) == 0
                               for h, o in zip(host, outs))
                    kernel_out = done
                    self._last_kernel_out = done
                if not done:
                    ev = torch.cuda.Event()
                    ev.record(cur)
                    s_out.wait_event(ev)
                    for h, o in zip(host, outs):
                        transfer.host_copy(h[t], o, s_out.cuda_stream)
        finally:
            # every DMA into the arena `host` arrays has landed before they can be dropped
            # (an exception above would otherwise return their blocks to the cache with
            # copies still writing into them)
            cur.wait_stream(s_out)
            cur.synchronize()
        return host

    def _bind_or_forward(self, bufs, axes, precision):
        try:  # validated once; re-launched on the same buffers every call
            return self.bind(bufs, level_axes=axes, precision=precision)
        except (ValueError, NotImplementedError):  # inputs the kernel reads through a copy
            return lambda stream=None: self.forward(bufs, level_axes=axes, stream=stream, precision=precision)

    # ---- persistence -------------------------------------------------------------
    _WEIGHTS = "weights.npz"
    _CONFIG = "dense_config.yaml"

    def dump(self, path: str):
        os.makedirs(path, exist_ok=True)
        arrays = {}
        p = self.params
        for i, (k, b) in enumerate(zip(p["hidden_kernels"], p["hidden_biases"])):
            arrays[f"hidden_{i}/kernel"] = k
            arrays[f"hidden_{i}/bias"] = b
        for o, (k, b) in enumerate(zip(p["out_kernels"], p["out_biases"])):
            arrays[f"output_{o}/kernel"] = k
            arrays[f"output_{o}/bias"] = b
            arrays[f"output_{o}/mean"] = p["out_mean"][o]
            arrays[f"output_{o}/sigma"] = p["out_sigma"][o]
        for v in range(len(p["in_mean"])):
            arrays[f"input_{v}/mean"] = p["in_mean"][v]
            arrays[f"input_{v}/sigma"] = p["in_sigma"][v]
        np.savez(os.path.join(path, self._WEIGHTS), **arrays)
        with open(os.path.join(path, self._CONFIG), "w") as f:
            yaml.safe_dump(self.config.to_dict(), f)

    @classmethod
    def load(cls, path: str) -> "DenseColumnModel":
        with open(os.path.join(path, cls._CONFIG)) as f:
            config = DenseModelConfig.from_dict(yaml.safe_load(f))
        z = np.load(os.path.join(path, cls._WEIGHTS), allow_pickle=False)
        p = dict(
            hidden_kernels=[z[f"hidden_{i}/kernel"] for i in range(config.n_hidden)],
            hidden_biases=[z[f"hidden_{i}/bias"] for i in range(config.n_hidden)],
            out_kernels=[z[f"output_{o}/kernel"] for o in range(len(config.out_nz))],
            out_biases=[z[f"output_{o}/bias"] for o in range(len(config.out_nz))],
            out_mean=[z[f"output_{o}/mean"] for o in range(len(config.out_nz))],
            out_sigma=[z[f"output_{o}/sigma"] for o in range(len(config.out_nz))],
            in_mean=[z[f"input_{v}/mean"] for v in range(len(config.in_nz))],
            in_sigma=[z[f"input_{v}/sigma"] for v in range(len(config.in_nz))],
        )
        return cls(config, p)


def _host_outputs(out, shapes):
    if out is None:
        from . import transfer

        # page-locked arena blocks (reused once the caller drops them)
        return [transfer.empty_host(sh, np.float32) for sh in shapes]
    out = list(out)
    if len(out) != len(shapes) or any(not (isinstance(o, np.ndarray) and o.dtype == np.float32 and o.shape == sh
                                           and o.flags.c_contiguous and o.flags.writeable)
                                      for o, sh in zip(out, shapes)):
        raise ValueError(f"out: writable contiguous float32 numpy arrays of shapes {shapes}")
    return out


class BoundForward:
    """A validated dense forward over fixed device buffers (see DenseColumnModel.bind)."""

    def __init__(self, model: "DenseColumnModel", inputs, in_layouts, outputs, out_layouts, ncol: int,
                 precision: str = "f32", in64: bool = False):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
        self.precision = precision
        self._prec = PRECISIONS[precision]
        self.model = model
        self.inputs = list(inputs)  # keep the tensors alive
        self.outputs = list(outputs)
        self._in_ptrs = (ctypes.c_void_p * len(inputs))(*[t.data_ptr() for t in inputs])
        self._out_ptrs = (ctypes.c_void_p * len(outputs))(*[t.data_ptr() for t in outputs])
        self._in_l = (_native.Layout * len(in_layouts))(*in_layouts)
        self._out_l = (_native.Layout * len(out_layouts))(*out_layouts)
        self._ncol = int(ncol)
        self._handle = model.handle()
        self._in64 = bool(in64)  # float64 inputs: fv3_dense_forward_f64in (exact f32 only)
        lib = _native.load()
        self._fn = lib.fv3_dense_forward_f64in if self._in64 else lib.fv3_dense_forward_ex
        model._last_bound = self

    def __call__(self, stream=None):
        """``stream``: a torch stream, a raw hipStream_t handle (int), or None (current)."""
        h = stream if isinstance(stream, int) else _device.stream_handle(stream, self.inputs + self.outputs)
        if self._handle not in self.model._handles.values():
            raise RuntimeError("BoundForward: the model was closed; bind again")
        if self._in64:
            st = self._fn(self._handle, self._in_ptrs, self._in_l, self._out_ptrs, self._out_l, self._ncol, h)
        else:
            st = self._fn(self._handle, self._in_ptrs, self._in_l, self._out_ptrs, self._out_l, self._ncol,
                          self._prec, h)
        if st:
            _native.check(st, "dense_forward")
        return self.outputs
