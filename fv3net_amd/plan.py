"""A launch plan: the launches of a timestep, bound once, issued by one C-ABI call.

The prognostic run applies the same state buffers every step (runtime/loop.py:604-628
around runtime/steppers/machine_learning.py:239-309).  The per-step launches are bound
once already (``DenseColumnModel.bind``, ``stepper.BoundEpilogue``,
``distributed.bind_*``); a ``LaunchPlan`` records them, in order, in a native plan
(csrc/plan.cpp, ``fv3_plan_*``) and replays them on the caller's stream with one foreign
call: on one rank's 6,912 columns the per-call host work of five separate calls took
longer than the kernels.  The plan holds references to the bound
objects, so their buffers stay allocated while it lives.
"""
import ctypes

from . import _device, _native

# bound reduction launch -> the plan op taking the same arguments (minus the stream)
_PLAN_OPS = {
    "fv3_area_weighted_sums_f64": "fv3_plan_add_area_weighted_sums_f64",
    "fv3_area_weighted_row_sums_f64": "fv3_plan_add_area_weighted_row_sums_f64",
    "fv3_level_sums_u8": "fv3_plan_add_level_sums_u8",
    "fv3_fold_rows": "fv3_plan_add_fold_rows",
    "fv3_step_partials_f64": "fv3_plan_add_step_partials_f64",
    "fv3_fold_rows_repeat": "fv3_plan_add_fold_rows_repeat",
}


class LaunchPlan:
    """``add(bound)`` for a BoundForward, a BoundEpilogue or a bound reduction
    (``distributed.bind_*``: the float64 sums, row sums, uint8 level sums and the row
    fold); ``copy(dst, src)`` for a device-to-device copy; calling the plan issues every
    op in order on the stream (a torch stream, a raw hipStream_t int, or None for the
    current one)."""

    def __init__(self, ops=()):
        self._lib = _native.load()
        h = ctypes.c_void_p()
        _native.check(self._lib.fv3_plan_create(ctypes.byref(h)), "plan_create")
        self._h = h.value
        self._keep = []
        for op in ops:
            self.add(op)

    def __len__(self) -> int:
        return int(self._lib.fv3_plan_size(self._h))

    def add(self, bound):
        from .dense import BoundForward
        from .stepper import BoundEpilogue

        lib = self._lib
        if isinstance(bound, BoundForward):
            st = lib.fv3_plan_add_dense_forward(
                self._h, bound._handle, ctypes.cast(bound._in_ptrs, ctypes.POINTER(ctypes.c_void_p)), bound._in_l,
                bound._out_ptrs, bound._out_l, bound._ncol, bound._prec, int(bound._in64))
            if not st:
                bound.model._plans.add(self)  # the model refuses close() while this plan lives
        elif isinstance(bound, BoundEpilogue):
            st = lib.fv3_plan_add_ml_epilogue(self._h, ctypes.byref(bound._io), *bound._args[1:])
        elif isinstance(bound, _device.BoundLaunch) and getattr(bound.fn, "__name__", None) in _PLAN_OPS:
            st = getattr(lib, _PLAN_OPS[bound.fn.__name__])(self._h, *bound.args)
        else:
            raise NotImplementedError(f"no plan op for {bound!r}")
        _native.check(st, "plan_add")
        self._keep.append(bound)
        return self

    def copy(self, dst, src):
        """Device-to-device copy of ``src``'s bytes into ``dst`` (contiguous CUDA tensors
        of equal byte size)."""
        n = src.numel() * src.element_size()
        if not (dst.is_cuda and src.is_cuda and dst.is_contiguous() and src.is_contiguous()
                and dst.numel() * dst.element_size() == n):
            raise ValueError("plan copy: contiguous CUDA tensors of equal byte size")
        _native.check(self._lib.fv3_plan_add_copy(self._h, dst.data_ptr(), src.data_ptr(), n), "plan_add_copy")
        self._keep.append((dst, src))
        return self

    def repeat(self, dst, src, times: int):
        """``times`` back-to-back copies of ``src``'s bytes into ``dst`` (contiguous CUDA
        tensors, dst holding exactly ``times`` copies), one launch."""
        n = src.numel() * src.element_size()
        if not (dst.is_cuda and src.is_cuda and dst.is_contiguous() and src.is_contiguous()
                and dst.numel() * dst.element_size() == n * times and n % 4 == 0):
            raise ValueError("plan repeat: contiguous CUDA tensors, dst = times x src bytes (a multiple of 4)")
        _native.check(self._lib.fv3_plan_add_repeat(self._h, dst.data_ptr(), src.data_ptr(), n, int(times)),
                      "plan_add_repeat")
        self._keep.append((dst, src))
        return self

    def __call__(self, stream=None):
        h = stream if isinstance(stream, int) else _device.stream_handle(stream)
        st = self._lib.fv3_plan_run(self._h, h)
        if st:
            _native.check(st, "plan_run")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fv3_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
