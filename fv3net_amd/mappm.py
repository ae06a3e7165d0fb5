"""Drop-in for the reference's f2py ``mappm`` module plus a device-resident API.

Reference: ``external/mappm/mappm/__init__.py`` exports ``mappm`` (and
``interpolate_2d``) compiled from ``mappm.f90``; ``vcm.cubedsphere.regridz``
calls ``mappm.mappm(p_in, f_in, p_out, 1, n_columns, iv, kord, dummy_ptop)``
with C-ordered ``(ncol, nlev)`` float64 arrays and gets ``(ncol, kn)`` float32
back (``regridz.py:268-275``, dtype pinned by ``tests/test_mappm.py:14,28,42``).
"""
import ctypes

import numpy as np

from . import _device, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def mappm_device(pe1, q1, pe2, iv: int = 1, kord: int = 1, out=None, stream=None, exact: bool = False):
    """Remap on device.  ``pe1 [km+1, ncol]``, ``q1 [km, ncol]``, ``pe2 [kn+1, ncol]``
    float32 CUDA tensors (column fastest, the Fortran pe1(i,k) order; strided views
    such as a column slice are read in place); returns ``q2 [kn, ncol]`` (or writes
    ``out``).  Asynchronous on the current stream.

    ``exact=False`` (default): north_star's floating-point contract (within 1e-5 rel of
    the reference; reciprocal divisions, FMA, hardware MAX / MIN, csrc/mappm_core.h) for
    finite inputs.  ``exact=True``: the reference build's arithmetic, bit for bit, for
    every input (NaNs included)."""
    _device.require_gpu()
    for a in (pe1, q1, pe2):
        if len(getattr(a, "shape", ())) != 2:
            raise ValueError("pe1, q1, pe2 must be 2-D [level, column]")
    pe1, l1, n1, kp1 = _device.column_view(pe1, 0)
    q1, lq, ncol, km = _device.column_view(q1, 0)
    pe2, l2, n2, kp2 = _device.column_view(pe2, 0)
    kn = kp2 - 1
    if kp1 != km + 1:
        raise ValueError("f_in must have a vertical dimension one shorter than p_in")
    if n1 != ncol or n2 != ncol:
        raise ValueError("All dimensions except vertical must be same size for p_in, f_in and p_out")
    if out is None:
        out = torch.empty((kn, ncol), dtype=torch.float32, device=q1.device)
    if tuple(out.shape) != (kn, ncol) or out.dtype != torch.float32:
        raise ValueError(f"out must be float32 ({kn}, {ncol})")
    lo, _, _ = _device.level_layout(out, 0)
    lib = _native.load()
    st = lib.fv3_mappm_ex(_device.ptr(pe1), l1, _device.ptr(q1), lq, _device.ptr(pe2), l2, _device.ptr(out), lo,
                          ncol, km, kn, int(iv), int(kord), 0.0, _native.arith(exact),
                          _device.stream_handle(stream, [pe1, q1, pe2, out]))
    _native.check(st, "mappm")
    return out


class MappmPlan:
    """A prepared ``mappm_device`` call on fixed device buffers: the argument checks,
    column layouts and stream handle are resolved once, so each ``plan()`` is a single
    C-ABI call (the per-call Python work of ``mappm_device`` is ~20 us, more than the
    C12 kernel itself).  The buffers must stay alive and keep their shapes; their
    contents may change between calls.  Same results as ``mappm_device``."""

    def __init__(self, pe1, q1, pe2, iv: int = 1, kord: int = 1, out=None, stream=None, exact: bool = False):
        self.out = mappm_device(pe1, q1, pe2, iv, kord, out=out, stream=stream, exact=exact)  # validates, first run
        views = [_device.column_view(a, 0) for a in (pe1, q1, pe2)]
        for name, a, v in zip(("pe1", "q1", "pe2"), (pe1, q1, pe2), views):
            if not (torch.is_tensor(a) and a.is_cuda and v[0].data_ptr() == a.data_ptr()):
                # a plan over a copy would keep remapping the stale snapshot
                raise ValueError(f"MappmPlan: {name} is read through a copy (host, float64 or an unaddressable "
                                 "layout); pass float32 CUDA buffers, or call mappm_device each time")
        (pe1, l1, _, _), (q1, lq, ncol, km), (pe2, l2, _, kp2) = views
        lo, _, _ = _device.level_layout(self.out, 0)
        self._keep = (pe1, q1, pe2)
        self._stream = stream
        self._fn = _native.load().fv3_mappm_ex
        self._args = (_device.ptr(pe1), l1, _device.ptr(q1), lq, _device.ptr(pe2), l2, _device.ptr(self.out), lo,
                      ncol, km, kp2 - 1, int(iv), int(kord), 0.0, _native.arith(exact), _device.stream_handle(stream))

    def __call__(self):
        if self._stream is not None:
            # a side-stream plan is ordered after the current stream's writes to the
            # bound buffers on EVERY call, not only when it was built
            _device.stream_handle(self._stream)
        _native.check(self._fn(*self._args), "mappm")
        return self.out


def _multi_args(pe1, q1s, pe2, iv, kord, outs, stream, exact):
    """Validated argument tuple of fv3_mappm_multi (+ the outputs and the tensors read)."""
    _device.require_gpu()
    q1s = list(q1s)
    if not 1 <= len(q1s) <= 64:
        raise ValueError("mappm_multi: 1..64 fields")
    for a in [pe1, pe2] + q1s:
        if len(getattr(a, "shape", ())) != 2:
            raise ValueError("pe1, q1, pe2 must be 2-D [level, column]")
    pe1, l1, n1, kp1 = _device.column_view(pe1, 0)
    pe2, l2, n2, kp2 = _device.column_view(pe2, 0)
    kn = kp2 - 1
    views = [_device.column_view(q, 0) for q in q1s]
    for _, _, ncol, km in views:
        if kp1 != km + 1:
            raise ValueError("f_in must have a vertical dimension one shorter than p_in")
        if ncol != n1 or n2 != n1:
            raise ValueError("All dimensions except vertical must be same size for p_in, f_in and p_out")
    ncol = n1
    if outs is None:
        outs = [torch.empty((kn, ncol), dtype=torch.float32, device=pe1.device) for _ in q1s]
    outs = list(outs)
    if len(outs) != len(q1s):
        raise ValueError("mappm_multi: one output per field")
    for o in outs:
        if tuple(o.shape) != (kn, ncol) or o.dtype != torch.float32:
            raise ValueError(f"out must be float32 ({kn}, {ncol})")
    lo = [_device.level_layout(o, 0)[0] for o in outs]
    nf = len(q1s)
    qp = (ctypes.c_void_p * nf)(*[_device.ptr(v[0]) for v in views])
    ql = (_native.Layout * nf)(*[v[1] for v in views])
    op = (ctypes.c_void_p * nf)(*[_device.ptr(o) for o in outs])
    ol = (_native.Layout * nf)(*lo)
    args = (_device.ptr(pe1), l1, qp, ql, _device.ptr(pe2), l2, op, ol, nf, ncol, views[0][3], kn, int(iv),
            int(kord), 0.0, _native.arith(exact), _device.stream_handle(stream))
    return args, outs, [pe1, pe2] + [v[0] for v in views]


def mappm_device_multi(pe1, q1s, pe2, iv: int = 1, kord: int = 1, out=None, stream=None, exact: bool = False):
    """``mappm_device`` for several fields on the same ``pe1`` / ``pe2`` (one reference
    ``mappm.mappm`` call per field, as ``coarsen_restarts_on_pressure`` issues them,
    coarsen_restarts.py:411-516): for kord <= 7 the fields go two per streaming pass,
    sharing the pressure-only arithmetic; with ``exact=True`` each result is
    bit-identical to ``mappm_device(..., exact=True)`` on that field (the default
    arithmetic as in ``mappm_device``).  Returns the list of ``[kn, ncol]`` outputs."""
    args, outs, keep = _multi_args(pe1, q1s, pe2, iv, kord, out, stream, exact)
    _native.check(_native.load().fv3_mappm_multi(*args), "mappm")
    _device.keep_for(stream, keep + outs)
    return outs


class MappmMultiPlan:
    """``MappmPlan`` for ``mappm_device_multi``: one C-ABI call per step on fixed
    float32 CUDA buffers (read in place; a copy would go stale, so it is refused)."""

    def __init__(self, pe1, q1s, pe2, iv: int = 1, kord: int = 1, out=None, stream=None, exact: bool = False):
        q1s = list(q1s)
        args, self.out, keep = _multi_args(pe1, q1s, pe2, iv, kord, out, stream, exact)
        for name, a, v in zip(["pe1", "pe2"] + [f"q1[{i}]" for i in range(len(q1s))], [pe1, pe2] + q1s, keep):
            if not (torch.is_tensor(a) and a.is_cuda and v.data_ptr() == a.data_ptr()):
                raise ValueError(f"MappmMultiPlan: {name} is read through a copy (host, float64 or an "
                                 "unaddressable layout); pass float32 CUDA buffers")
        self._keep = keep
        self._stream = stream
        self._fn = _native.load().fv3_mappm_multi
        self._args = args
        self()

    def __call__(self):
        if self._stream is not None:  # ordered after current-stream writes, every call
            _device.stream_handle(self._stream)
        _native.check(self._fn(*self._args), "mappm")
        return self.out


def mappm(pe1, q1, pe2, i1, i2, iv, kord, ptop):
    """f2py-compatible signature of ``mappm.mappm`` (mappm.f90:10).

    ``pe1 (ncol, km+1)``, ``q1 (ncol, km)``, ``pe2 (ncol, kn+1)`` host arrays.  As in the
    f2py signature (``pe1(i1:i2, km+1)``), the arrays hold exactly the columns
    ``i1..i2`` (1-based, inclusive): ``ncol == i2 - i1 + 1``; returns float32
    ``(ncol, kn)``.  The reference's own arithmetic (``exact=True``): this is the drop-in
    for the f2py module, bit-identical to it.
    """
    i1 = int(i1)
    i2 = int(i2)
    pe1 = np.asarray(pe1, dtype=np.float32)
    q1 = np.asarray(q1, dtype=np.float32)
    pe2 = np.asarray(pe2, dtype=np.float32)
    if pe1.ndim != 2 or q1.ndim != 2 or pe2.ndim != 2:
        raise ValueError("mappm expects 2-D (column, level) arrays")
    if not (pe1.shape[0] == q1.shape[0] == pe2.shape[0] == i2 - i1 + 1):
        raise ValueError(f"mappm: arrays hold {pe1.shape[0]} columns, i1..i2 = {i1}..{i2} names {i2 - i1 + 1}")
    res = mappm_device(pe1.T, q1.T, pe2.T, iv=int(iv), kord=int(kord), exact=True)
    return res.T.contiguous().cpu().numpy()
