"""ORACLE (test infrastructure only): mappm via ctypes.

Two independent CPU implementations of ``mappm`` (reference
``/root/reference/external/mappm/mappm/mappm.f90:10-126``):

* ``oracle_mappm``    — our plain-C restatement, ``oracle/mappm_oracle.c``.
* ``reference_mappm`` — the reference Fortran itself, compiled unmodified by
  ``oracle/Makefile`` into ``oracle/_ref/libmappm_ref.so`` (flang).  Its automatic
  arrays live on the stack, so it is called in chunks of <= 512 columns.

Both take column-fastest arrays: ``pe1[km+1, ncol]``, ``q1[km, ncol]``,
``pe2[kn+1, ncol]`` (float32) and return ``q2[kn, ncol]`` (float32), the same
layout the Fortran sees after f2py's C->F copy (``regridz.py:268-275``).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(_HERE, "_build", "liboracle.so")
REF_SO = os.path.join(_HERE, "_ref", "libmappm_ref.so")
_REF_CHUNK = 512

_oracle_lib = None
_ref_lib = None


def build():
    """Build the C restatement (and the flang reference when its sources exist)."""
    subprocess.run(["make", "-s", "-f", os.path.join(_HERE, "Makefile")], check=True)


def _load_oracle():
    global _oracle_lib
    if _oracle_lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        lib = ctypes.CDLL(ORACLE_SO)
        lib.oracle_mappm.restype = ctypes.c_int
        lib.oracle_mappm.argtypes = [
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
        ]
        _oracle_lib = lib
    return _oracle_lib


def reference_available() -> bool:
    return os.path.exists(REF_SO)


def _load_ref():
    global _ref_lib
    if _ref_lib is None:
        _ref_lib = ctypes.CDLL(REF_SO)
    return _ref_lib


def _prep(pe1, q1, pe2):
    pe1 = np.ascontiguousarray(pe1, dtype=np.float32)
    q1 = np.ascontiguousarray(q1, dtype=np.float32)
    pe2 = np.ascontiguousarray(pe2, dtype=np.float32)
    if pe1.ndim != 2 or q1.ndim != 2 or pe2.ndim != 2:
        raise ValueError("expected 2-D [level, column] arrays")
    km = q1.shape[0]
    kn = pe2.shape[0] - 1
    ncol = q1.shape[1]
    if pe1.shape != (km + 1, ncol) or pe2.shape[1] != ncol:
        raise ValueError("inconsistent shapes")
    return pe1, q1, pe2, km, kn, ncol


def oracle_mappm(pe1, q1, pe2, iv=1, kord=1):
    """C restatement of mappm.f90:10-126 (column-fastest arrays)."""
    pe1, q1, pe2, km, kn, ncol = _prep(pe1, q1, pe2)
    q2 = np.empty((kn, ncol), dtype=np.float32)
    rc = _load_oracle().oracle_mappm(
        km, pe1.ctypes.data, q1.ctypes.data, kn, pe2.ctypes.data, q2.ctypes.data,
        ncol, int(iv), int(kord),
    )
    if rc != 0:
        raise ValueError(f"oracle_mappm rejected km={km} kn={kn}")
    return q2


def reference_mappm(pe1, q1, pe2, iv=1, kord=1, ptop=0.0):
    """The reference Fortran ``mappm`` (flang build of mappm.f90), chunked."""
    pe1, q1, pe2, km, kn, ncol = _prep(pe1, q1, pe2)
    lib = _load_ref()
    q2 = np.empty((kn, ncol), dtype=np.float32)
    c_int = ctypes.c_int
    for s in range(0, ncol, _REF_CHUNK):
        e = min(ncol, s + _REF_CHUNK)
        n = e - s
        a = np.asfortranarray(pe1[:, s:e].T)  # Fortran (i, k): column fastest
        b = np.asfortranarray(q1[:, s:e].T)
        c = np.asfortranarray(pe2[:, s:e].T)
        out = np.zeros((n, kn), dtype=np.float32, order="F")
        lib.mappm_(
            ctypes.byref(c_int(km)), a.ctypes.data_as(ctypes.c_void_p),
            b.ctypes.data_as(ctypes.c_void_p), ctypes.byref(c_int(kn)),
            c.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
            ctypes.byref(c_int(1)), ctypes.byref(c_int(n)), ctypes.byref(c_int(int(iv))),
            ctypes.byref(c_int(int(kord))), ctypes.byref(ctypes.c_float(ptop)),
        )
        q2[:, s:e] = out.T
    return q2
