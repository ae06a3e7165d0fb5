"""CPU tests: pin the mappm oracle, and check the product's streaming algorithm
(compiled for the host, test-only) against it.  No GPU needed.

Reference KATs: external/vcm/tests/test_mappm.py:5-44.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle.mappm import oracle_mappm, reference_available, reference_mappm

HOST_SRC = os.path.join(ROOT, "tests", "native", "mappm_host.cpp")
HOST_SO = os.path.join(ROOT, "tests", "_build", "libmappm_host.so")


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return bool(same.all())


# --- test_mappm.py KATs (values copied as data) ---------------------------------
KATS = [
    # (p_in, f_in, p_out, expected)  test_mappm.py:5-16, 19-30, 33-44
    ([0.0, 1.0, 2.0, 3.0, 4.0, 5.0], [0.0, 1.0, 2.0, 3.0, 4.0], [0.5, 1.2, 2.4, 2.8, 3.2, 4.5],
     [0.35, 1.3, 2.1, 2.5, 3.35]),
    ([1.0, 2.0, 3.0, 4.0, 5.0], [1.5, 2.5, 3.5, 4.5], [0.0, 2.5, 3.5, 4.5, 50.0],
     [1.5, 3.0, 4.0, 4.502747]),
    ([1.0, 2.0, 3.0, 2.0, 5.0], [np.nan] * 4, [0.0, 2.5, 3.5, 4.5, 50.0], [np.nan] * 4),
]


@pytest.mark.parametrize("kat", KATS, ids=["identity", "out_of_bounds", "nans"])
def test_oracle_reproduces_reference_kats(kat):
    p_in, f_in, p_out, expected = (np.asarray(v, np.float64)[:, None] for v in kat)
    res = oracle_mappm(p_in, f_in, p_out, iv=1, kord=1)
    assert res.dtype == np.float32
    np.testing.assert_almost_equal(res, expected.astype(np.float32), decimal=5)


def test_oracle_matches_reference_golden_vectors():
    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    n = 0
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = oracle_mappm(pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord))
                    assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv)
                    n += 1
    for kord in (1, 10):
        res = oracle_mappm(g["c12_pe1"], g["c12_q"], g["c12_pe2"], 1, kord)
        assert _bits_equal(res, g[f"c12_k{kord}_iv1"])
    assert n == len(g["cases"]) * len(g["kords"]) * len(g["ivs"]) * 2


@pytest.mark.skipif(not reference_available(), reason="reference flang build not present")
@pytest.mark.parametrize("kord", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, -3])
def test_oracle_matches_live_reference(kord):
    rng = np.random.default_rng(kord + 100)
    for iv in (0, 1, -1, 2, -2):
        if iv == -2 and kord > 7:
            continue  # reference reads an uninitialised qs (mappm.f90:33,49): UB
        km, kn, ncol = 79, 50, 300
        delp = rng.uniform(100, 2000, (km, ncol)).astype(np.float32)
        pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                              300 + np.cumsum(delp, 0, dtype=np.float32)])
        pe2 = np.sort(rng.uniform(pe1[0] * 0.9, pe1[-1] * 1.02, (kn + 1, ncol)), axis=0).astype(np.float32)
        q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
        assert _bits_equal(oracle_mappm(pe1, q, pe2, iv, kord), reference_mappm(pe1, q, pe2, iv, kord))


# --- the product algorithm, host-compiled (test-only build) ----------------------
@pytest.fixture(scope="module")
def host_lib():
    os.makedirs(os.path.dirname(HOST_SO), exist_ok=True)
    # each process (pytest-xdist worker) builds its own file and renames it into place,
    # so no worker loads a library another one is still writing
    tmp = f"{HOST_SO}.{os.getpid()}.tmp"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                    "-o", tmp, HOST_SRC], check=True)
    own = f"{HOST_SO[:-3]}.{os.getpid()}.so"
    os.replace(tmp, own)
    lib = ctypes.CDLL(own)
    os.unlink(own)  # the mapping stays valid; nothing is left behind
    for fn in (lib.host_mappm, lib.host_mappm_cursor, lib.host_mappm_generic, lib.host_mappm_carry,
               lib.host_mappm_ring):
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    lib.host_mappm_cs_prefetch.restype = ctypes.c_int
    lib.host_mappm_cs_prefetch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.host_mappm_cs_tail.restype = ctypes.c_int
    lib.host_mappm_cs_tail.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    return lib


def _host(lib, pe1, q, pe2, iv, kord, cursor=False):
    pe1, q, pe2 = (np.ascontiguousarray(a, np.float32) for a in (pe1, q, pe2))
    out = np.empty((pe2.shape[0] - 1, q.shape[1]), np.float32)
    fn = {True: lib.host_mappm_cursor, False: lib.host_mappm, "generic": lib.host_mappm_generic,
          "carry": lib.host_mappm_carry, "ring": lib.host_mappm_ring}[cursor]
    rc = fn(q.shape[0], pe1.ctypes.data, q.ctypes.data, pe2.shape[0] - 1, pe2.ctypes.data, out.ctypes.data,
            q.shape[1], iv, kord)
    assert rc == 0
    return out


def test_streaming_algorithm_matches_golden(host_lib):
    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = _host(host_lib, pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord))
                    assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv)
                    if kord <= 7:  # the device mappm kernel's build (loads carried one level ahead)
                        res = _host(host_lib, pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord), cursor="carry")
                        assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv, "carry")
                        # the fast single-field kernel's build (window in register rings)
                        res = _host(host_lib, pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord), cursor="ring")
                        assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv, "ring")


@pytest.mark.parametrize("km", [4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 17, 33, 79, 80, 127])
def test_ring_window_is_bit_identical(host_lib, km):
    """The column with its window in register rings (mappm_ppm_column<.., RING>: the layer
    loop in groups of 5 ring phases) gives the shifting window's bits for every kord <= 7
    and iv, for level counts around the group boundaries, on rough columns with shared
    and unsorted output edges."""
    rng = np.random.default_rng(km)
    ncol = 64
    for kn in (max(1, km // 2), km, km + 7):
        for kord in (1, 2, 3, 4, 5, 6, 7):
            for iv in (0, 1, -1, 2):
                delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
                pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                      300 + np.cumsum(delp, 0, dtype=np.float32)])
                pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
                pe2[:, :3] = pe2[::-1, :3]
                q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
                with np.errstate(all="ignore"):
                    ref = _host(host_lib, pe1, q, pe2, iv, kord)
                    ring = _host(host_lib, pe1, q, pe2, iv, kord, cursor="ring")
                assert _bits_equal(ring, ref), (km, kn, kord, iv)


@pytest.mark.parametrize("kat", KATS, ids=["identity", "out_of_bounds", "nans"])
def test_streaming_algorithm_kats(host_lib, kat):
    p_in, f_in, p_out, expected = (np.asarray(v, np.float64)[:, None] for v in kat)
    res = _host(host_lib, p_in, f_in, p_out, 1, 1)
    np.testing.assert_almost_equal(res, expected.astype(np.float32), decimal=5)


@pytest.mark.parametrize("km,kn", [(4, 3), (5, 9), (6, 2), (79, 79), (79, 50), (127, 40)])
def test_streaming_algorithm_matches_oracle_random(host_lib, km, kn):
    rng = np.random.default_rng(km * 1000 + kn)
    for kord in (1, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17):
        for iv in (0, 1, -1, 2):
            ncol = 64
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
            # shared edges exercise the equality branches of the layer search
            m = min(km, kn) + 1
            pe2[: m // 2] = pe1[: m // 2]
            pe2 = np.sort(pe2, 0)
            q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            assert _bits_equal(_host(host_lib, pe1, q, pe2, iv, kord),
                               oracle_mappm(pe1, q, pe2, iv, kord)), (kord, iv)


@pytest.mark.parametrize("km,kn", [(4, 3), (5, 9), (6, 2), (79, 79), (79, 50), (127, 40)])
def test_output_driven_cursor_is_bit_identical(host_lib, km, kn):
    """The output-driven PpmCursor (fused coarsen kernel) == the streaming column ==
    the oracle, bit for bit, for every PPM kord and iv, incl. shared edges and
    output edges beyond the input column."""
    rng = np.random.default_rng(km * 7 + kn)
    for kord in (0, 1, 2, 3, 4, 5, 6, 7):
        for iv in (0, 1, -1, 2, -2):
            ncol = 64
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
            m = min(km, kn) + 1
            pe2[: m // 2] = pe1[: m // 2]
            pe2 = np.sort(pe2, 0)
            q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            cur = _host(host_lib, pe1, q, pe2, iv, kord, cursor=True)
            assert _bits_equal(cur, _host(host_lib, pe1, q, pe2, iv, kord)), (kord, iv)
            assert _bits_equal(cur, oracle_mappm(pe1, q, pe2, iv, kord)), (kord, iv)


def test_output_driven_cursor_golden(host_lib):
    g = np.load(os.path.join(GOLDEN, "mappm_golden.npz"))
    for ci in range(len(g["cases"])):
        pe1, pe2 = g[f"c{ci}_pe1"], g[f"c{ci}_pe2"]
        for kord in g["kords"]:
            if kord > 7:
                continue
            for iv in g["ivs"]:
                for qn in ("qs", "qr"):
                    res = _host(host_lib, pe1, g[f"c{ci}_{qn}"], pe2, int(iv), int(kord), cursor=True)
                    assert _bits_equal(res, g[f"c{ci}_{qn}_k{kord}_iv{iv}"]), (ci, qn, kord, iv)


@pytest.mark.parametrize("km,kn", [(4, 40), (79, 79), (79, 300), (20, 5)])
def test_streaming_degenerate_edges(host_lib, km, kn):
    """remap_layer_fast (the streaming consumer) == oracle bit for bit where the
    event mix per layer is extreme: zero-thickness input layers (repeated pe1),
    runs of repeated output edges, output grids much finer than the input (many
    inside-layer outputs per layer, each reusing the previous edge's position),
    output edges above the old top and below the old surface."""
    rng = np.random.default_rng(km * 31 + kn)
    for kord in (1, 4, 5, 6, 7, 10):
        for iv in (0, 1, -1):
            ncol = 64
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            delp[rng.random((km, ncol)) < 0.1] = 0.0  # zero-thickness layers
            delp[:2] = np.maximum(delp[:2], 1.0)       # keep the end cubics finite
            delp[-2:] = np.maximum(delp[-2:], 1.0)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = rng.uniform(pe1[0] * 0.7, pe1[-1] * 1.2, (kn + 1, ncol)).astype(np.float32)
            rep = rng.random((kn + 1, ncol)) < 0.2
            pe2[1:][rep[1:]] = pe2[:-1][rep[1:]]       # repeated output edges
            snap = rng.random((kn + 1, ncol)) < 0.2    # output edges on input edges
            idx = rng.integers(0, km + 1, (kn + 1, ncol))
            pe2[snap] = np.take_along_axis(pe1, idx, 0)[snap]
            pe2 = np.sort(pe2, 0)
            q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            with np.errstate(all="ignore"):
                exp = oracle_mappm(pe1, q, pe2, iv, kord)
            assert _bits_equal(_host(host_lib, pe1, q, pe2, iv, kord), exp), (kord, iv)


@pytest.mark.parametrize("km,kn", [(4, 40), (79, 79), (79, 300), (20, 5)])
def test_fast_consumer_equals_reference_loop_unsorted(host_lib, km, kn):
    """remap_layer_fast == remap_layer bit for bit on UNSORTED output edges too
    (outputs that step back above the current layer, leave and re-enter the column):
    the rearrangement assumes no ordering."""
    rng = np.random.default_rng(km * 17 + kn)
    for kord in (1, 4, 5, 6, 7):
        for iv in (0, 1, -1):
            ncol = 64
            # some input layers of negative thickness too (non-monotone pe1)
            delp = rng.uniform(-300 if iv else 1, 3000, (km, ncol)).astype(np.float32)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1.min() * 0.7, pe1.max() * 1.2, (kn + 1, ncol)), 0).astype(np.float32)
            swap = rng.random((kn, ncol)) < 0.15  # local inversions
            a, b = pe2[:-1].copy(), pe2[1:].copy()
            pe2[:-1][swap], pe2[1:][swap] = b[swap], a[swap]
            q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            with np.errstate(all="ignore"):
                fast = _host(host_lib, pe1, q, pe2, iv, kord)
                ref = _host(host_lib, pe1, q, pe2, iv, kord, cursor="generic")
            assert _bits_equal(fast, ref), (kord, iv)


@pytest.mark.parametrize("nf", [1, 2, 3, 4])
@pytest.mark.parametrize("km,kn", [(4, 40), (79, 79), (79, 50), (20, 5)])
def test_multi_field_streaming_bit_identical(host_lib, nf, km, kn):
    """mappm_ppm_columns<NF> (NF fields on one pressure column, the pressure-only
    divisions, positions and decisions shared) == the single-field streaming column
    for each field, bit for bit, for every PPM kord and iv, incl. degenerate edges."""
    import ctypes

    fn = host_lib.host_mappm_multi
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(km * 13 + kn * 7 + nf)
    ncol = 48
    for kord in (0, 1, 2, 3, 4, 5, 6, 7):
        for iv in (0, 1, -1, 2, -2):
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            delp[rng.random((km, ncol)) < 0.05] = 0.0
            delp[:2] = np.maximum(delp[:2], 1.0)
            delp[-2:] = np.maximum(delp[-2:], 1.0)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
            m = min(km, kn) + 1
            pe2[: m // 3] = pe1[: m // 3]
            pe2 = np.sort(pe2, 0)
            q = (rng.normal(0, 1, (nf, km, ncol)) * rng.choice([1e-4, 1, 300], (nf, km, ncol))).astype(np.float32)
            out = np.empty((nf, kn, ncol), np.float32)
            with np.errstate(all="ignore"):
                assert fn(nf, km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data, out.ctypes.data, ncol,
                          iv, kord) == 0
                for f in range(nf):
                    assert _bits_equal(out[f], _host(host_lib, pe1, q[f], pe2, iv, kord)), (nf, f, kord, iv)
                if nf == 2:  # the device pair kernel's build (loads carried one level ahead)
                    carry = np.empty_like(out)
                    cf = host_lib.host_mappm_pair_carry
                    cf.restype = ctypes.c_int
                    cf.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
                    assert cf(km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data, carry.ctypes.data, ncol, iv,
                              kord) == 0
                    assert _bits_equal(carry, out), (kord, iv, "carry")


@pytest.mark.parametrize("km,kn", [(4, 4), (5, 3), (6, 9), (7, 7), (8, 5), (9, 9), (17, 12), (33, 40), (79, 79),
                                   (79, 50), (127, 40)])
def test_cs_register_tail_is_bit_identical(host_lib, km, kn):
    """kord > 7 with the bottom NT edges of the tridiagonal solve held in registers (the
    device kernel's mappm_cs_column<.., NT>) gives the all-scratch column's bits, for every
    kord > 7 and iv (iv = -2 and km < NT + 1 take the all-scratch path), on columns with
    shared edges and unsorted output edges; and both match the oracle."""
    rng = np.random.default_rng(km * 7 + kn)
    ncol = 48
    for kord in (8, 9, 10, 11, 12, 13, 14, 15, 16, 17):
        for iv in (0, 1, -1, 2, -2):
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
            pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
            m = min(km, kn) + 1
            pe2[: m // 2] = pe1[: m // 2]
            pe2 = np.sort(pe2, 0)
            pe2[:, :4] = pe2[::-1, :4]  # a few columns with decreasing output edges
            q = (rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            ref = _host(host_lib, pe1, q, pe2, iv, kord)
            for nt in (8, 16, 32, 48):
                out = np.empty((kn, ncol), np.float32)
                assert host_lib.host_mappm_cs_tail(km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data,
                                                   out.ctypes.data, ncol, iv, kord, nt) == 0
                assert _bits_equal(out, ref), (kord, iv, nt)
            # the loads run ahead (mappm_cs_column<.., NT, PF>): same bits
            for nt, pf in ((0, 2), (0, 4), (0, 8), (16, 4)):
                out = np.empty((kn, ncol), np.float32)
                assert host_lib.host_mappm_cs_prefetch(km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data,
                                                       out.ctypes.data, ncol, iv, kord, nt, pf) == 0
                assert _bits_equal(out, ref), (kord, iv, nt, pf)


@pytest.mark.parametrize("nf", [1, 2])
@pytest.mark.parametrize("km,kn", [(4, 40), (79, 79), (79, 50), (20, 5), (12, 2), (79, 120)])
def test_two_lane_column_split_bit_identical(host_lib, nf, km, kn):
    """A column on two (and three) lanes (the small-grid pair kernels): outputs 1 .. kB-1 streamed from
    layer 1, kB .. kn from the layer where the single pass begins output kB, its window
    built from the local stencil (or, walk = 1 / out of the direct range, from layer 1).
    Every split point, both start modes, every PPM kord and iv, on columns with
    zero-thickness layers, shared edges, edges beyond both ends, unsorted and NaN edges
    anywhere (which the streamed checks send back to the single pass): the single pass's
    bits."""
    fn = host_lib.host_mappm_split
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    f3 = host_lib.host_mappm_split3
    f3.restype = ctypes.c_int
    f3.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    mf = host_lib.host_mappm_multi
    mf.restype = ctypes.c_int
    mf.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(km * 31 + kn * 3 + nf)
    ncol = 40
    kbs = sorted({0, 2, kn} | {int(k) for k in rng.integers(2, kn + 1, 3)}) if kn >= 2 else [0]
    for kord in (0, 1, 2, 3, 4, 5, 6, 7):
        for iv in (0, 1, -1, 2, -2):
            delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
            delp[rng.random((km, ncol)) < 0.05] = 0.0
            pe1 = np.concatenate([np.full((1, ncol), 300, np.float32),
                                  300 + np.cumsum(delp, 0, dtype=np.float32)])
            lo = rng.choice([0.5, 0.8, 1.0, 1.01], ncol)[None, :]
            hi = rng.choice([0.9, 1.0, 1.1, 2.0], ncol)[None, :]
            pe2 = np.sort(rng.uniform(pe1[0] * lo, pe1[-1] * hi, (kn + 1, ncol)), 0).astype(np.float32)
            m = min(km, kn) + 1
            pe2[: m // 3, :10] = pe1[: m // 3, :10]  # shared edges
            pe2 = np.sort(pe2, 0)
            pe2[:, 10:13] = pe2[::-1, 10:13]  # decreasing output edges: single pass
            pe1[km // 2, 13] = np.nan  # NaN input edge: single pass
            pe1[1:, 14] = pe1[:-1, 14]  # a repeated edge: zero-thickness first layer
            # unsorted edges only where one half of the split streams (the streamed checks
            # and the single-pass fix-up): the bottom input edge, just below the middle,
            # the bottom / top output edge, a NaN bottom input edge
            pe1[-1, 15] = pe1[km // 3, 15]
            pe1[km // 2 + 2, 16] = pe1[max(0, km // 2 - 6), 16]
            pe2[-1, 17] = pe2[0, 17]
            pe2[0, 18] = pe2[-1, 18]
            pe1[-1, 19] = np.nan
            # a raised run of input edges: the first lane stops inside it, the second starts
            # well below it (the two checked ranges do not meet: the fix-up)
            pe1[km // 4: km // 4 + 6, 20] += 1e7
            q = (rng.normal(0, 1, (nf, km, ncol)) * rng.choice([1e-4, 1, 300], (nf, km, ncol))).astype(np.float32)
            ref = np.empty((nf, kn, ncol), np.float32)
            with np.errstate(all="ignore"):
                assert mf(nf, km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data, ref.ctypes.data, ncol,
                          iv, kord) == 0
                for kb in kbs:
                    for walk in (0, 1):
                        out = np.full((nf, kn, ncol), 7.0, np.float32)
                        assert fn(nf, km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data, out.ctypes.data,
                                  ncol, iv, kord, kb, walk) == 0
                        assert _bits_equal(out, ref), (kord, iv, kb, walk)
                for walk in (0, 1):  # three lanes (outputs split at kn/3 + 1 and 2kn/3 + 1)
                    out = np.full((nf, kn, ncol), 7.0, np.float32)
                    assert f3(nf, km, pe1.ctypes.data, q.ctypes.data, kn, pe2.ctypes.data, out.ctypes.data,
                              ncol, iv, kord, walk) == 0
                    assert _bits_equal(out, ref), (kord, iv, "three lanes", walk)
