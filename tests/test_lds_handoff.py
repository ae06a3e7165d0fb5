"""Cross-wave LDS hand-offs ("LDS hand-offs"): every kernel that stages
values in LDS for other waves must order the writes before the reads with a barrier.  The
f32 dense kernel once read its normalisation constants before the waves that write them
had done so (round 4, commit 4588bbe): it picked up whatever an earlier kernel left in
LDS.  Here a test-only kernel (tests/native/lds_dirty.hip) fills every CU's LDS with a
pattern (NaN, inf, 0, 1e9) right before each checked kernel; results must not move by a
bit, and the clean results match the oracle.

Checked: the f32 dense kernel (8-wave and 16-column tiles), the bf16x3 / bf16x6 split
kernel (8- and 4-wave blocks, LDS-DMA and register staging), the pressure-level coarsen
(cell-per-wave 1- and 2-field passes, f = 8 and f = 2, and the 8-wave row kernel), the
level-parallel stepper epilogue, and mappm (level-parallel PPM, the kord > 7 LDS
scratch)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT, require_variant_kernels, set_variant
from oracle import coarsen as OC
from oracle.dense import dense_predict
from oracle.mappm import oracle_mappm
from tests.parity import assert_per_level

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tests", "_build", "liblds_dirty.so")
PATTERNS = [0x7FC00001, 0x7F800000, 0x00000000, 0x4E6E6B28]  # NaN, inf, 0, ~1e9 (f32 bits)


@pytest.fixture(scope="module")
def dirty(gpu):
    import torch

    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: __graft_entry__.build() compiles it")
    lib = ctypes.CDLL(LIB)
    lib.lds_dirty.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.lds_dirty.restype = ctypes.c_int
    sink = torch.zeros(1 << 16, dtype=torch.int32, device=gpu)

    def fill(pattern):
        assert lib.lds_dirty(pattern, sink.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0

    yield fill
    torch.cuda.synchronize()
    assert not sink.any()


def _same(a, b):
    import torch

    if torch.is_tensor(a):
        return a.shape == b.shape and torch.equal(a.view(torch.uint8), b.view(torch.uint8))
    return np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


def _stable(run, dirty):
    """run() after each LDS pattern gives the bits of a clean run (returned)."""
    import torch

    torch.cuda.synchronize()
    ref = [r.clone() for r in run()]
    torch.cuda.synchronize()
    for p in PATTERNS:
        dirty(p)
        got = run()
        torch.cuda.synchronize()
        for g, r in zip(got, ref):
            assert _same(g, r), f"LDS pattern {p:#010x} changed the result"
    return ref


def _samples(a):
    t, z, y, x = a.shape
    return a.transpose(0, 2, 3, 1).reshape(t * y * x, z)


@pytest.mark.parametrize("width,depth,precision", [(256, 3, "f32"), (32, 2, "f32"), (256, 5, "f32"),
                                                   (256, 3, "bf16x3"), (256, 3, "bf16x6"), (128, 2, "bf16x6")])
@pytest.mark.parametrize("res", [12, 48])
def test_dense_kernels_ignore_stale_lds(gpu, dirty, width, depth, precision, res):
    """C12 (one partial tile per block, the 4-wave split-kernel blocks) and C48; depth 5
    takes the f32 kernel's 16-column fallback."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    rng = np.random.default_rng(res + width)
    T = rng.normal(260, 15, (6, 79, res, res)).astype(np.float32)
    q = rng.uniform(0, 0.02, (6, 79, res, res)).astype(np.float32)
    cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [79, 79], [79, 79], width=width, depth=depth)
    m = DenseColumnModel.random(cfg, seed=3, sample_inputs=[_samples(T), _samples(q)], bias_scale=0.1)
    dT, dq = torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()
    ref = _stable(lambda: m.forward([dT, dq], level_axes=[1, 1], precision=precision), dirty)
    exp = dense_predict([_samples(T), _samples(q)], m.oracle_params(), np.float64)
    for g, r in zip(ref, exp):
        assert_per_level(_samples(g.cpu().numpy()), r, 1e-4 if precision == "bf16x3" else 1e-5)


@pytest.mark.parametrize("stage,waves", [("glds", "8"), ("glds", "4"), ("reg", "8")])
def test_split_kernel_staging_variants_ignore_stale_lds(gpu, dirty, stage, waves, monkeypatch):
    """The bf16x6 split kernel's LDS-DMA weight ring and per-wave input rows (glds) and the
    register-staged ring (reg), 8- and 4-wave blocks, on 4 persistent blocks so every
    block walks several tiles (the cross-tile input prefetch and the ring wrap)."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    set_variant(monkeypatch, "FV3_B3_STAGE", stage)
    set_variant(monkeypatch, "FV3_B3_WAVES", waves)
    set_variant(monkeypatch, "FV3_B3_GRID", "4")
    rng = np.random.default_rng(4)
    T = rng.normal(260, 15, (79, 2085)).astype(np.float32)
    q = rng.uniform(0, 0.02, (79, 2085)).astype(np.float32)
    cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [79, 79], [79, 79], width=256, depth=3)
    m = DenseColumnModel.random(cfg, seed=5, sample_inputs=[T.T, q.T], bias_scale=0.1)
    dT, dq = torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()
    ref = _stable(lambda: m.forward([dT, dq], level_axes=[0, 0], precision="bf16x6"), dirty)
    exp = dense_predict([T.T, q.T], m.oracle_params(), np.float64)
    for g, r in zip(ref, exp):
        assert_per_level(g.cpu().numpy().T, r, 1e-5)


@pytest.mark.parametrize("factor,n,path", [(8, 48, "cells"), (2, 16, "cells"), (4, 24, "rows")])
@pytest.mark.parametrize("nfields", [1, 2, 4])
def test_coarsen_ignores_stale_lds(gpu, dirty, factor, n, path, nfields, monkeypatch):
    """The coarsen kernels' LDS: the per-wave output ring and overflow flags of the
    cell-per-wave kernel (1- and 2-field passes), and the 8-wave row kernel's partial sums
    and coarse pressure edges; bit-exact vs oracle/coarsen.py."""
    from tests.remap_exact import coarsen_on_pressure

    set_variant(monkeypatch, "FV3_COARSEN_PATH", path)
    rng = np.random.default_rng(factor + n + nfields)
    base = np.linspace(200, 1800, 79)[None, :, None, None]
    delp = (base * rng.uniform(0.95, 1.05, (6, 79, n, n))).astype(np.float32)
    delp[:, :, :2, :2] *= rng.uniform(0.5, 1.5, (6, 79, 2, 2)).astype(np.float32)  # steep cells: overflow columns
    area = rng.uniform(0.5, 1.0, (6, n, n)).astype(np.float32)
    fields = {f"f{i}": (250 + rng.normal(0, 5, (6, 79, n, n))).astype(np.float32) for i in range(nfields)}

    def run():
        out, dc = coarsen_on_pressure(delp, area, fields, factor)
        return [out[k] for k in fields] + [dc]

    ref = _stable(run, dirty)
    exp, exp_dc = OC.coarsen_on_pressure(delp, area, list(fields.values()), factor)
    for g, r in zip(ref, list(exp) + [exp_dc]):
        g = g.cpu().numpy()
        assert np.array_equal(g.view(np.uint32), np.asarray(r, np.float32).view(np.uint32))


def test_level_parallel_epilogue_ignores_stale_lds(gpu, dirty, monkeypatch):
    """The stepper's level-parallel epilogue: per-level sum terms and NaN counts in LDS,
    summed per column after the barrier; bit-exact vs oracle/stepper.py."""
    import torch

    from fv3net_amd.stepper import ml_epilogue
    from oracle import stepper as OS

    set_variant(monkeypatch, "FV3_EPILOGUE_PATH", "levels")
    from tests.test_stepper import _state

    dq1, dq2, q, delp, T, precip = _state(np.random.default_rng(7), ncol=6912)
    dq1[5, 17] = np.nan
    names = {"net_moistening": "net_moistening_due_to_ml", "column_heating": "column_heating_due_to_ml"}

    keys = []

    def run():
        got = ml_epilogue(*(torch.from_numpy(a).cuda() for a in (dq1, dq2, q, delp, T)), 900.0,
                          torch.from_numpy(precip).cuda(), True, False, label="ml")
        keys[:] = [k for k in sorted(got) if torch.is_tensor(got[k])]
        return [got[k] for k in keys]

    ref = _stable(run, dirty)
    exp = OS.epilogue(dq1, dq2, q, delp, T, precip, 900.0, True, False)
    inv = {v: k for k, v in names.items()}
    checked = 0
    for k, g in zip(keys, ref):
        if inv.get(k, k) not in exp:
            continue
        r = exp[inv.get(k, k)]
        g = g.cpu().numpy()
        r = np.asarray(r).astype(g.dtype) if k.endswith("filled_frac") else np.asarray(r)
        assert np.array_equal(g.view(np.uint8), r.view(np.uint8)), k
        checked += 1
    assert checked >= 6


@pytest.mark.parametrize("kord,path", [(5, "levels"), (7, "levels"), (10, "lds")])
def test_mappm_ignores_stale_lds(gpu, dirty, kord, path, monkeypatch):
    """mappm's level-parallel PPM kernel (the column in LDS, the boundary layers on two
    threads) and the kord > 7 edge solve with its scratch in LDS; bit-exact vs the oracle."""
    import torch

    from tests.remap_exact import mappm_device

    if path == "lds":
        require_variant_kernels()
        set_variant(monkeypatch, "FV3_MAPPM_LDS", "1")
    else:
        set_variant(monkeypatch, "FV3_MAPPM_PATH", path)
    rng = np.random.default_rng(kord)
    km, kn, ncol = 79, 50, 700
    delp = rng.uniform(1, 3000, (km, ncol)).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    pe2 = np.sort(rng.uniform(pe1[0] * 0.8, pe1[-1] * 1.1, (kn + 1, ncol)), 0).astype(np.float32)
    qq = (rng.normal(0, 1, (km, ncol)) * 300).astype(np.float32)
    d1, dqq, d2 = (torch.from_numpy(a).cuda() for a in (pe1, qq, pe2))
    ref = _stable(lambda: [mappm_device(d1, dqq, d2, 1, kord)], dirty)
    assert np.array_equal(ref[0].cpu().numpy().view(np.uint32), oracle_mappm(pe1, qq, pe2, 1, kord).view(np.uint32))
