"""GPU parity of the fused DenseModel kernel against the numpy restatement of the
Keras graph (oracle/dense.py; reference external/fv3fit/fv3fit/keras/_models/dense.py:234-305).

Tolerance (north_star: "tendencies within 1e-5 rel of CPU reference"): for every
output variable AND every level of it, max over columns |gpu - ref64| <= 1e-5 * max
over columns |ref64| (tests/parity.py), with ref64 the float64 evaluation of the same graph; the float32 evaluation (Keras precision) must
satisfy the same bound, so the kernel is as close to the truth as Keras is.
"""
import numpy as np
import pytest

from conftest import set_variant

from oracle.dense import dense_predict
from tests.parity import assert_per_level

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _c48_state(rng, ntile=6, nz=79, n=48):
    T = rng.normal(260.0, 15.0, (ntile, nz, n, n)).astype(np.float32)
    q = rng.uniform(0.0, 0.02, (ntile, nz, n, n)).astype(np.float32)
    return T, q


def _to_samples(a):
    """(tile, z, y, x) -> [N, z] with N over (tile, y, x)."""
    t, z, y, x = a.shape
    return a.transpose(0, 2, 3, 1).reshape(t * y * x, z)


def _from_samples(a, t, y, x):
    return a.reshape(t, y, x, -1).transpose(0, 3, 1, 2)


def _check(gpu_out, ref64, ref32=None, rtol=RTOL):
    """Per output level (tests/parity.py): max over columns / max |ref| of that level."""
    for o, (g, r) in enumerate(zip(gpu_out, ref64)):
        assert_per_level(g, r, rtol, f"output {o}")
    if ref32 is not None:
        for o, (r32, r) in enumerate(zip(ref32, ref64)):
            assert_per_level(r32, r, rtol, f"float32 graph, output {o}")


def _model(cfg_kwargs, seed=1, bias_scale=0.1, samples=None):
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    cfg = DenseModelConfig(**cfg_kwargs)
    return DenseColumnModel.random(cfg, seed=seed, sample_inputs=samples, bias_scale=bias_scale)


def test_c48_2x256_tile_layout(gpu):
    """BASELINE config #2: DenseModel 2x256 predicting dQ1/dQ2 from T/q at C48 79L,
    inputs and outputs in (tile, z, y, x) layout (zero-copy stack/unstack)."""
    import torch

    rng = np.random.default_rng(0)
    T, q = _c48_state(rng)
    samples = [_to_samples(T), _to_samples(q)]
    m = _model(dict(input_variables=["air_temperature", "specific_humidity"],
                    output_variables=["dQ1", "dQ2"], in_nz=[79, 79], out_nz=[79, 79],
                    width=256, depth=3), samples=samples)
    outs = m.forward([torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()], level_axes=[1, 1])
    torch.cuda.synchronize()
    got = [_to_samples(o.cpu().numpy()) for o in outs]
    p = m.oracle_params()
    _check(got, dense_predict(samples, p, np.float64), dense_predict(samples, p, np.float32))


@pytest.mark.parametrize("width,depth", [(64, 2), (128, 3), (100, 4), (256, 2), (37, 3)])
def test_widths_depths_plain_layout(gpu, width, depth):
    import torch

    rng = np.random.default_rng(width + depth)
    n = 1000  # ragged: not a multiple of 16 or 64
    x1 = rng.normal(0, 3, (n, 20)).astype(np.float32)
    x2 = rng.normal(5, 1, (n, 7)).astype(np.float32)
    m = _model(dict(input_variables=["a", "b"], output_variables=["y1", "y2", "y3"], in_nz=[20, 7],
                    out_nz=[5, 33, 1], width=width, depth=depth), samples=[x1, x2])
    outs = m.forward([torch.from_numpy(x1.T.copy()).cuda(), torch.from_numpy(x2.T.copy()).cuda()])
    got = [o.cpu().numpy().T for o in outs]
    p = m.oracle_params()
    _check(got, dense_predict([x1, x2], p, np.float64))


def test_deep_model_falls_back_to_16_column_tiles(gpu):
    """A deep, many-feature model (6 x 84 input levels, 59 hidden layers of 256) whose
    32-column tiles would need more than 160 KiB of LDS (staged inputs + ~1 KiB of
    biases per hidden layer): the kernel runs 16-column tiles instead of failing
    (ADVICE r3), within the usual bound on a ragged grid."""
    import torch

    rng = np.random.default_rng(60)
    n = 531
    xs = [rng.normal(0, 1 + v, (n, 84)).astype(np.float32) for v in range(6)]
    m = _model(dict(input_variables=[f"x{v}" for v in range(6)], output_variables=["y1", "y2"], in_nz=[84] * 6,
                    out_nz=[79, 79], width=256, depth=60), samples=xs, bias_scale=0.01)
    outs = m.forward([torch.from_numpy(x.T.copy()).cuda() for x in xs])
    got = [o.cpu().numpy().T for o in outs]
    p = m.oracle_params()
    ref64, ref32 = dense_predict(xs, p, np.float64), dense_predict(xs, p, np.float32)
    # 59 layers amplify float32 rounding (measured 1.5e-4 on the GPU): the bound is the
    # numpy float32 graph's own worst level error against float64, with 3x headroom
    from tests.parity import per_level_errors

    for o, (g, r64, r32) in enumerate(zip(got, ref64, ref32)):
        f32_err = np.nanmax(per_level_errors(r32, r64)[0])
        assert_per_level(g, r64, max(RTOL, 3 * f32_err), f"deep model output {o} (float32 graph {f32_err:.2e})")


def test_clip_limits_mask_and_scalar_input(gpu):
    """ClipConfig on inputs (kept slice) and outputs (zero mask), OutputLimit clamps,
    and a 2-D (single-level) input."""
    import torch

    rng = np.random.default_rng(3)
    n = 777
    T = rng.normal(260, 15, (n, 79)).astype(np.float32)
    ps = rng.normal(1e5, 500, (n, 1)).astype(np.float32)
    cfg = dict(input_variables=["T", "ps"], output_variables=["dQ1", "dQ2"], in_nz=[79, 1],
               out_nz=[79, 79], width=128, depth=3,
               clip={"T": (10, 70), "dQ2": (5, 60)},
               output_limits={"dQ1": (-0.5, 0.5), "dQ2": (None, 0.1)})
    m = _model(cfg, samples=[T, ps], bias_scale=0.5)
    outs = m.forward([torch.from_numpy(T.T.copy()).cuda(), torch.from_numpy(ps[:, 0].copy()).cuda()],
                     level_axes=[0, None])
    got = [o.cpu().numpy().reshape(79, n).T for o in outs]
    ref = dense_predict([T, ps], m.oracle_params(), np.float64)
    _check(got, ref)
    assert (got[1][:, :5] == 0).all() and (got[1][:, 60:] == 0).all()
    assert got[0].max() <= 0.5 and got[0].min() >= -0.5 and got[1].max() <= 0.1


@pytest.mark.parametrize("n", [1, 15, 16, 17, 64, 65])
def test_tiny_and_ragged(gpu, n):
    import torch

    rng = np.random.default_rng(n)
    x = rng.normal(0, 1, (n, 79)).astype(np.float32)
    m = _model(dict(input_variables=["x"], output_variables=["y"], in_nz=[79], out_nz=[79],
                    width=256, depth=3))
    out = m.forward([torch.from_numpy(x.T.copy()).cuda()])[0].cpu().numpy().T
    # level magnitudes from 512 columns of the same model: with n = 1 a level's "max" is a
    # single dot product that may cancel towards zero
    wide = rng.normal(0, 1, (512, 79)).astype(np.float32)
    scale = np.abs(dense_predict([wide], m.oracle_params(), np.float64)[0]).max(axis=0)
    assert_per_level(out, dense_predict([x], m.oracle_params(), np.float64)[0], RTOL, "y", scale=scale)


def test_empty_and_bad_shapes(gpu):
    import torch

    m = _model(dict(input_variables=["x"], output_variables=["y"], in_nz=[10], out_nz=[3],
                    width=64, depth=2))
    out = m.forward([torch.zeros((10, 0), device="cuda")])[0]
    assert tuple(out.shape) == (3, 0)
    with pytest.raises(ValueError, match="levels"):
        m.forward([torch.zeros((9, 5), device="cuda")])


def test_c384_throughput_shape_and_determinism(gpu):
    """Full C384 column count (884,736): finite, deterministic across calls, and
    sampled columns match the float64 graph."""
    import torch

    rng = np.random.default_rng(384)
    ntile, nz, n = 6, 79, 384
    T = torch.from_numpy(rng.normal(260, 15, (ntile, nz, n, n)).astype(np.float32)).cuda()
    q = torch.from_numpy(rng.uniform(0, 0.02, (ntile, nz, n, n)).astype(np.float32)).cuda()
    sub = [_to_samples(T[:, :, :8, :8].cpu().numpy()), _to_samples(q[:, :, :8, :8].cpu().numpy())]
    m = _model(dict(input_variables=["T", "q"], output_variables=["dQ1", "dQ2"], in_nz=[79, 79],
                    out_nz=[79, 79], width=256, depth=3), samples=sub)
    a = m.forward([T, q], level_axes=[1, 1])
    b = m.forward([T, q], level_axes=[1, 1])
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
        assert torch.isfinite(x).all()
    got = [_to_samples(o[:, :, :8, :8].cpu().numpy()) for o in a]
    _check(got, dense_predict(sub, m.oracle_params(), np.float64))


def test_first_tile_after_other_kernels(gpu):
    """Regression: the f32 kernel's first tile per block stages its inputs with the
    normalisation constants that other waves write to LDS in the prologue; that staging
    once ran without a barrier, so a wave could read what an earlier kernel left in the
    LDS (seen as inf in one 32-column tile of a narrow model launched after a bf16x6
    launch).  Narrow and wide models, f32 and bf16x6, interleaved: every f32 result of
    the narrow model is bit-identical to the first and within 1e-5 of the float64 graph."""
    import torch

    rng = np.random.default_rng(77)
    T, q = _c48_state(rng)
    D = (np.linspace(200, 1800, 79)[None, :, None, None] * rng.uniform(0.95, 1.05, T.shape)).astype(np.float32)
    wide = _model(dict(input_variables=["T", "q"], output_variables=["dQ1", "dQ2"], in_nz=[79, 79],
                       out_nz=[79, 79], width=256, depth=3), samples=[_to_samples(T), _to_samples(q)])
    narrow = _model(dict(input_variables=["T", "D"], output_variables=["u", "v", "p", "d"], in_nz=[79, 79],
                         out_nz=[79, 79, 79, 1], width=32, depth=2), seed=5, samples=[_to_samples(T), _to_samples(D)])
    dT, dq, dD = (torch.from_numpy(a).cuda() for a in (T, q, D))
    first = None
    for _ in range(8):
        wide.forward([dT, dq], level_axes=[1, 1])
        wide.forward([dT, dq], level_axes=[1, 1], precision="bf16x6")
        got = narrow.forward([dT, dD], level_axes=[1, 1])
        torch.cuda.synchronize()
        if first is None:
            first = [g.clone() for g in got]
            ref = dense_predict([_to_samples(T), _to_samples(D)], narrow.oracle_params(), np.float64)
            _check([_to_samples(g.cpu().numpy()) for g in got], ref)
        for a, b in zip(got, first):
            assert torch.equal(a, b)


@pytest.mark.parametrize("precision", ["f32", "bf16x3", "bf16x6"])
def test_c384_columns_independent_of_position(gpu, precision):
    """A size-independent property at the full C384 grid (884,736 columns): the columns
    are 37 template columns repeated (37 is prime to every tile width, so each template
    lands on every lane, wave, tile and block position), and every copy's outputs carry
    exactly its template's bits.  The 37 templates are held to the float64 graph."""
    import torch

    rng = np.random.default_rng(3844)
    ntile, nz, n, nt = 6, 79, 384, 37
    tT = rng.normal(260, 15, (nt, nz)).astype(np.float32)
    tq = rng.uniform(0, 0.02, (nt, nz)).astype(np.float32)
    ncol = ntile * n * n
    pick = torch.arange(ncol, device="cuda") % nt
    # (tile, z, y, x) with column index (tile, y, x) -> template index % 37
    to_grid = lambda t: torch.from_numpy(t).cuda()[pick].reshape(ntile, n, n, nz).permute(0, 3, 1, 2).contiguous()  # noqa: E731
    T, q = to_grid(tT), to_grid(tq)
    m = _model(dict(input_variables=["T", "q"], output_variables=["dQ1", "dQ2"], in_nz=[79, 79],
                    out_nz=[79, 79], width=256, depth=3), samples=[tT, tq])
    outs = m.forward([T, q], level_axes=[1, 1], precision=precision)
    torch.cuda.synchronize()
    got = []
    for o in outs:
        cols = o.permute(0, 2, 3, 1).reshape(ncol, nz)  # [column, z]
        assert torch.equal(cols, cols[:nt][pick]), "a copy differs from its template"
        got.append(cols[:nt].cpu().numpy())
    _check(got, dense_predict([tT, tq], m.oracle_params(), np.float64), rtol=1e-4 if precision == "bf16x3" else RTOL)


@pytest.mark.parametrize("res,precision", [(7, "f32"), (48, "f32"), (7, "bf16x3"), (48, "bf16x3"), (7, "bf16x6"),
                                           (48, "bf16x6")])
def test_writes_stay_inside_outputs(gpu, res, precision):
    """Outputs as level slices of larger (tile, z, y, x) buffers pre-filled with NaN:
    the kernels write exactly the model's rows of the real columns (the f32 epilogue
    drops padding rows and columns past the end with range-checked buffer stores).
    C7: 294 columns, a ragged last tile for both kernels' tile widths."""
    import torch

    rng = np.random.default_rng(res)
    T, q = _c48_state(rng, n=res)
    samples = [_to_samples(T), _to_samples(q)]
    m = _model(dict(input_variables=["air_temperature", "specific_humidity"],
                    output_variables=["dQ1", "dQ2"], in_nz=[79, 79], out_nz=[79, 79],
                    width=256, depth=3), samples=samples)
    bigs = [torch.full((6, 90, res, res), float("nan"), device="cuda") for _ in range(2)]
    outs = [b[:, 5:84] for b in bigs]
    m.forward([torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()], level_axes=[1, 1],
              outputs=outs, out_level_axis=1, precision=precision)
    torch.cuda.synchronize()
    for b in bigs:
        assert torch.isnan(b[:, :5]).all() and torch.isnan(b[:, 84:]).all()
    got = [_to_samples(o.cpu().numpy()) for o in outs]
    _check(got, dense_predict(samples, m.oracle_params(), np.float64), rtol=1e-4 if precision == "bf16x3" else RTOL)


@pytest.mark.parametrize("res,width,ragged", [(12, 256, False), (48, 256, False), (7, 128, True), (12, 64, False)])
def test_float64_inputs_read_in_place(gpu, res, width, ragged):
    """A float64 state goes to fv3_dense_forward_f64in (cast in the kernel's staging):
    bit-identical to casting to float32 first, on the (tile, z, y, x) layout and on a
    strided row-band view, for widths 64-256."""
    import torch

    rng = np.random.default_rng(res + width)
    T = rng.normal(260.0, 15.0, (6, 79, res, res))
    q = rng.uniform(0.0, 0.02, (6, 79, res, res))
    m = _model(dict(input_variables=["air_temperature", "specific_humidity"],
                    output_variables=["dQ1", "dQ2"], in_nz=[79, 79], out_nz=[79, 79],
                    width=width, depth=3),
               samples=[_to_samples(T.astype(np.float32)), _to_samples(q.astype(np.float32))])
    Td, qd = torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()
    if ragged:  # a row band of every tile: strided columns
        Td, qd = Td[:, :, 1:6], qd[:, :, 1:6]
    a = m.forward([Td, qd], level_axes=[1, 1])
    b = m.forward([Td.to(torch.float32), qd.to(torch.float32)], level_axes=[1, 1])
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert x.dtype == torch.float32
        assert torch.equal(x, y)


def test_bind_float64_state_sees_updates(gpu):
    """bind() on a float64 state reads it in place: an in-place state update (the
    stepper's add_tendency) is seen by the next call."""
    import torch

    rng = np.random.default_rng(4)
    T = torch.from_numpy(rng.normal(260.0, 15.0, (6, 79, 8, 8))).cuda()
    q = torch.from_numpy(rng.uniform(0.0, 0.02, (6, 79, 8, 8))).cuda()
    cfg = dict(input_variables=["T", "q"], output_variables=["dQ1", "dQ2"], in_nz=[79, 79], out_nz=[79, 79],
               width=256, depth=3)
    m = _model(cfg)
    b = m.bind([T, q], level_axes=[1, 1])
    T.add_(1.5)
    got = [o.clone() for o in b()]
    ref = m.forward([T.to(torch.float32), q.to(torch.float32)], level_axes=[1, 1])
    for x, y in zip(got, ref):
        assert torch.equal(x, y)


@pytest.mark.parametrize("ncol,precision", [(1000, "f32"), (1000, "bf16x3"), (13824 + 37, "f32"),
                                            (13824 + 37, "bf16x3"), (1000, "bf16x6"), (13824 + 37, "bf16x6")])
@pytest.mark.parametrize("tr", ["1", "0"])
def test_residual_outputs_stay_inside(gpu, ncol, precision, tr, monkeypatch):
    """Regression for the memory fault fixed in round 1 (residual outputs read one level
    past a 79-level input): an emulator-style model whose output is input + de-normalised
    difference (Difference.backward), residual input an EXACT-size [79, ncol] tensor,
    ragged last tile for both kernels, outputs written into NaN-filled level slices.  The
    split kernel with its transposed output layer (FV3_B3_TR=1: 16-byte residual loads and
    stores at 1,000 columns, dword ones at 13,861, whose rows are not 16-byte aligned) and
    without (0)."""
    import torch

    if precision == "f32" and tr == "0":
        pytest.skip("the exact-f32 kernel has one output layer")
    set_variant(monkeypatch, "FV3_B3_TR", tr)

    rng = np.random.default_rng(ncol)
    x = rng.normal(250.0, 10.0, (ncol, 79)).astype(np.float32)
    w = rng.uniform(0.0, 0.02, (ncol, 79)).astype(np.float32)
    cfg = dict(input_variables=["x", "w"], output_variables=["dx", "dw"], in_nz=[79, 79], out_nz=[79, 79],
               width=256, depth=3, output_residuals={"dx": "x", "dw": "w"})
    m = _model(cfg, samples=[x, w])
    xd = torch.from_numpy(x.T.copy()).cuda()
    wd = torch.from_numpy(w.T.copy()).cuda()
    assert xd.numel() == 79 * ncol and xd.untyped_storage().nbytes() == 4 * 79 * ncol
    bigs = [torch.full((90, ncol), float("nan"), device="cuda") for _ in range(2)]
    outs = [b[5:84] for b in bigs]
    m.forward([xd, wd], outputs=outs, precision=precision)
    torch.cuda.synchronize()
    for b in bigs:
        assert torch.isnan(b[:5]).all() and torch.isnan(b[84:]).all()
    y = dense_predict([x, w], m.oracle_params(), np.float64)
    ref = [x.astype(np.float64) + y[0], w.astype(np.float64) + y[1]]
    got = [o.cpu().numpy().T for o in outs]
    _check(got, ref, rtol=1e-4 if precision == "bf16x3" else RTOL)


def test_bind_refuses_snapshot_inputs(gpu):
    """bind() would re-run on a copy that never sees the caller's in-place updates when
    the kernel cannot read an input in place (float64 state on bf16x3, numpy): refused
    (ADVICE r1)."""
    import torch

    rng = np.random.default_rng(5)
    T = torch.from_numpy(rng.normal(260.0, 15.0, (6, 79, 8, 8))).cuda()
    q = torch.from_numpy(rng.uniform(0.0, 0.02, (6, 79, 8, 8))).cuda()
    m = _model(dict(input_variables=["T", "q"], output_variables=["dQ1", "dQ2"], in_nz=[79, 79],
                    out_nz=[79, 79], width=256, depth=3))
    with pytest.raises(ValueError, match="copy"):
        m.bind([T, q], level_axes=[1, 1], precision="bf16x3")
    with pytest.raises(ValueError, match="copy"):
        m.bind([T.float(), q.float().cpu().numpy()], level_axes=[1, 1])
    b = m.bind([T.float(), q.float()], level_axes=[1, 1], precision="bf16x3")  # float32 device: in place
    assert len(b()) == 2
