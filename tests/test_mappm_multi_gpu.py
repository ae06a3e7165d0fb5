"""Several fields remapped onto the same edges (fv3_mappm_multi): every field's result
is bit-identical to a single-field mappm call on it, and to the oracle.  Bar: bit-exact.

The reference issues one mappm.mappm call per variable on shared p_in / p_out
(external/vcm/vcm/cubedsphere/coarsen_restarts.py:411-516 -> regridz.py:164-279);
csrc/mappm_multi.h computes the pressure-only part once per pair of fields.
"""
import numpy as np
import pytest

from conftest import set_variant

from oracle.mappm import oracle_mappm
from tests.test_mappm_gpu import _bits_equal, _columns

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["split", "split3", "serial", "levels"])
def path(request, monkeypatch):
    """`split`: pairs of fields on the two-field streaming kernel, each column on two
    lanes (FV3_MAPPM_SPLIT=1; the default for pairs from ~87,000 to 147,456 columns on 256
    CUs); `split3`: three lanes per column (FV3_MAPPM_SPLIT=3; the default for pairs from
    10,240 columns up to ~87,000); `serial`: the same kernel one lane per column
    (FV3_MAPPM_SPLIT=0, the default above 147,456); `levels`: the small-grid kernel, one
    field per launch (the default for pairs below 10,240 columns and single fields below
    20,480).  Single-field calls under a forced FV3_MAPPM_PATH keep that path's kernel."""
    set_variant(monkeypatch, "FV3_MAPPM_PATH", "levels" if request.param == "levels" else "serial")
    if request.param != "levels":
        set_variant(monkeypatch, "FV3_MAPPM_SPLIT", {"split": "1", "split3": "3"}.get(request.param, "0"))
    return request.param


def _fields(rng, km, ncol, n):
    return [(rng.normal(0, 1, (km, ncol)) * rng.choice([1e-4, 1, 300], (km, ncol))).astype(np.float32)
            for _ in range(n)]


@pytest.mark.parametrize("km,kn,ncol,nf", [(4, 3, 1, 2), (5, 9, 257, 3), (79, 50, 1000, 2), (79, 79, 777, 5),
                                           (127, 40, 300, 4)])
def test_multi_equals_single_and_oracle(gpu, path, km, kn, ncol, nf):
    from tests.remap_exact import mappm_device, mappm_device_multi

    rng = np.random.default_rng(km * 7 + kn + ncol + nf)
    pe1, q0, pe2 = _columns(rng, km, kn, ncol)
    qs = [q0] + _fields(rng, km, ncol, nf - 1)
    for kord in (1, 4, 5, 6, 7, 10):
        for iv in (0, 1, -1, 2):
            outs = mappm_device_multi(pe1, qs, pe2, iv, kord)
            assert len(outs) == nf
            for f, (q, o) in enumerate(zip(qs, outs)):
                got = o.cpu().numpy()
                assert _bits_equal(got, mappm_device(pe1, q, pe2, iv, kord).cpu().numpy()), (kord, iv, f)
                assert _bits_equal(got, oracle_mappm(pe1, q, pe2, iv, kord)), (kord, iv, f)


def test_multi_c384_pair_kernel_sampled(gpu, monkeypatch):
    """Config #3 size (6*384*384 columns, 79 -> 79) through the two-field kernel:
    whole arrays equal to the single-field kernel, sampled columns to the oracle."""
    import torch

    from tests.remap_exact import mappm_device, mappm_device_multi

    set_variant(monkeypatch, "FV3_MAPPM_PATH", "serial")
    rng = np.random.default_rng(385)
    ncol, km = 6 * 384 * 384, 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    pe = []
    for _ in range(2):
        delp = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
        pe.append(np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)]))
    qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
    d = [torch.from_numpy(a).cuda() for a in pe + qs]
    outs = mappm_device_multi(d[0], d[2:], d[1], 1, 1)
    for q, o in zip(d[2:], outs):
        assert torch.equal(o.view(torch.int32), mappm_device(d[0], q, d[1], 1, 1).view(torch.int32))
    idx = np.sort(rng.choice(ncol, 2048, replace=False))
    for q, o in zip(qs, outs):
        ref = oracle_mappm(pe[0][:, idx], q[:, idx], pe[1][:, idx], 1, 1)
        assert _bits_equal(o.cpu().numpy()[:, idx], ref)


def test_multi_tile_layout_in_place(gpu, monkeypatch):
    """(tile, z, y, x) fields read and written in place, each with its own layout (an
    output written into a slice of a larger array)."""
    import torch

    from tests.remap_exact import mappm_device_multi

    set_variant(monkeypatch, "FV3_MAPPM_PATH", "serial")
    rng = np.random.default_rng(8)
    ntile, km, ny, nx = 6, 79, 12, 12
    ncol = ntile * ny * nx
    pe1, q0, pe2 = _columns(rng, km, km, ncol)
    q1 = _fields(rng, km, ncol, 1)[0]
    to_t = lambda a: torch.from_numpy(np.ascontiguousarray(  # noqa: E731
        a.reshape(a.shape[0], ntile, ny * nx).transpose(1, 0, 2).reshape(ntile, a.shape[0], ny, nx))).cuda()
    from_t = lambda t: t.cpu().numpy().reshape(ntile, -1, ny * nx).transpose(1, 0, 2).reshape(t.shape[1], ncol)  # noqa
    big = torch.zeros((ntile, 2 * km, ny, nx), device="cuda")
    outs = [big[:, :km], big[:, km:]]
    # the multi API takes [level, column] 2-D views: build them from the tile arrays
    pe1_t, pe2_t, qa, qb = (to_t(a) for a in (pe1, pe2, q0, q1))
    flat = lambda t: t.permute(1, 0, 2, 3).reshape(t.shape[1], -1)  # noqa: E731  (a copy for tile data)
    res = mappm_device_multi(flat(pe1_t), [flat(qa), flat(qb)], flat(pe2_t), 1, 1)
    for q, r in zip((q0, q1), res):
        assert _bits_equal(r.cpu().numpy(), oracle_mappm(pe1, q, pe2, 1, 1))
    # strided in-place outputs through the C ABI with per-field layouts
    from fv3net_amd import _device, _native
    import ctypes

    lays = [_device.level_layout(t, 1)[0] for t in (pe1_t, pe2_t, qa, qb, outs[0], outs[1])]
    qp = (ctypes.c_void_p * 2)(qa.data_ptr(), qb.data_ptr())
    ql = (_native.Layout * 2)(lays[2], lays[3])
    op = (ctypes.c_void_p * 2)(outs[0].data_ptr(), outs[1].data_ptr())
    ol = (_native.Layout * 2)(lays[4], lays[5])
    st = _native.load().fv3_mappm_multi(pe1_t.data_ptr(), lays[0], qp, ql, pe2_t.data_ptr(), lays[1], op, ol, 2,
                                         ncol, km, km, 1, 1, 0.0, _native.ARITH_EXACT, _device.stream_handle())
    _native.check(st)
    for q, o in zip((q0, q1), outs):
        assert _bits_equal(from_t(o), oracle_mappm(pe1, q, pe2, 1, 1))


def test_multi_plan_tracks_contents_and_refuses_copies(gpu, path):
    import torch

    from tests.remap_exact import MappmMultiPlan

    rng = np.random.default_rng(24)
    pe1, q0, pe2 = _columns(rng, 79, 50, 864)
    q1 = _fields(rng, 79, 864, 1)[0]
    d = [torch.from_numpy(a).cuda() for a in (pe1, pe2, q0, q1)]
    plan = MappmMultiPlan(d[0], d[2:], d[1], 1, 4)
    for q, o in zip((q0, q1), plan()):
        assert _bits_equal(o.cpu().numpy(), oracle_mappm(pe1, q, pe2, 1, 4))
    d[3].mul_(2.0)
    out = plan()
    assert _bits_equal(out[1].cpu().numpy(), oracle_mappm(pe1, q1 * 2, pe2, 1, 4))
    assert _bits_equal(out[0].cpu().numpy(), oracle_mappm(pe1, q0, pe2, 1, 4))
    with pytest.raises(ValueError, match="copy"):
        MappmMultiPlan(d[0], [d[2], d[3].double()], d[1], 1, 1)
    with pytest.raises(ValueError, match="copy"):
        MappmMultiPlan(d[0], [q0], d[1], 1, 1)


def test_multi_errors(gpu):
    import torch

    from tests.remap_exact import mappm_device_multi

    z = lambda *s: torch.zeros(s, device="cuda")  # noqa: E731
    assert [tuple(o.shape) for o in mappm_device_multi(z(80, 0), [z(79, 0)] * 3, z(51, 0))] == [(50, 0)] * 3
    with pytest.raises(ValueError, match="1..64"):
        mappm_device_multi(z(80, 3), [], z(51, 3))
    with pytest.raises(ValueError, match="one shorter"):
        mappm_device_multi(z(80, 3), [z(79, 3), z(78, 3)], z(51, 3))
    with pytest.raises(ValueError, match="same size"):
        mappm_device_multi(z(80, 3), [z(79, 3), z(79, 4)], z(51, 3))
    with pytest.raises(ValueError, match="one output per field"):
        mappm_device_multi(z(80, 3), [z(79, 3), z(79, 3)], z(51, 3), out=[z(50, 3)])
    torch.cuda.synchronize()


def test_multi_on_a_side_stream(gpu, path):
    """A call on another stream waits for the current stream (host inputs are copied
    there) and keeps its temporaries alive until that stream is done: same bits."""
    import torch

    from tests.remap_exact import mappm_device, mappm_device_multi

    rng = np.random.default_rng(31)
    pe1, q0, pe2 = _columns(rng, 79, 50, 3000)
    q1 = _fields(rng, 79, 3000, 1)[0]
    side = torch.cuda.Stream()
    outs = mappm_device_multi(pe1, [q0, q1], pe2, 1, 1, stream=side)
    one = mappm_device(pe1, q1, pe2, 1, 1, stream=side)
    side.synchronize()
    for q, o in zip((q0, q1), outs):
        assert _bits_equal(o.cpu().numpy(), oracle_mappm(pe1, q, pe2, 1, 1))
    assert _bits_equal(one.cpu().numpy(), oracle_mappm(pe1, q1, pe2, 1, 1))


@pytest.mark.parametrize("kn", [79, 50, 2, 1])
def test_two_lane_pair_kernel_rank_share_size(gpu, kn, monkeypatch):
    """One rank's share of C384 at world 8 (110,592 columns, the two-lane kernel by
    default): whole arrays bit-identical to the one-lane pair kernel and sampled
    columns to the oracle, on columns that take every start of the second lane (a
    direct window, output kB above the top or below the bottom, kB's layer near either
    end) and columns that the streamed checks send back to the single pass (unsorted
    pe2, a NaN edge, an unsorted bottom input or output edge, a raised run of input
    edges); a zero-thickness layer stays on two lanes.  The unsorted and NaN columns can
    fail the reference's layer search (undefined behaviour, excluded from oracle parity,
    DESIGN.md §4): there the two kernels must agree with each other only."""
    import torch

    from tests.remap_exact import mappm_device_multi

    rng = np.random.default_rng(110592 + kn)
    ncol, km = 110592, 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    delp = (base * rng.uniform(0.9, 1.1, (km, ncol))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    top, bot = pe1[0], pe1[-1]
    a = rng.choice([-0.3, 0.0, 0.0, 0.5], ncol)
    b = rng.choice([0.4, 1.0, 1.0, 1.3], ncol)
    a, b = np.minimum(a, b - 0.05), b
    frac = np.sort(rng.uniform(a, b, (kn + 1, ncol)), 0)
    pe2 = (top + (bot - top) * frac).astype(np.float32)
    pe2[:, :64] = pe2[::-1, :64]  # decreasing
    pe1[40, 64:96] = np.nan
    pe1[20, 96:128] = pe1[19, 96:128]  # a zero-thickness layer: still sorted
    # unsorted only where one lane streams (the streamed checks and the single-pass
    # fix-up): the bottom input edge, a raised run of input edges (the two lanes' checked
    # ranges do not meet), the bottom output edge
    pe1[-1, 160:192] = pe1[30, 160:192]
    pe1[20:26, 192:224] += 1e7
    pe2[-1, 224:256] = pe2[0, 224:256]
    qs = [rng.normal(250, 10, (km, ncol)).astype(np.float32), rng.uniform(0, 0.02, (km, ncol)).astype(np.float32)]
    d = [torch.from_numpy(x).cuda() for x in (pe1, pe2, *qs)]
    default = mappm_device_multi(d[0], d[2:], d[1], 1, 1)
    res = {}
    for split in ("1", "0", "3"):  # two lanes, one, three
        set_variant(monkeypatch, "FV3_MAPPM_SPLIT", split)
        res[split] = mappm_device_multi(d[0], d[2:], d[1], 1, 1)
    for x, y, z, w in zip(res["1"], res["0"], default, res["3"]):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))
        assert torch.equal(x.view(torch.int32), z.view(torch.int32))
        assert torch.equal(w.view(torch.int32), y.view(torch.int32))
    idx = np.concatenate([np.arange(96, 160), np.sort(rng.choice(np.arange(256, ncol), 1500, replace=False))])
    for q, o in zip(qs, res["1"]):
        with np.errstate(all="ignore"):
            ref = oracle_mappm(pe1[:, idx], q[:, idx], pe2[:, idx], 1, 1)
        assert _bits_equal(o.cpu().numpy()[:, idx], ref)


@pytest.mark.parametrize("ncol", [27648, 55296, 110592])
def test_single_field_split_lanes_default(gpu, ncol, monkeypatch):
    """One field (fv3_mappm_ex) on the split kernels the host picks by size (three lanes at
    27,648 and 55,296 columns, two at 110,592) and forced to two / three lanes: whole
    arrays bit-identical to one lane per column on sorted columns and, over the unsorted /
    NaN / raised-run columns (the streamed checks' fix-up), to the multi-field single pass
    (the one-lane pair kernel); sampled sorted columns equal the oracle."""
    import torch

    from tests.remap_exact import mappm_device

    rng = np.random.default_rng(ncol)
    km, kn = 79, 79
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    delp = (base * rng.uniform(0.9, 1.1, (km, ncol))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    frac = np.sort(rng.uniform(-0.1, 1.1, (kn + 1, ncol)), 0)
    pe2 = (pe1[0] + (pe1[-1] - pe1[0]) * frac).astype(np.float32)
    bad = np.arange(0, 160)
    pe2[:, :32] = pe2[::-1, :32]
    pe1[40, 32:64] = np.nan
    pe1[20:26, 64:96] += 1e7
    pe1[-1, 96:128] = pe1[30, 96:128]
    pe2[-1, 128:160] = pe2[0, 128:160]
    q = rng.normal(250, 10, (km, ncol)).astype(np.float32)
    d = [torch.from_numpy(x).cuda() for x in (pe1, q, pe2)]
    runs = {}
    for name, env in (("default", {}), ("two", {"FV3_MAPPM_SPLIT1": "2"}), ("three", {"FV3_MAPPM_SPLIT1": "3"}),
                      ("one", {"FV3_MAPPM_PATH": "serial", "FV3_MAPPM_SPLIT1": "0"})):
        for k in ("FV3_MAPPM_SPLIT1", "FV3_MAPPM_PATH"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            set_variant(monkeypatch, k, v)
        runs[name] = mappm_device(d[0], d[1], d[2], 1, 1).cpu().numpy()
    good = np.setdiff1d(np.arange(ncol), bad)
    for name in ("default", "two", "three"):
        assert _bits_equal(runs[name][:, good], runs["one"][:, good]), name
    # the unsorted columns: the fix-up's single pass is the multi-field streaming code's
    # (the one-lane pair kernel on two copies of the field)
    monkeypatch.delenv("FV3_MAPPM_SPLIT1", raising=False)
    set_variant(monkeypatch, "FV3_MAPPM_PATH", "serial")
    set_variant(monkeypatch, "FV3_MAPPM_SPLIT", "0")
    from tests.remap_exact import mappm_device_multi
    multi = mappm_device_multi(d[0], [d[1], d[1]], d[2], 1, 1)[0].cpu().numpy()
    for name in ("default", "two", "three"):
        assert _bits_equal(runs[name][:, bad], multi[:, bad]), name
    idx = np.sort(rng.choice(good, 1000, replace=False))
    assert _bits_equal(runs["default"][:, idx], oracle_mappm(pe1[:, idx], q[:, idx], pe2[:, idx], 1, 1))


@pytest.mark.parametrize("km,kn", [(4, 2), (4, 3), (5, 9), (12, 2), (40, 79)])
def test_split_defaults_small_level_counts(gpu, km, kn, monkeypatch):
    """The split kernels the host picks at 30,000 columns (one field: three lanes, or two
    for kn = 2; a pair: three lanes) on few or unequal level counts, including kn = 2
    (the smallest a split takes) and km = 4 (no direct start window): bit-identical to
    one lane per column, and to the oracle on sampled columns."""
    import torch

    from tests.remap_exact import mappm_device, mappm_device_multi

    rng = np.random.default_rng(km * 100 + kn)
    ncol = 30000
    pe1, q0, pe2 = _columns(rng, km, kn, ncol)
    q1 = _fields(rng, km, ncol, 1)[0]
    d = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (pe1, q0, q1, pe2)]
    for kord in (1, 5, 7):
        for iv in (0, 1):
            monkeypatch.delenv("FV3_MAPPM_PATH", raising=False)
            monkeypatch.delenv("FV3_MAPPM_SPLIT", raising=False)
            one_default = mappm_device(d[0], d[1], d[3], iv, kord).cpu().numpy()
            pair_default = [o.cpu().numpy() for o in mappm_device_multi(d[0], [d[1], d[2]], d[3], iv, kord)]
            set_variant(monkeypatch, "FV3_MAPPM_PATH", "serial")
            set_variant(monkeypatch, "FV3_MAPPM_SPLIT", "0")
            one_ref = mappm_device(d[0], d[1], d[3], iv, kord).cpu().numpy()
            pair_ref = [o.cpu().numpy() for o in mappm_device_multi(d[0], [d[1], d[2]], d[3], iv, kord)]
            assert _bits_equal(one_default, one_ref), (kord, iv)
            for a, b in zip(pair_default, pair_ref):
                assert _bits_equal(a, b), (kord, iv)
            idx = np.sort(rng.choice(ncol, 300, replace=False))
            assert _bits_equal(one_default[:, idx], oracle_mappm(pe1[:, idx], q0[:, idx], pe2[:, idx], iv, kord))
