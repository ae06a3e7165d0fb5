"""The fv3fit Predictor boundary: registry, stack semantics, ConstantOutputPredictor
(CPU), and the MI355X DenseColumnPredictor end to end (GPU).

Mirrors external/fv3fit/tests/test_stacking.py:24-94, test_io.py / test_register_model.py
(duplicate names, name file), test_constant_predictor.py, and pure_keras.py:98-118.
"""
import os

import numpy as np
import pytest

from conftest import set_variant

from tests.parity import assert_per_level

from fv3net_amd import dataset as D
from fv3net_amd import predictor as P
from fv3net_amd.predictor import SAMPLE_DIM_NAME, Z_DIM_NAMES, stack


def _gridded(zdim, ydim=10, xdim=10):
    var = np.array([[[(100 * k) + (10 * j) + i for i in range(xdim)] for j in range(ydim)] for k in range(zdim)],
                   dtype=np.float64)
    return D.Dataset({"var": D.DataArray(var, ["z", "y", "x"],
                                         coords={"z": range(zdim), "y": range(ydim), "x": range(xdim)})})


@pytest.mark.parametrize("zdim", [1, 10])
def test_stack_dims(zdim):
    ds = _gridded(zdim)
    out = stack(ds, unstacked_dims=Z_DIM_NAMES)
    assert set(out.dims) == {SAMPLE_DIM_NAME, "z"}
    assert out["var"].dims[0] == SAMPLE_DIM_NAME
    assert out["var"].shape == (100, zdim)


def test_stack_order_is_alphabetical_and_bit_exact():
    """sample s = ix * ny + iy: stack dims are iterated sorted (x before y), C order."""
    ds = _gridded(3, ydim=4, xdim=5)
    out = stack(ds, unstacked_dims=["z"]).data_vars["var"].data
    v = ds["var"].values  # (z, y, x)
    for ix in range(5):
        for iy in range(4):
            np.testing.assert_array_equal(out[ix * 4 + iy], v[:, iy, ix])


def test_stack_no_stacked_dims():
    ds = _gridded(10)
    out = stack(ds, unstacked_dims=["x", "y", "z"])
    assert list(out["var"].dims) == [SAMPLE_DIM_NAME, "x", "y", "z"]
    assert out["var"].shape[0] == 1


def test_stack_no_unstacked_dims():
    ds = _gridded(10)
    out = stack(ds)
    assert list(out["var"].dims) == [SAMPLE_DIM_NAME]
    assert out["var"].shape[0] == 1000


@pytest.mark.parametrize("dims", [("time", "x", "y", "z"), ("time", "z", "y", "x")])
def test_multiple_unstacked_dims_are_alphabetically_ordered(dims):
    ds = D.Dataset({"var1": D.DataArray(np.zeros([2, 12, 12, 15]), dims)})
    out = stack(ds, unstacked_dims=["x", "y", "z"])
    assert list(out["var1"].dims) == [SAMPLE_DIM_NAME, "x", "y", "z"]


def test_stack_refuses_broadcast():
    ds = D.Dataset({"a": D.DataArray(np.zeros((3, 4, 5)), ["z", "y", "x"]),
                    "b": D.DataArray(np.zeros((3, 4)), ["z", "y"])})
    with pytest.raises(ValueError, match="broadcast"):
        stack(ds, unstacked_dims=["z"])


def test_register_duplicate_name_raises():
    with pytest.raises(ValueError, match="already registered"):
        P.register("constant-output")(type("X", (), {}))


def test_constant_output_predictor_roundtrip(tmp_path):
    ds = D.Dataset({"a": D.DataArray(np.random.rand(5, 3, 4), ["z", "y", "x"]),
                    "b": D.DataArray(np.random.rand(3, 4), ["y", "x"])})
    p = P.ConstantOutputPredictor(["a", "b"], ["out_z", "out_s"])
    p.set_outputs(out_z=np.arange(5.0), out_s=2.5)
    out = p.predict(ds)
    assert out["out_z"].dims == ("z", "y", "x")
    assert out["out_s"].dims == ("y", "x")
    np.testing.assert_array_equal(out["out_z"].values[:, 1, 2], np.arange(5.0))
    assert (out["out_s"].values == 2.5).all()
    P.dump(p, str(tmp_path / "m"))
    with open(tmp_path / "m" / "name") as f:
        assert f.read() == "constant-output"
    q = P.load(str(tmp_path / "m"))
    np.testing.assert_array_equal(q.predict(ds)["out_z"].values, out["out_z"].values)


def test_constant_predictor_missing_input_raises_keyerror():
    ds = D.Dataset({"a": D.DataArray(np.zeros((5, 3, 4)), ["z", "y", "x"])})
    p = P.ConstantOutputPredictor(["a", "missing"], ["o"])
    with pytest.raises(KeyError):
        p.predict(ds)


def test_predictor_rejects_unknown_kwargs():
    with pytest.raises(TypeError):
        P.ConstantOutputPredictor.__mro__[1].__init__(P.ConstantOutputPredictor(["a"], ["b"]), ["a"], ["b"],
                                                     bogus=1)


def test_dense_model_dump_load_roundtrip(tmp_path):
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [7, 7], [7, 7], width=16, depth=3,
                           clip={"T": (1, 6)}, output_limits={"dQ2": (None, 0.5)})
    m = DenseColumnModel.random(cfg, seed=3, bias_scale=0.1)
    pred = P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)
    P.dump(pred, str(tmp_path / "dense"))
    with open(tmp_path / "dense" / "name") as f:
        assert f.read() == "mi355x-dense"
    q = P.load(str(tmp_path / "dense"))
    assert q.model.config == cfg
    for k in ("hidden_kernels", "out_kernels", "in_mean", "out_sigma"):
        for a, b in zip(m.params[k], q.model.params[k]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_dense_predictor_end_to_end(gpu):
    """DenseColumnPredictor.predict on a (z, y, x) state == the Keras graph applied
    per column (oracle), same dims/coords as the input, float32."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from oracle.dense import dense_predict

    rng = np.random.default_rng(5)
    nz, ny, nx = 79, 48, 48
    T = rng.normal(260, 15, (nz, ny, nx)).astype(np.float64)
    q = rng.uniform(0, 0.02, (nz, ny, nx)).astype(np.float64)
    ps = rng.normal(1e5, 300, (ny, nx))
    X = D.Dataset({"air_temperature": D.DataArray(T, ["z", "y", "x"], coords={"x": np.arange(nx)}),
                   "specific_humidity": D.DataArray(q, ["z", "y", "x"]),
                   "surface_pressure": D.DataArray(ps, ["y", "x"])})
    cfg = DenseModelConfig(["air_temperature", "specific_humidity", "surface_pressure"],
                           ["dQ1", "dQ2", "total_precip"], [79, 79, 1], [79, 79, 1], width=256, depth=3)
    sT = T.transpose(1, 2, 0).reshape(-1, nz)
    sq = q.transpose(1, 2, 0).reshape(-1, nz)
    sps = ps.reshape(-1, 1)
    m = DenseColumnModel.random(cfg, seed=2, sample_inputs=[sT, sq, sps], bias_scale=0.1)
    pred = P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)
    out = pred.predict(X)
    assert out["dQ1"].dims == ("z", "y", "x") and out["total_precip"].dims == ("y", "x")
    assert out["dQ1"].values.dtype == np.float32
    ref = dense_predict([sT, sq, sps], m.oracle_params(), np.float64)
    got1 = out["dQ1"].values.transpose(1, 2, 0).reshape(-1, nz)
    got3 = out["total_precip"].values.reshape(-1, 1)
    for g, r in ((got1, ref[0]), (got3, ref[2])):
        assert_per_level(g, r, 1e-5)
    np.testing.assert_array_equal(out.coords["x"], np.arange(nx))
    # device-resident input stays on device
    Xd = D.Dataset({k: D.DataArray(torch.from_numpy(X[k].values.astype(np.float32)).cuda(), X[k].dims)
                    for k in X})
    outd = pred.predict(Xd)
    assert isinstance(outd["dQ1"].data, torch.Tensor) and outd["dQ1"].data.is_cuda
    with pytest.raises(KeyError):
        pred.predict(D.Dataset({"air_temperature": X["air_temperature"]}))


@pytest.mark.gpu
def test_dense_predictor_host_arrays_arena_path(gpu):
    """numpy inputs take the host-call path (copies to device buffers kept per shape, the
    bound kernel, DMA back into arrays of the library's page-locked arena):
    bit-identical to the device-resident predict on the float32 values, for float64 and
    float32 arrays, read-only arrays, repeated calls (fresh outputs each call), a shape
    change, and small arrays."""
    import torch

    from fv3net_amd import transfer
    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    rng = np.random.default_rng(8)
    cfg = DenseModelConfig(["air_temperature", "specific_humidity"], ["dQ1", "dQ2"], [79, 79], [79, 79],
                           width=256, depth=3)
    T = rng.normal(260, 15, (79, 48, 48))
    q = rng.uniform(0, 0.02, (79, 48, 48))
    m = DenseColumnModel.random(cfg, seed=3, sample_inputs=[T.reshape(79, -1).T, q.reshape(79, -1).T])
    pred = P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m)

    def device_ref(T, q):
        Xd = D.Dataset({"air_temperature": D.DataArray(torch.from_numpy(T.astype(np.float32)).cuda(), ["z", "y", "x"]),
                        "specific_humidity": D.DataArray(torch.from_numpy(q.astype(np.float32)).cuda(),
                                                         ["z", "y", "x"])})
        o = pred.predict(Xd)
        return [o[k].data.cpu().numpy() for k in ("dQ1", "dQ2")]

    def host(T, q):
        X = D.Dataset({"air_temperature": D.DataArray(T, ["z", "y", "x"]),
                       "specific_humidity": D.DataArray(q, ["z", "y", "x"])})
        o = pred.predict(X)
        assert all(isinstance(o[k].values, np.ndarray) and o[k].values.dtype == np.float32 for k in ("dQ1", "dQ2"))
        return [o[k].values for k in ("dQ1", "dQ2")]

    ref = device_ref(T, q)
    first = host(T, q)
    for g, r in zip(first, ref):
        assert (g.view(np.uint32) == r.view(np.uint32)).all()
    ro_T, ro_q = T.copy(), q.copy()
    ro_T.flags.writeable = False
    ro_q.flags.writeable = False
    again = host(ro_T, ro_q)
    for g, a, r in zip(again, first, ref):
        assert g is not a and (g.view(np.uint32) == r.view(np.uint32)).all()
    T32, q32 = T.astype(np.float32), q.astype(np.float32)
    for g, r in zip(host(T32, q32), ref):
        assert (g.view(np.uint32) == r.view(np.uint32)).all()
    # another shape (a smaller rank subdomain), then small arrays
    for shape in ((79, 24, 48), (79, 4, 5)):
        Ts, qs = T[:, :shape[1], :shape[2]].copy(), q[:, :shape[1], :shape[2]].copy()
        for g, r in zip(host(Ts, qs), device_ref(Ts, qs)):
            assert (g.view(np.uint32) == r.view(np.uint32)).all(), shape
    # outputs of the numpy path live in the library's page-locked arena
    assert transfer.is_arena(first[0]) and transfer.is_arena(again[1])
    torch.cuda.synchronize()


def test_load_without_name_file_tries_every_registered_type(tmp_path):
    """io.py:76-88: a missing ``name`` file warns and tries each registered class."""
    ds = D.Dataset({"a": D.DataArray(np.random.rand(5, 3, 4), ["z", "y", "x"])})
    p = P.ConstantOutputPredictor(["a"], ["o"])
    p.set_outputs(o=np.arange(5.0))
    P.dump(p, str(tmp_path / "m"))
    (tmp_path / "m" / "name").unlink()
    with pytest.warns(UserWarning, match="one-by-one"):
        q = P.load(str(tmp_path / "m"))
    np.testing.assert_array_equal(q.predict(ds)["o"].values, p.predict(ds)["o"].values)


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [("tile", "z", "y", "x"), ("y", "x", "z")])
def test_dense_predictor_level_axis_anywhere(gpu, dims):
    """(tile, z, y, x) is read in place (level axis 1); (y, x, z) goes through the
    permute path.  Output dims follow the input's order; values == per-column oracle."""
    import torch

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig
    from oracle.dense import dense_predict

    rng = np.random.default_rng(11)
    sizes = {"tile": 2, "z": 9, "y": 5, "x": 6}
    shape = [sizes[d] for d in dims]
    T = rng.normal(260, 15, shape).astype(np.float32)
    q = rng.uniform(0, 0.02, shape).astype(np.float32)
    X = D.Dataset({"T": D.DataArray(torch.from_numpy(T).cuda(), list(dims)),
                   "q": D.DataArray(torch.from_numpy(q).cuda(), list(dims))})
    cfg = DenseModelConfig(["T", "q"], ["dQ1", "pr"], [9, 9], [9, 1], width=64, depth=3)
    zax = dims.index("z")
    cols = lambda a: np.moveaxis(a, zax, -1).reshape(-1, 9)
    m = DenseColumnModel.random(cfg, seed=4, sample_inputs=[cols(T), cols(q)], bias_scale=0.1)
    out = P.DenseColumnPredictor(cfg.input_variables, cfg.output_variables, m).predict(X)
    assert out["dQ1"].dims == tuple(dims)
    assert out["pr"].dims == tuple(d for d in dims if d != "z")
    ref = dense_predict([cols(T), cols(q)], m.oracle_params(), np.float64)
    g1 = cols(out["dQ1"].data.cpu().numpy())
    g2 = out["pr"].data.cpu().numpy().reshape(-1, 1)
    for g, r in ((g1, ref[0]), (g2, ref[1])):
        assert_per_level(g, r, 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel_out", ["1", "0"])
@pytest.mark.parametrize("groups,ntile", [("tiles", 6), ("two", 6), ("two", 5)])
def test_forward_host_tile_pipeline_bit_identical(gpu, dtype, kernel_out, groups, ntile, monkeypatch):
    """DenseColumnModel.forward_host over (tile, z, y, x) numpy arrays: the tile blocks
    pipelined over two streams, one tile per group or two halves of the tile axis (the
    thresholds lowered so a C12 state takes the path; 5 tiles: halves of 2 and 3), give
    the bits of the device-resident forward of the same values, on repeated calls, with
    fresh outputs each call; the out-copies by the fv3_copy_to_host kernel into the
    arena pages (FV3_D2H_KERNEL=1) or by the copy engines (0); a level-leading array
    (no block axis) takes the one-call path."""
    import torch

    set_variant(monkeypatch, "FV3_D2H_KERNEL", kernel_out)
    if groups == "two":
        set_variant(monkeypatch, "FV3_HOST_TWO_GROUPS_MIB", "0")

    from fv3net_amd.dense import DenseColumnModel, DenseModelConfig

    rng = np.random.default_rng(12)
    cfg = DenseModelConfig(["T", "q"], ["dQ1", "dQ2"], [79, 79], [79, 79], width=256, depth=3)
    T = rng.normal(260, 15, (ntile, 79, 12, 12)).astype(dtype)
    q = rng.uniform(0, 0.02, (ntile, 79, 12, 12)).astype(dtype)
    m = DenseColumnModel.random(cfg, seed=4, sample_inputs=[T[0].reshape(79, -1).T, q[0].reshape(79, -1).T])
    ref = m.forward([torch.from_numpy(T).cuda(), torch.from_numpy(q).cuda()], level_axes=[1, 1])
    ref = [r.cpu().numpy() for r in ref]
    if groups == "tiles":
        m._PIPELINE_MIN_BYTES = 0
    a = m.forward_host([T, q], [1, 1])
    b = m.forward_host([T, q], [1, 1])
    assert m._host_call[3] is not None  # the pipelined path
    assert len(m._host_call[2]) == (ntile if groups == "tiles" else 2)
    # fresh outputs live in the page-locked arena, so FV3_D2H_KERNEL=1 takes the kernel
    assert m._last_kernel_out == (kernel_out == "1")
    assert a[0] is not b[0]
    for x, y, r in zip(a, b, ref):
        assert x.shape == r.shape and x.dtype == np.float32
        assert (x.view(np.uint32) == r.view(np.uint32)).all()
        assert (y.view(np.uint32) == r.view(np.uint32)).all()
    outs = [np.full(T.shape, np.nan, np.float32), np.full(T.shape, np.nan, np.float32)]
    c = m.forward_host([T, q], [1, 1], out=outs)
    assert c[0] is outs[0]
    for x, r in zip(outs, ref):
        assert (x.view(np.uint32) == r.view(np.uint32)).all()
    with pytest.raises(ValueError):
        m.forward_host([T, q], [1, 1], out=[outs[0]])
    one = m.forward_host([np.ascontiguousarray(T[0]), np.ascontiguousarray(q[0])], [0, 0])
    assert m._host_call[3] is None
    for x, r in zip(one, ref):
        assert (x.view(np.uint32) == r[0].view(np.uint32)).all()
