"""DenseColumnPredictor's per-layout plan (predictor.py ``_plan``): the layout decisions
of a call are cached per (names, dims, shapes, array kinds) of the input Dataset, so a
prognostic run's repeated calls skip them.  Checked on the CPU with a stand-in model whose
host forward is plain numpy (output = per-column function of the inputs): a cached plan
gives the uncached call's result, and a new layout (dim order, shape, an extra variable)
gets a plan of its own."""
import numpy as np
import pytest

from fv3net_amd import dataset as D
from fv3net_amd.dense import DenseModelConfig
from fv3net_amd.predictor import DenseColumnPredictor


class _NumpyModel:
    def __init__(self, nz=5):
        self.config = DenseModelConfig(["a", "b"], ["y", "s"], [nz, nz], [nz, 1], width=8, depth=2)
        self.calls = 0

    def forward_host(self, arrays, axes):
        self.calls += 1
        a = np.moveaxis(arrays[0], axes[0], 0).astype(np.float64)
        b = np.moveaxis(arrays[1], axes[1], 0).astype(np.float64)
        y = np.moveaxis((2 * a - b).astype(np.float32), 0, axes[0])
        s = np.moveaxis((a * b).sum(0, keepdims=True).astype(np.float32), 0, axes[0])
        return [np.ascontiguousarray(y), np.ascontiguousarray(s)]


def _expected(a_zyx, b_zyx):
    return (2 * a_zyx - b_zyx).astype(np.float32), (a_zyx * b_zyx).sum(0).astype(np.float32)


@pytest.mark.parametrize("dims", [("z", "y", "x"), ("y", "x", "z"), ("x", "z", "y")])
def test_cached_plan_matches_first_call_and_layouts_do_not_mix(dims):
    rng = np.random.default_rng(0)
    m = _NumpyModel()
    p = DenseColumnPredictor(["a", "b"], ["y", "s"], m)
    a, b = rng.normal(size=(5, 4, 6)), rng.normal(size=(5, 4, 6))
    perm = [("z", "y", "x").index(d) for d in dims]
    X = D.Dataset({"a": D.DataArray(np.transpose(a, perm), dims), "b": D.DataArray(np.transpose(b, perm), dims)},
                  coords={"x": np.arange(6.0)})
    ey, es = _expected(a, b)
    for _ in range(3):  # first call builds the plan, the others replay it
        out = p.predict(X)
        assert out["y"].dims == dims
        np.testing.assert_array_equal(out["y"].data, np.transpose(ey, perm))
        assert out["s"].dims == tuple(d for d in dims if d != "z")
        np.testing.assert_array_equal(out["s"].data, es if dims.index("y") < dims.index("x") else es.T)
        np.testing.assert_array_equal(out["y"].coords["x"], np.arange(6.0))
    assert len(p._plans) == 1
    # another layout through the same predictor: a plan of its own, right result
    X2 = D.Dataset({"a": D.DataArray(a, ("z", "y", "x")), "b": D.DataArray(b, ("z", "y", "x"))})
    np.testing.assert_array_equal(p.predict(X2)["y"].data, ey)
    assert len(p._plans) == 1 + (dims != ("z", "y", "x"))
    # an extra variable changes the output dim order rule's input: new plan, same values
    X3 = D.Dataset({"w": D.DataArray(np.zeros((6, 4)), ("x", "y")), "a": D.DataArray(a, ("z", "y", "x")),
                    "b": D.DataArray(b, ("z", "y", "x"))})
    out3 = p.predict(X3)
    assert out3["y"].dims == ("x", "y", "z")
    np.testing.assert_array_equal(out3["y"].data, np.transpose(ey, (2, 1, 0)))


def test_plan_cache_keeps_validation_errors():
    m = _NumpyModel()
    p = DenseColumnPredictor(["a", "b"], ["y", "s"], m)
    X = D.Dataset({"a": D.DataArray(np.zeros((5, 4, 6)), ("z", "y", "x")),
                   "b": D.DataArray(np.zeros((5, 4)), ("z", "y"))})
    for _ in range(2):  # a failing layout is never cached
        with pytest.raises(ValueError):
            p.predict(X)
    with pytest.raises(KeyError):
        p.predict(D.Dataset({"a": D.DataArray(np.zeros((5, 4, 6)), ("z", "y", "x"))}))
    assert not getattr(p, "_plans", {})
