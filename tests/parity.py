"""Shared tolerance checks for the floating-point parity tests.

``assert_per_level``: the north_star bound ("tendencies within 1e-5 rel") applied to
EVERY output level on its own: for level k, max_c |gpu - ref| <= rtol * max_c |ref|.
A bound over all levels at once would let a level whose values are 1e3x smaller than
the column maximum (dQ2 aloft) be off by 100% and pass.  A level whose reference is
identically zero (a clip mask) must come out exactly zero.
"""
import numpy as np


def per_level_errors(got, ref, scale=None):
    """got, ref: [N, z] (sample-major) or [N] -> per-level relative errors (NaN where
    the reference level is all zero) and the absolute errors of those zero levels.
    ``scale`` [z]: per-level magnitudes taken from a larger sample of the same model
    (a batch of one or two columns has no level scale of its own: one value that a
    dot product happens to cancel towards zero is not the level's magnitude)."""
    g = np.asarray(got, dtype=np.float64)
    r = np.asarray(ref, dtype=np.float64)
    if g.shape != r.shape:
        raise AssertionError(f"shape {g.shape} != reference {r.shape}")
    if g.ndim == 1:
        g, r = g[:, None], r[:, None]
    err = np.abs(g - r).max(axis=0)
    scale = np.abs(r).max(axis=0) if scale is None else np.maximum(np.abs(r).max(axis=0), np.ravel(scale))
    zero = scale == 0
    rel = np.where(zero, np.nan, err / np.where(zero, 1.0, scale))
    return rel, err[zero]


def assert_per_level(got, ref, rtol, what="", scale=None):
    if np.asarray(ref).size == 0:
        return
    rel, zero_err = per_level_errors(got, ref, scale)
    assert np.isfinite(np.asarray(got, dtype=np.float64)).all() or not np.isfinite(ref).all(), f"{what}: non-finite"
    assert (zero_err == 0).all(), f"{what}: levels whose reference is zero are not zero ({zero_err.max():.3e})"
    if np.isfinite(rel).any():
        k = int(np.nanargmax(rel))
        assert rel[k] <= rtol, f"{what}: level {k} max rel err {rel[k]:.3e} > {rtol}"
