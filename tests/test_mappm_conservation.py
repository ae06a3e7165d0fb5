"""Column-mass conservation of the remap, a size-independent property checked at the
full BASELINE sizes (C384: 884,736 columns) where a whole-grid oracle comparison would
take too long on the CPU.

The PPM / cs sub-grid profiles integrate to q1 * dp1 over each input layer
(mappm.f90:58-124 sums whole layers as q1 * dp1 and the partial pieces as integrals of
the layer's parabola), so when the output edges span the input column, sum(q2 * dp2)
equals sum(q1 * dp1) up to float32 rounding.  One caveat is the reference's own: an
output layer whose top edge is at or above pe1(1) takes q1(1) whole (mappm.f90:62-64),
so the first output edge is placed one float32 step inside the column.  Measured on the
oracle: <= 4.1e-8 relative for every kord 1-17 and iv; the bar here is 1e-6.
"""
import numpy as np
import pytest

from oracle.mappm import oracle_mappm

RTOL = 1e-6  # column mass, relative; the oracle itself holds 4.1e-8


def _columns_np(rng, km, kn, ncol, positive=False):
    base = np.linspace(200, 1800, km, dtype=np.float32)[:, None]
    delp = (base * rng.uniform(0.99, 1.01, (km, ncol))).astype(np.float32)
    pe1 = np.concatenate([np.full((1, ncol), 300, np.float32), 300 + np.cumsum(delp, 0, dtype=np.float32)])
    frac = np.linspace(0.0, 1.0, kn + 1)[:, None]
    pe2 = (pe1[0] + (pe1[-1] - pe1[0]) * frac).astype(np.float32)
    pe2[0] = np.nextafter(pe1[0], np.float32(np.inf))
    pe2[-1] = pe1[-1]
    q = (rng.uniform(0, 0.02, (km, ncol)) if positive else rng.normal(250, 10, (km, ncol))).astype(np.float32)
    return pe1, q, pe2


def _mass(q, pe):
    return (np.asarray(q, np.float64) * np.diff(np.asarray(pe, np.float64), axis=0)).sum(0)


@pytest.mark.parametrize("kn", [79, 50, 120])
@pytest.mark.parametrize("positive", [False, True], ids=["temperature", "tracer"])
def test_oracle_conserves_column_mass(kn, positive):
    """Pins the property on the oracle (CPU): every kord and iv."""
    rng = np.random.default_rng(kn + 7 * positive)
    pe1, q, pe2 = _columns_np(rng, 79, kn, 400, positive)
    m1 = _mass(q, pe1)
    for kord in range(1, 18):
        for iv in (0, 1, -1, 2):
            m2 = _mass(oracle_mappm(pe1, q, pe2, iv, kord), pe2)
            rel = np.abs(m2 - m1) / np.abs(m1)
            assert rel.max() <= RTOL, (kord, iv, rel.max())


def _columns_dev(seed, km, kn, ncol, positive=False):
    """The same construction on the device (float32 cumsum there; the property does not
    depend on the exact edges)."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    base = torch.linspace(200, 1800, km, device="cuda")[:, None]
    delp = base * (0.99 + 0.02 * torch.rand((km, ncol), generator=g, device="cuda"))
    pe1 = torch.cat([torch.full((1, ncol), 300.0, device="cuda"), 300.0 + torch.cumsum(delp, 0)])
    frac = torch.linspace(0.0, 1.0, kn + 1, device="cuda", dtype=torch.float64)[:, None]
    pe2 = (pe1[0].double() + (pe1[-1].double() - pe1[0].double()) * frac).float()
    pe2[0] = torch.nextafter(pe1[0], torch.tensor(float("inf"), device="cuda"))
    pe2[-1] = pe1[-1]
    if positive:
        q = 0.02 * torch.rand((km, ncol), generator=g, device="cuda")
    else:
        q = 250.0 + 10.0 * torch.randn((km, ncol), generator=g, device="cuda")
    return pe1.contiguous(), q.contiguous(), pe2.contiguous()


def _mass_dev(q, pe):
    return (q.double() * (pe[1:].double() - pe[:-1].double())).sum(0)


def _check_dev(q1, pe1, q2, pe2):
    import torch

    assert bool(torch.isfinite(q2).all())
    m1, m2 = _mass_dev(q1, pe1), _mass_dev(q2, pe2)
    rel = float(((m2 - m1).abs() / m1.abs()).max())
    assert rel <= RTOL, rel


NCOL_C384 = 6 * 384 * 384


@pytest.mark.gpu
@pytest.mark.parametrize("kord,iv,kn", [(1, 1, 79), (10, 1, 79), (1, 1, 50), (10, 0, 120), (5, -1, 79)])
def test_c384_column_mass_conserved(gpu, kord, iv, kn):
    """Every one of the 884,736 columns at the bench size (the kord 1 and kord 10 legs),
    through the product kernels that size selects."""
    import torch

    from tests.remap_exact import mappm_device

    pe1, q, pe2 = _columns_dev(kord * 100 + kn, 79, kn, NCOL_C384)
    q2 = mappm_device(pe1, q, pe2, iv, kord)
    torch.cuda.synchronize()
    _check_dev(q, pe1, q2, pe2)


@pytest.mark.gpu
def test_c384_two_field_pass_conserves_both(gpu):
    """The two-field pass (predict + mappm's remap of both tendencies) at C384."""
    import torch

    from tests.remap_exact import mappm_device_multi

    pe1, q, pe2 = _columns_dev(11, 79, 79, NCOL_C384)
    _, t, _ = _columns_dev(12, 79, 79, NCOL_C384, positive=True)
    outs = mappm_device_multi(pe1, [q, t], pe2, 1, 1)
    torch.cuda.synchronize()
    _check_dev(q, pe1, outs[0], pe2)
    _check_dev(t, pe1, outs[1], pe2)


@pytest.mark.gpu
@pytest.mark.parametrize("kord", [1, 10])
def test_c384_columns_independent_of_position(gpu, kord):
    """37 template columns (edges and values) repeated over the 884,736 columns: every
    copy's remap carries exactly its template's bits, whichever lane, wave, scratch slot
    or level tail serves it."""
    import torch

    from tests.remap_exact import mappm_device, mappm_device_multi

    nt = 37
    pe1, q, pe2 = _columns_dev(kord + 41, 79, 79, nt)
    _, t, _ = _columns_dev(kord + 42, 79, 79, nt, positive=True)
    pick = torch.arange(NCOL_C384, device="cuda") % nt
    rep = lambda a: a[:, pick].contiguous()  # noqa: E731
    P1, Q, P2, Tq = rep(pe1), rep(q), rep(pe2), rep(t)
    outs = [mappm_device(P1, Q, P2, 1, kord)] + list(mappm_device_multi(P1, [Q, Tq], P2, 1, kord))
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert torch.equal(o, o[:, :nt][:, pick]), i
    assert torch.equal(outs[0], outs[1])  # the two-field pass: bit-identical to one field
