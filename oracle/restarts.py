"""ORACLE (test infrastructure only): numpy restatement of
coarsen_restarts_on_pressure for the fv_core, fv_tracer and fv_srf_wnd categories.

Reference (paths under /root/reference/external/vcm/vcm):
* coarsen_restarts_on_pressure            cubedsphere/coarsen_restarts.py:152-225
* _coarse_grain_fv_core_on_pressure       :411-516  phis/delp/DZ plain area-weighted;
                                                      W, T (+ua, va) masked on pressure;
                                                      u (dx), v (dy) edge-weighted on pressure
* _coarse_grain_fv_tracer_on_pressure     :840-887  every tracer masked on pressure
* _coarse_grain_fv_srf_wnd                :890-913  u_srf, v_srf plain area-weighted
* _impose_hydrostatic_balance             :916-938  DZ = hydrostatic_dz(T, sphum, delp);
                                                      phis = g (top height + sum DZ)
* hydrostatic_dz / height_at_interface / dz_and_top_to_phis
                                          calc/thermo/vertically_dependent.py:211-228, 69-100, 182-186
* constants                               calc/thermo/constants.py:2-4,17

Arrays carry the restart files' dims, (tile, Time, z, y, x) and (tile, Time, y, x),
with Time of length 1, as the reference's regression data does.  Pinned by that data:
tests/test_restarts.py checks every variable of
_coarsen_restarts_regression_tests/reference/pressure-level-{with,without}-agrid-winds-
{fv_core,fv_tracer,fv_srf_wnd}.res.json (tests/golden/restarts_kat.npz) at the
reference test's tolerance.

dtype flow (numpy promotion, as the reference's xarray arithmetic does it): float64
restart data times float32 area stays float64; the pressure-level fields are float32
(mappm output); in hydrostatic_dz the virtual temperature T (1 + c q) is float32 (a
Python float against float32 arrays) and everything else float64.  dz.sum over the
vertical (not the innermost axis) adds level by level.
"""
import numpy as np

from . import coarsen as OC

GRAVITY = 9.80665  # calc/thermo/constants.py:2
RDGAS = 287.05     # :3
RVGAS = 461.5      # :4

FRACTION_TRACERS = ["cld_amt"]  # coarsen_restarts.py:56
NON_FRACTION_TRACERS = ["sphum", "liq_wat", "rainwat", "ice_wat", "snowwat", "graupel", "o3mr", "sgs_tke"]


def hydrostatic_dz(T, q, delp):
    """(tile, z, y, x); vertically_dependent.py:211-228."""
    pi = OC.pressure_at_interface(delp)
    tv = T * (1 + (RVGAS / RDGAS - 1) * q)
    dlogp = np.diff(np.log(pi), axis=1)
    return -dlogp * RDGAS * tv / GRAVITY


def height_top(dz, phis):
    """Top value of height_at_interface (vertically_dependent.py:69-100): the reverse
    cumsum of [-dz, phis / g] along the vertical, i.e. phis/g - dz[km-1] - ... - dz[0]."""
    h = phis / GRAVITY
    for k in range(dz.shape[1] - 1, -1, -1):
        h = h + (-dz[:, k])
    return h


def impose_hydrostatic_balance(core, sphum):
    dz = hydrostatic_dz(core["T"], sphum, core["delp"])
    top = height_top(core["DZ"], core["phis"])
    s = dz[:, 0].copy()
    for k in range(1, dz.shape[1]):
        s = s + dz[:, k]
    return dz, GRAVITY * (top + s)


def coarsen_restarts_on_pressure(factor, grid_spec, restarts, coarsen_agrid_winds=False, iv=1, kord=1):
    """grid_spec: area (tile, y, x), dx (tile, y+1, x), dy (tile, y, x+1);
    restarts: {"fv_core.res": {...}, "fv_tracer.res": {...}, ["fv_srf_wnd.res": {...}]}."""
    notime = lambda d: {k: np.asarray(v)[:, 0] for k, v in d.items()}
    core = notime(restarts["fv_core.res"])
    tracer = notime(restarts["fv_tracer.res"])
    area, dx, dy = (np.asarray(grid_spec[k]) for k in ("area", "dx", "dy"))
    delp = core["delp"]
    masked = ["W", "T"] + (["ua", "va"] if coarsen_agrid_winds else [])
    if coarsen_agrid_winds and not ("ua" in core and "va" in core):
        raise ValueError("If 'coarsen_agrid_winds' is active, 'ua' and 'va' "
                         "must be present in the 'fv_core.res' restart files.")
    out_core = {}
    out_core["phis"] = OC.weighted_block_average(core["phis"], area, factor)
    for name in ("delp", "DZ"):
        out_core[name] = OC.weighted_block_average(core[name], area[:, None], factor)
    regridded, _ = OC.coarsen_on_pressure(delp, area, [core[n] for n in masked], factor, iv, kord)
    out_core.update(zip(masked, regridded))
    (out_core["u"],) = OC.coarsen_edges_on_pressure(delp, dx, [core["u"]], factor, "x", iv, kord)
    (out_core["v"],) = OC.coarsen_edges_on_pressure(delp, dy, [core["v"]], factor, "y", iv, kord)
    # only the listed tracers come out (cld_amt first: xr.merge order, :859-887); a
    # missing one is the reference's KeyError on ds_regridded[...]
    names = FRACTION_TRACERS + NON_FRACTION_TRACERS
    missing = [n for n in names if n not in tracer]
    if missing:
        raise KeyError(f"fv_tracer.res lacks {missing}")
    regridded, _ = OC.coarsen_on_pressure(delp, area, [tracer[n] for n in names], factor, iv, kord)
    out_tracer = dict(zip(names, regridded))
    out_core["DZ"], out_core["phis"] = impose_hydrostatic_balance(out_core, out_tracer["sphum"])
    result = {"fv_core.res": out_core, "fv_tracer.res": out_tracer}
    if "fv_srf_wnd.res" in restarts:
        srf = notime(restarts["fv_srf_wnd.res"])
        result["fv_srf_wnd.res"] = {n: OC.weighted_block_average(srf[n], area, factor) for n in ("u_srf", "v_srf")}
    return {cat: {k: v[:, None] for k, v in d.items()} for cat, d in result.items()}


# the reference regression test's inputs (external/vcm/tests/test_coarsen_restarts.py:23-30,
# regenerated as external/synth does, synth/core.py:63-67: seed 0 per single-chunk variable)
KAT_FACTOR = 2
KAT_RANGES = {"delp": (3, 5), "area": (0.5, 1), "dx": (0.5, 1), "dy": (0.5, 1)}
KAT_SCHEMA = {  # _coarsen_restarts_regression_tests/schemas/*.json: shapes and dtypes
    "fv_core.res": {"u": (6, 1, 7, 5, 4), "v": (6, 1, 7, 4, 5), "W": (6, 1, 7, 4, 4), "DZ": (6, 1, 7, 4, 4),
                    "T": (6, 1, 7, 4, 4), "delp": (6, 1, 7, 4, 4), "phis": (6, 1, 4, 4),
                    "ua": (6, 1, 7, 4, 4), "va": (6, 1, 7, 4, 4)},
    "fv_tracer.res": {n: (6, 1, 7, 4, 4) for n in ["sphum", "liq_wat", "rainwat", "ice_wat", "snowwat", "graupel",
                                                   "o3mr", "sgs_tke", "cld_amt"]},
    "fv_srf_wnd.res": {"u_srf": (6, 1, 4, 4), "v_srf": (6, 1, 4, 4)},
}
KAT_GRID = {"area": (6, 4, 4), "dx": (6, 5, 4), "dy": (6, 4, 5)}  # float32


def kat_inputs():
    restarts = {cat: {n: OC.synth_uniform(*KAT_RANGES.get(n, (-1000, 1000)), shape, np.float64)
                      for n, shape in vs.items()} for cat, vs in KAT_SCHEMA.items()}
    grid = {n: OC.synth_uniform(*KAT_RANGES[n], shape, np.float32) for n, shape in KAT_GRID.items()}
    return grid, restarts
