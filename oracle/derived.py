"""ORACLE (test infrastructure only): numpy restatement of the derived-variable arithmetic
behind fv3fit's DerivedModel and TransformedPredictor, with the reference's dtype flow
(NumPy weak Python-float scalars, numpy reduction order).  Arrays are [z, ...] with the
vertical axis first (the stacked (z, y, x) layout); 2-D arrays drop it.

Reference (paths under /root/reference/external/vcm/vcm):
* DerivedMapping entries   derived_mapping.py:123-127 (evaporation), 264-410
* DataTransform registry   data_transform.py:65-323
* thermo                   calc/thermo/local.py:25-28 (latent_heat_vaporization),
                           69-82 (latent_heat_flux_to_evaporation), 195-208
                           (internal_energy), 317-360 (MSE / temperature tendency);
                           calc/thermo/vertically_dependent.py:18-38 (mass_integrate /
                           mass_cumsum / mass_divergence), 279-325 (column integrals)
* flux form                calc/flux_form.py:7-100
* clouds                   calc/clouds.py:7-66
* constants                calc/thermo/constants.py

xarray's float reductions skip NaN: ``.sum`` is np.nansum (from the identity +0, rows of
the leading axis added in order), ``.cumsum`` np.nancumsum (from the first term).
Parity pinned by the restated expressions only: the reference's DerivedMapping /
DataTransform tests need xarray (absent here), so beyond the expressions this is
"parity unpinned" — the HIP kernels are checked bitwise against it.
"""
import numpy as np

GRAVITY = 9.80665
RDGAS = 287.05
CP = 1004
LV0 = 2.5e6
H_LIQ = 4185.5
H_VAP = 1846
T_FREEZE = 273.15
DEFAULT_SURFACE_TEMPERATURE = T_FREEZE + 15
KG_M2S_TO_MM_DAY = (1e3 * 86400) / 997.0
CLIMIT1 = 1.0e-3
CLIMIT2 = 5.0e-2


def latent_heat_vaporization(t):
    return LV0 + (H_LIQ - H_VAP) * (t - T_FREEZE)


def latent_heat_flux_to_evaporation(lhf, surface_temperature=DEFAULT_SURFACE_TEMPERATURE):
    return lhf / latent_heat_vaporization(surface_temperature)


def internal_energy(t):
    return (CP - RDGAS) * t


def _nan0(x):
    return np.where(np.isnan(x), np.zeros((), x.dtype), x)


def mass_integrate(da, delp):
    x = _nan0(da * delp / GRAVITY)
    out = np.zeros(x.shape[1:], x.dtype)
    for k in range(x.shape[0]):
        out = out + x[k]
    return out


def mass_cumsum(da, delp):
    return np.nancumsum(da * delp / GRAVITY, axis=0)


def mass_divergence(da_interface, delp):
    return GRAVITY * np.diff(da_interface, axis=0) / delp


def column_integrated_heating_from_isochoric_transition(dt_dt, delp):
    return (CP - RDGAS) * mass_integrate(dt_dt, delp)


def minus_column_integrated_moistening(dq_dt, delp):
    return KG_M2S_TO_MM_DAY * mass_integrate(dq_dt * -1, delp)


def moist_static_energy_tendency(q1, q2, temperature=T_FREEZE):
    return (CP - RDGAS) * q1 + latent_heat_vaporization(temperature) * q2


def temperature_tendency(qm, q2, temperature=T_FREEZE):
    return (qm - latent_heat_vaporization(temperature) * q2) / (CP - RDGAS)


def gridcell_to_incloud_condensate(cf, condensate, climit1=CLIMIT1, climit2=CLIMIT2):
    scaling_ratio = 1.0 / np.where(cf > climit2, cf, np.asarray(climit2, cf.dtype))
    return np.where(cf <= climit1, condensate, condensate * scaling_ratio)


def incloud_to_gridcell_condensate(cf, incloud, climit1=CLIMIT1, climit2=CLIMIT2):
    rect = np.where(cf > climit2, cf, np.asarray(climit2, cf.dtype))
    return np.where(cf <= climit1, incloud, incloud * rect)


def isclose(x, c, rtol=1e-05, atol=1e-08):
    """np.isclose(x, c) as numpy 1.x evaluates it on a float array and a Python number
    (value-based casting: in x's dtype); NaN / inf never close to a finite c."""
    x = np.asarray(x)
    return np.abs(x - x.dtype.type(c)) <= x.dtype.type(atol + rtol * abs(c))


def _rectify(x):
    return np.where(x >= 0, x, np.zeros((), x.dtype))


def tendency_to_flux(tendency, toa_net_flux, surface_upward_flux, delp, rectify=True):
    """flux_form.py:7-42 -> (interface fluxes [z], downward surface flux)."""
    flux = -mass_cumsum(tendency, delp)
    flux = np.concatenate([np.zeros((1,) + flux.shape[1:], flux.dtype), flux])
    flux += toa_net_flux  # in place: the tendency's dtype
    down = flux[-1] + surface_upward_flux
    if rectify:
        down = _rectify(down)
    return flux[:-1], down


def tendency_to_implied_surface_downward_flux(tendency, toa_net_flux, surface_upward_flux, delp, rectify=True):
    down = toa_net_flux + surface_upward_flux - mass_integrate(tendency, delp)
    return _rectify(down) if rectify else down


def flux_to_tendency(net_flux, surface_downward_flux, surface_upward_flux, delp):
    sfc = surface_downward_flux - surface_upward_flux
    full = np.concatenate([net_flux, sfc[None].astype(np.result_type(net_flux, sfc))])
    return -mass_divergence(full, delp)


# -------------------------------------------------------------- DerivedMapping entries
def derived(name, m):
    """The DerivedMapping value of ``name`` over the mapping ``m`` (name -> array),
    honouring use_nonderived_if_exists."""
    delp = m.get("pressure_thickness_of_atmospheric_layer")
    nonderived = {"Q1", "Q2", "pQ1", "pQ2", "water_vapor_path"}
    if name in nonderived and name in m:
        return m[name]
    if name in ("pQ1", "pQ2"):
        return np.zeros_like(delp)
    if name in ("Q1", "Q2"):
        d, p = "d" + name, "p" + name
        return m[d] + derived(p, m) if d in m else derived(p, m)
    if name == "internal_energy":
        return internal_energy(m["air_temperature"])
    if name == "column_integrated_dQ1":
        return column_integrated_heating_from_isochoric_transition(m["dQ1"], delp)
    if name == "column_integrated_dQ2":
        return -minus_column_integrated_moistening(m["dQ2"], delp)
    if name == "column_integrated_Q1":
        return column_integrated_heating_from_isochoric_transition(m["Q1"], delp)
    if name == "column_integrated_Q2":
        return -minus_column_integrated_moistening(m["Q2"], delp)
    if name == "water_vapor_path":
        return mass_integrate(m["specific_humidity"], delp)
    if name == "evaporation":
        return latent_heat_flux_to_evaporation(m["latent_heat_flux"])
    if name == "upward_heat_flux_at_surface":
        return (m["total_sky_upward_shortwave_flux_at_surface"] + m["total_sky_upward_longwave_flux_at_surface"]
                + m["sensible_heat_flux"])
    if name == "net_shortwave_sfc_flux_derived":
        return (1 - m["surface_diffused_shortwave_albedo"]) * m[
            "override_for_time_adjusted_total_sky_downward_shortwave_flux_at_surface"]
    if name == "downward_shortwave_sfc_flux_via_transmissivity":
        return m["shortwave_transmissivity_of_atmospheric_column"] * m[DSW_TOA]
    if name == "net_shortwave_sfc_flux_via_transmissivity":
        return (1 - m["surface_diffused_shortwave_albedo"]) * derived("downward_shortwave_sfc_flux_via_transmissivity",
                                                                      m)
    if name in ("is_land", "is_sea", "is_sea_ice"):
        return np.where(isclose(m["land_sea_mask"], {"is_land": 1, "is_sea": 0, "is_sea_ice": 2}[name]), 1.0, 0.0)
    if name == "incloud_water_mixing_ratio":
        return gridcell_to_incloud_condensate(m["cloud_amount"], m["cloud_water_mixing_ratio"])
    if name == "incloud_ice_mixing_ratio":
        return gridcell_to_incloud_condensate(m["cloud_amount"], m["cloud_ice_mixing_ratio"])
    raise NotImplementedError(name)


# ---------------------------------------------------------------- DataTransform registry
DELP = "pressure_thickness_of_atmospheric_layer"
DSW_TOA = "total_sky_downward_shortwave_flux_at_top_of_atmosphere"
ULW_SFC = "total_sky_upward_longwave_flux_at_surface"
ULW_TOA = "total_sky_upward_longwave_flux_at_top_of_atmosphere"
USW_SFC = "total_sky_upward_shortwave_flux_at_surface"
USW_TOA = "total_sky_upward_shortwave_flux_at_top_of_atmosphere"
COL_T_NUDGE = "storage_of_internal_energy_path_due_to_fine_res_temperature_nudging"
LHF = "latent_heat_flux"
SHF = "sensible_heat_flux"


def _toa(ds, include_nudging):
    toa = ds[DSW_TOA] - ds[USW_TOA] - ds[ULW_TOA]
    if include_nudging:
        toa += ds[COL_T_NUDGE]
    return toa


def _sfc_up(ds):
    return ds[LHF] + ds[SHF] + ds[USW_SFC] + ds[ULW_SFC]


def apply_transform(name, ds, **kw):
    """data_transform.py's registered function ``name`` on a dict of arrays (updated)."""
    ds = dict(ds)
    if name in ("tapered_dQ1", "tapered_dQ2"):
        src = name.split("_")[1]
        from oracle.composite import vertical_tapering_scale_factors

        s = vertical_tapering_scale_factors(ds[src].shape[0], kw["cutoff"], kw["rate"])
        ds[name] = s.reshape((-1,) + (1,) * (ds[src].ndim - 1)) * ds[src]
    elif name == "Qm_from_Q1_Q2":
        ds["Qm"] = moist_static_energy_tendency(ds["Q1"], ds["Q2"])
    elif name == "Q1_from_Qm_Q2":
        ds["Q1"] = temperature_tendency(ds["Qm"], ds["Q2"])
    elif name == "Qm_from_Q1_Q2_temperature_dependent":
        ds["Qm"] = moist_static_energy_tendency(ds["Q1"], ds["Q2"], temperature=ds["air_temperature"])
    elif name == "Q1_from_Qm_Q2_temperature_dependent":
        ds["Q1"] = temperature_tendency(ds["Qm"], ds["Q2"], temperature=ds["air_temperature"])
    elif name == "Q1_from_dQ1_pQ1":
        ds["Q1"] = ds["dQ1"] + ds["pQ1"]
    elif name == "Q2_from_dQ2_pQ2":
        ds["Q2"] = ds["dQ2"] + ds["pQ2"]
    elif name == "Qm_flux_from_Qm_tendency":
        toa = _toa(ds, kw.get("include_temperature_nudging", True))
        ds["Qm_flux"], ds["implied_downward_radiative_flux_at_surface"] = tendency_to_flux(
            ds["Qm"], toa, _sfc_up(ds), ds[DELP], kw.get("rectify_downward_radiative_flux", True))
    elif name == "Q2_flux_from_Q2_tendency":
        ds["Q2_flux"], ds["implied_surface_precipitation_rate"] = tendency_to_flux(
            ds["Q2"], np.zeros_like(ds[LHF]), latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP],
            kw.get("rectify_surface_precipitation_rate", True))
    elif name == "Qm_tendency_from_Qm_flux":
        ds["Qm"] = flux_to_tendency(ds["Qm_flux"], ds["implied_downward_radiative_flux_at_surface"], _sfc_up(ds),
                                    ds[DELP])
    elif name == "Q2_tendency_from_Q2_flux":
        ds["Q2"] = flux_to_tendency(ds["Q2_flux"], ds["implied_surface_precipitation_rate"],
                                    latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP])
    elif name == "implied_downward_radiative_flux_at_surface":
        toa = _toa(ds, kw.get("include_temperature_nudging", True))
        ds[name] = tendency_to_implied_surface_downward_flux(ds["Qm"], toa, _sfc_up(ds), ds[DELP],
                                                             kw.get("rectify", True))
    elif name == "implied_surface_precipitation_rate":
        ds[name] = tendency_to_implied_surface_downward_flux(
            ds["Q2"], np.zeros_like(ds[LHF]), latent_heat_flux_to_evaporation(ds[LHF]), ds[DELP],
            kw.get("rectify", True))
    elif name == "cloud_water_mixing_ratio_from_incloud":
        ds["cloud_water_mixing_ratio"] = incloud_to_gridcell_condensate(ds["cloud_amount"],
                                                                        ds["incloud_water_mixing_ratio"])
    elif name == "cloud_ice_mixing_ratio_from_incloud":
        ds["cloud_ice_mixing_ratio"] = incloud_to_gridcell_condensate(ds["cloud_amount"],
                                                                      ds["incloud_ice_mixing_ratio"])
    else:
        raise NotImplementedError(name)
    return ds


# ---------------------------------------------------------------------------------
# D-grid wind rotation (vcm/cubedsphere/rotate.py:9-56, coarsen.py:54-75) and the
# wind-parallel projections (derived_mapping.py:129-187).  Pinned by the reference KATs
# external/vcm/tests/test__rotate.py:7-34 (rotate_xy_winds at 45 degrees),
# test_derived_mapping.py:86-90 (zero coefficients) and :33-58 (projection cases).
# Arrays carry their dims explicitly: (ndarray, dims); coefficients broadcast by name.
# ---------------------------------------------------------------------------------
EDGE_TO_CENTER_DIMS = {"x_interface": "x", "y_interface": "y"}


def shift_edge_var_to_center(a, dims):
    """coarsen.py:54-75: 0.5 * (edge + edge.shift(1)) without the first edge, along the
    first of x_interface / y_interface the array has; returns (array, centred dims)."""
    for d in EDGE_TO_CENTER_DIMS:
        if d in dims:
            ax = dims.index(d)
            n = a.shape[ax]
            hi = np.take(a, np.arange(1, n), axis=ax)
            lo = np.take(a, np.arange(0, n - 1), axis=ax)
            return 0.5 * (hi + lo), tuple(EDGE_TO_CENTER_DIMS[x] if x == d else x for x in dims)
    raise ValueError("Variable to shift to center must be centered on one horizontal axis and edge-valued on the "
                     "other.")


def _bcast(a, dims, out_dims):
    """``a`` (dims ``dims``) transposed and expanded to ``out_dims`` (a view)."""
    own = [d for d in out_dims if d in dims]
    a = np.transpose(a, [dims.index(d) for d in own])
    shape = [a.shape[own.index(d)] if d in dims else 1 for d in out_dims]
    return a.reshape(shape)


def rotate_xy_winds(coeffs, xc, yc, dims):
    """rotate.py:40-56: eastward = eu xc + ev yc, northward = nu xc + nv yc (numpy's
    promotion), in ``dims`` (xc and yc already in them).  coeffs: 4 (array, dims)."""
    c = [_bcast(a, d, dims) for a, d in coeffs]
    east = c[0] * xc + c[1] * yc
    north = c[2] * xc + c[3] * yc
    shape = np.broadcast_shapes(xc.shape, yc.shape)
    return np.broadcast_to(east, shape).copy(), np.broadcast_to(north, shape).copy()


def center_and_rotate_xy_winds(coeffs, x, x_dims, y, y_dims):
    """rotate.py:9-37: both components centred, then rotated; results in the centred x
    component's dims (northward transposed to the centred y component's)."""
    xc, cx = shift_edge_var_to_center(x, tuple(x_dims))
    yc, cy = shift_edge_var_to_center(y, tuple(y_dims))
    yc_in_x = np.transpose(yc, [cy.index(d) for d in cx])
    east, north = rotate_xy_winds(coeffs, xc, yc_in_x, cx)
    return (east, cx), (np.transpose(north, [cx.index(d) for d in cy]).copy(), cy)


def parallel_to_wind(wind, tendency):
    """derived_mapping.py:163-174: sign(wind / tendency) * abs(tendency)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.sign(wind / tendency) * abs(tendency)


def horizontal_wind_tendency_parallel_to_horizontal_wind(E, dQu, N, dQv):
    """derived_mapping.py:177-187 (np.linalg.norm of the stacked pair: one scalar)."""
    return (E * dQu + N * dQv) / np.linalg.norm((E, N))


# ---------------------------------------------------------------------------------
# Solar zenith angle (vcm/calc/_zenith_angle.py:54-244).  Pinned by the reference KATs
# external/vcm/tests/test__zenith_angle.py:9-90 (twelve points, the invalid-calendar
# ValueError, the DataArray name and the radian-units conversion).  Times are
# datetime.datetime (proleptic Gregorian) or JulianDate (the Julian calendar that
# cftime.DatetimeJulian holds; cftime is absent here).
# ---------------------------------------------------------------------------------
RAD_PER_DEG = np.pi / 180.0


class JulianDate:
    """A Julian-calendar date whose differences are exact timedeltas (the part of
    cftime.DatetimeJulian _days_from_2000 uses)."""

    def __init__(self, year, month, day, hour=0, minute=0, second=0):
        self.year, self.month, self.day, self.hour, self.minute, self.second = year, month, day, hour, minute, second

    def _seconds(self):
        a = (14 - self.month) // 12
        y = self.year + 4800 - a
        m = self.month + 12 * a - 3
        jdn = self.day + (153 * m + 2) // 5 + 365 * y + y // 4 - 32083
        return ((jdn * 24 + self.hour) * 60 + self.minute) * 60 + self.second

    def __sub__(self, other):
        import datetime

        return datetime.timedelta(seconds=self._seconds() - other._seconds())


def days_from_2000(model_time, julian_types=(JulianDate,)):
    import datetime

    flat = np.asarray(model_time, dtype=object).ravel()
    date_type = type(flat[0])
    if date_type not in (datetime.datetime,) + tuple(julian_types):
        raise ValueError(f"model_time has an invalid date type. It must be either datetime.datetime or "
                         f"cftime.DatetimeJulian. Got {date_type}.")
    epoch = date_type(2000, 1, 1, 12, 0)
    diff = np.array([t - epoch for t in flat], dtype=object).reshape(np.shape(model_time))
    return np.asarray(diff).astype("timedelta64[us]") / np.timedelta64(1, "D")


def _gmst(days):
    jc = days / 36525.0
    theta = 67310.54841 + jc * (876600 * 3600 + 8640184.812866 + jc * (0.093104 - jc * 6.2 * 10e-6))
    return np.deg2rad(theta / 240.0) % (2 * np.pi)


def _sun_ecliptic_longitude(days):
    jc = days / 36525.0
    mean_anomaly = np.deg2rad(357.52910 + 35999.05030 * jc - 0.0001559 * jc * jc - 0.00000048 * jc * jc * jc)
    mean_longitude = np.deg2rad(280.46645 + 36000.76983 * jc + 0.0003032 * (jc ** 2))
    d_l = np.deg2rad((1.914600 - 0.004817 * jc - 0.000014 * (jc ** 2)) * np.sin(mean_anomaly)
                     + (0.019993 - 0.000101 * jc) * np.sin(2 * mean_anomaly) + 0.000290 * np.sin(3 * mean_anomaly))
    return mean_longitude + d_l


def _obliquity_star(jc):
    return np.deg2rad(23.0 + 26.0 / 60 + 21.406 / 3600.0
                      - (46.836769 * jc - 0.0001831 * (jc ** 2) + 0.00200340 * (jc ** 3) - 0.576e-6 * (jc ** 4)
                         - 4.34e-8 * (jc ** 5)) / 3600.0)


def _right_ascension_declination(days):
    eps = _obliquity_star(days / 36525.0)
    eclon = _sun_ecliptic_longitude(days)
    x = np.cos(eclon)
    y = np.cos(eps) * np.sin(eclon)
    z = np.sin(eps) * np.sin(eclon)
    r = np.sqrt(1.0 - z * z)
    return 2 * np.arctan2(y, (x + r)), np.arctan2(z, r)


def cos_zenith_angle(model_time, lon, lat, julian_types=(JulianDate,)):
    """_zenith_angle.py:54-93, 225-244 for numpy inputs (degrees), broadcast like numpy."""
    days = days_from_2000(model_time, julian_types)
    lon_rad, lat_rad = lon * RAD_PER_DEG, lat * RAD_PER_DEG
    ra, dec = _right_ascension_declination(days)
    h_angle = _gmst(days) + lon_rad - ra
    return np.sin(lat_rad) * np.sin(dec) + np.cos(lat_rad) * np.cos(dec) * np.cos(h_angle)
