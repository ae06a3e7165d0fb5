"""ORACLE (test infrastructure only): numpy restatement of the ML stepper's
post-prediction epilogue with the reference's dtype flow (f32 model outputs, state
in the state's dtype, Python-float constants, NumPy weak-scalar promotion).

Reference (paths under /root/reference/workflows/prognostic_c48_run/runtime):
* non_negative_sphum                       steppers/machine_learning.py:67-74
* update_moisture_tendency_to_ensure...    steppers/machine_learning.py:77-80
* update_temperature_tendency_to_conserve  steppers/machine_learning.py:83-88
  (vcm moist_static_energy_tendency / temperature_tendency,
   external/vcm/vcm/calc/thermo/local.py:317-360, latent_heat_vaporization :25-28
   at the default temperature 273.15 K)
* non_negative_sphum_mse_conserving        steppers/machine_learning.py:91-99
* PureMLStepper.__call__ limiter + diags   steppers/machine_learning.py:255-303
* compute_diagnostics (net moistening/heating) diagnostics/compute.py:77-106
* mass_integrate                           external/vcm/vcm/calc/thermo/vertically_dependent.py:18-22
* column_integrated_heating_from_iso{baric,choric}_transition  vertically_dependent.py:255-301
* fillna_tendency                          loop.py:103-110
* add_tendency                             loop.py:202-219
* precipitation_sum                        diagnostics/compute.py:21-39
Constants: external/vcm/vcm/calc/thermo/constants.py.

Arrays are [z, column] (the stacked (z, y, x) state); column sums run over z in
order, NaN-skipping like xarray's sum (numpy reduces a non-contiguous outer axis
row by row).
"""
import numpy as np

GRAVITY = 9.80665
RDGAS = 287.05
CP = 1004
LV0 = 2.5e6
H_LIQ = 4185.5
H_VAP = 1846
T_FREEZE = 273.15


def latent_heat_vaporization(t=T_FREEZE):
    return LV0 + (H_LIQ - H_VAP) * (t - T_FREEZE)


def mass_integrate(da, delp):
    x = da * delp / GRAVITY
    x = np.where(np.isnan(x), np.zeros((), x.dtype), x)
    out = np.zeros(x.shape[1:], x.dtype)  # numpy's add.reduce starts from +0.0
    for k in range(x.shape[0]):
        out = out + x[k]
    return out


def heating(dt_dt, delp, hydrostatic):
    c = CP if hydrostatic else (CP - RDGAS)
    return c * mass_integrate(dt_dt, delp)


def limiter(sphum, dq1, dq2, dt, mse_conserving):
    if mse_conserving:
        q2_new = np.where(sphum + dq2 * dt >= 0, dq2, -sphum / dt)
        cv = CP - RDGAS
        lv = latent_heat_vaporization()
        mse = cv * dq1 + lv * dq2
        q1_new = (mse - lv * q2_new) / cv
    else:
        delta = dq2 * dt
        ratio = (-sphum) / (dt * dq2)
        keep = sphum + delta >= 0
        q1_new = np.where(keep, dq1, ratio * dq1)
        q2_new = np.where(keep, dq2, ratio * dq2)
    return q1_new, q2_new


def fillna(t):
    filled = np.where(np.isnan(t), np.zeros((), t.dtype), t)
    frac = (t != filled).astype(np.int64).sum(axis=0) / t.shape[0]
    return filled, frac


def epilogue(dq1, dq2, sphum, delp, temperature, physics_precip, dt, mse_conserving=True, hydrostatic=False):
    """Everything the prognostic loop does with a (dQ1, dQ2) prediction, per column."""
    dt = float(dt)
    q1n, q2n = limiter(sphum, dq1, dq2, dt, mse_conserving)
    out = {
        "dQ1": q1n,
        "dQ2": q2n,
        "column_integrated_dQ1_change_non_neg_sphum_constraint": heating(q1n - dq1, delp, hydrostatic),
        "column_integrated_dQ2_change_non_neg_sphum_constraint": mass_integrate(q2n - dq2, delp),
        "specific_humidity_limiter_active": np.where(dq2 != q2n, 1, 0).astype(np.uint8),
        "net_moistening": mass_integrate(q2n, delp),
        "column_heating": heating(q1n, delp, hydrostatic),
    }
    q1f, frac1 = fillna(q1n)
    q2f, frac2 = fillna(q2n)
    out["dQ1_filled_frac"] = frac1
    out["dQ2_filled_frac"] = frac2
    out["air_temperature"] = temperature + q1f * dt
    out["specific_humidity"] = sphum + q2f * dt
    m_per_mm = 1 / 1000
    total = physics_precip + (-out["net_moistening"] * dt * m_per_mm)
    out["total_precipitation"] = np.where(total >= 0, total, 0)
    return out


# ---------------------------------------------------------------------------------
# The whole PureMLStepper step for an arbitrary prediction (machine_learning.py:239-309,
# runtime/names.py:31-65), its get_diagnostics (diagnostics/compute.py:77-161) and the
# loop's apply (loop.py:103-145, 202-219, 615-628).  Arrays are [z, column].
# ---------------------------------------------------------------------------------
TENDENCY_TO_STATE_NAME = {"dQ1": "air_temperature", "dQ2": "specific_humidity", "dQu": "eastward_wind",
                          "dQv": "northward_wind", "dQx_wind": "x_wind", "dQy_wind": "y_wind",
                          "dQp": "pressure_thickness_of_atmospheric_layer"}
TENDENCY_NAMES = set(TENDENCY_TO_STATE_NAME) | {"dQu", "dQv"}
TOTAL_PRECIP_RATE = "total_precipitation_rate"


def is_state_update_variable(key, state):
    return (key in state and key not in TENDENCY_NAMES) or key == TOTAL_PRECIP_RATE


def pure_ml_step(prediction, state, dt, mse_conserving=True, hydrostatic=False, label="machine_learning"):
    """-> (tendency, diagnostics, state_updates, stepper_diags, applied) where
    stepper_diags is get_diagnostics' dict and applied the loop's updated state +
    filled fractions + the float64 A-grid wind tendencies handed to the wrapper."""
    dt = float(dt)
    sphum, delp = state["specific_humidity"], state["pressure_thickness_of_atmospheric_layer"]
    tendency, updates, diags = {}, {}, {}
    for k, v in prediction.items():
        if is_state_update_variable(k, state):
            updates[k] = v
        elif k in TENDENCY_NAMES:
            tendency[k] = v
        else:
            diags[k] = v
    diags.update(updates)
    zeros = np.zeros_like(sphum)
    dq1 = tendency.get("dQ1", zeros)
    dq2 = tendency.get("dQ2", zeros)
    q1n, q2n = limiter(sphum, dq1, dq2, dt, mse_conserving)
    if "dQ1" in tendency:
        diags["column_integrated_dQ1_change_non_neg_sphum_constraint"] = heating(q1n - tendency["dQ1"], delp,
                                                                                  hydrostatic)
        tendency["dQ1"] = q1n
    if "dQ2" in tendency:
        diags["column_integrated_dQ2_change_non_neg_sphum_constraint"] = mass_integrate(q2n - tendency["dQ2"], delp)
        tendency["dQ2"] = q2n
    diags["specific_humidity_limiter_active"] = np.where(dq2 != q2n, 1, 0).astype(np.uint8)
    # get_diagnostics: compute_diagnostics + compute_ml_momentum_diagnostics
    zd = np.zeros_like(delp)
    sd = {f"net_moistening_due_to_{label}": mass_integrate(tendency.get("dQ2", zd), delp),
          f"column_heating_due_to_{label}": heating(tendency.get("dQ1", zd), delp, hydrostatic)}
    if "dQp" in tendency:
        sd[f"net_mass_tendency_due_to_{label}"] = mass_integrate(np.ones_like(tendency["dQp"]), tendency["dQp"])
    sd["dQ1"] = tendency.get("dQ1", zd)
    sd["dQ2"] = tendency.get("dQ2", zd)
    for w in ("dQu", "dQv"):
        sd[w] = tendency.get(w, zd)
        sd[f"column_integrated_{w}_stress"] = mass_integrate(sd[w], delp)
    # apply: fillna, add_tendency (A-grid winds go to the wrapper as float64), precipitation_sum
    applied, fracs = {}, {}
    for name, t in tendency.items():
        filled, fracs[f"{name}_filled_frac"] = fillna(t)
        if name in ("dQu", "dQv"):
            applied[name] = filled.astype(np.float64)
        else:
            sname = TENDENCY_TO_STATE_NAME[name]
            applied[sname] = state[sname] + filled * dt
    if "total_precipitation" in state:
        net = sd[f"net_moistening_due_to_{label}"]
        total = state["total_precipitation"] + (-net * dt * (1 / 1000))
        applied["total_precipitation"] = np.where(total >= 0, total, 0)
    return tendency, diags, updates, sd, (applied, fracs)
