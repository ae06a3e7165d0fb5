"""ORACLE (test infrastructure only): numpy restatement of the microphysics emulator
hook's masks and Zhao-Carr fixers, for same-dtype [feature, sample] arrays.

Reference (paths under /root/reference/external/emulation/emulation):
* RangeMask / LevelMask                        masks.py:23-70
* squash_water_water_conserving, _apply_squash zhao_carr.py:57-84
* infer_gscond_cloud_from_conservation         zhao_carr.py:72-76
* _limit_net_condensation_conserving            zhao_carr.py:87-101
* ice_water_flag (the numba loop)               zhao_carr.py:108-133
* latent_heat_phase_dependent, apply_condensation zhao_carr.py:136-161
* _update_with_net_condensation + the gscond masks zhao_carr.py:164-259
* _get_classify_output                          zhao_carr.py:214-219
* enforce_conservative_precpd (+ the strict TOA->surface loop) zhao_carr.py:262-352
* conservative_precip_simple                    zhao_carr.py:355-371
Pinned by the reference's own KATs (tests/test_emulation_hook.py mirrors
external/emulation/tests/test_zhao_carr.py:15-66 and test_mask.py:7-50).
"""
import numpy as np

GRAVITY = 9.80665
CP = 1.0046e3
LV = 2.5e6
RHO_WATER = 1000.0
HFUS = 3.3358e5
CLASS_NAMES = ["negative_tendency", "positive_tendency", "zero_cloud", "zero_tendency"]  # sorted

QC_IN, QV_IN, T_IN, DELP = ("cloud_water_mixing_ratio_input", "specific_humidity_input", "air_temperature_input",
                            "pressure_thickness_of_atmospheric_layer")
QC_GS, QV_GS, T_GS = ("cloud_water_mixing_ratio_after_gscond", "specific_humidity_after_gscond",
                      "air_temperature_after_gscond")
QC_PR, QV_PR, T_PR, PRECIP = ("cloud_water_mixing_ratio_after_precpd", "specific_humidity_after_precpd",
                              "air_temperature_after_precpd", "total_precipitation")


def range_mask(x, lo=None, hi=None):
    if lo is not None:
        x = np.maximum(x, lo)
    if hi is not None:
        x = np.minimum(x, hi)
    return x


def level_mask(field, state_field, start, stop):
    out = np.copy(field)
    out[slice(start, stop)] = state_field[slice(start, stop)]
    return out


def squash(cloud, humidity, bound):
    cloud_out = np.where(cloud < bound, 0, cloud)
    return cloud_out, humidity + (cloud - cloud_out)


def infer_cloud(state, emulator):
    return state[QC_IN] - (emulator[QV_GS] - state[QV_IN])


def limit_net_condensation(state, net):
    cond = np.where(net > 0, net, 0.0)
    evap = np.where(net < 0, net, 0.0)
    return np.maximum(evap, -state[QC_IN]) + np.minimum(cond, state[QV_IN])


def apply_condensation(state, net, lv):
    return {QC_GS: state[QC_IN] + net, QV_GS: state[QV_IN] - net, T_GS: state[T_IN] + lv * net / CP}


def gscond_update(state, cloud_out, limit=True, lv=LV):
    net = cloud_out - state[QC_IN]
    if limit:
        net = limit_net_condensation(state, net)
    return apply_condensation(state, net, lv)


def ice_water_flag(tc, cloud):
    """The numba loop, over the last axis of 2-D arrays."""
    n, z = tc.shape
    iw = np.zeros_like(tc)
    for i in range(n):
        for k in range(z - 1, -1, -1):
            t = tc[i, k]
            if t < -15:
                iw[i, k] = 1.0
            elif t > 0.0:
                iw[i, k] = 0.0
            elif k < z - 1 and iw[i, k + 1] == 1 and float(cloud[i, k]) > 1e-20:
                iw[i, k] = 1.0
    return iw


def ice_water_flag_fast(tc, cloud):
    """The same recurrence vectorised over rows (for large arrays in the tests)."""
    n, z = tc.shape
    iw = np.zeros_like(tc)
    nxt = np.zeros(n, dtype=bool)
    for k in range(z - 1, -1, -1):
        t = tc[:, k]
        cold = t < -15
        mid = ~cold & ~(t > 0.0)
        v = cold | (mid & (k < z - 1) & nxt & (cloud[:, k].astype(np.float64) > 1e-20))
        iw[:, k] = v
        nxt = v
    return iw


def phase_dependent(state, emulator):
    tc = state[T_IN] - 273.16
    iw = ice_water_flag_fast(tc, state[QC_IN])
    return gscond_update(state, emulator[QC_GS], limit=False, lv=2.5e6 + iw * HFUS)


def classify(logits, axis=0):
    one_hot = logits == np.max(logits, axis=axis, keepdims=True)
    d = {name: np.take(one_hot, i, axis) for i, name in enumerate(CLASS_NAMES)}
    d["nontrivial_tendency"] = d["positive_tendency"] | d["negative_tendency"]
    return d


def strict_precip(condensate_to_precip, precip_to_vapor):
    """_strict_conservative_precip_from_TOA_to_surface: levels from the last (TOA) down."""
    c_to_p = np.maximum(condensate_to_precip, 0)
    p_to_v = np.maximum(precip_to_vapor, 0)
    total = np.zeros(p_to_v.shape[1])
    for k in range(p_to_v.shape[0] - 1, -1, -1):
        total += c_to_p[k]
        lim = np.minimum(total, p_to_v[k])
        total -= lim
        p_to_v[k, :] = lim
    return c_to_p, p_to_v, total


def precpd_conservative(state, emulator):
    cloud_change = emulator[QC_PR] - state[QC_GS]
    humidity_change = emulator[QV_PR] - state[QV_GS]
    delp = state[DELP]
    src = -1 * cloud_change * delp / GRAVITY
    sink = humidity_change * delp / GRAVITY
    c_to_p, p_to_v, total = strict_precip(src, sink)
    evap = p_to_v / delp * GRAVITY
    return {QC_PR: state[QC_GS] + (-1 * c_to_p) / delp * GRAVITY, QV_PR: state[QV_GS] + evap,
            T_PR: state[T_GS] + LV / CP * -1 * evap, PRECIP: total / RHO_WATER}


def precip_simple(state, emulator):
    before = np.sum((state[QV_GS] + state[QC_GS]) * state[DELP] / GRAVITY, axis=0)
    after = np.sum((emulator[QV_PR] + emulator[QC_PR]) * state[DELP] / GRAVITY, axis=0)
    return (before - after) / RHO_WATER
