"""ORACLE (test infrastructure only): numpy restatement of the composite predictors'
arithmetic and of the online transformer Adapter, with the reference's dtype flow.

Reference (paths under /root/reference):
* EnsembleModel.predict   external/fv3fit/fv3fit/_shared/models.py:253-260
  xr.concat(outputs, dim="member").mean / .median(dim="member"): xarray 0.19 skips NaN
  for floats, i.e. numpy's nanmean / nanmedian over the member axis (bottleneck is not
  pinned in constraints.txt, so numpy's).
* TaperConfig.apply       external/fv3fit/fv3fit/_shared/config.py:21-29
  vertical_tapering_scale_factors  external/vcm/vcm/calc/calc.py:45-49
* Adapter.predict         workflows/prognostic_c48_run/runtime/transformers/fv3fit.py:66-83
  non_negative_sphum_mse_conserving  runtime/steppers/machine_learning.py:77-99
  (vcm moist_static_energy_tendency / temperature_tendency, vcm/calc/thermo/local.py:317-360)

Pinned by the reference's own KATs (tests/test_composite.py): test_ensemble.py:8-28
(median 3.0 / mean 8/3 of constant members) and test_tapered_model.py:12-29 (taper of
constant outputs).  The Adapter has no reference KAT (its tests need the fv3gfs
wrapper): parity unpinned beyond the restated expressions.
"""
from collections import defaultdict

import numpy as np

from oracle.stepper import CP, RDGAS, latent_heat_vaporization

SPHUM = "specific_humidity"
TEMP = "air_temperature"


def member_reduce(members, reduction):
    """members: list of same-shaped arrays -> nanmean / nanmedian over the member axis."""
    stacked = np.stack([np.asarray(m) for m in members])
    if reduction == "mean":
        return np.nanmean(stacked, axis=0)
    if reduction == "median":
        return np.nanmedian(stacked, axis=0)
    raise NotImplementedError(reduction)


def vertical_tapering_scale_factors(n_levels, cutoff, rate):
    z_arr = np.arange(n_levels)
    scaled = np.exp((z_arr[slice(None, cutoff)] - cutoff) / rate)
    unscaled = np.ones(n_levels - cutoff)
    return np.hstack([scaled, unscaled])


def taper(data, level_axis, cutoff, rate):
    """scaling * data with the scaling's dim first (xarray's broadcast order):
    returns (moved level axis first) float64 result."""
    x = np.moveaxis(np.asarray(data), level_axis, 0)
    s = vertical_tapering_scale_factors(x.shape[0], cutoff, rate)
    return s.reshape((-1,) + (1,) * (x.ndim - 1)) * x


def adapter_predict(prediction, inputs, tendency_predictions, state_predictions, timestep,
                    limit_negative_humidity=True):
    """Adapter.predict on plain arrays (prediction: output name -> array; inputs: state
    name -> array)."""
    tendency_names = defaultdict(list)
    for k, v in tendency_predictions.items():
        tendency_names[v].append(k)
    state_names = {v: k for k, v in state_predictions.items()}
    tendencies = {k: sum([prediction[item] for item in v]) for k, v in tendency_names.items()}
    state_updates = {k: prediction[v] for k, v in state_names.items()}
    if limit_negative_humidity:
        if SPHUM not in tendencies:
            raise NotImplementedError("Cannot limit specific humidity tendencies if specific humidity "
                                      "updates not being predicted.")
        sphum, q2 = inputs[SPHUM], tendencies[SPHUM]
        q2_new = np.where(sphum + q2 * timestep >= 0, q2, -sphum / timestep)
        tendencies[SPHUM] = q2_new
        q1 = tendencies.get(TEMP)
        if q1 is not None:
            cv = CP - RDGAS
            lv = latent_heat_vaporization()
            mse = cv * q1 + lv * q2
            tendencies[TEMP] = (mse - lv * q2_new) / cv
    for name in tendencies:
        state_updates[name] = inputs[name] + tendencies[name] * timestep
    return state_updates
