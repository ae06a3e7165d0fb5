// fv3net_amd — the stepper epilogue's per-level and per-column arithmetic, shared by the
// standalone epilogue kernels (stepper.hip) and the dense kernel's fused stepper
// epilogue (dense.hip, fv3_dense_stepper_f64in): one definition, so the fused path
// carries the standalone path's bits by construction.  See stepper.hip for the
// reference lines each piece follows.
#pragma once

#include "common.h"

namespace fv3 {
namespace epi {

constexpr double kGravity = 9.80665;  // vcm/calc/thermo/constants.py
constexpr double kRdgas = 287.05;
constexpr double kCp = 1004.0;
constexpr double kLv = 2.5e6;         // latent_heat_vaporization(273.15 K)

template <typename DT>
struct EpilogueArgs {
    const float* dq1;
    const float* dq2;
    const DT* sphum;
    const DT* delp;
    const DT* temp;
    const DT* precip;      // [col] physics precipitation, or NULL
    DT* dq1_out;           // [z][col] limited tendencies (pre-fill), or NULL
    DT* dq2_out;
    uint8_t* active;       // [z][col] limiter flag, or NULL
    DT* temp_out;          // [z][col] T + fill(dQ1) dt, or NULL (may alias temp)
    DT* sphum_out;         // [z][col] q + fill(dQ2) dt, or NULL (may alias sphum)
    DT* col;               // [8][col] column diagnostics (see fv3net_amd.h), or NULL
    fv3_layout lay;        // every [z][col] array
    int64_t ncol, col_ld;  // column diagnostics: row stride
    int nz, mse, hydrostatic;
    int has_dq1, has_dq2;  // the prediction holds dQ1 / dQ2 (else the inputs are zeros, machine_learning.py:258-259)
    double dt;
};

template <typename DT>
__device__ __forceinline__ DT nan0(DT x) { return x != x ? DT(0) : x; }

// One level of one column: the limiter, the limited / filled tendencies and the updated
// state written, and the level's terms of the four column sums returned (each already
// nan0'd: the sums add them in level order from +0.0).
template <typename DT>
struct EpiLevel {
    DT h, m, nm, ch;  // mass_integrate terms: heating change, moistening change, net moistening, column heating
    bool nan1, nan2;
};

template <typename DT>
__device__ __forceinline__ EpiLevel<DT> epi_level(const EpilogueArgs<DT>& a, int64_t i, float q1, float q2, DT sp,
                                                  DT dp, DT t)
{
    const float dtf = (float)a.dt;  // f32 array * Python float -> f32
    const DT dtd = (DT)a.dt;
    const float cvf = (float)(kCp - kRdgas), lvf = (float)kLv;
    const DT cv = (DT)(kCp - kRdgas), lv = (DT)kLv, g = (DT)kGravity;
    DT q1n, q2n;
    if (a.mse) {
        // update_moisture_tendency_to_ensure_non_negative_humidity (machine_learning.py:77-80)
        const float d = q2 * dtf;
        q2n = (sp + (DT)d >= (DT)0) ? (DT)q2 : (-sp) / dtd;
        // update_temperature_tendency_to_conserve_mse (:83-88)
        const float m = cvf * q1 + lvf * q2;
        q1n = ((DT)m - lv * q2n) / cv;
    } else {
        // non_negative_sphum (:67-74)
        const float delta = q2 * dtf;
        const DT ratio = (-sp) / (DT)(dtf * q2);
        const bool keep = sp + (DT)delta >= (DT)0;
        q1n = keep ? (DT)q1 : ratio * (DT)q1;
        q2n = keep ? (DT)q2 : ratio * (DT)q2;
    }
    EpiLevel<DT> r;
    // mass_integrate terms: (x * delp) / g, NaN-skipping sum from +0.0
    r.h = nan0((q1n - (DT)q1) * dp / g);
    r.m = nan0((q2n - (DT)q2) * dp / g);
    // compute_diagnostics reads the tendency dict: zeros for a tendency the model lacks
    r.nm = nan0(q2n * dp / g);
    r.ch = nan0(q1n * dp / g);
    if (a.dq1_out) {
        a.dq1_out[i] = q1n;
        a.dq2_out[i] = q2n;
    }
    if (a.active) a.active[i] = ((DT)q2 != q2n) ? 1 : 0;
    // fillna_tendency + add_tendency
    // (only the tendencies the model predicts are applied, loop.py:202-219)
    r.nan1 = q1n != q1n;
    r.nan2 = q2n != q2n;
    if (a.temp_out) a.temp_out[i] = a.has_dq1 ? t + (r.nan1 ? (DT)0 : q1n) * dtd : t;
    if (a.sphum_out) a.sphum_out[i] = a.has_dq2 ? sp + (r.nan2 ? (DT)0 : q2n) * dtd : sp;
    return r;
}

// the column diagnostics from the four sums and the filled-level counts
template <typename DT>
__device__ __forceinline__ void epi_column_out(const EpilogueArgs<DT>& a, int64_t c, int s, DT sum, int n)
{
    const DT cv = (DT)(kCp - kRdgas);
    const DT ch = a.hydrostatic ? (DT)kCp : cv;
    DT* o = a.col + c;
    switch (s) {
    case 0:
        o[0 * a.col_ld] = ch * sum;                    // column_integrated_dQ1_change_non_neg_sphum_constraint
        o[4 * a.col_ld] = (DT)((double)n / a.nz);      // dQ1_filled_frac
        break;
    case 1:
        o[1 * a.col_ld] = sum;                         // column_integrated_dQ2_change_non_neg_sphum_constraint
        o[5 * a.col_ld] = (DT)((double)n / a.nz);      // dQ2_filled_frac
        break;
    case 2:
        o[2 * a.col_ld] = sum;                         // net_moistening_due_to_<label>
        if (a.precip) {
            const DT total = a.precip[c] + ((-sum) * (DT)a.dt) * (DT)(1.0 / 1000);
            o[6 * a.col_ld] = total >= (DT)0 ? total : (DT)0;  // total_precipitation
        }
        break;
    default:
        o[3 * a.col_ld] = ch * sum;                    // column_heating_due_to_<label>
    }
}

// the kernel arguments of one epilogue call (the C ABI's fv3_epilogue_io and flags)
template <typename DT>
inline EpilogueArgs<DT> make_args(const fv3_epilogue_io& io, fv3_layout lay, int64_t ncol, int nz, double dt,
                                  int mse_conserving, int hydrostatic, int flags)
{
    EpilogueArgs<DT> a;
    a.dq1 = io.dq1;
    a.dq2 = io.dq2;
    a.sphum = (const DT*)io.sphum;
    a.delp = (const DT*)io.delp;
    a.temp = (const DT*)io.temperature;
    a.precip = (const DT*)io.physics_precip;
    a.dq1_out = (DT*)io.dq1_out;
    a.dq2_out = (DT*)io.dq2_out;
    a.active = io.limiter_active;
    a.temp_out = (DT*)io.temperature_out;
    a.sphum_out = (DT*)io.sphum_out;
    a.col = (DT*)io.column;
    a.lay = lay;
    a.ncol = ncol;
    a.col_ld = io.column_ld > 0 ? io.column_ld : ncol;
    a.nz = nz;
    a.mse = mse_conserving != 0;
    a.hydrostatic = hydrostatic != 0;
    a.has_dq1 = (flags & FV3_EPI_HAS_DQ1) != 0;
    a.has_dq2 = (flags & FV3_EPI_HAS_DQ2) != 0;
    a.dt = dt;
    return a;
}

}  // namespace epi
}  // namespace fv3
