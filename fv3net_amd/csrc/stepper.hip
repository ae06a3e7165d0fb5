// fv3net_amd — the ML stepper's epilogue, one pass per column on gfx950.
//
// Everything the prognostic loop does with a (dQ1, dQ2) prediction, fused:
//   humidity limiter, MSE-conserving or legacy
//       workflows/prognostic_c48_run/runtime/steppers/machine_learning.py:67-99, 258-299
//       (vcm moist_static_energy_tendency / temperature_tendency,
//        external/vcm/vcm/calc/thermo/local.py:317-360)
//   limiter diagnostics (column heating / moistening change, limiter_active)
//       machine_learning.py:267-303
//   compute_diagnostics: net moistening, column heating   diagnostics/compute.py:77-106
//       (vcm mass_integrate, vertically_dependent.py:18-22, 255-301)
//   fillna_tendency + filled fraction                       loop.py:103-110
//   add_tendency: T += dQ1 dt, q += dQ2 dt                   loop.py:202-219
//   precipitation_sum                                        diagnostics/compute.py:21-39
// Level-parallel (a thread per (column, level set), the column sums added in level order
// by one thread per (sum, column) from LDS), or one thread per column walking the levels
// in order where the levels are too many for the LDS.
// The arithmetic replays the reference's dtype flow: f32 model tendencies combined
// with Python-float constants stay f32, anything mixed with the state is in the
// state's dtype DT, column sums run over z in order from +0.0 skipping NaN (xarray's
// sum).  Bit-identical to oracle/stepper.py.
// Roofline: HBM-bound: (2*4 + 3*sizeof(DT)) B read + (2 + 2)*sizeof(DT) + 1 B written per
// level (inputs dQ1, dQ2, sphum, delp, T; outputs dQ1, dQ2, T, q, limiter flag).
#include "common.h"

namespace fv3 {
namespace {

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

// One thread per column walking the levels in order: the kernel for levels too many for
// the level-parallel kernel's LDS (FV3_EPILOGUE_PATH=columns forces it).
template <typename DT>
__global__ __launch_bounds__(64) void ml_epilogue_kernel(EpilogueArgs<DT> a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const int64_t off = col_offset(a.lay, c);
    DT s_h = 0, s_m = 0, s_nm = 0, s_ch = 0;
    int n1 = 0, n2 = 0;
    // Levels are fetched in batches of U, the next batch issued before the current one
    // is processed.  The explicit batches also keep the loads ahead of the stores, which
    // the compiler may not reorder itself since temp_out / sphum_out may alias temp /
    // sphum.  The z sums stay in level order.
    constexpr int U = 8;
    float b_q1[2][U], b_q2[2][U];
    DT b_sp[2][U], b_dp[2][U], b_t[2][U];
    const bool want_t = a.temp_out != nullptr;
    auto fetch = [&](int buf, int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + u < a.nz ? k0 + u : a.nz - 1;  // clamped: re-reads the last level
            const int64_t i = off + (int64_t)k * a.lay.ld;
            b_q1[buf][u] = a.dq1[i];
            b_q2[buf][u] = a.dq2[i];
            b_sp[buf][u] = a.sphum[i];
            b_dp[buf][u] = a.delp[i];
            b_t[buf][u] = want_t ? a.temp[i] : (DT)0;
        }
    };
    auto level = [&](int k, float q1, float q2, DT sp, DT dp, DT t) {
        const EpiLevel<DT> r = epi_level(a, off + (int64_t)k * a.lay.ld, q1, q2, sp, dp, t);
        s_h = s_h + r.h;
        s_m = s_m + r.m;
        if (a.has_dq2) s_nm = s_nm + r.nm;
        if (a.has_dq1) s_ch = s_ch + r.ch;
        n1 += r.nan1;
        n2 += r.nan2;
    };
    fetch(0, 0);
    for (int k0 = 0; k0 < a.nz; k0 += 2 * U) {
        if (k0 + U < a.nz) fetch(1, k0 + U);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < a.nz) level(k0 + u, b_q1[0][u], b_q2[0][u], b_sp[0][u], b_dp[0][u], b_t[0][u]);
        if (k0 + U >= a.nz) break;
        if (k0 + 2 * U < a.nz) fetch(0, k0 + 2 * U);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + U + u < a.nz)
                level(k0 + U + u, b_q1[1][u], b_q2[1][u], b_sp[1][u], b_dp[1][u], b_t[1][u]);
    }
    if (a.col) {
        epi_column_out(a, c, 0, s_h, n1);
        epi_column_out(a, c, 1, s_m, n2);
        epi_column_out(a, c, 2, s_nm, 0);
        epi_column_out(a, c, 3, s_ch, 0);
    }
}

// Level-parallel: a block of kEpiCols columns x kEpiLanes level lanes.  Each thread runs
// the levels lane, lane + kEpiLanes, ... of its column (every level's work is
// independent) and leaves the four sum terms in LDS; then one thread per (sum, column)
// adds its column's terms in level order from +0.0, the same additions as the column
// kernel.  One rank's 6,912 columns are 108 waves in the column kernel (one per CU, a
// serial 79-level chain each: 44 us); here 1,728.
// kEpiU levels per thread per pass: 5 covers 79 levels in one pass of loads (3 took
// two dependent rounds of them; one rank's 6,912 columns, tools/ab.py)
constexpr int kEpiCols = 16, kEpiLanes = 16;
template <typename DT, int kEpiU>
__global__ __launch_bounds__(kEpiCols * kEpiLanes) void ml_epilogue_levels_kernel(EpilogueArgs<DT> a)
{
    extern __shared__ __align__(16) unsigned char epi_smem[];
    DT* terms = reinterpret_cast<DT*>(epi_smem);                    // [4][nz][kEpiCols]
    int* cnt = reinterpret_cast<int*>(terms + 4 * a.nz * kEpiCols);  // [2][kEpiCols]
    const int cl = threadIdx.x % kEpiCols, lane = threadIdx.x / kEpiCols;
    const int64_t c = (int64_t)blockIdx.x * kEpiCols + cl;
    if (threadIdx.x < 2 * kEpiCols) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (c < a.ncol) {
        const int64_t off = col_offset(a.lay, c);
        const bool want_t = a.temp_out != nullptr;
        int n1 = 0, n2 = 0;
        // kEpiU levels' loads issued before any of their stores (temp_out / sphum_out may
        // alias temp / sphum, so the compiler keeps loads behind earlier stores)
        for (int k0 = lane; k0 < a.nz; k0 += kEpiU * kEpiLanes) {
            float q1[kEpiU], q2[kEpiU];
            DT sp[kEpiU], dp[kEpiU], t[kEpiU];
#pragma unroll
            for (int u = 0; u < kEpiU; ++u) {
                int k = k0 + u * kEpiLanes;
                k = k < a.nz ? k : a.nz - 1;  // clamped: re-reads a level, never used
                const int64_t i = off + (int64_t)k * a.lay.ld;
                q1[u] = a.dq1[i];
                q2[u] = a.dq2[i];
                sp[u] = a.sphum[i];
                dp[u] = a.delp[i];
                t[u] = want_t ? a.temp[i] : (DT)0;
            }
#pragma unroll
            for (int u = 0; u < kEpiU; ++u) {
                const int k = k0 + u * kEpiLanes;
                if (k < a.nz) {
                    const EpiLevel<DT> r = epi_level(a, off + (int64_t)k * a.lay.ld, q1[u], q2[u], sp[u], dp[u], t[u]);
                    terms[(0 * a.nz + k) * kEpiCols + cl] = r.h;
                    terms[(1 * a.nz + k) * kEpiCols + cl] = r.m;
                    terms[(2 * a.nz + k) * kEpiCols + cl] = r.nm;
                    terms[(3 * a.nz + k) * kEpiCols + cl] = r.ch;
                    n1 += r.nan1;
                    n2 += r.nan2;
                }
            }
        }
        if (n1) atomicAdd(&cnt[cl], n1);
        if (n2) atomicAdd(&cnt[kEpiCols + cl], n2);
    }
    __syncthreads();
    if (a.col && threadIdx.x < 4 * kEpiCols && c < a.ncol) {
        const int s = lane;  // 0..3: which sum
        const bool on = s < 2 || (s == 2 ? a.has_dq2 : a.has_dq1);
        DT sum = 0;
        if (on) {
            const DT* tp = terms + (int64_t)s * a.nz * kEpiCols + cl;
            for (int k = 0; k < a.nz; ++k) sum = sum + tp[k * kEpiCols];
        }
        epi_column_out(a, c, s, sum, s < 2 ? cnt[s * kEpiCols + cl] : 0);
    }
}

constexpr size_t kEpiMaxSmem = 48 << 10;  // f64 state: nz <= 95
constexpr int64_t kEpiLevelsMaxCols = 32768;
size_t epi_levels_smem(int nz, size_t dt_size) { return 4 * (size_t)nz * kEpiCols * dt_size + 2 * kEpiCols * sizeof(int); }

template <typename DT>
int epilogue_impl(const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz, double dt, int mse_conserving,
                  int hydrostatic, int flags, void* stream)
{
    clear_error();
    FV3_REQUIRE(io, "ml_epilogue: NULL io");
    FV3_REQUIRE(ncol >= 0 && nz >= 1, "ml_epilogue: bad sizes ncol=%lld nz=%d", (long long)ncol, nz);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(io->dq1 && io->dq2 && io->sphum && io->delp && io->temperature,
                "ml_epilogue: dQ1, dQ2, specific humidity, delp and air temperature are required");
    FV3_REQUIRE(layout_ok(lay, ncol), "ml_epilogue: bad layout");
    FV3_REQUIRE(!io->dq1_out == !io->dq2_out, "ml_epilogue: dq1_out and dq2_out go together");
    EpilogueArgs<DT> a;
    a.dq1 = io->dq1;
    a.dq2 = io->dq2;
    a.sphum = (const DT*)io->sphum;
    a.delp = (const DT*)io->delp;
    a.temp = (const DT*)io->temperature;
    a.precip = (const DT*)io->physics_precip;
    a.dq1_out = (DT*)io->dq1_out;
    a.dq2_out = (DT*)io->dq2_out;
    a.active = io->limiter_active;
    a.temp_out = (DT*)io->temperature_out;
    a.sphum_out = (DT*)io->sphum_out;
    a.col = (DT*)io->column;
    a.lay = lay;
    a.ncol = ncol;
    a.col_ld = io->column_ld > 0 ? io->column_ld : ncol;
    a.nz = nz;
    a.mse = mse_conserving != 0;
    a.hydrostatic = hydrostatic != 0;
    a.has_dq1 = (flags & FV3_EPI_HAS_DQ1) != 0;
    a.has_dq2 = (flags & FV3_EPI_HAS_DQ2) != 0;
    a.dt = dt;
    // level-parallel on small grids (one rank's share of C96 over 8, 6,912 columns: step
    // 0.092 -> 0.061 ms), the column kernel on large ones (full C96, 55,296 columns:
    // 0.2065 vs 0.2080 ms) (tools/ab.py, profiles/r04j_epi_ab.log);
    // FV3_EPILOGUE_PATH=levels|columns forces one
    const size_t smem = epi_levels_smem(nz, sizeof(DT));
    const char* path = fv3::variant_env("FV3_EPILOGUE_PATH");
    bool levels = ncol <= kEpiLevelsMaxCols;
    if (path && path[0] == 'c') levels = false;
    if (path && path[0] == 'l') levels = true;
    if (levels && smem <= kEpiMaxSmem) {
        const int64_t grid = (ncol + kEpiCols - 1) / kEpiCols;
        auto kfn = ml_epilogue_levels_kernel<DT, 5>;
#if FV3_VARIANT_KERNELS
        const char* u = fv3::variant_env("FV3_EPI_U");  // A/B: 3 (round 4) | 5
        if (u && u[0] == '3') kfn = ml_epilogue_levels_kernel<DT, 3>;
#endif
        hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(kEpiCols * kEpiLanes), smem, (hipStream_t)stream, a);
    } else {
        const int block = 64;  // one wave: C96's 864 waves spread over every CU (256-thread blocks left 40 idle)
        const int64_t grid = (ncol + block - 1) / block;
        hipLaunchKernelGGL(ml_epilogue_kernel<DT>, dim3((unsigned)grid), dim3(block), 0, (hipStream_t)stream, a);
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

// The prediction's other tendencies (runtime/names.py:31-50), one pass per column:
//   TEND_WIND (dQu, dQv): compute_ml_momentum_diagnostics (diagnostics/compute.py:140-161)
//       column_integrated_dQ{u,v}_stress = mass_integrate(dQ, delp) = sum (dQ delp) / g
//       (float32 * state dtype -> DT), fillna + filled fraction (loop.py:103-123), and the
//       filled tendency cast to float64 as prepare_agrid_wind_tendencies does
//       (loop.py:126-145; the A->D-grid transform after it belongs to the fv3gfs wrapper)
//   TEND_MASS (dQp): net_mass_tendency = mass_integrate(ones_like(dQp), dQp)
//       (compute.py:107-115) = sum (1 * dQp) / g in float32 (all-float32 operands),
//       fillna + filled fraction, add_tendency delp + fill(dQp) dt (loop.py:202-219)
// Column sums over z in order from +0.0 skipping NaN; HBM-bound.
template <typename DT>
struct TendArgs {
    const float* t;
    const DT* delp;   // TEND_WIND: the integral's weights; TEND_MASS: the state updated
    double* filled;   // TEND_WIND: [z][col] float64 filled tendency, or NULL
    DT* state_out;    // TEND_MASS: [z][col] delp + fill(dQp) dt, or NULL (may alias delp)
    void* integral;   // [col]: DT (TEND_WIND) or float (TEND_MASS), or NULL
    DT* frac;         // [col] filled fraction, or NULL
    fv3_layout lay;
    int64_t ncol;
    int nz, mode;
    double dt;
};

template <typename DT>
__global__ __launch_bounds__(64) void tendency_columns_kernel(TendArgs<DT> a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const int64_t off = col_offset(a.lay, c);
    const DT g = (DT)kGravity;
    const float gf = (float)kGravity, dtf = (float)a.dt;
    DT sd = 0;
    float sf = 0.0f;
    int n = 0;
    for (int k = 0; k < a.nz; ++k) {
        const int64_t i = off + (int64_t)k * a.lay.ld;
        const float t = a.t[i];
        const DT dp = a.delp[i];
        const bool isnan_ = t != t;
        n += isnan_;
        const float tf = isnan_ ? 0.0f : t;
        if (a.mode == FV3_TEND_WIND) {
            sd = sd + nan0((DT)t * dp / g);
            if (a.filled) a.filled[i] = (double)tf;
        } else {
            sf = sf + nan0(1.0f * t / gf);
            if (a.state_out) a.state_out[i] = dp + (DT)(tf * dtf);
        }
    }
    if (a.integral) {
        if (a.mode == FV3_TEND_WIND) static_cast<DT*>(a.integral)[c] = sd;
        else static_cast<float*>(a.integral)[c] = sf;
    }
    if (a.frac) a.frac[c] = (DT)((double)n / a.nz);
}

template <typename DT>
int tendency_impl(const float* t, const void* delp, double* filled, void* state_out, void* integral, void* frac,
                  fv3_layout lay, int64_t ncol, int nz, int mode, double dt, void* stream)
{
    clear_error();
    FV3_REQUIRE(ncol >= 0 && nz >= 1, "tendency_columns: bad sizes ncol=%lld nz=%d", (long long)ncol, nz);
    FV3_REQUIRE(mode == FV3_TEND_WIND || mode == FV3_TEND_MASS, "tendency_columns: unknown mode %d", mode);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(t && delp, "tendency_columns: the tendency and delp are required");
    FV3_REQUIRE(layout_ok(lay, ncol), "tendency_columns: bad layout");
    TendArgs<DT> a{t, (const DT*)delp, filled, (DT*)state_out, integral, (DT*)frac, lay, ncol, nz, mode, dt};
    const int64_t grid = (ncol + 63) / 64;
    hipLaunchKernelGGL(tendency_columns_kernel<DT>, dim3((unsigned)grid), dim3(64), 0, (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_ml_epilogue(const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz, int state_f64,
                               double dt, int mse_conserving, int hydrostatic, void* stream)
{
    return fv3_ml_epilogue_ex(io, lay, ncol, nz, state_f64, dt, mse_conserving, hydrostatic,
                              FV3_EPI_HAS_DQ1 | FV3_EPI_HAS_DQ2, stream);
}

extern "C" int fv3_ml_epilogue_ex(const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz, int state_f64,
                                  double dt, int mse_conserving, int hydrostatic, int flags, void* stream)
{
    return state_f64 ? fv3::epilogue_impl<double>(io, lay, ncol, nz, dt, mse_conserving, hydrostatic, flags, stream)
                     : fv3::epilogue_impl<float>(io, lay, ncol, nz, dt, mse_conserving, hydrostatic, flags, stream);
}

extern "C" int fv3_tendency_columns(const float* tendency, const void* delp, double* filled_out, void* state_out,
                                    void* integral, void* filled_frac, fv3_layout lay, int64_t ncol, int nz,
                                    int state_f64, int mode, double dt, void* stream)
{
    return state_f64 ? fv3::tendency_impl<double>(tendency, delp, filled_out, state_out, integral, filled_frac, lay,
                                                  ncol, nz, mode, dt, stream)
                     : fv3::tendency_impl<float>(tendency, delp, filled_out, state_out, integral, filled_frac, lay,
                                                 ncol, nz, mode, dt, stream);
}
