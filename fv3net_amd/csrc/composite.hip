// fv3net_amd — the arithmetic of the composite predictors and of the online
// transformer Adapter around the build's predictor, on gfx950.
//
//   member_reduce   EnsembleModel.predict (external/fv3fit/fv3fit/_shared/models.py:253-260):
//                   xr.concat(outputs, "member").mean / .median(dim="member"), i.e. numpy's
//                   nanmean / nanmedian over the leading member axis (xarray 0.19 skips NaN
//                   for floats; bottleneck is not pinned, constraints.txt)
//   scale_levels    TaperedModel.predict (:95-100) -> TaperConfig.apply
//                   (_shared/config.py:21-29): float64 scale factors along taper_dim times the
//                   prediction (vcm.vertical_tapering_scale_factors, vcm/calc/calc.py:45-49)
//   adapter_apply   runtime/transformers/fv3fit.py:66-83 Adapter.predict: tendencies summed
//                   over the model outputs mapped to one state variable, the MSE-conserving
//                   humidity limiter (steppers/machine_learning.py:77-99) and
//                   state + tendency * timestep
//
// All three are elementwise over contiguous arrays (member_reduce, adapter_apply) or over
// [level][column] views (scale_levels): one thread per element, grid-stride, coalesced.
// HBM-bound; the arithmetic replays numpy's dtype flow and order, so results are
// bit-identical to the numpy restatements in oracle/composite.py.
#include "common.h"

namespace fv3 {
namespace {

constexpr double kRdgas = 287.05;  // vcm/calc/thermo/constants.py
constexpr double kCp = 1004.0;
constexpr double kLv = 2.5e6;      // latent_heat_vaporization(273.15 K)

constexpr int kMaxMembers = 32;

template <typename T>
struct MemberArgs {
    const T* m[kMaxMembers];
    int nm, op;
    int64_t n;
    T* out;
};

template <typename T>
__device__ __forceinline__ bool is_nan(T x) { return x != x; }

template <typename T>
__global__ __launch_bounds__(256) void member_reduce_kernel(MemberArgs<T> a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        if (a.op == FV3_REDUCE_MEAN) {
            // np.nanmean: NaN -> 0, add.reduce along the member axis in member order from
            // the identity +0.0 (so an all-(-0.0) column sums to +0.0), divided by the
            // non-NaN count (a correctly rounded division; 0 / 0 = NaN when every member
            // is NaN)
            T s = T(0);
            int cnt = 0;
            for (int j = 0; j < a.nm; ++j) {
                const T v = a.m[j][i];
                cnt += !is_nan(v);
                s = s + (is_nan(v) ? T(0) : v);
            }
            a.out[i] = s / (T)cnt;
        } else {
            // np.nanmedian (< 600 members: numpy.ma.median of the NaN-masked values):
            // sort the unmasked values, low = v[(c - 1) / 2], high = v[c / 2], then
            // ma.sum([low, high]) / 2 in the array's dtype: the sum runs from the identity
            // +0.0 (also for odd counts, where low == high); NaN when every member is NaN
            T v[kMaxMembers];
            int c = 0;
            for (int j = 0; j < a.nm; ++j) {
                const T x = a.m[j][i];
                if (is_nan(x)) continue;
                int p = c++;
                while (p > 0 && v[p - 1] > x) {
                    v[p] = v[p - 1];
                    --p;
                }
                v[p] = x;
            }
            if (c == 0) {
                a.out[i] = (T)NAN;
            } else {
                const int h = c / 2, l = (c % 2) ? h : h - 1;
                a.out[i] = ((T(0) + v[l]) + v[h]) / (T)2;
            }
        }
    }
}

template <typename T>
struct ScaleArgs {
    const T* x;
    fv3_layout lay;
    const double* s;  // [nz] float64 factors
    double* out;      // [nz][ncol] contiguous
    int64_t ncol;
    int nz;
};

template <typename T>
__global__ __launch_bounds__(256) void scale_levels_kernel(ScaleArgs<T> a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const int64_t off = col_offset(a.lay, c);
    for (int k = 0; k < a.nz; ++k)  // scaling * data: float64 DataArray times the prediction
        a.out[(int64_t)k * a.ncol + c] = a.s[k] * (double)a.x[off + (int64_t)k * a.lay.ld];
}

struct AdapterArgs {
    fv3_adapter_target t[FV3_ADAPTER_MAX_TARGETS];
    int nt, limit, q_index, t_index, state_f64;
    int64_t n;
    double dt;
};

// numpy's dtype flow in double arithmetic: a float32 intermediate is the double result
// rounded to float (exact for + - * / of float32 operands: 53 >= 2 * 24 + 2 bits, so the
// double rounding is innocuous), a Python-float constant takes the array operand's dtype
// (NumPy weak scalars)
__device__ __forceinline__ double as_dtype(double x, bool f64) { return f64 ? x : (double)(float)x; }

__device__ __forceinline__ double load_as(const void* p, bool f64, int64_t i)
{
    return f64 ? static_cast<const double*>(p)[i] : (double)static_cast<const float*>(p)[i];
}

// sum([prediction[item] for item in v]): Python's sum starts from the integer 0, so the
// first term fixes the dtype (0 + -0.0 = +0.0) and the sum widens at the first float64
// term (xarray aligns, numpy promotes pairwise in order)
__device__ __forceinline__ double tendency_sum(const fv3_adapter_target& t, int64_t i, bool& wide)
{
    wide = t.pred_f64 & 1u;
    double s = 0.0 + load_as(t.preds[0], wide, i);
    for (int p = 1; p < t.n_preds; ++p) {
        const bool w = (t.pred_f64 >> p) & 1u;
        wide = wide || w;
        s = as_dtype(s + load_as(t.preds[p], w, i), wide);
    }
    return s;
}

__global__ __launch_bounds__(256) void adapter_apply_kernel(AdapterArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const double cv = kCp - kRdgas, lv = kLv, dt = a.dt;
    const bool sw = a.state_f64 != 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        double q2 = 0.0, q2n = 0.0;
        bool wq = false;
        if (a.limit) {
            // update_moisture_tendency_to_ensure_non_negative_humidity (machine_learning.py:77-80):
            // xr.where(sphum + q2 * dt >= 0, q2, -sphum / dt), dtype promote(q2, sphum)
            const fv3_adapter_target& tq = a.t[a.q_index];
            q2 = tendency_sum(tq, i, wq);
            const double sp = load_as(tq.state, sw, i);
            const double step = as_dtype(q2 * as_dtype(dt, wq), wq);
            q2n = (as_dtype(sp + step, wq || sw) >= 0.0) ? q2 : as_dtype((-sp) / as_dtype(dt, sw), sw);
        }
        for (int g = 0; g < a.nt; ++g) {
            const fv3_adapter_target& t = a.t[g];
            const double x = load_as(t.state, sw, i);
            double tend;
            bool wt;
            if (a.limit && g == a.q_index) {
                tend = q2n, wt = wq || sw;
            } else if (a.limit && g == a.t_index) {
                // update_temperature_tendency_to_conserve_mse (:83-88): vcm
                // moist_static_energy_tendency (cv * q1 + lv * q2) and temperature_tendency
                // ((mse - lv * q2_new) / cv)
                bool w1;
                const double q1 = tendency_sum(t, i, w1);
                const bool wm = w1 || wq, wn = wq || sw;
                const double mse = as_dtype(as_dtype(as_dtype(cv, w1) * q1, w1) + as_dtype(as_dtype(lv, wq) * q2, wq), wm);
                const double lq = as_dtype(as_dtype(lv, wn) * q2n, wn);
                wt = wm || wn;
                tend = as_dtype(as_dtype(mse - lq, wt) / as_dtype(cv, wt), wt);
            } else {
                tend = tendency_sum(t, i, wt);
            }
            // inputs[name] + tendency * timestep
            const bool wo = wt || sw;
            const double y = as_dtype(x + as_dtype(tend * as_dtype(dt, wt), wt), wo);
            if (wo)
                static_cast<double*>(t.out)[i] = y;
            else
                static_cast<float*>(t.out)[i] = (float)y;
        }
    }
}

inline unsigned elementwise_grid(int64_t n)
{
    const int64_t g = (n + 255) / 256;
    return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_member_reduce(const void* const* members, int n_members, int64_t n, int dtype_f64, int op,
                                 void* out, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(n_members >= 1 && n_members <= kMaxMembers, "member_reduce: 1..%d members, got %d", kMaxMembers,
                n_members);
    FV3_REQUIRE(op == FV3_REDUCE_MEAN || op == FV3_REDUCE_MEDIAN, "member_reduce: unknown reduction %d", op);
    FV3_REQUIRE(n >= 0, "member_reduce: negative size");
    if (n == 0) return FV3_OK;
    FV3_REQUIRE(members && out, "member_reduce: NULL array");
    for (int j = 0; j < n_members; ++j) FV3_REQUIRE(members[j], "member_reduce: member %d is NULL", j);
    const unsigned grid = elementwise_grid(n);
    if (dtype_f64) {
        MemberArgs<double> a{};
        for (int j = 0; j < n_members; ++j) a.m[j] = static_cast<const double*>(members[j]);
        a.nm = n_members, a.op = op, a.n = n, a.out = static_cast<double*>(out);
        hipLaunchKernelGGL(member_reduce_kernel<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    } else {
        MemberArgs<float> a{};
        for (int j = 0; j < n_members; ++j) a.m[j] = static_cast<const float*>(members[j]);
        a.nm = n_members, a.op = op, a.n = n, a.out = static_cast<float*>(out);
        hipLaunchKernelGGL(member_reduce_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_scale_levels(const void* x, int x_f64, fv3_layout lay, const double* scale, int64_t ncol, int nz,
                                double* out, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ncol >= 0 && nz >= 1, "scale_levels: bad sizes ncol=%lld nz=%d", (long long)ncol, nz);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(x && scale && out, "scale_levels: NULL array");
    FV3_REQUIRE(layout_ok(lay, ncol), "scale_levels: bad layout");
    const unsigned grid = (unsigned)((ncol + 255) / 256);
    if (x_f64) {
        ScaleArgs<double> a{static_cast<const double*>(x), lay, scale, out, ncol, nz};
        hipLaunchKernelGGL(scale_levels_kernel<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    } else {
        ScaleArgs<float> a{static_cast<const float*>(x), lay, scale, out, ncol, nz};
        hipLaunchKernelGGL(scale_levels_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_adapter_apply(const fv3_adapter_target* targets, int n_targets, int64_t n, int state_f64,
                                 double dt, int limit, int sphum_target, int temp_target, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(targets && n_targets >= 1 && n_targets <= FV3_ADAPTER_MAX_TARGETS,
                "adapter_apply: 1..%d targets, got %d", FV3_ADAPTER_MAX_TARGETS, n_targets);
    FV3_REQUIRE(n >= 0, "adapter_apply: negative size");
    if (limit) {
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, sphum_target >= 0 && sphum_target < n_targets,
                         "Cannot limit specific humidity tendencies if specific humidity updates not being "
                         "predicted.");
        FV3_REQUIRE(temp_target < n_targets && temp_target != sphum_target, "adapter_apply: bad temperature target");
    }
    auto wide = [&](int g) { return (targets[g].pred_f64 & ((1u << targets[g].n_preds) - 1u)) != 0u; };
    for (int g = 0; g < n_targets; ++g) {
        const fv3_adapter_target& t = targets[g];
        FV3_REQUIRE(t.n_preds >= 1 && t.n_preds <= FV3_ADAPTER_MAX_PREDS, "adapter_apply: target %d has %d "
                    "predictions (1..%d)", g, t.n_preds, FV3_ADAPTER_MAX_PREDS);
        FV3_REQUIRE(t.state && t.out, "adapter_apply: target %d: NULL state or output", g);
        for (int p = 0; p < t.n_preds; ++p) FV3_REQUIRE(t.preds[p], "adapter_apply: target %d: NULL prediction", g);
    }
    for (int g = 0; g < n_targets; ++g) {
        // the output's numpy dtype: state + tendency * dt, the limited tendencies promoted
        // with the humidity state and, for temperature, with the humidity tendency
        bool wt = wide(g);
        if (limit && (g == sphum_target || g == temp_target)) wt = wt || wide(sphum_target) || state_f64;
        const bool wo = wt || state_f64;
        FV3_REQUIRE((targets[g].out_f64 != 0) == wo, "adapter_apply: target %d output must be float%d", g,
                    wo ? 64 : 32);
    }
    if (n == 0) return FV3_OK;
    AdapterArgs a{};
    for (int g = 0; g < n_targets; ++g) a.t[g] = targets[g];
    a.nt = n_targets, a.limit = limit != 0, a.q_index = limit ? sphum_target : -1;
    a.t_index = limit ? temp_target : -1, a.n = n, a.dt = dt, a.state_f64 = state_f64 != 0;
    hipLaunchKernelGGL(adapter_apply_kernel, dim3(elementwise_grid(n)), dim3(256), 0, (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
