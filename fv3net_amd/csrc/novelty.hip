// fv3net_amd — the out-of-sample composite's column work on gfx950: the min-max novelty
// score of every column and the taper applied to the base model's outputs.
//
// Replaces
//   MinMaxNoveltyDetector.predict            external/fv3fit/fv3fit/sklearn/_min_max_novelty_detector.py:86-115
//     pack (clip, variables' features in order)        _shared/packer.py:106-127
//     MinMaxScaler.transform: X *= scale_; X += min_   (in X's dtype, in place)
//     score = max(max_f X - 1, 0) + max(-1 * min_f X, 0)
//   taper_mask / taper_ramp / taper_decay   external/fv3fit/fv3fit/_shared/taper_function.py:6-35
//   OutOfSampleModel.predict's  base_predict[v] * taper_values   _shared/models.py:386-400
// One thread per column; the features are read through the fv3_layout of each variable
// (the stacked sample order is a zero-copy view).  The arithmetic follows numpy's dtype
// flow: the scaler's in-place products round to X's dtype after each operation, np.max /
// np.min / np.maximum / np.clip propagate NaN, the mask taper is int64 and a float32
// output times it is float64.  HBM-bound (features read once, one score written).
#include <cmath>

#include "common.h"

namespace fv3 {
namespace {

template <typename T>
__device__ __forceinline__ T load_as(const void* p, int f64, int64_t i)
{
    return f64 ? (T) static_cast<const double*>(p)[i] : (T) static_cast<const float*>(p)[i];
}

// numpy's NaN-propagating max / min / maximum
template <typename T>
__device__ __forceinline__ T np_max(T a, T b) { return (a != a || b != b) ? (a != a ? a : b) : (a > b ? a : b); }
template <typename T>
__device__ __forceinline__ T np_min(T a, T b) { return (a != a || b != b) ? (a != a ? a : b) : (a < b ? a : b); }

struct NovArgs {
    fv3_nov_var vars[FV3_NOV_MAX_VARS];
    int n_vars;
    const void* scale;  // [n_features] MinMaxScaler.scale_
    const void* mn;     // [n_features] MinMaxScaler.min_
    int scale_f64;
    int64_t ncol;
    void* score;        // [ncol] in X's dtype T
};

// T: X's dtype (the packed features' promoted dtype); S: the scaler's; the in-place
// ufuncs compute in promote(T, S) and round to T
template <typename T, typename S>
__global__ __launch_bounds__(256) void minmax_scores_kernel(NovArgs a)
{
    using P = typename std::conditional<(sizeof(T) >= sizeof(S)), T, S>::type;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const S* scale = static_cast<const S*>(a.scale);
    const S* mn = static_cast<const S*>(a.mn);
    T mx_v = T(0), mn_v = T(0);
    bool first = true;
    int f = 0;
    for (int v = 0; v < a.n_vars; ++v) {
        const fv3_nov_var& d = a.vars[v];
        const int64_t off = col_offset(d.layout, c);
        for (int k = 0; k < d.nfeat; ++k, ++f) {
            const T x = load_as<T>(d.data, d.data_f64, off + (int64_t)(d.z0 + k) * d.layout.ld);
            T s = (T)((P)x * (P)scale[f]);
            s = (T)((P)s + (P)mn[f]);
            if (first) {
                mx_v = s;
                mn_v = s;
                first = false;
            } else {
                mx_v = np_max(mx_v, s);
                mn_v = np_min(mn_v, s);
            }
        }
    }
    const T larger = np_max((T)(mx_v - T(1)), T(0));
    const T smaller = np_max((T)(T(-1) * mn_v), T(0));
    static_cast<T*>(a.score)[c] = larger + smaller;
}

struct TaperArgs {
    const void* score;
    int score_f64;
    int64_t ncol;
    int mode;
    double p0, p1;   // mask: cutoff; ramp: ramp_min, ramp_max; decay: threshold, rate
    void* taper;     // [ncol]: int64 (mask) or the score's dtype, or NULL
    fv3_taper_field fields[FV3_NOV_MAX_FIELDS];
    int n_fields;
};

// the taper value of one column in its numpy dtype TV (int64 for the mask)
template <typename ST>
__device__ __forceinline__ double taper_value(const TaperArgs& a, ST s)
{
    if (a.mode == FV3_TAPER_MASK) return s > (ST)a.p0 ? 0.0 : 1.0;  // xr.where(score > cutoff, 0, 1)
    if (a.mode == FV3_TAPER_RAMP) {
        // (ramp_max - score) / (ramp_max - ramp_min), then np.clip(., 0, 1): the Python
        // floats enter as the score's dtype, their difference taken in double first
        const ST u = ((ST)a.p1 - s) / (ST)(a.p1 - a.p0);
        return (double)np_min(np_max(u, (ST)0), (ST)1);
    }
    // np.minimum(rate ** (score - threshold), 1)
    const ST e = s - (ST)a.p0;
    const ST pw = sizeof(ST) == 8 ? (ST)pow((double)a.p1, (double)e) : (ST)powf((float)a.p1, (float)e);
    return (double)np_min(pw, (ST)1);
}

template <typename ST>
__global__ __launch_bounds__(64) void taper_columns_kernel(TaperArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const ST s = static_cast<const ST*>(a.score)[c];
    const double t = taper_value(a, s);  // exact in double: 0 / 1, or a value of ST
    const bool mask = a.mode == FV3_TAPER_MASK;
    if (a.taper) {
        if (mask) static_cast<int64_t*>(a.taper)[c] = (int64_t)t;
        else static_cast<ST*>(a.taper)[c] = (ST)t;
    }
    // base_predict[v] * taper_values: promote(output dtype, taper dtype) (int64 -> f64)
    for (int i = 0; i < a.n_fields; ++i) {
        const fv3_taper_field& fd = a.fields[i];
        const int64_t io = col_offset(fd.in_layout, c), oo = col_offset(fd.out_layout, c);
        const bool out64 = fd.in_f64 || mask || sizeof(ST) == 8;
        for (int k = 0; k < fd.nz; ++k) {
            const int64_t ii = io + (int64_t)k * fd.in_layout.ld, oi = oo + (int64_t)k * fd.out_layout.ld;
            if (out64) {
                const double x = fd.in_f64 ? static_cast<const double*>(fd.in)[ii] : (double)static_cast<const float*>(fd.in)[ii];
                static_cast<double*>(fd.out)[oi] = x * t;
            } else {
                static_cast<float*>(fd.out)[oi] = static_cast<const float*>(fd.in)[ii] * (float)t;
            }
        }
    }
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_minmax_scores(const fv3_nov_var* vars, int n_vars, const void* scale, const void* min,
                                 int scale_f64, int x_f64, int64_t ncol, void* score, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(n_vars >= 1 && n_vars <= FV3_NOV_MAX_VARS, "minmax_scores: 1..%d variables (got %d)",
                FV3_NOV_MAX_VARS, n_vars);
    FV3_REQUIRE(vars && scale && min && (score || ncol == 0), "minmax_scores: NULL array");
    FV3_REQUIRE(ncol >= 0, "minmax_scores: ncol must be >= 0");
    if (ncol == 0) return FV3_OK;
    NovArgs a{};
    int nf = 0;
    for (int v = 0; v < n_vars; ++v) {
        FV3_REQUIRE(vars[v].data && vars[v].nfeat >= 1 && vars[v].z0 >= 0 && layout_ok(vars[v].layout, ncol),
                    "minmax_scores: bad variable %d", v);
        a.vars[v] = vars[v];
        nf += vars[v].nfeat;
    }
    FV3_REQUIRE(nf >= 1, "minmax_scores: no features");
    a.n_vars = n_vars;
    a.scale = scale;
    a.mn = min;
    a.scale_f64 = scale_f64;
    a.ncol = ncol;
    a.score = score;
    const dim3 grid((unsigned)((ncol + 255) / 256)), block(256);
    hipStream_t s = (hipStream_t)stream;
    if (x_f64 && scale_f64) hipLaunchKernelGGL((minmax_scores_kernel<double, double>), grid, block, 0, s, a);
    else if (x_f64) hipLaunchKernelGGL((minmax_scores_kernel<double, float>), grid, block, 0, s, a);
    else if (scale_f64) hipLaunchKernelGGL((minmax_scores_kernel<float, double>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((minmax_scores_kernel<float, float>), grid, block, 0, s, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_taper_columns(const void* score, int score_f64, int64_t ncol, int mode, double p0, double p1,
                                 void* taper_out, const fv3_taper_field* fields, int n_fields, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(mode == FV3_TAPER_MASK || mode == FV3_TAPER_RAMP || mode == FV3_TAPER_DECAY,
                "taper_columns: unknown taper %d", mode);
    FV3_REQUIRE(n_fields >= 0 && n_fields <= FV3_NOV_MAX_FIELDS, "taper_columns: 0..%d fields (got %d)",
                FV3_NOV_MAX_FIELDS, n_fields);
    FV3_REQUIRE(ncol >= 0 && (score || ncol == 0), "taper_columns: bad scores");
    if (ncol == 0) return FV3_OK;
    TaperArgs a{};
    a.score = score;
    a.score_f64 = score_f64;
    a.ncol = ncol;
    a.mode = mode;
    a.p0 = p0;
    a.p1 = p1;
    a.taper = taper_out;
    for (int i = 0; i < n_fields; ++i) {
        FV3_REQUIRE(fields && fields[i].in && fields[i].out && fields[i].nz >= 1 &&
                        layout_ok(fields[i].in_layout, ncol) && layout_ok(fields[i].out_layout, ncol),
                    "taper_columns: bad field %d", i);
        a.fields[i] = fields[i];
    }
    a.n_fields = n_fields;
    const dim3 grid((unsigned)((ncol + 63) / 64)), block(64);
    hipStream_t s = (hipStream_t)stream;
    if (score_f64) hipLaunchKernelGGL(taper_columns_kernel<double>, grid, block, 0, s, a);
    else hipLaunchKernelGGL(taper_columns_kernel<float>, grid, block, 0, s, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
