// fv3net_amd — the microphysics emulator hook's post-processing on gfx950.
//
// What external/emulation does to the emulator's prediction before it goes back to the
// Fortran state, on the hook's [feature, sample] arrays (_emulate/microphysics.py:83-101):
//   fv3_range_mask            RangeMask: np.maximum / np.minimum clamps      masks.py:23-39
//   fv3_time_blend            TimeMask: state * alpha + emulator * (1 - alpha)
//                                                         _emulate/microphysics.py:37-47
//   fv3_classify_one_hot      _get_classify_output: one-hot of the class logits where
//                             they equal their max over the class axis, plus
//                             nontrivial = positive | negative                 zhao_carr.py:214-219
//   fv3_zc_infer_gscond_cloud infer_gscond_cloud_from_conservation          zhao_carr.py:72-76
//   fv3_zc_squash             squash_water_water_conserving (gscond/precpd)  zhao_carr.py:57-69
//   fv3_zc_zero_where         mask_zero_cloud_classifier_precpd's select      zhao_carr.py:240-247
//   fv3_zc_gscond_update      the cloud choice of enforce_conservative_gscond,
//                             mask_where_fortran_cloud_identical / _vanishes_gscond,
//                             mask_zero_cloud_classifier, mask_zero_tend_classifier, then
//                             _update_with_net_condensation (limit + liquid-phase
//                             condensation); or enforce_conservative_phase_dependent
//                             (no limit, latent heat from the ice-water flag)  zhao_carr.py:79-245
//   fv3_zc_ice_water_flag     ice_water_flag (the numba loop: per row of a 2-D array, a
//                             right-to-left recurrence along the last axis)   zhao_carr.py:108-133
//   fv3_zc_precpd_conservative enforce_conservative_precpd with
//                             _strict_conservative_precip_from_TOA_to_surface zhao_carr.py:277-352
//   fv3_zc_precip_simple      conservative_precip_simple                     zhao_carr.py:355-371
// Arithmetic in the arrays' dtype T (float or double) with numpy's semantics: np.maximum /
// np.minimum propagate NaN, np.where selects, Python-float constants take T, sums over the
// feature axis add level by level.  All HBM-bound elementwise or column passes; coalesced
// along the sample axis.
#include <cmath>

#include "common.h"

namespace fv3 {
namespace {

constexpr double kGravity = 9.80665;  // physcons.f, zhao_carr.py:36-39
constexpr double kCp = 1.0046e3;
constexpr double kLv = 2.5e6;
constexpr double kRhoWater = 1000.0;
constexpr double kHfus = 3.3358e5;    // latent_heat_phase_dependent, zhao_carr.py:136-139

// numpy's maximum / minimum: NaN in either operand propagates (the first one wins)
template <typename T>
__device__ __forceinline__ T np_max(T a, T b) { return (a >= b || a != a) ? a : b; }
template <typename T>
__device__ __forceinline__ T np_min(T a, T b) { return (a <= b || a != a) ? a : b; }

__device__ __forceinline__ int64_t gid() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

template <typename T>
__global__ __launch_bounds__(256) void range_mask_kernel(const T* x, T* out, int64_t n, T lo, T hi, int has_lo,
                                                         int has_hi)
{
    const int64_t i = gid();
    if (i >= n) return;
    T v = x[i];
    if (has_lo) v = np_max(v, lo);
    if (has_hi) v = np_min(v, hi);
    out[i] = v;
}

// logits [n_class][inner] -> masks [n_class + 1][inner]: one-hot where logit == max over
// classes (ties: every maximal class), the last mask = masks[pos] | masks[neg]
template <typename T>
__global__ __launch_bounds__(256) void classify_kernel(const T* logits, int n_class, int64_t inner, uint8_t* masks,
                                                       int pos, int neg)
{
    const int64_t i = gid();
    if (i >= inner) return;
    T m = logits[i];
    for (int c = 1; c < n_class; ++c) {  // np.max: NaN propagates
        const T v = logits[(int64_t)c * inner + i];
        m = (m != m) ? m : ((v != v || v > m) ? v : m);
    }
    for (int c = 0; c < n_class; ++c) masks[(int64_t)c * inner + i] = logits[(int64_t)c * inner + i] == m;
    masks[(int64_t)n_class * inner + i] = masks[(int64_t)pos * inner + i] | masks[(int64_t)neg * inner + i];
}

template <typename T>
__global__ __launch_bounds__(256) void infer_cloud_kernel(const T* qc_in, const T* qv_in, const T* qv_gscond,
                                                          T* qc_out, int64_t n)
{
    const int64_t i = gid();
    if (i >= n) return;
    const T humidity_change = qv_gscond[i] - qv_in[i];
    qc_out[i] = qc_in[i] - humidity_change;
}

template <typename T>
__global__ __launch_bounds__(256) void squash_kernel(const T* cloud, const T* humidity, T bound, T* cloud_out,
                                                     T* humidity_out, int64_t n)
{
    const int64_t i = gid();
    if (i >= n) return;
    const T c = cloud[i];
    const T co = (c < bound) ? (T)0 : c;
    humidity_out[i] = humidity[i] + (c - co);
    cloud_out[i] = co;
}

// np.where(class, 0, cloud) (mask_zero_cloud_classifier_precpd, zhao_carr.py:240-247)
template <typename T>
__global__ __launch_bounds__(256) void zero_where_kernel(const uint8_t* klass, const T* cloud, T* out, int64_t n)
{
    const int64_t i = gid();
    if (i >= n) return;
    out[i] = klass[i] ? (T)0 : cloud[i];
}

template <typename T>
struct GscondArgs {
    const T *qc_in, *qv_in, *t_in, *qc_fortran, *qc_emu;
    const uint8_t* klass;  // the class one-hot the mode reads, or NULL
    const uint8_t* ice;    // ice_water_flag (0/1) for the phase-dependent mode, or NULL
    T *qc_out, *qv_out, *t_out;
    int64_t n;
    int mode;
};

template <typename T>
__global__ __launch_bounds__(256) void gscond_kernel(GscondArgs<T> a)
{
    const int64_t i = gid();
    if (i >= a.n) return;
    const T qc = a.qc_in[i], qv = a.qv_in[i], emu = a.qc_emu[i];
    T cloud, net, lv;
    switch (a.mode) {
        case FV3_ZC_CLOUD_IDENTICAL: cloud = (a.qc_fortran[i] == qc) ? qc : emu; break;
        case FV3_ZC_CLOUD_VANISHES: cloud = (a.qc_fortran[i] < (T)1e-15) ? (T)0 : emu; break;
        case FV3_ZC_CLOUD_CLASS_ZERO: cloud = a.klass[i] ? (T)0 : emu; break;
        case FV3_ZC_CLOUD_CLASS_NOTEND: cloud = a.klass[i] ? qc : emu; break;
        default: cloud = emu; break;  // FV3_ZC_CLOUD_EMULATOR, FV3_ZC_PHASE_DEPENDENT
    }
    net = cloud - qc;
    if (a.mode == FV3_ZC_PHASE_DEPENDENT) {
        lv = (T)kLv + (T)a.ice[i] * (T)kHfus;  // hvap + iw * hfus
    } else {
        // _limit_net_condensation_conserving (zhao_carr.py:90-101)
        const T condensation = (net > (T)0) ? net : (T)0;
        const T evaporation = (net < (T)0) ? net : (T)0;
        net = np_max(evaporation, -qc) + np_min(condensation, qv);
        lv = (T)kLv;
    }
    // apply_condensation (zhao_carr.py:149-161)
    a.qc_out[i] = qc + net;
    a.qv_out[i] = qv - net;
    a.t_out[i] = a.t_in[i] + lv * net / (T)kCp;
}

// ice_water_flag: rows of a (nrows, z) array, each a recurrence from its last element
// to its first.  Element k: t < -15 -> 1; t > 0 -> 0; otherwise iw[k+1] if k < z-1 and
// cloud[k] > 1e-20 (a "pass"), else 0.  So iw[k] is decided by the nearest non-pass
// element at or after k: 1 if it is cold (< -15), else 0.  Three passes: per chunk the
// nearest non-pass (suffix min in LDS) and whether the chunk's first element is decided
// inside the chunk; a per-row walk over the chunks from the right; the final values.
constexpr int kIceChunk = 256;
constexpr int kNone = 0x7fffffff;

template <typename T>
__device__ __forceinline__ int ice_code(const T* tc, const T* cloud, int64_t k, int64_t z, T off)
{
    const T t = tc[k] - off;  // temperature_celsius = T - 273.16
    if (t < (T)-15) return 1;  // cold: 1
    if (t > (T)0) return 0;    // warm: 0
    return (k < z - 1 && (double)cloud[k] > 1e-20) ? 2 : 0;  // pass (inherit) / 0 (numba: f64 compare)
}

// suffix "nearest non-pass index" within this block's chunk; returns it (or kNone)
template <typename T>
__device__ int ice_nearest(const T* tc, const T* cloud, int64_t z, int64_t k0, T off, int* sh, int* code_out)
{
    const int tid = threadIdx.x;
    const int64_t k = k0 + tid;
    const int code = k < z ? ice_code(tc, cloud, k, z, off) : 0;
    *code_out = code;
    sh[tid] = (k < z && code != 2) ? tid : kNone;
    __syncthreads();
    for (int o = 1; o < kIceChunk; o <<= 1) {  // suffix min
        const int v = (tid + o < kIceChunk) ? sh[tid + o] : kNone;
        __syncthreads();
        sh[tid] = min(sh[tid], v);
        __syncthreads();
    }
    return sh[tid];
}

template <typename T>
__global__ __launch_bounds__(kIceChunk) void ice_pass1(const T* tc, const T* cloud, int64_t z, T off,
                                                       uint8_t* chunk_state, int64_t nchunk)
{
    __shared__ int sh[kIceChunk];
    __shared__ int codes[kIceChunk];
    const int64_t row = blockIdx.y, c = blockIdx.x;
    const T* t = tc + row * z;
    const T* cl = cloud + row * z;
    int code;
    const int near = ice_nearest(t, cl, z, c * kIceChunk, off, sh, &code);
    codes[threadIdx.x] = code;
    __syncthreads();
    if (threadIdx.x == 0)  // 0 / 1 decided inside the chunk, 2: inherits from the next chunk
        chunk_state[row * nchunk + c] = (near == kNone) ? 2 : (uint8_t)(codes[near] == 1);
}

__global__ __launch_bounds__(256) void ice_pass2(uint8_t* chunk_state, int64_t nchunk)
{
    // one block per row: the chunk states through LDS in pieces, one thread walks them
    // right to left; chunk_state[c] becomes the value its first element resolves to
    __shared__ uint8_t s[4096];
    uint8_t* st = chunk_state + (int64_t)blockIdx.x * nchunk;
    uint8_t carry = 0;
    for (int64_t hi = nchunk; hi > 0; hi -= 4096) {
        const int64_t lo = hi > 4096 ? hi - 4096 : 0;
        for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) s[j - lo] = st[j];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int64_t j = hi - 1; j >= lo; --j) {
                if (s[j - lo] == 2) s[j - lo] = carry;
                carry = s[j - lo];
            }
        __syncthreads();
        for (int64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) st[j] = s[j - lo];
        __syncthreads();
    }
}

template <typename T>
__global__ __launch_bounds__(kIceChunk) void ice_pass3(const T* tc, const T* cloud, int64_t z, T off,
                                                       const uint8_t* resolved, int64_t nchunk, T* iw)
{
    __shared__ int sh[kIceChunk];
    __shared__ int codes[kIceChunk];
    const int64_t row = blockIdx.y, c = blockIdx.x;
    const T* t = tc + row * z;
    const T* cl = cloud + row * z;
    int code;
    const int near = ice_nearest(t, cl, z, c * kIceChunk, off, sh, &code);
    codes[threadIdx.x] = code;
    __syncthreads();
    const int64_t k = c * kIceChunk + threadIdx.x;
    if (k >= z) return;
    // no decided element left in the chunk: the next chunk's first element's value
    const uint8_t v = (near == kNone) ? resolved[row * nchunk + c + 1] : (uint8_t)(codes[near] == 1);
    iw[row * z + k] = (T)v;
}

// enforce_conservative_precpd: per column (one thread), levels from TOA (index nz-1)
// down; the precipitation total accumulates in float64 (np.zeros(num_samples)) while the
// limited evaporation is stored back into the T-typed array (zhao_carr.py:277-311)
template <typename T>
struct PrecpdArgs {
    const T *qc_gs, *qv_gs, *t_gs, *qc_emu, *qv_emu, *delp;
    T *qc_out, *qv_out, *t_out;
    double* precip;
    int64_t ncol;
    int nz;
};

template <typename T>
__global__ __launch_bounds__(64) void precpd_kernel(PrecpdArgs<T> a)
{
    const int64_t c = gid();
    if (c >= a.ncol) return;
    double total = 0.0;
    for (int k = a.nz - 1; k >= 0; --k) {
        const int64_t i = (int64_t)k * a.ncol + c;
        const T dp = a.delp[i];
        const T cloud_change = a.qc_emu[i] - a.qc_gs[i];
        const T humidity_change = a.qv_emu[i] - a.qv_gs[i];
        const T source = ((T)-1 * cloud_change) * dp / (T)kGravity;  // mixing_ratio_to_mass
        const T sink = humidity_change * dp / (T)kGravity;
        const T c_to_p = np_max(source, (T)0);
        const T p_to_v = np_max(sink, (T)0);
        total += (double)c_to_p;
        const double evap = np_min(total, (double)p_to_v);
        total -= evap;
        const T limited = (T)evap;  // limited_p_to_v[k, :] = limited_evap
        const T evaporation = limited / dp * (T)kGravity;  // mass_to_mixing_ratio
        const T cooling = (T)(kLv / kCp * -1) * evaporation;
        a.qc_out[i] = a.qc_gs[i] + ((T)-1 * c_to_p) / dp * (T)kGravity;
        a.qv_out[i] = a.qv_gs[i] + evaporation;
        a.t_out[i] = a.t_gs[i] + cooling;
    }
    a.precip[c] = total / kRhoWater;  // liquid_water_equivalent (float64)
}

// conservative_precip_simple: column water before - after, in T, levels added in order
template <typename T>
__global__ __launch_bounds__(64) void precip_simple_kernel(const T* qv_gs, const T* qc_gs, const T* qv_emu,
                                                           const T* qc_emu, const T* delp, T* precip, int64_t ncol,
                                                           int nz)
{
    const int64_t c = gid();
    if (c >= ncol) return;
    T before = 0, after = 0;
    for (int k = 0; k < nz; ++k) {
        const int64_t i = (int64_t)k * ncol + c;
        const T wb = (qv_gs[i] + qc_gs[i]) * delp[i] / (T)kGravity;
        const T wa = (qv_emu[i] + qc_emu[i]) * delp[i] / (T)kGravity;
        before = k ? before + wb : wb;
        after = k ? after + wa : wa;
    }
    precip[c] = (before - after) / (T)kRhoWater;
}

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

}  // namespace
}  // namespace fv3

using namespace fv3;

#define FV3_DISPATCH(f64, CALL) ((f64) ? CALL(double) : CALL(float))

// TimeMask's blend with numpy's dtype flow: each product in its array's dtype (the
// Python-float weight cast to it, NumPy's weak scalars), the sum in the promoted dtype
template <typename TS, typename TE, typename TO>
__global__ __launch_bounds__(256) void time_blend_kernel(const TS* __restrict__ s, const TE* __restrict__ e,
                                                         TO* __restrict__ out, int64_t n, TS alpha, TE beta)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const TS a = s[i] * alpha;
        const TE b = e[i] * beta;
        out[i] = (TO)a + (TO)b;
    }
}

template <typename TS, typename TE, typename TO>
static void launch_blend(const void* s, const void* e, void* out, int64_t n, double alpha, hipStream_t st)
{
    hipLaunchKernelGGL((time_blend_kernel<TS, TE, TO>), dim3(grid_for(n, 256)), dim3(256), 0, st, (const TS*)s,
                       (const TE*)e, (TO*)out, n, (TS)alpha, (TE)(1.0 - alpha));
}

extern "C" int fv3_time_blend(const void* state, int state_f64, const void* emulator, int emulator_f64, void* out,
                              int64_t n, double alpha, void* stream)
{
    clear_error();
    FV3_REQUIRE(n >= 0, "time_blend: n must be >= 0");
    if (n == 0) return FV3_OK;
    FV3_REQUIRE(state && emulator && out, "time_blend: NULL array");
    hipStream_t st = (hipStream_t)stream;
    if (state_f64 && emulator_f64) launch_blend<double, double, double>(state, emulator, out, n, alpha, st);
    else if (state_f64) launch_blend<double, float, double>(state, emulator, out, n, alpha, st);
    else if (emulator_f64) launch_blend<float, double, double>(state, emulator, out, n, alpha, st);
    else launch_blend<float, float, float>(state, emulator, out, n, alpha, st);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_range_mask(const void* x, void* out, int64_t n, double lo, double hi, int has_lo, int has_hi,
                              int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(n >= 0 && x && out, "range_mask: bad arguments");
    if (n == 0) return FV3_OK;
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(range_mask_kernel<double>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const double*)x,
                           (double*)out, n, lo, hi, has_lo, has_hi);
    else
        hipLaunchKernelGGL(range_mask_kernel<float>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const float*)x,
                           (float*)out, n, (float)lo, (float)hi, has_lo, has_hi);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_classify_one_hot(const void* logits, int n_class, int64_t inner, unsigned char* masks,
                                    int positive, int negative, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(n_class >= 1 && inner >= 0 && positive >= 0 && positive < n_class && negative >= 0 &&
                    negative < n_class,
                "classify_one_hot: bad arguments");
    if (inner == 0) return FV3_OK;
    FV3_REQUIRE(logits && masks, "classify_one_hot: NULL array");
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(classify_kernel<double>, dim3(grid_for(inner, 256)), dim3(256), 0, s,
                           (const double*)logits, n_class, inner, masks, positive, negative);
    else
        hipLaunchKernelGGL(classify_kernel<float>, dim3(grid_for(inner, 256)), dim3(256), 0, s,
                           (const float*)logits, n_class, inner, masks, positive, negative);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_infer_gscond_cloud(const void* qc_in, const void* qv_in, const void* qv_gscond, void* qc_out,
                                         int64_t n, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(n >= 0 && qc_in && qv_in && qv_gscond && qc_out, "zc_infer_gscond_cloud: bad arguments");
    if (n == 0) return FV3_OK;
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(infer_cloud_kernel<double>, dim3(grid_for(n, 256)), dim3(256), 0, s,
                           (const double*)qc_in, (const double*)qv_in, (const double*)qv_gscond, (double*)qc_out, n);
    else
        hipLaunchKernelGGL(infer_cloud_kernel<float>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const float*)qc_in,
                           (const float*)qv_in, (const float*)qv_gscond, (float*)qc_out, n);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_squash(const void* cloud, const void* humidity, double bound, void* cloud_out,
                             void* humidity_out, int64_t n, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(n >= 0 && cloud && humidity && cloud_out && humidity_out, "zc_squash: bad arguments");
    if (n == 0) return FV3_OK;
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(squash_kernel<double>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const double*)cloud,
                           (const double*)humidity, bound, (double*)cloud_out, (double*)humidity_out, n);
    else
        hipLaunchKernelGGL(squash_kernel<float>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const float*)cloud,
                           (const float*)humidity, (float)bound, (float*)cloud_out, (float*)humidity_out, n);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_zero_where(const unsigned char* class_mask, const void* cloud, void* out, int64_t n, int f64,
                                 void* stream)
{
    clear_error();
    FV3_REQUIRE(n >= 0 && class_mask && cloud && out, "zc_zero_where: bad arguments");
    if (n == 0) return FV3_OK;
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(zero_where_kernel<double>, dim3(grid_for(n, 256)), dim3(256), 0, s, class_mask,
                           (const double*)cloud, (double*)out, n);
    else
        hipLaunchKernelGGL(zero_where_kernel<float>, dim3(grid_for(n, 256)), dim3(256), 0, s, class_mask,
                           (const float*)cloud, (float*)out, n);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_gscond_update(int mode, const void* qc_in, const void* qv_in, const void* t_in,
                                    const void* qc_fortran_gscond, const void* qc_emulator,
                                    const unsigned char* class_mask, const unsigned char* ice_flag, void* qc_out,
                                    void* qv_out, void* t_out, int64_t n, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(mode >= FV3_ZC_CLOUD_EMULATOR && mode <= FV3_ZC_PHASE_DEPENDENT, "zc_gscond_update: bad mode %d",
                mode);
    FV3_REQUIRE(n >= 0 && qc_in && qv_in && t_in && qc_emulator && qc_out && qv_out && t_out,
                "zc_gscond_update: NULL array");
    FV3_REQUIRE(!(mode == FV3_ZC_CLOUD_IDENTICAL || mode == FV3_ZC_CLOUD_VANISHES) || qc_fortran_gscond,
                "zc_gscond_update: this mode needs the Fortran gscond cloud");
    FV3_REQUIRE(!(mode == FV3_ZC_CLOUD_CLASS_ZERO || mode == FV3_ZC_CLOUD_CLASS_NOTEND) || class_mask,
                "zc_gscond_update: this mode needs a class mask");
    FV3_REQUIRE(mode != FV3_ZC_PHASE_DEPENDENT || ice_flag, "zc_gscond_update: the phase mode needs the ice flag");
    if (n == 0) return FV3_OK;
    hipStream_t s = (hipStream_t)stream;
#define FV3_GSCOND(T)                                                                                          \
    do {                                                                                                       \
        GscondArgs<T> a{(const T*)qc_in, (const T*)qv_in,       (const T*)t_in, (const T*)qc_fortran_gscond,   \
                        (const T*)qc_emulator, class_mask, ice_flag, (T*)qc_out, (T*)qv_out, (T*)t_out, n, mode}; \
        hipLaunchKernelGGL(gscond_kernel<T>, dim3(grid_for(n, 256)), dim3(256), 0, s, a);                      \
    } while (0)
    if (f64)
        FV3_GSCOND(double);
    else
        FV3_GSCOND(float);
#undef FV3_GSCOND
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_ice_water_flag(const void* temperature, const void* cloud, double offset, void* iw,
                                     int64_t nrows, int64_t z, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(nrows >= 0 && z >= 0 && nrows <= 65535, "zc_ice_water_flag: bad shape (%lld, %lld)",
                (long long)nrows, (long long)z);
    if (nrows == 0 || z == 0) return FV3_OK;
    FV3_REQUIRE(temperature && cloud && iw, "zc_ice_water_flag: NULL array");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nchunk = (z + kIceChunk - 1) / kIceChunk;
    FV3_REQUIRE(nchunk < 0x7fffffff, "zc_ice_water_flag: rows too long");
    void* buf = nullptr;
    FV3_HIP(hipMallocAsync(&buf, (size_t)(nrows * nchunk), s));
    uint8_t* st = (uint8_t*)buf;
    const dim3 grid((unsigned)nchunk, (unsigned)nrows);
    if (f64) {
        hipLaunchKernelGGL(ice_pass1<double>, grid, dim3(kIceChunk), 0, s, (const double*)temperature,
                           (const double*)cloud, z, offset, st, nchunk);
    } else {
        hipLaunchKernelGGL(ice_pass1<float>, grid, dim3(kIceChunk), 0, s, (const float*)temperature,
                           (const float*)cloud, z, (float)offset, st, nchunk);
    }
    FV3_LAUNCH_CHECK();
    hipLaunchKernelGGL(ice_pass2, dim3((unsigned)nrows), dim3(256), 0, s, st, nchunk);
    FV3_LAUNCH_CHECK();
    if (f64) {
        hipLaunchKernelGGL(ice_pass3<double>, grid, dim3(kIceChunk), 0, s, (const double*)temperature,
                           (const double*)cloud, z, offset, st, nchunk, (double*)iw);
    } else {
        hipLaunchKernelGGL(ice_pass3<float>, grid, dim3(kIceChunk), 0, s, (const float*)temperature,
                           (const float*)cloud, z, (float)offset, st, nchunk, (float*)iw);
    }
    FV3_LAUNCH_CHECK();
    FV3_HIP(hipFreeAsync(buf, s));
    return FV3_OK;
}

extern "C" int fv3_zc_precpd_conservative(const void* qc_gscond, const void* qv_gscond, const void* t_gscond,
                                          const void* qc_emulator, const void* qv_emulator, const void* delp,
                                          void* qc_out, void* qv_out, void* t_out, double* precip, int nz,
                                          int64_t ncol, int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(nz >= 1 && ncol >= 0, "zc_precpd_conservative: bad shape (%d, %lld)", nz, (long long)ncol);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(qc_gscond && qv_gscond && t_gscond && qc_emulator && qv_emulator && delp && qc_out && qv_out &&
                    t_out && precip,
                "zc_precpd_conservative: NULL array");
    hipStream_t s = (hipStream_t)stream;
#define FV3_PRECPD(T)                                                                                           \
    do {                                                                                                        \
        PrecpdArgs<T> a{(const T*)qc_gscond, (const T*)qv_gscond, (const T*)t_gscond, (const T*)qc_emulator,    \
                        (const T*)qv_emulator, (const T*)delp, (T*)qc_out, (T*)qv_out, (T*)t_out, precip, ncol, nz}; \
        hipLaunchKernelGGL(precpd_kernel<T>, dim3(grid_for(ncol, 64)), dim3(64), 0, s, a);                      \
    } while (0)
    if (f64)
        FV3_PRECPD(double);
    else
        FV3_PRECPD(float);
#undef FV3_PRECPD
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_zc_precip_simple(const void* qv_gscond, const void* qc_gscond, const void* qv_emulator,
                                    const void* qc_emulator, const void* delp, void* precip, int nz, int64_t ncol,
                                    int f64, void* stream)
{
    clear_error();
    FV3_REQUIRE(nz >= 1 && ncol >= 0, "zc_precip_simple: bad shape (%d, %lld)", nz, (long long)ncol);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(qv_gscond && qc_gscond && qv_emulator && qc_emulator && delp && precip,
                "zc_precip_simple: NULL array");
    hipStream_t s = (hipStream_t)stream;
    if (f64)
        hipLaunchKernelGGL(precip_simple_kernel<double>, dim3(grid_for(ncol, 64)), dim3(64), 0, s,
                           (const double*)qv_gscond, (const double*)qc_gscond, (const double*)qv_emulator,
                           (const double*)qc_emulator, (const double*)delp, (double*)precip, ncol, nz);
    else
        hipLaunchKernelGGL(precip_simple_kernel<float>, dim3(grid_for(ncol, 64)), dim3(64), 0, s,
                           (const float*)qv_gscond, (const float*)qc_gscond, (const float*)qv_emulator,
                           (const float*)qc_emulator, (const float*)delp, (float*)precip, ncol, nz);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
