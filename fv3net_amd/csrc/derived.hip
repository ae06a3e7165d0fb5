// fv3net_amd — the derived-variable arithmetic behind fv3fit's DerivedModel and
// TransformedPredictor (external/fv3fit/fv3fit/_shared/models.py:110-220, 279-337), for the
// catalogue entries a dQ1/dQ2 model feeds:
//
//   vcm.DerivedMapping   external/vcm/vcm/derived_mapping.py:123-127, 264-410
//     Q1 / Q2 (= dQ + pQ), internal_energy, column_integrated_{dQ1,dQ2,Q1,Q2},
//     water_vapor_path, evaporation, upward_heat_flux_at_surface, incloud_*_mixing_ratio
//   vcm.DataTransform    external/vcm/vcm/data_transform.py:65-323
//     Q{1,2}_from_dQ{1,2}_pQ{1,2}, Qm <-> Q1 (optionally temperature dependent),
//     Q2 / Qm flux form <-> tendency, implied surface precipitation / downward radiative
//     flux, tapered_dQ{1,2} (csrc/composite.hip fv3_scale_levels), condensate conversions
//   with vcm/calc/thermo (local.py:25-28, 69-82, 195-208, 317-360, vertically_dependent.py:
//   18-38, 279-325), vcm/calc/flux_form.py:7-100 and vcm/calc/clouds.py:7-66.
//
// Two kernels, both HBM-bound:
//   derived_elementwise_kernel  one thread per element of contiguous arrays, grid-stride
//   derived_columns_kernel      one thread per column walking its levels in order (mass
//                               integrals, cumulative sums, vertical differences), every
//                               level a coalesced row of the [level][column] layout
// Every operand is float32 or float64.  The arithmetic runs in double and each numpy
// intermediate is rounded to its numpy dtype (as_dtype): float32 + - * / computed in double
// and rounded once give the float32 operation's bits (53 >= 2 * 24 + 2), and a float64
// operand meeting a float32 one reproduces numpy's promotion.  Python-float constants take
// the array's dtype (NumPy weak scalars), reductions follow numpy's order (nansum from +0,
// nancumsum from the first term), so results are bit-identical to oracle/derived.py.
#include "common.h"

namespace fv3 {
namespace {

constexpr double kGravity = 9.80665;  // vcm/calc/thermo/constants.py
constexpr double kRdgas = 287.05;
constexpr double kCp = 1004.0;
constexpr double kLv0 = 2.5e6;
constexpr double kHLiq = 4185.5, kHVap = 1846.0;
constexpr double kTFreeze = 273.15;

__device__ __forceinline__ double as_dtype(double x, bool f64) { return f64 ? x : (double)(float)x; }

__device__ __forceinline__ double ld(const void* p, bool f64, int64_t i)
{
    return f64 ? static_cast<const double*>(p)[i] : (double)static_cast<const float*>(p)[i];
}

__device__ __forceinline__ void st(void* p, bool f64, int64_t i, double v)
{
    if (f64)
        static_cast<double*>(p)[i] = v;
    else
        static_cast<float*>(p)[i] = (float)v;
}

// latent_heat_vaporization(T) (local.py:25-28) in T's dtype
__device__ __forceinline__ double lv_of(double t, bool w)
{
    return as_dtype(as_dtype(kLv0, w) + as_dtype(as_dtype(kHLiq - kHVap, w) * as_dtype(t - as_dtype(kTFreeze, w), w), w),
                    w);
}

constexpr int kMaxIn = 8;

struct EwArgs {
    const void* in[kMaxIn];
    int f64[kMaxIn];
    int n_in, op, out_f64;
    void* out;
    int64_t n;
    double p[4];
};

__global__ __launch_bounds__(256) void derived_elementwise_kernel(EwArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool w0 = a.f64[0], w1 = a.f64[1], w2 = a.f64[2];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        // a missing operand (NULL) is zeros_like(...) of its dtype
        const double x = a.in[0] ? ld(a.in[0], w0, i) : 0.0;
        const double y = a.n_in > 1 && a.in[1] ? ld(a.in[1], w1, i) : 0.0;
        double r = 0.0;
        switch (a.op) {
        case FV3_EW_ADD:  // x + y (+ z + ...), left to right
        {
            bool w = w0;
            r = x;
            for (int j = 1; j < a.n_in; ++j) {
                w = w || a.f64[j];
                r = as_dtype(r + (a.in[j] ? ld(a.in[j], a.f64[j], i) : 0.0), w);
            }
            break;
        }
        case FV3_EW_SUB:  // x - y - z ...
        {
            bool w = w0;
            r = x;
            for (int j = 1; j < a.n_in; ++j) {
                w = w || a.f64[j];
                r = as_dtype(r - (a.in[j] ? ld(a.in[j], a.f64[j], i) : 0.0), w);
            }
            break;
        }
        case FV3_EW_IADD:  // x += y: computed in the promoted dtype, stored in x's
            r = as_dtype(as_dtype(x + y, w0 || w1), w0);
            break;
        case FV3_EW_SCALE:  // c * x
            r = as_dtype(as_dtype(a.p[0], w0) * x, w0);
            break;
        case FV3_EW_DIV_SCALAR:  // x / c
            r = as_dtype(x / as_dtype(a.p[0], w0), w0);
            break;
        case FV3_EW_MSE:  // moist_static_energy_tendency(q1, q2[, T]) (local.py:317-337)
        case FV3_EW_TEMP_TEND:  // temperature_tendency(qm, q2[, T]) (local.py:340-360)
        {
            double lvq;
            bool wl;
            if (a.n_in > 2) {  // temperature dependent: latent_heat_vaporization(T) * q2
                const double t = ld(a.in[2], w2, i);
                wl = w2 || w1;
                lvq = as_dtype(lv_of(t, w2) * y, wl);
            } else {  // the default 273.15 K: a Python float constant
                wl = w1;
                lvq = as_dtype(as_dtype(kLv0 + (kHLiq - kHVap) * (kTFreeze - kTFreeze), w1) * y, w1);
            }
            const bool w = w0 || wl;
            if (a.op == FV3_EW_MSE)
                r = as_dtype(as_dtype(as_dtype(kCp - kRdgas, w0) * x, w0) + lvq, w);
            else
                r = as_dtype(as_dtype(x - lvq, w) / as_dtype(kCp - kRdgas, w), w);
            break;
        }
        case FV3_EW_INCLOUD_TO_GRIDCELL:  // clouds.py:40-66: x = cloud fraction, y = in-cloud
        case FV3_EW_GRIDCELL_TO_INCLOUD:  // clouds.py:7-37: x = cloud fraction, y = grid-cell
        {
            const double c1 = a.p[0], c2 = a.p[1];
            const double rect = x > as_dtype(c2, w0) ? x : as_dtype(c2, w0);  // cf.where(cf > climit2, climit2)
            const bool w = w0 || w1;
            double other;
            if (a.op == FV3_EW_INCLOUD_TO_GRIDCELL)
                other = as_dtype(y * rect, w);
            else
                other = as_dtype(y * as_dtype(as_dtype(1.0, w0) / rect, w0), w);  // y * (1.0 / rect)
            r = x <= as_dtype(c1, w0) ? y : other;
            break;
        }
        case FV3_EW_MUL:  // x * y
            r = as_dtype(x * y, w0 || w1);
            break;
        case FV3_EW_ONE_MINUS_MUL:  // (1 - x) * y (derived_mapping.py:194-195)
            r = as_dtype(as_dtype(1.0 - x, w0) * y, w0 || w1);
            break;
        case FV3_EW_SIGN_PARALLEL:  // sign(x / y) * abs(y) (derived_mapping.py:163-174)
        {
            const bool w = w0 || w1;
            const double q = as_dtype(x / y, w);
            const double sg = q > 0.0 ? 1.0 : q < 0.0 ? -1.0 : q == 0.0 ? 0.0 : q;  // np.sign (NaN stays)
            r = as_dtype(sg * fabs(y), w);
            break;
        }
        case FV3_EW_PROJECT:  // (x * y + z * u) / norm (derived_mapping.py:177-187)
        {
            const bool w2_ = a.f64[2], w3 = a.f64[3];
            const double z = ld(a.in[2], w2_, i), u = ld(a.in[3], w3, i);
            const bool wa = w0 || w1, wb = w2_ || w3, ws = wa || wb, wr = ws || a.p[1] != 0.0;
            const double s = as_dtype(as_dtype(x * y, wa) + as_dtype(z * u, wb), ws);
            r = as_dtype(s / a.p[0], wr);
            break;
        }
        case FV3_EW_ISCLOSE_ONEHOT:  // xr.where(isclose(x, p0), 1.0, 0.0): float64 one-hot
        {
            // np.isclose within_tol: |x - y| <= atol + rtol |y| in x's dtype (p1 = rtol,
            // p2 = atol); NaN and infinities are never close to a finite p0
            const double c = as_dtype(a.p[0], w0);
            const double tol = as_dtype(a.p[2] + a.p[1] * fabs(a.p[0]), w0);
            r = fabs(as_dtype(x - c, w0)) <= tol ? 1.0 : 0.0;
            break;
        }
        }
        st(a.out, a.out_f64, i, r);
    }
}

// ---------------------------------------------------------------------------------
// column operations: fields [level][column] under an fv3_layout, 2-D fields one level
// ---------------------------------------------------------------------------------
struct ColArgs {
    fv3_field in[kMaxIn];
    fv3_field out[2];
    int n_in, op;
    int64_t ncol;
    int nz;
    double p[4];
};

__device__ __forceinline__ double fld(const fv3_field& f, int64_t off, int k)
{
    return f.data ? ld(f.data, f.f64, off + (int64_t)k * f.lay.ld) : 0.0;
}

// nan0(x * delp / g) in promote(x, delp)
__device__ __forceinline__ double mass_term(double x, double d, bool w)
{
    const double t = as_dtype(as_dtype(x * d, w) / as_dtype(kGravity, w), w);
    return t != t ? 0.0 : t;
}

// sum_z nan0(s x delp / g) in numpy's order: the reduction's identity +0 plus, over a
// leading or middle z, the levels added in order; over the contiguous last axis (z-last
// arrays, pairwise != 0) numpy's pairwise_sum: 8 interleaved partial sums combined as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the remainder (nz <= 128)
__device__ __forceinline__ double column_sum(const fv3_field& X, int64_t ox, const fv3_field& D, int64_t od, int nz,
                                             double sgn, bool w, bool pairwise)
{
    auto term = [&](int k) { return mass_term(sgn * fld(X, ox, k), fld(D, od, k), w); };
    if (!pairwise || nz < 8) {
        double s = 0.0;
        for (int k = 0; k < nz; ++k) s = as_dtype(s + term(k), w);
        return s;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = term(j);
    int i = 8;
    for (const int lim = nz - nz % 8; i < lim; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = as_dtype(r[j] + term(i + j), w);
    }
    double res = as_dtype(as_dtype(as_dtype(r[0] + r[1], w) + as_dtype(r[2] + r[3], w), w) +
                              as_dtype(as_dtype(r[4] + r[5], w) + as_dtype(r[6] + r[7], w), w),
                          w);
    for (; i < nz; ++i) res = as_dtype(res + term(i), w);
    return as_dtype(0.0 + res, w);
}

__global__ __launch_bounds__(256) void derived_columns_kernel(ColArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const fv3_field& X = a.in[0];
    const fv3_field& D = a.in[1];
    const int64_t ox = col_offset(X.lay, c), od = col_offset(D.lay, c);
    const bool wx = X.f64, wd = D.f64, wp = wx || wd;
    switch (a.op) {
    case FV3_COL_MASS_INTEGRAL: {
        // p0 * (sum_z nan0(s * x * delp / g)), s = +-1, p0 NaN: no scale; p1 != 0: negated
        // (p3 != 0: pairwise, z-last)
        const double sgn = a.p[0] < 0 ? -1.0 : 1.0;
        double s = column_sum(X, ox, D, od, a.nz, sgn, wp, a.p[3] != 0.0);
        if (a.p[1] == a.p[1]) s = as_dtype(as_dtype(a.p[1], wp) * s, wp);
        if (a.p[2] != 0.0) s = -s;
        st(const_cast<void*>(a.out[0].data), a.out[0].f64, col_offset(a.out[0].lay, c), s);
        break;
    }
    case FV3_COL_TENDENCY_TO_FLUX:
    case FV3_COL_IMPLIED_SURFACE_FLUX: {
        // flux_form.py:7-73.  in[2] = TOA net flux (NULL: zeros of its dtype), in[3] =
        // surface upward flux; p0 != 0: rectify.  TENDENCY_TO_FLUX writes out[0] = the
        // interface fluxes above each level (in promote(tendency, delp)) and out[1] = the
        // downward surface flux; IMPLIED_SURFACE_FLUX writes out[0] = the downward flux.
        const fv3_field& T = a.in[2];
        const fv3_field& U = a.in[3];
        const int64_t ot = col_offset(T.lay, c), ou = col_offset(U.lay, c);
        const bool wt = T.f64, wu = U.f64;
        const double toa = fld(T, ot, 0), up = fld(U, ou, 0);
        double down;
        bool wdn;
        if (a.op == FV3_COL_TENDENCY_TO_FLUX) {
            // flux = -nancumsum(x delp / g), padded with 0.0 on top, += toa (in place:
            // stays in the tendency's dtype)
            const fv3_field& F = a.out[0];
            const int64_t of = col_offset(F.lay, c);
            double cum = 0.0;
            st(const_cast<void*>(F.data), F.f64, of, as_dtype(as_dtype(0.0 + toa, wp || wt), wp));
            for (int k = 0; k < a.nz; ++k) {
                const double t = mass_term(fld(X, ox, k), fld(D, od, k), wp);
                cum = k == 0 ? t : as_dtype(cum + t, wp);  // nancumsum starts from the first term
                const double f = as_dtype(as_dtype(-cum + toa, wp || wt), wp);
                if (k + 1 < a.nz)
                    st(const_cast<void*>(F.data), F.f64, of + (int64_t)(k + 1) * F.lay.ld, f);
                else
                    down = f;
            }
            wdn = wp || wu;
            down = as_dtype(down + up, wdn);
        } else {
            // TOA net flux + surface upward flux - mass_integrate(x) (p1 != 0: pairwise)
            const double s = column_sum(X, ox, D, od, a.nz, 1.0, wp, a.p[1] != 0.0);
            const bool wtu = wt || wu;
            wdn = wtu || wp;
            down = as_dtype(as_dtype(toa + up, wtu) - s, wdn);
        }
        if (a.p[0] != 0.0 && !(down >= 0.0)) down = 0.0;  // .where(down >= 0, 0)
        const fv3_field& O = a.op == FV3_COL_TENDENCY_TO_FLUX ? a.out[1] : a.out[0];
        st(const_cast<void*>(O.data), O.f64, col_offset(O.lay, c), down);
        break;
    }
    case FV3_COL_FLUX_TO_TENDENCY: {
        // flux_form.py:76-100: in[0] = interface fluxes (levels), in[2] = downward and
        // in[3] = upward surface flux; tendency = -(g * diff(concat(flux, down - up)) / delp)
        const fv3_field& Dn = a.in[2];
        const fv3_field& U = a.in[3];
        const bool wn = Dn.f64 || U.f64, wc = wx || wn, wo = wc || wd;
        const double sfc = as_dtype(fld(Dn, col_offset(Dn.lay, c), 0) - fld(U, col_offset(U.lay, c), 0), wn);
        const fv3_field& O = a.out[0];
        const int64_t oo = col_offset(O.lay, c);
        double prev = fld(X, ox, 0);
        for (int k = 0; k < a.nz; ++k) {
            const double next = k + 1 < a.nz ? fld(X, ox, k + 1) : sfc;
            const double diff = as_dtype(next - prev, wc);
            const double div = as_dtype(as_dtype(as_dtype(kGravity, wc) * diff, wc) / fld(D, od, k), wo);
            st(const_cast<void*>(O.data), O.f64, oo + (int64_t)k * O.lay.ld, -div);
            prev = next;
        }
        break;
    }
    }
}

// ---------------------------------------------------------------------------------
// strided operands over a result of up to FV3_MAX_DIMS dims (xarray's alignment by dim
// name): the D-grid wind rotation and the solar zenith angle
// ---------------------------------------------------------------------------------
struct Shape {
    int ndim;
    int64_t n[FV3_MAX_DIMS];
};

// the element offset of result element i in an operand with strides st
__device__ __forceinline__ void unravel(const Shape& sh, int64_t i, int64_t* idx)
{
    for (int d = sh.ndim - 1; d >= 0; --d) {
        const int64_t q = i / sh.n[d];
        idx[d] = i - q * sh.n[d];
        i = q;
    }
}

__device__ __forceinline__ int64_t offset(const Shape& sh, const int64_t* idx, const int64_t* st)
{
    int64_t o = 0;
    for (int d = 0; d < sh.ndim; ++d) o += idx[d] * st[d];
    return o;
}

struct RotArgs {
    Shape sh;
    int64_t n;
    fv3_strided x, y, c[4];
    int64_t xs, ys;
    void* east;
    void* north;
    int east_f64, north_f64;
};

// rotate.py:9-56: centre both D-grid components (coarsen.py:54-75: 0.5 * (edge +
// edge.shift(1)) dropping the first edge, i.e. 0.5 * (e[j + 1] + e[j])), then the 2x2
// rotation by the grid's coefficients; one thread per centred element
__global__ __launch_bounds__(256) void center_rotate_kernel(RotArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool wx = a.x.f64, wy = a.y.f64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        int64_t idx[FV3_MAX_DIMS];
        unravel(a.sh, i, idx);
        const int64_t ox = offset(a.sh, idx, a.x.stride), oy = offset(a.sh, idx, a.y.stride);
        const double xc = as_dtype(0.5 * as_dtype(ld(a.x.data, wx, ox + a.xs) + ld(a.x.data, wx, ox), wx), wx);
        const double yc = as_dtype(0.5 * as_dtype(ld(a.y.data, wy, oy + a.ys) + ld(a.y.data, wy, oy), wy), wy);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            void* out = r ? a.north : a.east;
            if (!out) continue;
            const fv3_strided& cu = a.c[2 * r];
            const fv3_strided& cv = a.c[2 * r + 1];
            const bool wu = cu.f64 || wx, wv = cv.f64 || wy;
            const double pu = as_dtype(ld(cu.data, cu.f64, offset(a.sh, idx, cu.stride)) * xc, wu);
            const double pv = as_dtype(ld(cv.data, cv.f64, offset(a.sh, idx, cv.stride)) * yc, wv);
            st(out, r ? a.north_f64 : a.east_f64, i, as_dtype(pu + pv, wu || wv));
        }
    }
}

// sum of squares, stage 1: block b sums a fixed strided subset in float64, then a fixed
// tree; stage 2 folds the block partials in a fixed tree (deterministic for a given n)
constexpr int kSqBlocks = 512;

__device__ double block_sum(double v, double* lds)
{
    lds[threadIdx.x] = v;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) lds[threadIdx.x] += lds[threadIdx.x + s];
        __syncthreads();
    }
    return lds[0];
}

struct SqArgs {
    const void* in[kMaxIn];
    int f64[kMaxIn];
    int n_arr;
    int64_t n;
};

__global__ __launch_bounds__(256) void sum_squares_stage1(SqArgs a, double* partial)
{
    __shared__ double lds[256];
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int j = 0; j < a.n_arr; ++j)
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
            const double v = ld(a.in[j], a.f64[j], i);
            s += v * v;
        }
    const double t = block_sum(s, lds);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void sum_squares_stage2(const double* partial, int nb, double* out)
{
    __shared__ double lds[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
    const double t = block_sum(s, lds);
    if (threadIdx.x == 0) out[0] = t;
}

struct ZenArgs {
    Shape sh;
    int64_t n;
    fv3_strided lon, lat;
    int lon_rad, lat_rad;
    int64_t tst[FV3_MAX_DIMS];
    const double* terms;  // [4][nt]: gmst, ra, sin(dec), cos(dec)
    int64_t nt;
    double* out;
};

// degrees -> radians in the operand's dtype (lon * RAD_PER_DEG; np.rad2deg first for a
// radian-valued DataArray)
__device__ __forceinline__ double to_rad(double v, bool w, bool rad_units)
{
    constexpr double kRadPerDeg = 3.141592653589793 / 180.0, kDegPerRad = 180.0 / 3.141592653589793;
    if (rad_units) v = as_dtype(v * as_dtype(kDegPerRad, w), w);
    return as_dtype(v * as_dtype(kRadPerDeg, w), w);
}

__global__ __launch_bounds__(256) void cos_zenith_kernel(ZenArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool wo = a.lon.f64, wa = a.lat.f64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        int64_t idx[FV3_MAX_DIMS];
        unravel(a.sh, i, idx);
        const int64_t t = offset(a.sh, idx, a.tst);
        const double lon = to_rad(ld(a.lon.data, wo, offset(a.sh, idx, a.lon.stride)), wo, a.lon_rad);
        const double lat = to_rad(ld(a.lat.data, wa, offset(a.sh, idx, a.lat.stride)), wa, a.lat_rad);
        const double gmst = a.terms[t], ra = a.terms[a.nt + t];
        const double sdec = a.terms[2 * a.nt + t], cdec = a.terms[3 * a.nt + t];
        const double sl = wa ? sin(lat) : (double)sinf((float)lat);
        const double cl = wa ? cos(lat) : (double)cosf((float)lat);
        const double h = (gmst + lon) - ra;  // local mean sidereal time - right ascension
        a.out[i] = sl * sdec + cl * cdec * cos(h);
    }
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_derived_elementwise(int op, const void* const* in, const int* in_f64, int n_in, void* out,
                                       int out_f64, int64_t n, const double* params, int n_params, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(n >= 0, "derived_elementwise: negative size");
    FV3_REQUIRE(n_in >= 1 && n_in <= kMaxIn && in && in_f64, "derived_elementwise: 1..%d inputs", kMaxIn);
    FV3_REQUIRE(n_params >= 0 && n_params <= 4 && (n_params == 0 || params), "derived_elementwise: bad parameters");
    FV3_REQUIRE(op >= FV3_EW_ADD && op <= FV3_EW_PROJECT, "derived_elementwise: unknown op %d", op);
    const bool unary = op == FV3_EW_SCALE || op == FV3_EW_DIV_SCALAR || op == FV3_EW_ISCLOSE_ONEHOT;
    const int need = op == FV3_EW_ISCLOSE_ONEHOT ? 3
                   : (op == FV3_EW_SCALE || op == FV3_EW_DIV_SCALAR) ? 1
                   : (op == FV3_EW_INCLOUD_TO_GRIDCELL || op == FV3_EW_GRIDCELL_TO_INCLOUD || op == FV3_EW_PROJECT) ? 2
                                                                                                       : 0;
    FV3_REQUIRE(n_params >= need, "derived_elementwise: op %d needs %d parameters", op, need);
    FV3_REQUIRE((op == FV3_EW_MSE || op == FV3_EW_TEMP_TEND) ? (n_in == 2 || n_in == 3)
                : unary ? n_in == 1
                : (op == FV3_EW_ADD || op == FV3_EW_SUB) ? n_in >= 2
                : op == FV3_EW_PROJECT ? n_in == 4 : n_in == 2,
                "derived_elementwise: op %d got %d inputs", op, n_in);
    if (n == 0) return FV3_OK;
    FV3_REQUIRE(out, "derived_elementwise: NULL output");
    EwArgs a{};
    for (int j = 0; j < n_in; ++j) {
        a.in[j] = in[j];
        a.f64[j] = in_f64[j] != 0;
        // only the elementwise sums take a missing operand (zeros_like)
        FV3_REQUIRE(in[j] || ((op == FV3_EW_ADD || op == FV3_EW_SUB) && j > 0),
                    "derived_elementwise: input %d is NULL", j);
    }
    a.n_in = n_in, a.op = op, a.out = out, a.out_f64 = out_f64 != 0, a.n = n;
    for (int j = 0; j < n_params; ++j) a.p[j] = params[j];
    const int64_t g = (n + 255) / 256;
    const unsigned grid = (unsigned)(g < 8192 ? g : 8192);
    hipLaunchKernelGGL(derived_elementwise_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_derived_columns(int op, const fv3_field* in, int n_in, const fv3_field* out, int n_out,
                                   int64_t ncol, int nz, const double* params, int n_params, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ncol >= 0 && nz >= 1, "derived_columns: bad sizes ncol=%lld nz=%d", (long long)ncol, nz);
    FV3_REQUIRE(op >= FV3_COL_MASS_INTEGRAL && op <= FV3_COL_FLUX_TO_TENDENCY, "derived_columns: unknown op %d", op);
    const int want_in = op == FV3_COL_MASS_INTEGRAL ? 2 : 4;
    const int want_out = op == FV3_COL_TENDENCY_TO_FLUX ? 2 : 1;
    const int want_p = op == FV3_COL_MASS_INTEGRAL ? 4 : (op == FV3_COL_FLUX_TO_TENDENCY ? 0 : (op == FV3_COL_IMPLIED_SURFACE_FLUX ? 2 : 1));
    FV3_REQUIRE(in && n_in == want_in && out && n_out == want_out && n_params >= want_p && (want_p == 0 || params),
                "derived_columns: op %d takes %d inputs, %d outputs, %d parameters", op, want_in, want_out, want_p);
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED,
                     nz <= 128 || !((op == FV3_COL_MASS_INTEGRAL && params[3] != 0.0) ||
                                    (op == FV3_COL_IMPLIED_SURFACE_FLUX && params[1] != 0.0)),
                     "derived_columns: pairwise (z-last) sums of more than 128 levels");
    if (ncol == 0) return FV3_OK;
    ColArgs a{};
    for (int j = 0; j < n_in; ++j) {
        // the TOA net flux may be missing (zeros_like(latent_heat_flux)); nothing else
        FV3_REQUIRE(in[j].data || (j == 2 && op != FV3_COL_FLUX_TO_TENDENCY), "derived_columns: input %d is NULL", j);
        FV3_REQUIRE(!in[j].data || layout_ok(in[j].lay, ncol), "derived_columns: input %d: bad layout", j);
        a.in[j] = in[j];
    }
    for (int j = 0; j < n_out; ++j) {
        FV3_REQUIRE(out[j].data && layout_ok(out[j].lay, ncol), "derived_columns: output %d: NULL or bad layout", j);
        a.out[j] = out[j];
    }
    a.n_in = n_in, a.op = op, a.ncol = ncol, a.nz = nz;
    for (int j = 0; j < n_params && j < 4; ++j) a.p[j] = params[j];
    hipLaunchKernelGGL(derived_columns_kernel, dim3((unsigned)((ncol + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

namespace {
bool shape_ok(int ndim, const int64_t* shape, fv3::Shape& sh, int64_t& n)
{
    if (ndim < 1 || ndim > FV3_MAX_DIMS || !shape) return false;
    sh.ndim = ndim;
    n = 1;
    for (int d = 0; d < ndim; ++d) {
        if (shape[d] < 0) return false;
        sh.n[d] = shape[d];
        n *= shape[d];
    }
    return true;
}

unsigned ew_grid(int64_t n)
{
    const int64_t g = (n + 255) / 256;
    return (unsigned)(g < 8192 ? g : 8192);
}
}  // namespace

extern "C" int fv3_center_rotate_winds(int ndim, const int64_t* shape, fv3_strided x_wind, int64_t x_stag,
                                       fv3_strided y_wind, int64_t y_stag, const fv3_strided* coeff, void* eastward,
                                       int east_f64, void* northward, int north_f64, void* stream)
{
    using namespace fv3;
    clear_error();
    RotArgs a{};
    FV3_REQUIRE(shape_ok(ndim, shape, a.sh, a.n), "center_rotate_winds: 1..%d dims of size >= 0", FV3_MAX_DIMS);
    FV3_REQUIRE(coeff, "center_rotate_winds: NULL coefficients");
    if (a.n == 0) return FV3_OK;
    FV3_REQUIRE(x_wind.data && y_wind.data, "center_rotate_winds: NULL wind");
    FV3_REQUIRE(x_stag != 0 && y_stag != 0, "center_rotate_winds: zero staggered stride");
    a.x = x_wind, a.y = y_wind, a.xs = x_stag, a.ys = y_stag;
    for (int j = 0; j < 4; ++j) a.c[j] = coeff[j];
    const bool wx = x_wind.f64, wy = y_wind.f64;
    if (eastward) {
        FV3_REQUIRE(coeff[0].data && coeff[1].data, "center_rotate_winds: NULL eastward coefficient");
        const bool w = (coeff[0].f64 || wx) || (coeff[1].f64 || wy);
        FV3_REQUIRE((east_f64 != 0) == w, "center_rotate_winds: eastward must be float%d (numpy's promotion)",
                    w ? 64 : 32);
    }
    if (northward) {
        FV3_REQUIRE(coeff[2].data && coeff[3].data, "center_rotate_winds: NULL northward coefficient");
        const bool w = (coeff[2].f64 || wx) || (coeff[3].f64 || wy);
        FV3_REQUIRE((north_f64 != 0) == w, "center_rotate_winds: northward must be float%d (numpy's promotion)",
                    w ? 64 : 32);
    }
    a.east = eastward, a.north = northward, a.east_f64 = east_f64 != 0, a.north_f64 = north_f64 != 0;
    hipLaunchKernelGGL(center_rotate_kernel, dim3(ew_grid(a.n)), dim3(256), 0, (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_sum_squares(const void* const* in, const int* in_f64, int n_arr, int64_t n, double* out,
                               void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(in && in_f64 && out && n_arr >= 1 && n_arr <= kMaxIn && n >= 0, "sum_squares: bad arguments");
    SqArgs a{};
    for (int j = 0; j < n_arr; ++j) {
        FV3_REQUIRE(in[j] || n == 0, "sum_squares: input %d is NULL", j);
        a.in[j] = in[j];
        a.f64[j] = in_f64[j] != 0;
    }
    a.n_arr = n_arr, a.n = n;
    hipStream_t s = (hipStream_t)stream;
    double* partial = nullptr;
    FV3_HIP(hipMallocAsync((void**)&partial, kSqBlocks * sizeof(double), s));
    hipLaunchKernelGGL(sum_squares_stage1, dim3(kSqBlocks), dim3(256), 0, s, a, partial);
    hipLaunchKernelGGL(sum_squares_stage2, dim3(1), dim3(256), 0, s, partial, kSqBlocks, out);
    const hipError_t e = hipGetLastError();
    FV3_HIP(hipFreeAsync(partial, s));
    FV3_HIP(e);
    return FV3_OK;
}

extern "C" int fv3_cos_zenith(int ndim, const int64_t* shape, fv3_strided lon, int lon_rad, fv3_strided lat,
                              int lat_rad, const int64_t* time_stride, const double* terms, int64_t n_times,
                              double* out, void* stream)
{
    using namespace fv3;
    clear_error();
    ZenArgs a{};
    FV3_REQUIRE(shape_ok(ndim, shape, a.sh, a.n), "cos_zenith: 1..%d dims of size >= 0", FV3_MAX_DIMS);
    if (a.n == 0) return FV3_OK;
    FV3_REQUIRE(lon.data && lat.data && time_stride && terms && out && n_times >= 1, "cos_zenith: NULL operand");
    a.lon = lon, a.lat = lat, a.lon_rad = lon_rad != 0, a.lat_rad = lat_rad != 0;
    int64_t tmax = 0;
    for (int d = 0; d < ndim; ++d) {
        FV3_REQUIRE(time_stride[d] >= 0, "cos_zenith: negative time stride");
        a.tst[d] = time_stride[d];
        tmax += (shape[d] - 1) * time_stride[d];
    }
    FV3_REQUIRE(tmax < n_times, "cos_zenith: time strides address %lld of %lld time values", (long long)tmax + 1,
                (long long)n_times);
    a.terms = terms, a.nt = n_times, a.out = out;
    hipLaunchKernelGGL(cos_zenith_kernel, dim3(ew_grid(a.n)), dim3(256), 0, (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
