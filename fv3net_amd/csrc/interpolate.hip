// fv3net_amd — vertical interpolation of columns to new levels on gfx950.
//
// Replaces (paths under /root/reference):
//   fv3_interpolate_2d       external/mappm/mappm/interpolate_2d.f90:1-27 (f2py
//                            mappm.interpolate_2d, called by vcm/interpolate.py:176-180
//                            for per-column output levels, interpolate_1d :100-145)
//   fv3_interpolate_levels   vcm/interpolate.py:148-173: metpy.interpolate.interpolate_1d
//                            for one set of output levels shared by every column
//                            (MetPy is not vendored; its published algorithm is restated
//                            below and pinned by the reference's test KATs)
//   fv3_pressure_midpoint_log  vcm/calc/thermo/vertically_dependent.py:153-178
//                            (interpolate_to_pressure_levels, vcm/interpolate.py:77-97)
//
// Layout: every array is level-major, element (level k, column c) at [k * ld + c]
// (the stacked [z][column] state, no transposes); one thread per column, so each
// level is a coalesced row.  Memory-bound: n_in * 2 + n_out values per column.
//
// interpolate_2d semantics (Fortran, real*8): out = fill; for every output level the
// interval loop runs k = 1..n_in-1 with NO early exit, so the LAST k that matches any
// of  x_k <= xp < x_k+1 -> y_k (1-w) + y_k+1 w,  x_k == xp -> y_k,  x_k+1 == xp -> y_k+1
// decides.  Scanning k downwards and stopping at the first match is the same thing.
#define FV3_HD __host__ __device__
#include "common.h"

namespace fv3 {
namespace {

__global__ __launch_bounds__(256) void interpolate_2d_kernel(const double* __restrict__ xp, int64_t ld_xp,
                                                             const double* __restrict__ x, int64_t ld_x,
                                                             const double* __restrict__ y, int64_t ld_y,
                                                             double* __restrict__ out, int64_t ld_out, int64_t ncol,
                                                             int n_in, int n_out, double fill)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncol) return;
    for (int j = 0; j < n_out; ++j) {
        const double p = xp[(int64_t)j * ld_xp + c];
        double r = fill;
        for (int k = n_in - 2; k >= 0; --k) {
            const double x0 = x[(int64_t)k * ld_x + c];
            const double x1 = x[(int64_t)(k + 1) * ld_x + c];
            if (x0 <= p && p < x1) {
                const double w = (p - x0) / (x1 - x0);
                r = y[(int64_t)k * ld_y + c] * (1.0 - w) + y[(int64_t)(k + 1) * ld_y + c] * w;
                break;
            } else if (x0 == p) {
                r = y[(int64_t)k * ld_y + c];
                break;
            } else if (x1 == p) {
                r = y[(int64_t)(k + 1) * ld_y + c];
                break;
            }
        }
        out[(int64_t)j * ld_out + c] = r;
    }
}

// metpy.interpolate.interpolate_1d for ascending column coordinates xp (the reference
// requires x increasing, vcm/interpolate.py:108) and levels sorted ascending:
//   minv = searchsorted(xp, level, 'left'); above = clamp(minv, 1, n-1); below = above-1
//   v = var[below] + (var[above] - var[below]) * ((level - xp[below]) / (xp[above] - xp[below]))
//   fill where minv == n or level < xp[below]
// with numpy's promotion (float64 levels): the coordinate difference in TX, the value
// difference in TV, everything else in float64.  `reverse`: output level j is written
// to n_out-1-j (metpy returns descending-input levels reversed).
template <typename TX, typename TV>
__global__ __launch_bounds__(256) void interpolate_levels_kernel(const TX* __restrict__ xp, int64_t ld_xp,
                                                                 const TV* __restrict__ var, int64_t ld_v,
                                                                 const double* __restrict__ levels, int n_out,
                                                                 int reverse, double* __restrict__ out,
                                                                 int64_t ld_out, int64_t ncol, int n_in, double fill)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncol) return;
    int minv = 0;  // levels ascend, so the insertion point only moves up
    for (int j = 0; j < n_out; ++j) {
        const double lv = levels[j];
        while (minv < n_in && (double)xp[(int64_t)minv * ld_xp + c] < lv) ++minv;
        const int above = minv == n_in ? n_in - 1 : (minv == 0 ? 1 : minv);
        const int below = above - 1;
        const TX xb = xp[(int64_t)below * ld_xp + c], xa = xp[(int64_t)above * ld_xp + c];
        const TV vb = var[(int64_t)below * ld_v + c], va = var[(int64_t)above * ld_v + c];
        const TV dv = va - vb;
        const TX dx = xa - xb;
        const double ratio = (lv - (double)xb) / (double)dx;
        double r = (double)vb + (double)dv * ratio;
        if (minv == n_in || lv < (double)xb) r = fill;
        out[(int64_t)(reverse ? n_out - 1 - j : j) * ld_out + c] = r;
    }
}

// pressure_at_midpoint_log: pi = cumsum([ptop, delp]); out = delp / diff(log(pi)), in T
template <typename T>
__global__ __launch_bounds__(256) void pressure_midpoint_log_kernel(const T* __restrict__ delp, int64_t ld_in,
                                                                    T* __restrict__ out, int64_t ld_out,
                                                                    int64_t ncol, int nz, double ptop)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncol) return;
    T pi = (T)ptop;
    T lp = log(pi);
    for (int k = 0; k < nz; ++k) {
        const T d = delp[(int64_t)k * ld_in + c];
        pi = pi + d;
        const T l1 = log(pi);
        out[(int64_t)k * ld_out + c] = d / (l1 - lp);
        lp = l1;
    }
}

unsigned nblocks(int64_t ncol) { return (unsigned)((ncol + 255) / 256); }

}  // namespace
}  // namespace fv3

extern "C" int fv3_interpolate_2d(const double* xp, int64_t ld_xp, const double* x, int64_t ld_x, const double* y,
                                  int64_t ld_y, double* out, int64_t ld_out, int64_t ncol, int n_in, int n_out,
                                  double fill_value, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ncol >= 0 && n_in >= 1 && n_out >= 0, "interpolate_2d: bad sizes");
    if (ncol == 0 || n_out == 0) return FV3_OK;
    FV3_REQUIRE(xp && x && y && out, "interpolate_2d: NULL array");
    FV3_REQUIRE(ncol < ((int64_t)1 << 40), "interpolate_2d: too many columns");
    hipLaunchKernelGGL(interpolate_2d_kernel, dim3(nblocks(ncol)), dim3(256), 0, (hipStream_t)stream, xp, ld_xp, x,
                       ld_x, y, ld_y, out, ld_out, ncol, n_in, n_out, fill_value);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_interpolate_levels(const void* xp, int64_t ld_xp, const void* var, int64_t ld_v, int dtypes,
                                      const double* levels, int n_out, int reverse, double* out, int64_t ld_out,
                                      int64_t ncol, int n_in, double fill_value, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(dtypes >= 0 && dtypes <= 3, "interpolate_levels: dtypes = xp_f64 | var_f64 << 1");
    FV3_REQUIRE(ncol >= 0 && n_out >= 0, "interpolate_levels: bad sizes");
    FV3_REQUIRE(n_in >= 2, "interpolate_levels: need at least 2 input levels (got %d)", n_in);
    if (ncol == 0 || n_out == 0) return FV3_OK;
    FV3_REQUIRE(xp && var && levels && out, "interpolate_levels: NULL array");
    hipStream_t s = (hipStream_t)stream;
#define FV3_INTERP_LEVELS(TX, TV)                                                                                  \
    hipLaunchKernelGGL((interpolate_levels_kernel<TX, TV>), dim3(nblocks(ncol)), dim3(256), 0, s, (const TX*)xp, \
                       ld_xp, (const TV*)var, ld_v, levels, n_out, reverse, out, ld_out, ncol, n_in, fill_value)
    switch (dtypes) {
        case 0: FV3_INTERP_LEVELS(float, float); break;
        case 1: FV3_INTERP_LEVELS(double, float); break;
        case 2: FV3_INTERP_LEVELS(float, double); break;
        default: FV3_INTERP_LEVELS(double, double); break;
    }
#undef FV3_INTERP_LEVELS
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_pressure_midpoint_log(const void* delp, int dtype, int64_t ld_in, void* out, int64_t ld_out,
                                         int64_t ncol, int nz, double ptop, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(dtype == 0 || dtype == 1, "pressure_midpoint_log: dtype must be 0 (float32) or 1 (float64)");
    FV3_REQUIRE(ncol >= 0 && nz >= 0, "pressure_midpoint_log: bad sizes");
    if (ncol == 0 || nz == 0) return FV3_OK;
    FV3_REQUIRE(delp && out, "pressure_midpoint_log: NULL array");
    hipStream_t s = (hipStream_t)stream;
    if (dtype == 0)
        hipLaunchKernelGGL(pressure_midpoint_log_kernel<float>, dim3(nblocks(ncol)), dim3(256), 0, s,
                           (const float*)delp, ld_in, (float*)out, ld_out, ncol, nz, ptop);
    else
        hipLaunchKernelGGL(pressure_midpoint_log_kernel<double>, dim3(nblocks(ncol)), dim3(256), 0, s,
                           (const double*)delp, ld_in, (double*)out, ld_out, ncol, nz, ptop);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
