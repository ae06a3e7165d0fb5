// fv3net_amd — the rest of coarsen_restarts_on_pressure on gfx950.
//
// The masked pressure-level variables go through the fused regrid_coarsen kernels
// (csrc/coarsen.hip).  What coarsen_restarts_on_pressure
// (external/vcm/vcm/cubedsphere/coarsen_restarts.py:152-225) does besides:
//
//   weighted_block_average_kernel   the plain area-weighted averages of phis, delp, DZ
//                                   (coarsen_restarts.py:439, 480-486) and of the surface
//                                   winds u_srf, v_srf (:890-913):
//                                   sum(obj * w) / sum(w) over f x f blocks
//                                   (cubedsphere/coarsen.py:183-218), obj in its own dtype
//                                   (float64 restart data), w float32, NaN-skipping sums in
//                                   numpy's order (blocks.h).
//   hydrostatic_balance_kernel      _impose_hydrostatic_balance (coarsen_restarts.py:916-938):
//                                   DZ = hydrostatic_dz(T, sphum, delp)
//                                   (calc/thermo/vertically_dependent.py:211-228) and
//                                   phis = g (top height + sum DZ) (:182-186), top height from
//                                   height_at_interface(DZ_coarse, phis_coarse) (:69-100).
//
// Both are HBM-bound elementwise/column passes over the coarse grid or one pass over the
// fine field: one thread per coarse cell (per level) or per coarse column.
#include <cmath>

#include "blocks.h"
#include "common.h"

namespace fv3 {
namespace {

constexpr int kMaxAvgFields = 16;
constexpr double kGravity = 9.80665;  // calc/thermo/constants.py:2
constexpr double kRdGas = 287.05;     // :3
constexpr double kRvGas = 461.5;      // :4

template <typename T>
struct BlockAvgArgs {
    const T* fields[kMaxAvgFields];
    T* out[kMaxAvgFields];
    const float* weights;  // (tile, ny, nx)
    int n_fields, ntile, nz, ny, nx, f;
};

// one thread per coarse cell (tile, k, Y, X) of one field (blockIdx.y)
template <typename T>
__global__ __launch_bounds__(256) void weighted_block_average_kernel(BlockAvgArgs<T> a)
{
    const int nyc = a.ny / a.f, nxc = a.nx / a.f, f = a.f;
    const int64_t n = (int64_t)a.ntile * a.nz * nyc * nxc;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int X = (int)(i % nxc);
    int64_t r = i / nxc;
    const int Y = (int)(r % nyc);
    r /= nyc;
    const int tile = (int)(r / a.nz);  // r = tile * nz + k
    const int64_t plane = (int64_t)a.ny * a.nx;
    const T* src = a.fields[blockIdx.y] + r * plane + (int64_t)(Y * f) * a.nx + (int64_t)X * f;
    const float* w = a.weights + (int64_t)tile * plane + (int64_t)(Y * f) * a.nx + (int64_t)X * f;
    auto at = [&](int j) { return (int64_t)(j / f) * a.nx + j % f; };
    // (obj * weights) in obj's dtype; weights.coarsen().sum() in float32 (coarsen.py:213-215)
    const T num = block_sum<T>(f, [&](int j) { return nan0(src[at(j)] * (T)w[at(j)]); });
    const float den = block_sum<float>(f, [&](int j) { return nan0(w[at(j)]); });
    a.out[blockIdx.y][i] = num / (T)den;
}

struct HydroArgs {
    const float* T;       // coarse temperature (tile, km, ny, nx), float32 (pressure-level path)
    const float* q;       // coarse specific humidity, float32
    const double* delp;   // coarse delp, float64
    const double* dz;     // area-weighted coarse DZ, float64
    const double* phis;   // area-weighted coarse phis (tile, ny, nx), float64
    double* dz_out;       // hydrostatic DZ
    double* phis_out;     // adjusted phis
    int64_t plane;        // ny * nx
    int ntile, km;
    double ptop;
};

// one thread per coarse column; every level load is a coalesced row across the wave
__global__ __launch_bounds__(256) void hydrostatic_balance_kernel(HydroArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)a.ntile * a.plane) return;
    const int64_t tile = i / a.plane, p = i - tile * a.plane;
    const int64_t base = tile * a.km * a.plane + p;
    // height_at_interface (vertically_dependent.py:69-100): reverse cumsum of
    // [-DZ, phis / g] (NaN-skipping, like xarray's cumsum); its top value
    double h = nan0(a.phis[i] / kGravity);
    for (int k = a.km - 1; k >= 0; --k) h = h + nan0(-a.dz[base + (int64_t)k * a.plane]);
    // hydrostatic_dz (:211-228): pi = cumsum([ptop, delp]); tv = T (1 + (Rv/Rd - 1) q) in
    // float32 (a Python float against float32 arrays); dz = -dlogp Rd tv / g in float64
    const float c = (float)(kRvGas / kRdGas - 1.0);
    double pi = a.ptop;
    double lp = log(pi);
    double dzsum = 0.0;
    for (int k = 0; k < a.km; ++k) {
        const int64_t o = base + (int64_t)k * a.plane;
        pi = pi + nan0(a.delp[o]);
        const double lp1 = log(pi);
        const double dlogp = lp1 - lp;
        lp = lp1;
        const float tv = a.T[o] * (1.0f + c * a.q[o]);
        const double dz = -dlogp * kRdGas * (double)tv / kGravity;
        a.dz_out[o] = dz;
        dzsum = dzsum + nan0(dz);  // dz.sum(dim): NaN-skipping, level order
    }
    // dz_and_top_to_phis (:182-186)
    a.phis_out[i] = kGravity * (h + dzsum);
}

template <typename T>
int block_average_impl(const T* const* fields, T* const* out, int n_fields, const float* weights, int ntile, int nz,
                       int ny, int nx, int factor, void* stream)
{
    clear_error();
    FV3_REQUIRE(n_fields >= 0 && n_fields <= kMaxAvgFields, "weighted_block_average: n_fields must be in [0, %d]",
                kMaxAvgFields);
    FV3_REQUIRE(ntile >= 1 && nz >= 1 && ny >= 1 && nx >= 1, "weighted_block_average: bad shape (%d, %d, %d, %d)",
                ntile, nz, ny, nx);
    FV3_REQUIRE(factor >= 1 && factor <= 8, "weighted_block_average: coarsening factor must be in [1, 8]");
    FV3_REQUIRE(ny % factor == 0 && nx % factor == 0, "weighted_block_average: %dx%d not divisible by factor %d",
                ny, nx, factor);
    FV3_REQUIRE(weights, "weighted_block_average: NULL weights");
    if (n_fields == 0) return FV3_OK;
    FV3_REQUIRE(fields && out, "weighted_block_average: NULL field tables");
    BlockAvgArgs<T> a{};
    for (int v = 0; v < n_fields; ++v) {
        FV3_REQUIRE(fields[v] && out[v], "weighted_block_average: NULL field/output %d", v);
        a.fields[v] = fields[v];
        a.out[v] = out[v];
    }
    a.weights = weights;
    a.n_fields = n_fields;
    a.ntile = ntile;
    a.nz = nz;
    a.ny = ny;
    a.nx = nx;
    a.f = factor;
    const int64_t n = (int64_t)ntile * nz * (ny / factor) * (nx / factor);
    const int64_t blocks = (n + 255) / 256;
    FV3_REQUIRE(blocks < (int64_t)0x7fffffff, "weighted_block_average: grid too large");
    hipLaunchKernelGGL((weighted_block_average_kernel<T>), dim3((unsigned)blocks, (unsigned)n_fields), dim3(256), 0,
                       (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_weighted_block_average(const float* const* fields, float* const* out, int n_fields,
                                          const float* weights, int ntile, int nz, int ny, int nx, int factor,
                                          void* stream)
{
    return fv3::block_average_impl<float>(fields, out, n_fields, weights, ntile, nz, ny, nx, factor, stream);
}

extern "C" int fv3_weighted_block_average_f64(const double* const* fields, double* const* out, int n_fields,
                                              const float* weights, int ntile, int nz, int ny, int nx, int factor,
                                              void* stream)
{
    return fv3::block_average_impl<double>(fields, out, n_fields, weights, ntile, nz, ny, nx, factor, stream);
}

extern "C" int fv3_hydrostatic_balance(const float* temperature, const float* sphum, const double* delp,
                                       const double* dz, const double* phis, double* dz_out, double* phis_out,
                                       int ntile, int km, int ny, int nx, double ptop_toa, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ntile >= 1 && km >= 1 && ny >= 1 && nx >= 1, "hydrostatic_balance: bad shape (%d, %d, %d, %d)",
                ntile, km, ny, nx);
    FV3_REQUIRE(temperature && sphum && delp && dz && phis && dz_out && phis_out, "hydrostatic_balance: NULL pointer");
    HydroArgs a{temperature, sphum, delp, dz, phis, dz_out, phis_out, (int64_t)ny * nx, ntile, km, ptop_toa};
    const int64_t n = (int64_t)ntile * ny * nx;
    hipLaunchKernelGGL(hydrostatic_balance_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, a);
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
