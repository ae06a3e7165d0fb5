// fv3net_amd — vertical remap `mappm` on gfx950.
//
// Replaces the f2py-wrapped Fortran mappm (external/mappm/mappm/mappm.f90:10-126)
// as called by vcm.cubedsphere.regrid_vertical (external/vcm/vcm/cubedsphere/regridz.py:273).
//
// One thread per column; the column-fastest [level][column] layout (Fortran's
// pe1(i,k)) makes every per-level load a coalesced 256 B wave access.  The
// per-column algorithm is the one-pass streaming formulation in mappm_core.h:
// kord <= 7 runs entirely in registers (no LDS, no scratch); kord > 7 solves
// cs_profile's tridiagonal edge system into LDS (2 x (km+2) floats per column,
// [level][lane] so every access is bank-conflict free), then streams.
// Roofline: HBM-bound at (km+1 + km + kn+1 + kn) * 4 B per column, with ~150
// VALU ops per input level (including ~7 IEEE divides) close behind.
#define FV3_HD __host__ __device__
#include "common.h"
#include "mappm_core.h"

#include <cstdlib>

namespace fv3 {
namespace {

// The remap consumer emits q2(k) for k = 1, 2, ... and asks for next_edge(k) for
// k = 2, 3, ... strictly in order, so both walk running pointers: no per-lane 64-bit
// index multiply per output level.
struct DevCol {
    const float* pe1_;
    const float* q1_;
    const float* pe2_;
    float* q2_;
    int64_t ld_pe1, ld_q1, ld_pe2, ld_q2;
    int kn;
    const float* pe2_next;  // pe2(k + 1) for the next next_edge(k)
    __device__ __forceinline__ float q1(int k) const { return q1_[(int64_t)(k - 1) * ld_q1]; }
    __device__ __forceinline__ float pe1(int k) const { return pe1_[(int64_t)(k - 1) * ld_pe1]; }
    __device__ __forceinline__ float pe2(int k) const { return pe2_[(int64_t)(k - 1) * ld_pe2]; }
    __device__ __forceinline__ void emit(int, float v)
    {
        *q2_ = v;
        q2_ += ld_q2;
    }
    __device__ __forceinline__ float next_edge(int k)
    {
        if (k + 1 > kn + 1) return 0.0f;
        const float r = *pe2_next;
        pe2_next += ld_pe2;
        return r;
    }
};

struct LdsScr {
    float* base;  // [2][km+3][blockDim]
    int stride;   // blockDim.x
    int plane;    // (km+3) * blockDim.x
    __device__ __forceinline__ float& e(int k) { return base[k * stride]; }
    __device__ __forceinline__ float& g(int k) { return base[plane + k * stride]; }
};

// The same [2][km+3][column] scratch in global memory (stream-ordered allocation):
// coalesced like the column arrays, and unlike LDS (42 KB per 64 columns at km = 79,
// i.e. 3 waves per CU) it leaves occupancy to the VGPR budget.
struct GlobalScr {
    float* base;     // scratch + column
    int64_t stride;  // padded column count
    int64_t plane;   // (km+3) * stride
    __device__ __forceinline__ float& e(int k) { return base[k * stride]; }
    __device__ __forceinline__ float& g(int k) { return base[plane + k * stride]; }
};

struct MappmArgs {
    const float* pe1;
    const float* q1;
    const float* pe2;
    float* q2;
    fv3_layout l_pe1, l_q1, l_pe2, l_q2;
    int64_t ncol;
    int km, kn, iv, kord;
    float* scratch;  // kord > 7: [2][km+3][grid * block] (NULL: the LDS path)
};

__device__ __forceinline__ DevCol make_col(const MappmArgs& a, int64_t c)
{
    DevCol d;
    d.pe1_ = a.pe1 + col_offset(a.l_pe1, c);
    d.q1_ = a.q1 + col_offset(a.l_q1, c);
    d.pe2_ = a.pe2 + col_offset(a.l_pe2, c);
    d.q2_ = a.q2 + col_offset(a.l_q2, c);
    d.ld_pe1 = a.l_pe1.ld;
    d.ld_q1 = a.l_q1.ld;
    d.ld_pe2 = a.l_pe2.ld;
    d.ld_q2 = a.l_q2.ld;
    d.kn = a.kn;
    d.pe2_next = d.pe2_ + 2 * d.ld_pe2;
    return d;
}

__global__ __launch_bounds__(256) void mappm_ppm_kernel(MappmArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    DevCol col = make_col(a, c);
    mappm_ppm_column(col, a.km, a.kn, a.iv, a.kord);
}

__global__ __launch_bounds__(64) void mappm_cs_kernel(MappmArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    LdsScr scr{lds + threadIdx.x, (int)blockDim.x, (a.km + 3) * (int)blockDim.x};
    DevCol col = make_col(a, c);
    mappm_cs_column(col, scr, a.km, a.kn, a.iv, a.kord);
}

__global__ __launch_bounds__(256) void mappm_cs_global_kernel(MappmArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    GlobalScr scr{a.scratch + c, stride, (int64_t)(a.km + 3) * stride};
    DevCol col = make_col(a, c);
    mappm_cs_column(col, scr, a.km, a.kn, a.iv, a.kord);
}

}  // namespace

int launch_mappm(MappmArgs a, hipStream_t stream)
{
    if (a.ncol == 0) return FV3_OK;
    if (a.kord > 7 && !getenv("FV3_MAPPM_LDS")) {
        const int block = 256;
        const int64_t grid = (a.ncol + block - 1) / block;
        FV3_HIP(hipMallocAsync((void**)&a.scratch, sizeof(float) * 2 * (size_t)(a.km + 3) * (size_t)grid * block,
                               stream));
        hipLaunchKernelGGL(mappm_cs_global_kernel, dim3((unsigned)grid), dim3(block), 0, stream, a);
        FV3_LAUNCH_CHECK();
        FV3_HIP(hipFreeAsync(a.scratch, stream));
        return FV3_OK;
    }
    if (a.kord > 7) {
        const int block = 64;
        const size_t lds = sizeof(float) * 2 * (size_t)(a.km + 3) * block;
        FV3_REQUIRE(lds <= 160 * 1024, "mappm: km=%d too large for the kord>7 LDS path", a.km);
        const int64_t grid = (a.ncol + block - 1) / block;
        hipLaunchKernelGGL(mappm_cs_kernel, dim3((unsigned)grid), dim3(block), lds, stream, a);
    } else {
        const int block = 256;
        const int64_t grid = (a.ncol + block - 1) / block;
        hipLaunchKernelGGL(mappm_ppm_kernel, dim3((unsigned)grid), dim3(block), 0, stream, a);
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

}  // namespace fv3

using fv3::MappmArgs;

extern "C" int fv3_mappm_ex(const float* pe1, fv3_layout pe1_l, const float* q1, fv3_layout q1_l,
                            const float* pe2, fv3_layout pe2_l, float* q2, fv3_layout q2_l,
                            int64_t ncol, int km, int kn, int iv, int kord, float ptop,
                            void* stream)
{
    (void)ptop;  // unused by the reference too (regridz.py:270)
    fv3::clear_error();
    FV3_REQUIRE(ncol >= 0, "mappm: ncol must be >= 0 (got %lld)", (long long)ncol);
    FV3_REQUIRE(km >= 4, "mappm: km must be >= 4 (got %d)", km);
    FV3_REQUIRE(kn >= 1, "mappm: kn must be >= 1 (got %d)", kn);
    FV3_REQUIRE(ncol == 0 || (pe1 && q1 && pe2 && q2), "mappm: NULL array");
    FV3_REQUIRE(ncol == 0 || (fv3::layout_ok(pe1_l, ncol) && fv3::layout_ok(q1_l, ncol) &&
                              fv3::layout_ok(pe2_l, ncol) && fv3::layout_ok(q2_l, ncol)),
                "mappm: invalid column layout");
    FV3_REQUIRE(ncol / 256 < (int64_t)0x7fffffff, "mappm: ncol too large");
    MappmArgs a{pe1, q1, pe2, q2, pe1_l, q1_l, pe2_l, q2_l, ncol, km, kn, iv, kord, nullptr};
    return fv3::launch_mappm(a, (hipStream_t)stream);
}

extern "C" int fv3_mappm(const float* pe1, const float* q1, const float* pe2, float* q2,
                         int64_t ncol, int km, int kn, int iv, int kord, float ptop, void* stream)
{
    const fv3_layout l = fv3::plain_layout(ncol > 0 ? ncol : 1);
    return fv3_mappm_ex(pe1, l, q1, l, pe2, l, q2, l, ncol, km, kn, iv, kord, ptop, stream);
}
