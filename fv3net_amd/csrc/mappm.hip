// fv3net_amd — vertical remap `mappm` on gfx950.
//
// Replaces the f2py-wrapped Fortran mappm (external/mappm/mappm/mappm.f90:10-126)
// as called by vcm.cubedsphere.regrid_vertical (external/vcm/vcm/cubedsphere/regridz.py:273).
//
// One thread per column; the column-fastest [level][column] layout (Fortran's
// pe1(i,k)) makes every per-level load a coalesced 256 B wave access.  The
// per-column algorithm is the one-pass streaming formulation in mappm_core.h:
// kord <= 7 runs entirely in registers (no LDS, no scratch) -- or, below
// kLevelsMaxCols columns, one block per column with a lane per level; kord > 7 solves
// cs_profile's tridiagonal edge system into a [2][km+3][column] scratch in global
// memory (coalesced; LDS kept behind FV3_MAPPM_LDS), then streams.
// Roofline: HBM-bound at (km+1 + km + kn+1 + kn) * 4 B per column, with ~150
// VALU ops per input level (including ~7 IEEE divides) close behind.
#define FV3_HD __host__ __device__
#include "common.h"
#include "mappm_core.h"
#include "mappm_multi.h"

#include <algorithm>
#include <cstdlib>

namespace fv3 {

// launch arguments, shared by the exact and the fast-arithmetic translation units
// (mappm.hip, mappm_fast.hip: the same kernels under mappm_core.h's two policies)
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

struct MappmPairArgs {
    const float* pe1;
    const float* pe2;
    fv3_layout l_pe1, l_pe2;
    const float* q1[2];
    float* q2[2];
    fv3_layout l_q1[2], l_q2[2];
    int64_t ncol;
    int km, kn, iv, kord;
};

namespace FV3_ARITH_NS {
int launch_mappm(MappmArgs a, hipStream_t stream);
int launch_mappm_pairs(const MappmPairArgs& a, hipStream_t stream);
}  // namespace FV3_ARITH_NS
#ifndef FV3_FAST_ARITH
namespace fast {  // mappm_fast.hip
int launch_mappm(MappmArgs a, hipStream_t stream);
int launch_mappm_pairs(const MappmPairArgs& a, hipStream_t stream);
}  // namespace fast
#endif

namespace FV3_ARITH_NS {  // kernels named fv3::exact::... / fv3::fast::... in traces
namespace {

// The remap consumer emits q2(k) for k = 1, 2, ... and asks for next_edge(k) for
// k = 2, 3, ... strictly in order, so both walk running pointers: no per-lane 64-bit
// index multiply per output level.
#ifndef FV3_MAPPM_EDGE_AHEAD
#define FV3_MAPPM_EDGE_AHEAD 1  // next_edge's load one call ahead (0: tools A/B builds)
#endif

struct DevCol {
    const float* pe1_;
    const float* q1_;
    const float* pe2_;
    float* q2_;
    int64_t ld_pe1, ld_q1, ld_pe2, ld_q2;
    int kn;
    const float* pe2_next;  // the edge after nb
    float nb;               // pe2(k + 1) for the next next_edge(k), loaded one call ahead
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
#if FV3_MAPPM_EDGE_AHEAD
        const float r = nb;
        pe2_next += ld_pe2;
        nb = (k + 2 <= kn + 1) ? *pe2_next : 0.0f;
#else
        const float r = *pe2_next;
        pe2_next += ld_pe2;
#endif
        return r;
    }
};

// DevCol with buffer loads: q1(k) / pe1(k) at a uniform level k are one
// `buffer_load_dword` of (resource over the array) + (the lane's byte offset, VGPR) +
// (the level's byte offset, SGPR soffset), so every load in flight holds one data VGPR
// and no 64-bit address (DevCol's each hold an address pair, which the compiler does not
// fold into a uniform-base form by itself).  The host checks every array spans < 4 GiB.
// emit / next_edge walk per-lane pointers as in DevCol.
typedef __amdgpu_buffer_rsrc_t MRsrc;
__device__ __forceinline__ MRsrc mrsrc(const void* p)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0xffffffffu, 0x00020000);
}
__device__ __forceinline__ float bload(MRsrc r, uint32_t voff, uint32_t soff)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}

struct DevColBuf {
    MRsrc r_pe1, r_q1;
    uint32_t o_pe1, o_q1;     // lane byte offsets
    uint32_t lb_pe1, lb_q1;   // level strides in bytes
    const float* pe2_;
    float* q2_;
    int64_t ld_pe2, ld_q2;
    int kn;
    const float* pe2_next;  // the edge after nb
    float nb;               // pe2(k + 1) for the next next_edge(k), loaded one call ahead
    __device__ __forceinline__ float q1(int k) const { return bload(r_q1, o_q1, (uint32_t)(k - 1) * lb_q1); }
    __device__ __forceinline__ float pe1(int k) const { return bload(r_pe1, o_pe1, (uint32_t)(k - 1) * lb_pe1); }
    __device__ __forceinline__ float pe2(int k) const { return pe2_[(int64_t)(k - 1) * ld_pe2]; }
    __device__ __forceinline__ void emit(int, float v)
    {
        *q2_ = v;
        q2_ += ld_q2;
    }
    __device__ __forceinline__ float next_edge(int k)
    {
        if (k + 1 > kn + 1) return 0.0f;
#if FV3_MAPPM_EDGE_AHEAD
        const float r = nb;
        pe2_next += ld_pe2;
        nb = (k + 2 <= kn + 1) ? *pe2_next : 0.0f;
#else  // A/B variant builds: loaded at the call
        const float r = *pe2_next;
        pe2_next += ld_pe2;
#endif
        return r;
    }
};

// GlobalScr through buffer loads / stores (the host checks the scratch is < 4 GiB);
// e(k) / g(k) are proxies: read as a float, assigned by a store
struct GlobalScrBuf {
    MRsrc r;
    uint32_t o;   // lane byte offset
    uint32_t sb;  // level stride in bytes
    uint32_t pb;  // plane stride in bytes
    struct Ref {
        MRsrc r;
        uint32_t o, so;
        __device__ __forceinline__ operator float() const { return bload(r, o, so); }
        __device__ __forceinline__ Ref& operator=(float v)
        {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)o, (int)so, 0);
            return *this;
        }
    };
    __device__ __forceinline__ Ref e(int k) const { return Ref{r, o, (uint32_t)k * sb}; }
    __device__ __forceinline__ Ref g(int k) const { return Ref{r, o, pb + (uint32_t)k * sb}; }
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
    d.nb = d.kn >= 2 ? *d.pe2_next : 0.0f;
    return d;
}

// DevColBuf of column c: q1 / pe1 through buffer loads at 32-bit offsets (the host checks
// fits_c32), pe2 / q2 through per-lane pointers as in DevCol
__device__ __forceinline__ DevColBuf make_col_buf(const MappmArgs& a, int64_t c)
{
    DevColBuf d;
    d.r_pe1 = mrsrc(a.pe1);
    d.r_q1 = mrsrc(a.q1);
    d.o_pe1 = (uint32_t)(col_offset(a.l_pe1, c) * 4);
    d.o_q1 = (uint32_t)(col_offset(a.l_q1, c) * 4);
    d.lb_pe1 = (uint32_t)(a.l_pe1.ld * 4);
    d.lb_q1 = (uint32_t)(a.l_q1.ld * 4);
    d.pe2_ = a.pe2 + col_offset(a.l_pe2, c);
    d.q2_ = a.q2 + col_offset(a.l_q2, c);
    d.ld_pe2 = a.l_pe2.ld;
    d.ld_q2 = a.l_q2.ld;
    d.kn = a.kn;
    d.pe2_next = d.pe2_ + 2 * d.ld_pe2;
    d.nb = a.kn >= 2 ? *d.pe2_next : 0.0f;
    return d;
}

// buffer operations at 32-bit byte offsets reach every element of an array in layout l
// over ncol columns and nlev levels: its last column's offset plus nlev levels < 4 GiB
inline bool fits_c32(const fv3_layout& l, int64_t ncol, int nlev)
{
    if (l.ld < 0 || l.blk_stride < 0) return false;
    const int64_t c = ncol - 1;
    const int64_t off = (l.ncol_blk <= 0 || c < l.ncol_blk) ? c : (c / l.ncol_blk) * l.blk_stride + c % l.ncol_blk;
    return 4 * (off + (int64_t)nlev * l.ld) < (1ll << 32) - 4;
}

// the single-field column's window in register rings (mappm_core.h, RING): on the fast
// arithmetic only, where it measured faster (0.384 -> 0.367 ms at C384 kord 1)
#ifdef FV3_FAST_ARITH
constexpr bool kRingWindow = true;
#else
constexpr bool kRingWindow = false;
#endif

// K1: kord 1 and iv 1 (the default of regrid_vertical and of the pressure-level coarsen)
// as compile-time constants, so every branch of mappm.f90 on kord / iv folds away
// BUF: q1 / pe1 through buffer loads at SGPR level offsets (DevColBuf), when every array
// fits 32-bit offsets; else 64-bit addresses.  C384 kord 1: fast 0.370 -> 0.368 ms, exact
// 0.501 -> 0.497 (profiles/r06zt_mappm_buf_ab.log)
#ifndef FV3_MAPPM_PPM_WPE
#define FV3_MAPPM_PPM_WPE 0  // register target in waves per SIMD (0: the compiler's, 66 VGPRs, 7 waves;
                             // 8 spills 5 and measured 0.365 -> 0.398 ms, profiles/r06zu_mappm_wpe_ab.log)
#endif
#if FV3_MAPPM_PPM_WPE
#define FV3_PPM_WPE_ATTR __attribute__((amdgpu_waves_per_eu(FV3_MAPPM_PPM_WPE, FV3_MAPPM_PPM_WPE)))
#else
#define FV3_PPM_WPE_ATTR
#endif
template <bool K1, bool BUF>
__global__ __launch_bounds__(256) FV3_PPM_WPE_ATTR void mappm_ppm_kernel(MappmArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    if constexpr (BUF) {
        DevColBuf col = make_col_buf(a, c);
        mappm_ppm_column<DevColBuf, true, true, kRingWindow>(col, a.km, a.kn, K1 ? 1 : a.iv, K1 ? 1 : a.kord);
    } else {
        DevCol col = make_col(a, c);
        mappm_ppm_column<DevCol, true, true, kRingWindow>(col, a.km, a.kn, K1 ? 1 : a.iv, K1 ? 1 : a.kord);
    }
}

bool is_k1(int iv, int kord) { return iv == 1 && kord == 1; }

// tools/ab.py, kord 1 79->79: C48 (13,824 columns) 142 -> 38 us, C96
// (55,296) 168 -> 118 us; at C384 the serial kernel (0.70 ms) wins.
constexpr int64_t kLevelsMaxCols = 65536;

// No-op edge source for remap_one (the level-parallel kernel finishes one output
// layer per lane, so the next edge is never read).
struct NoEdge {
    __device__ __forceinline__ float next_edge(int) const { return 0.0f; }
};

// kord <= 7 with one BLOCK per column and one lane per level: the latency-bound
// case (config #1: 864 columns = 14 waves of the one-lane-per-column kernel, each
// walking 79 levels serially).  ppm_profile is a local stencil, so each phase below
// evaluates one of mappm_ppm_column's per-level expressions for every level at once,
// with the same helpers and operands, into LDS; the remap then gives each output
// layer its own lane, which replays remap_one over the input layers it overlaps
// (mappm.f90:58-124 for one k).  The streaming code starts output k's layer search
// where output k-1 ended; with non-decreasing pe1 and pe2 that is the first L with
// pe2(k) <= pe1(L+1), found here by bisection.  A column whose edges are not
// non-decreasing (or hold NaNs) runs the serial streaming code on lane 0 instead, so
// every input gives the serial kernel's (bit-exact) result.
//
// LDS: 9 (km+2) + (kn+2) floats, 1-based levels.
__global__ __launch_bounds__(128) void mappm_ppm_levels_kernel(MappmArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int km = a.km, kn = a.kn, n = km + 2;
    const int tid = threadIdx.x, nt = blockDim.x;
    float* const q = lds;
    float* const pe = lds + n;
    float* const dp = lds + 2 * n;
    float* const dc = lds + 3 * n;
    float* const al = lds + 4 * n;  // AL(k); al[km+1] holds ar_km
    float* const h2 = lds + 5 * n;
    float* const pal = lds + 6 * n;  // final layer coefficients
    float* const par = lds + 7 * n;
    float* const pa6 = lds + 8 * n;
    float* const pe2 = lds + 9 * n;
    const int64_t c = blockIdx.x;
    DevCol col = make_col(a, c);

    for (int k = tid + 1; k <= km + 1; k += nt) {
        pe[k] = col.pe1(k);
        if (k <= km) q[k] = col.q1(k);
    }
    for (int k = tid + 1; k <= kn + 1; k += nt) pe2[k] = col.pe2(k);
    __syncthreads();
    int sorted = 1;
    for (int k = tid + 1; k <= km; k += nt) {
        dp[k] = pe[k + 1] - pe[k];
        sorted &= pe[k] <= pe[k + 1];
    }
    for (int k = tid + 1; k <= kn; k += nt) sorted &= pe2[k] <= pe2[k + 1];
    if (!__syncthreads_and(sorted)) {
        if (tid == 0) mappm_ppm_column(col, km, kn, a.iv, a.kord);
        return;
    }
    const int iv = a.iv, kord = a.kord;
    const bool huynh = kord >= 7;
    // dc(k), k = 2..km-1 (mappm.f90:658-668)
    for (int k = tid + 2; k <= km - 1; k += nt) dc[k] = ppm_dc(q[k - 1], q[k], q[k + 1], dp[k - 1], dp[k], dp[k + 1]);
    __syncthreads();
    // ALraw(m), m = 3..km-1 (mappm.f90:674-683)
    for (int m = tid + 3; m <= km - 1; m += nt)
        al[m] = ppm_al(dp[m - 2], dp[m - 1], dp[m], dp[m + 1], q[m - 1], q[m], dc[m - 1], dc[m]);
    __syncthreads();
    if (tid == 0) {  // top: area-preserving cubic (mappm.f90:689-725), as in mappm_ppm_column
        float al1, al2, dc1;
        ppm_top_cubic(q[1], q[2], dp[1], dp[2], al[3], iv, al1, al2, dc1);
        dc[1] = dc1;
        al[1] = al1;
        al[2] = al2;
    }
    if (tid == (1 % nt)) {  // bottom: area-preserving cubic (mappm.f90:729-761)
        float alm, ar, dcm;
        ppm_bottom_cubic(q[km], q[km - 1], dp[km], dp[km - 1], al[km - 1], iv, alm, ar, dcm);
        dc[km] = dcm;
        al[km] = alm;
        al[km + 1] = ar;
    }
    __syncthreads();
    if (huynh) {  // h2(k), k = 2..km-1 (mappm.f90:784-795)
        for (int k = tid + 2; k <= km - 1; k += nt) h2[k] = ppm_h2(dc[k - 1], dc[k + 1], dp[k - 1], dp[k], dp[k + 1]);
        __syncthreads();
    }
    int lmt = kord - 3;
    lmt = lmt > 0 ? lmt : 0;
    if (iv == 0) lmt = lmt < 2 ? lmt : 2;
    // final coefficients of every layer (the top of mappm_ppm_column's L loop)
    for (int L = tid + 1; L <= km; L += nt) {
        Ppm p{q[L], al[L], al[L + 1], 0.0f};  // al[km+1] = ar_km
        const float dcL = dc[L];
        if (L <= 2 || L >= km - 1) {
            p.a6 = a6_of(p);
            ppm_limit(dcL, p, 0);
        } else if (huynh) {
            ppm_huynh(p, dcL, h2[L - 1], h2[L + 1]);
            if (iv == 0) ppm_limit(dcL, p, 2);
        } else {
            if (kord != 4) p.a6 = a6_of(p);
            if (kord != 6) ppm_limit(dcL, p, lmt);
        }
        pal[L] = p.al;
        par[L] = p.ar;
        pa6[L] = p.a6;
    }
    __syncthreads();
    // one output layer per lane
    const ColumnEnds ends{pe[1], pe[km + 1], q[1], q[km]};
    NoEdge none;
    for (int k = tid + 1; k <= kn; k += nt) {
        RemapState s{k, false, 0.0f, 0.0f, pe2[k], pe2[k + 1]};
        float val = 0.0f;
        bool done = false;
        if (!(s.t <= ends.pe_top) && !(s.t >= ends.pe_bot)) {
            int lo = 1, hi = km;  // first L in [1, km] with t <= pe1(L+1); exists since t < pe_bot
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s.t <= pe[mid + 1]) hi = mid; else lo = mid + 1;
            }
            for (int L = lo; L <= km && !done; ++L) {
                const LayerView v{pe[L], pe[L + 1], dp[L], q[L], Ppm{q[L], pal[L], par[L], pa6[L]}};
                done = remap_one(s, v, ends, none, val);
            }
            if (!done) {  // below the last input layer (mappm.f90:115-121); s.accum is set here
                const float delp = s.b - ends.pe_bot;
                if (delp > 0.0f) {
                    s.qsum = s.qsum + delp * ends.q_bot;
                    s.dpsum = s.dpsum + delp;
                }
                val = FV3_DIVQ(s.qsum, s.dpsum);
            }
        } else {
            val = (s.t <= ends.pe_top) ? ends.q_top : ends.q_bot;
        }
        col.q2_[(int64_t)(k - 1) * col.ld_q2] = val;
    }
}

#ifdef FV3_FAST_ARITH
#define FV3_MAPPM_CS 0  // kord > 7 always takes the exact kernels (launch_arith): none here
#else
#define FV3_MAPPM_CS 1
#endif

#if FV3_MAPPM_CS && FV3_VARIANT_KERNELS  // the solve's scratch in LDS (A/B: FV3_MAPPM_LDS)
__global__ __launch_bounds__(64) void mappm_cs_kernel(MappmArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    LdsScr scr{lds + threadIdx.x, (int)blockDim.x, (a.km + 3) * (int)blockDim.x};
    DevCol col = make_col(a, c);
    mappm_cs_column(col, scr, a.km, a.kn, a.iv, a.kord);
}
#endif

#if FV3_MAPPM_CS
// NT > 0: the bottom NT edges of the solve stay in registers (mappm_cs_column), 6 NT
// fewer scratch accesses per column; the scratch keeps its full [2][km+3] shape
// PF > 0: loads run PF levels ahead in the solve, one layer ahead in the main loop
// (mappm_cs_column).  C32: buffer loads / stores at 32-bit offsets (DevColBuf / GlobalScrBuf).
template <int NT, int PF, bool C32, int KORD = 0>
__global__ __launch_bounds__(256) void mappm_cs_global_kernel(MappmArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if constexpr (C32) {
        GlobalScrBuf scr{mrsrc(a.scratch), (uint32_t)(c * 4), (uint32_t)(stride * 4),
                         (uint32_t)((a.km + 3) * stride * 4)};
        DevColBuf d = make_col_buf(a, c);
        mappm_cs_column<DevColBuf, GlobalScrBuf, NT, PF, KORD>(d, scr, a.km, a.kn, a.iv, a.kord);
    } else {
        GlobalScr scr{a.scratch + c, stride, (int64_t)(a.km + 3) * stride};
        DevCol col = make_col(a, c);
        mappm_cs_column<DevCol, GlobalScr, NT, PF>(col, scr, a.km, a.kn, a.iv, a.kord);
    }
}

// register-tail depth of the kord > 7 kernel (every depth gives the same bits).  Measured
// on MI355X (tools/ab.py, profiles/r04c_mappm_nt.log), C384 79 -> 79: at
// 884,736 columns NT = 0 / 16 / 32 / 48 take 0.89 / 0.97 / 1.12 / 1.24 ms (the registers
// cost occupancy: 60 -> 78 / 100 / 132 VGPRs, 8 -> 6 / 4 / 3 waves per SIMD, and the
// launch needs it more than the scratch bytes saved); at one rank's 110,592 columns,
// where occupancy is not the limit, 0.232 / 0.223 / 0.218 / 0.212 ms.  So the tail is
// used on small grids only.  FV3_MAPPM_CS_NT=0|16|32|48 forces a depth (A/B).
const void* cs_global_kernel(const MappmArgs& a, int64_t nlanes)
{
    const int64_t ncol = a.ncol;
    int nt = ncol < 262144 ? 48 : 0;
    // load distance (tools/ab.py; C384 79 -> 79 kord 10, buffer operations):
    // before the rolling subgrid flags (profiles/r04l_mappm_pf.log) 884,736 columns PF =
    // 0 / 2 / 4 / 8 0.909 / 0.761 / 0.798 / 0.836 ms (64-bit addresses, PF = 0: 0.871),
    // 110,592 columns (register tail) 0.224 / 0.185 / 0.182 / 0.182 ms; with them
    // (profiles/r04q_mappm_kord_ab.log) PF = 2 / 4 0.772 / 0.765 ms and 0.175 / 0.170 ms
    int pf = 4;
#if FV3_VARIANT_KERNELS
    if (const char* e = fv3::variant_env("FV3_MAPPM_CS_NT")) nt = atoi(e);
    if (const char* e = fv3::variant_env("FV3_MAPPM_CS_PF")) pf = atoi(e);
#endif
    // buffer operations at 32-bit byte offsets when every array (and the scratch) spans
    // < 4 GiB: the last column's offset plus km levels
    auto fits = [&](const fv3_layout& l, int nlev) { return fits_c32(l, ncol, nlev); };
    bool c32 = fits(a.l_pe1, a.km + 1) && fits(a.l_q1, a.km) && 4 * nlanes * 2 * (int64_t)(a.km + 3) < (1ll << 32) - 4;
    if (const char* e = fv3::variant_env("FV3_MAPPM_CS_C32")) c32 = c32 && atoi(e) != 0;
#if FV3_VARIANT_KERNELS  // the other depths and load distances (A/B)
#define FV3_CS_PF(NT_, C_)                                                        \
    switch (pf) {                                                                 \
    case 0: return (const void*)mappm_cs_global_kernel<NT_, 0, C_>;               \
    case 4: return (const void*)mappm_cs_global_kernel<NT_, 4, C_>;               \
    case 8: return (const void*)mappm_cs_global_kernel<NT_, 8, C_>;               \
    default: return (const void*)mappm_cs_global_kernel<NT_, 2, C_>;              \
    }
    if (pf != 4 || (nt != 0 && nt != 48)) {
        if (c32) {
            if (nt == 8) { FV3_CS_PF(8, true) }
            if (nt == 16) { FV3_CS_PF(16, true) }
            if (nt) { FV3_CS_PF(48, true) } else { FV3_CS_PF(0, true) }
        }
        if (nt) { FV3_CS_PF(48, false) }
        FV3_CS_PF(0, false)
    }
#undef FV3_CS_PF
#endif
    // kord 10 under the register tail at the default load distance: the column
    // specialised for it (0.170 -> 0.168 ms at 110,592 columns; on the full grid the
    // specialised build measured slower, 0.772 -> 0.806 ms at PF = 2, so it is not used
    // there; profiles/r04q_mappm_kord_ab.log).  FV3_MAPPM_CS_KORD=0: the generic column.
    const char* ke = fv3::variant_env("FV3_MAPPM_CS_KORD");
    if (c32 && nt == 48 && (a.kord == 10 || a.kord == -10) && !(ke && atoi(ke) == 0))
        return (const void*)mappm_cs_global_kernel<48, 4, true, 10>;
    if (c32) return nt ? (const void*)mappm_cs_global_kernel<48, 4, true> : (const void*)mappm_cs_global_kernel<0, 4, true>;
    return nt ? (const void*)mappm_cs_global_kernel<48, 4, false> : (const void*)mappm_cs_global_kernel<0, 4, false>;
}
#endif  // FV3_MAPPM_CS

}  // namespace



// kord <= 7: the level-parallel kernel while one lane per column leaves the chip
// mostly idle (FV3_MAPPM_PATH=serial|levels overrides, for tests and A/B).
bool use_levels_kernel(const MappmArgs& a, int64_t max_cols = kLevelsMaxCols)
{
    const char* p = fv3::variant_env("FV3_MAPPM_PATH");
    if (p && p[0] == 's') return false;
    if (a.km > 1000 || a.kn > 1000) return false;
    if (p && p[0] == 'l') return true;
    return a.ncol < max_cols;
}

// Pairs of fields: the pair kernel on two or three lanes per column beats the
// level-parallel kernel (one field per launch) from ~10,000 columns
// (tools/ab.py, profiles/r05zr_mappm_small_lanes.log and
// r05zs_mappm_small_lanes.log, two fields, levels / three lanes: 6,912 columns 47 / 59 us,
// 10,368 63 / 59 us, C48 13,824 77 / 60 us, C96 55,296 252 / 86 us)
constexpr int64_t kLevelsMaxColsPairs = 10240;

bool launch_split_single(const MappmArgs& a, hipStream_t stream);  // below the split kernels

int launch_mappm(MappmArgs a, hipStream_t stream)
{
    if (a.ncol == 0) return FV3_OK;
#if FV3_MAPPM_CS
    if (a.kord > 7 && !(FV3_VARIANT_KERNELS && fv3::variant_env("FV3_MAPPM_LDS"))) {
        const int block = 256;
        const int64_t grid = (a.ncol + block - 1) / block;
        FV3_HIP(hipMallocAsync((void**)&a.scratch, sizeof(float) * 2 * (size_t)(a.km + 3) * (size_t)grid * block,
                               stream));
        void* kargs[] = {&a};
        FV3_HIP(hipLaunchKernel(cs_global_kernel(a, grid * block), dim3((unsigned)grid), dim3(block), kargs, 0, stream));
        FV3_LAUNCH_CHECK();
        FV3_HIP(hipFreeAsync(a.scratch, stream));
        return FV3_OK;
    }
#endif
    if (a.kord > 7) {
#if FV3_MAPPM_CS && FV3_VARIANT_KERNELS
        const int block = 64;
        const size_t lds = sizeof(float) * 2 * (size_t)(a.km + 3) * block;
        FV3_REQUIRE(lds <= 160 * 1024, "mappm: km=%d too large for the kord>7 LDS path", a.km);
        const int64_t grid = (a.ncol + block - 1) / block;
        hipLaunchKernelGGL(mappm_cs_kernel, dim3((unsigned)grid), dim3(block), lds, stream, a);
#else
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, false, "mappm: kord > 7 runs on the exact kernels only");
#endif
    } else if (launch_split_single(a, stream)) {
        // one field on two or three lanes per column
    } else if (use_levels_kernel(a)) {
        const int block = a.km + 1 > 64 ? 128 : 64;
        const size_t lds = sizeof(float) * (9 * (size_t)(a.km + 2) + (size_t)(a.kn + 2));
        FV3_REQUIRE(lds <= 64 * 1024, "mappm: km=%d kn=%d too large for the level-parallel path", a.km, a.kn);
        FV3_REQUIRE(a.ncol <= 0x7fffffff, "mappm: ncol too large for the level-parallel path");
        hipLaunchKernelGGL(mappm_ppm_levels_kernel, dim3((unsigned)a.ncol), dim3(block), lds, stream, a);
    } else {
        const int block = 256;
        const int64_t grid = (a.ncol + block - 1) / block;
        // q1 / pe1 by buffer loads wherever they fit 32-bit offsets (FV3_MAPPM_PPM_BUF=0:
        // 64-bit addresses, A/B)
        bool buf = fits_c32(a.l_pe1, a.ncol, a.km + 1) && fits_c32(a.l_q1, a.ncol, a.km);
        if (const char* e = fv3::variant_env("FV3_MAPPM_PPM_BUF")) buf = buf && atoi(e) != 0;
        const bool k1 = is_k1(a.iv, a.kord);
        const void* kfn = k1 ? (buf ? (const void*)mappm_ppm_kernel<true, true> : (const void*)mappm_ppm_kernel<true, false>)
                             : (buf ? (const void*)mappm_ppm_kernel<false, true> : (const void*)mappm_ppm_kernel<false, false>);
        void* kargs[] = {&a};
        FV3_HIP(hipLaunchKernel(kfn, dim3((unsigned)grid), dim3(block), kargs, 0, stream));
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

// ---- two fields on one column's edges (fv3_mappm_multi) ----

// DevCol for mappm_ppm_columns<NF> (NF = 1, 2): fields f emit output k in turn, so each
// keeps its own running output pointer
template <int NF>
struct DevColN {
    const float* pe1_;
    const float* pe2_;
    const float* q1_[NF];
    float* q2_[NF];
    int64_t ld_pe1, ld_pe2, ld_q1[NF], ld_q2[NF];
    int kn;
    const float* pe2_next;
    float nb;  // as DevCol::nb
    __device__ __forceinline__ float q1(int f, int k) const { return q1_[f][(int64_t)(k - 1) * ld_q1[f]]; }
    __device__ __forceinline__ float pe1(int k) const { return pe1_[(int64_t)(k - 1) * ld_pe1]; }
    __device__ __forceinline__ float pe2(int k) const { return pe2_[(int64_t)(k - 1) * ld_pe2]; }
    __device__ __forceinline__ void emit(int f, int, float v)
    {
        *q2_[f] = v;
        q2_[f] += ld_q2[f];
    }
    __device__ __forceinline__ float next_edge(int k)
    {
        if (k + 1 > kn + 1) return 0.0f;
#if FV3_MAPPM_EDGE_AHEAD
        const float r = nb;
        pe2_next += ld_pe2;
        nb = (k + 2 <= kn + 1) ? *pe2_next : 0.0f;
#else
        const float r = *pe2_next;
        pe2_next += ld_pe2;
#endif
        return r;
    }
};
using DevColPair = DevColN<2>;

template <bool K1>
__global__ __launch_bounds__(256) void mappm_ppm_pair_kernel(MappmPairArgs a)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.ncol) return;
    DevColPair d;
    d.pe1_ = a.pe1 + col_offset(a.l_pe1, c);
    d.pe2_ = a.pe2 + col_offset(a.l_pe2, c);
    d.ld_pe1 = a.l_pe1.ld;
    d.ld_pe2 = a.l_pe2.ld;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        d.q1_[f] = a.q1[f] + col_offset(a.l_q1[f], c);
        d.q2_[f] = a.q2[f] + col_offset(a.l_q2[f], c);
        d.ld_q1[f] = a.l_q1[f].ld;
        d.ld_q2[f] = a.l_q2[f].ld;
    }
    d.kn = a.kn;
    d.pe2_next = d.pe2_ + 2 * d.ld_pe2;
    d.nb = d.kn >= 2 ? *d.pe2_next : 0.0f;
#ifndef FV3_MAPPM_PAIR_CARRY
#define FV3_MAPPM_PAIR_CARRY 1  // 0: tools A/B builds
#endif
    mappm_ppm_columns<2, DevColPair, FV3_MAPPM_PAIR_CARRY != 0>(d, a.km, a.kn, K1 ? 1 : a.iv, K1 ? 1 : a.kord);
}

// Small grids with one lane per column left the SIMDs short of waves (one rank's share
// of C384 at world 8, 110,592 columns: 1.7 waves per SIMD, the serial remap's latency
// unhidden).  Here each column runs on TWO lanes: the first streams outputs 1 .. kB - 1,
// the second kB .. kn from the input layer where the single pass begins output kB
// (mappm_multi.h, "two lanes per column").  A block is two waves over the same 64
// columns, wave 0 the first halves and wave 1 the second, so every lane of a wave is in
// the same phase of its column (neighbouring columns' remap events mostly coincide; with
// the halves mixed in one wave they diverge at every level).  The second lane finds its
// start layer in two rounds of loads; both lanes check the sortedness that start layer
// relies on on the edges they stream, and after the block barrier the first lane re-runs
// the single pass on any column the checks did not prove (unsorted or NaN edges).  The
// host runs this kernel for kn >= 2 only, on NF = 2 fields (fv3_mappm_multi's pairs) or
// one (fv3_mappm_ex).
template <int NF, bool K1>
__global__ __launch_bounds__(128) void mappm_ppm_pair_split_kernel(MappmPairArgs a)
{
    const int iv = K1 ? 1 : a.iv, kord = K1 ? 1 : a.kord;
    __shared__ int s_ok[64], s_l0[64];
    const int lane = threadIdx.x & 63;
    const int part = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = c0 < a.ncol;
    const int64_t c = valid ? c0 : a.ncol - 1;  // spare lanes only pass the barrier
    DevColN<NF> d;
    d.pe1_ = a.pe1 + col_offset(a.l_pe1, c);
    d.pe2_ = a.pe2 + col_offset(a.l_pe2, c);
    d.ld_pe1 = a.l_pe1.ld;
    d.ld_pe2 = a.l_pe2.ld;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        d.q1_[f] = a.q1[f] + col_offset(a.l_q1[f], c);
        d.q2_[f] = a.q2[f] + col_offset(a.l_q2[f], c);
        d.ld_q1[f] = a.l_q1[f].ld;
        d.ld_q2[f] = a.l_q2[f].ld;
    }
    d.kn = a.kn;
    const int km = a.km, kn = a.kn;
    const int kB = kn / 2 + 1;
    // this lane's outputs [kf, kl] and first input layer (one call site for every lane)
    int kf = 1, kl = kB - 1, Lf = 1;
    if (part == 1) {
        kf = kB;
        kl = kn;
        const float t = d.pe2(kB);
        Lf = split_first_layer(d, km, t, split_count_sorted(d, km, t));
    }
    SplitCheck chk{1, km};
    if (valid) {
        // the output pointers and the edge cursor where the single pass has them once
        // output kf - 1 is written
        float* q2c[NF];
        for (int f = 0; f < NF; ++f) {
            q2c[f] = d.q2_[f];
            d.q2_[f] += (int64_t)(kf - 1) * d.ld_q2[f];
        }
        d.pe2_next = d.pe2_ + (int64_t)(kf + 1) * d.ld_pe2;
        d.nb = (kf + 2 <= kn + 1) ? *d.pe2_next : 0.0f;
        mappm_ppm_columns<NF, DevColN<NF>, FV3_MAPPM_PAIR_CARRY != 0, true>(d, km, kn, iv, kord, kf, kl, Lf, &chk);
        for (int f = 0; f < NF; ++f) d.q2_[f] = q2c[f];
    }
    if (part == 1) {
        s_ok[lane] = chk.mono;
        s_l0[lane] = Lf;
    }
    __syncthreads();
    if (part == 0 && valid && !split_exact(chk, SplitCheck{s_ok[lane], km}, s_l0[lane], km)) {
        // the fix-up: this column's single pass, over what the halves wrote
        d.pe2_next = d.pe2_ + 2 * d.ld_pe2;
        d.nb = kn >= 2 ? *d.pe2_next : 0.0f;
        mappm_ppm_columns<NF, DevColN<NF>, FV3_MAPPM_PAIR_CARRY != 0>(d, km, kn, iv, kord);
    }
}

// The same on THREE lanes per column (three waves over 64 columns; outputs split at
// kB1 = kn / 3 + 1 and kB2 = 2 kn / 3 + 1, each later lane starting where the single pass
// begins its first output): more waves for grids too small to fill the SIMDs even on
// two.  The host runs it for kn >= 3 only.
template <int NF, bool K1>
__global__ __launch_bounds__(192) void mappm_ppm_pair_split3_kernel(MappmPairArgs a)
{
    const int iv = K1 ? 1 : a.iv, kord = K1 ? 1 : a.kord;
    __shared__ int s_ok[2][64], s_l0[2][64], s_exit[64];
    const int lane = threadIdx.x & 63;
    const int part = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = c0 < a.ncol;
    const int64_t c = valid ? c0 : a.ncol - 1;  // spare lanes only pass the barrier
    DevColN<NF> d;
    d.pe1_ = a.pe1 + col_offset(a.l_pe1, c);
    d.pe2_ = a.pe2 + col_offset(a.l_pe2, c);
    d.ld_pe1 = a.l_pe1.ld;
    d.ld_pe2 = a.l_pe2.ld;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        d.q1_[f] = a.q1[f] + col_offset(a.l_q1[f], c);
        d.q2_[f] = a.q2[f] + col_offset(a.l_q2[f], c);
        d.ld_q1[f] = a.l_q1[f].ld;
        d.ld_q2[f] = a.l_q2[f].ld;
    }
    d.kn = a.kn;
    const int km = a.km, kn = a.kn;
    const int kB1 = kn / 3 + 1, kB2 = 2 * kn / 3 + 1;
    int kf = 1, kl = kB1 - 1, Lf = 1;
    if (part > 0) {
        kf = part == 1 ? kB1 : kB2;
        kl = part == 1 ? kB2 - 1 : kn;
        const float t = d.pe2(kf);
        Lf = split_first_layer(d, km, t, split_count_sorted(d, km, t));
    }
    SplitCheck chk{1, km};
    if (valid) {
        float* q2c[NF];
        for (int f = 0; f < NF; ++f) {
            q2c[f] = d.q2_[f];
            d.q2_[f] += (int64_t)(kf - 1) * d.ld_q2[f];
        }
        d.pe2_next = d.pe2_ + (int64_t)(kf + 1) * d.ld_pe2;
        d.nb = (kf + 2 <= kn + 1) ? *d.pe2_next : 0.0f;
        mappm_ppm_columns<NF, DevColN<NF>, FV3_MAPPM_PAIR_CARRY != 0, true>(d, km, kn, iv, kord, kf, kl, Lf, &chk);
        for (int f = 0; f < NF; ++f) d.q2_[f] = q2c[f];
    }
    if (part > 0) {
        s_ok[part - 1][lane] = chk.mono;
        s_l0[part - 1][lane] = Lf;
    }
    if (part == 1) s_exit[lane] = chk.l_exit;
    __syncthreads();
    if (part == 0 && valid &&
        !split3_exact(chk, SplitCheck{s_ok[0][lane], s_exit[lane]}, SplitCheck{s_ok[1][lane], km}, s_l0[0][lane],
                      s_l0[1][lane], km)) {
        // the fix-up: this column's single pass, over what the lanes wrote
        d.pe2_next = d.pe2_ + 2 * d.ld_pe2;
        d.nb = kn >= 2 ? *d.pe2_next : 0.0f;
        mappm_ppm_columns<NF, DevColN<NF>, FV3_MAPPM_PAIR_CARRY != 0>(d, km, kn, iv, kord);
    }
}

// Where the two-lane kernel pays (tools/ab.py, one box, interleaved; one
// lane per column vs two).  With whole-column sortedness scans up front
// (profiles/r05r_mappm_split.log): 65,536 columns 142.7 vs 115.4 us, 110,592 (one rank's
// C384 band at world 8) 165.7 vs 161.5 us, 147,456 213 vs 228 us, C384 0.78 vs 1.06 ms.
// With the start layer searched and the checks on the streamed edges
// (profiles/r05zi_mappm_split.log): 65,536 columns 142.7 vs 99 us, 110,592 165.8 vs
// 142 us, 147,456 215 vs 215 us, 221,184 262 vs 280 us, C384 0.78 vs 0.93 ms.  Above the
// level-parallel kernel's range and below kSplitMaxCols columns it runs by default;
// FV3_MAPPM_SPLIT=0|1 forces it off / on (A/B, tests).
constexpr int64_t kSplitMaxCols = 147456;
// Three lanes (profiles/r05zq_mappm_split3.log, one / two / three lanes): 65,536 columns
// 142.7 / 99 / 86.5 us, 110,592 166 / 141 / 150.5 us, 147,456 214 / 213 / 194 us.  Both
// split kernels hold 4 waves per SIMD (124-126 VGPRs); three lanes pay while all their
// waves are resident at once (3 ncol / 64 <= 4 waves x 4 SIMDs x CUs), which 110,592
// columns exceed.
constexpr int kSplitWavesPerSimd = 4;

// CUs of the current device, queried once (thread-safe static initialisation)
int device_cus()
{
    static const int n_cu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    return n_cu;
}

// lanes per column of the pair kernel: 1, 2 or 3 (FV3_MAPPM_SPLIT=0|1|3 forces one)
int split_lanes(int64_t ncol, int kn)
{
    const int n_cu = device_cus();
    const char* p = fv3::variant_env("FV3_MAPPM_SPLIT");
    int n = ncol < kSplitMaxCols ? 2 : 1;
    if (n == 2 && 3 * ncol <= (int64_t)64 * kSplitWavesPerSimd * 4 * n_cu) n = 3;
    if (p && p[0] == '0') n = 1;
    if (p && p[0] == '1') n = 2;
    if (p && p[0] == '3') n = 3;
    if (n == 3 && kn < 3) n = 2;
    if (n == 2 && kn < 2) n = 1;
    return n;
}

// One field (fv3_mappm_ex, kord <= 7) on the split kernels (profiles/r05zw_mappm_single_lanes.log,
// levels / one lane / two / three lanes, us): 13,824 columns 38.6 / 105 / 70 / 49.6,
// 27,648 67.8 / 108 / 76 / 56.6, C96 55,296 126 / 110 / 81 / 70, 82,944 184 / 127 / 113 /
// 98, 110,592 242 / 128 / 115 / 119, 147,456 320 / 152 / 139 / 149, 221,184 589 / 190 /
// 204 / 210.  The one-field split kernels hold 5 waves per SIMD (91 VGPRs): three lanes
// while all their waves are resident (3 ncol / 64 <= 5 x 4 SIMDs x CUs), then two while
// theirs are, from 20,480 columns (the level-parallel kernel below).  FV3_MAPPM_SPLIT1=0|2|3
// forces none / two / three lanes (A/B); a forced FV3_MAPPM_PATH keeps its kernel.
// Returns false where the host keeps the level-parallel or one-lane kernel.
constexpr int64_t kSplit1MinCols = 20480;
constexpr int kSplit1WavesPerSimd = 5;

bool launch_split_single(const MappmArgs& a, hipStream_t stream)
{
    if (a.kord > 7 || a.kn < 2) return false;
    const char* p = variant_env("FV3_MAPPM_SPLIT1");
    int lanes = 0;
    if (p) {
        lanes = atoi(p);
    } else if (!variant_env("FV3_MAPPM_PATH") && a.ncol >= kSplit1MinCols) {
        const int64_t resident = (int64_t)64 * kSplit1WavesPerSimd * 4 * device_cus();
        lanes = 3 * a.ncol <= resident ? 3 : (2 * a.ncol <= resident ? 2 : 0);
    }
    if (lanes == 3 && a.kn < 3) lanes = 2;
    if (lanes != 2 && lanes != 3) return false;
    MappmPairArgs pa{a.pe1, a.pe2, a.l_pe1, a.l_pe2, {a.q1, nullptr}, {a.q2, nullptr}, {a.l_q1, {}}, {a.l_q2, {}},
                     a.ncol, a.km, a.kn, a.iv, a.kord};
    const int64_t grid = (a.ncol + 63) / 64;
    const bool k1 = is_k1(a.iv, a.kord);
    if (lanes == 3)
        hipLaunchKernelGGL((k1 ? mappm_ppm_pair_split3_kernel<1, true> : mappm_ppm_pair_split3_kernel<1, false>),
                           dim3((unsigned)grid), dim3(192), 0, stream, pa);
    else
        hipLaunchKernelGGL((k1 ? mappm_ppm_pair_split_kernel<1, true> : mappm_ppm_pair_split_kernel<1, false>),
                           dim3((unsigned)grid), dim3(128), 0, stream, pa);
    return true;
}

// pairs of fields on the streaming kord <= 7 kernel (fv3_mappm_multi)
int launch_mappm_pairs(const MappmPairArgs& a, hipStream_t s)
{
    const int lanes = split_lanes(a.ncol, a.kn);
    const bool k1 = is_k1(a.iv, a.kord);
    if (lanes == 3) {  // three lanes per column: 192 threads per 64 columns
        const int64_t grid = (a.ncol + 63) / 64;
        hipLaunchKernelGGL((k1 ? mappm_ppm_pair_split3_kernel<2, true> : mappm_ppm_pair_split3_kernel<2, false>),
                           dim3((unsigned)grid), dim3(192), 0, s, a);
    } else if (lanes == 2) {  // two lanes per column: 128 threads per 64 columns
        const int64_t grid = (a.ncol + 63) / 64;
        hipLaunchKernelGGL((k1 ? mappm_ppm_pair_split_kernel<2, true> : mappm_ppm_pair_split_kernel<2, false>),
                           dim3((unsigned)grid), dim3(128), 0, s, a);
    } else {
        const int block = 256;
        const int64_t grid = (a.ncol + block - 1) / block;
        hipLaunchKernelGGL((k1 ? mappm_ppm_pair_kernel<true> : mappm_ppm_pair_kernel<false>), dim3((unsigned)grid),
                           dim3(block), 0, s, a);
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

}  // namespace FV3_ARITH_NS
}  // namespace fv3

#ifndef FV3_FAST_ARITH  // the C ABI: one definition, dispatching on the arithmetic
using fv3::MappmArgs;

namespace {
// FV3_ARITH_FAST covers the ppm_profile path (kord <= 7) only.  cs_profile (kord > 7)
// flattens a layer or switches its Huynh constraint on flags (extm, ext5, ext6,
// mappm.f90:269-288) computed from the solved edges, a discontinuous choice: 1-ulp
// changes to the edges flip it (tools/remap_fast_study.py, C384 kord 10: 7e-3 per level,
// 1 % of the values moved).  So kord > 7 always runs the exact arithmetic.
int launch_arith(const MappmArgs& a, int arith, hipStream_t s)
{
    return arith == FV3_ARITH_FAST && a.kord <= 7 ? fv3::fast::launch_mappm(a, s) : fv3::exact::launch_mappm(a, s);
}
}  // namespace

extern "C" int fv3_mappm_ex(const float* pe1, fv3_layout pe1_l, const float* q1, fv3_layout q1_l,
                            const float* pe2, fv3_layout pe2_l, float* q2, fv3_layout q2_l,
                            int64_t ncol, int km, int kn, int iv, int kord, float ptop, int arith,
                            void* stream)
{
    (void)ptop;  // unused by the reference too (regridz.py:270)
    fv3::clear_error();
    FV3_REQUIRE(arith == FV3_ARITH_EXACT || arith == FV3_ARITH_FAST, "mappm: unknown arithmetic %d", arith);
    FV3_REQUIRE(ncol >= 0, "mappm: ncol must be >= 0 (got %lld)", (long long)ncol);
    FV3_REQUIRE(km >= 4, "mappm: km must be >= 4 (got %d)", km);
    FV3_REQUIRE(kn >= 1, "mappm: kn must be >= 1 (got %d)", kn);
    FV3_REQUIRE(ncol == 0 || (pe1 && q1 && pe2 && q2), "mappm: NULL array");
    FV3_REQUIRE(ncol == 0 || (fv3::layout_ok(pe1_l, ncol) && fv3::layout_ok(q1_l, ncol) &&
                              fv3::layout_ok(pe2_l, ncol) && fv3::layout_ok(q2_l, ncol)),
                "mappm: invalid column layout");
    FV3_REQUIRE(ncol / 256 < (int64_t)0x7fffffff, "mappm: ncol too large");
    MappmArgs a{pe1, q1, pe2, q2, pe1_l, q1_l, pe2_l, q2_l, ncol, km, kn, iv, kord, nullptr};
    return launch_arith(a, arith, (hipStream_t)stream);
}

// the f2py signature of the reference's mappm.mappm: the reference's arithmetic
extern "C" int fv3_mappm(const float* pe1, const float* q1, const float* pe2, float* q2,
                         int64_t ncol, int km, int kn, int iv, int kord, float ptop, void* stream)
{
    const fv3_layout l = fv3::plain_layout(ncol > 0 ? ncol : 1);
    return fv3_mappm_ex(pe1, l, q1, l, pe2, l, q2, l, ncol, km, kn, iv, kord, ptop, FV3_ARITH_EXACT, stream);
}

extern "C" int fv3_mappm_multi(const float* pe1, fv3_layout pe1_l, const float* const* q1, const fv3_layout* q1_l,
                               const float* pe2, fv3_layout pe2_l, float* const* q2, const fv3_layout* q2_l,
                               int n_fields, int64_t ncol, int km, int kn, int iv, int kord, float ptop, int arith,
                               void* stream)
{
    fv3::clear_error();
    FV3_REQUIRE(arith == FV3_ARITH_EXACT || arith == FV3_ARITH_FAST, "mappm: unknown arithmetic %d", arith);
    FV3_REQUIRE(n_fields >= 1 && n_fields <= 64, "mappm_multi: n_fields must be in 1..64 (got %d)", n_fields);
    FV3_REQUIRE(q1 && q1_l && q2 && q2_l, "mappm_multi: NULL field array");
    FV3_REQUIRE(ncol >= 0, "mappm: ncol must be >= 0 (got %lld)", (long long)ncol);
    FV3_REQUIRE(km >= 4, "mappm: km must be >= 4 (got %d)", km);
    FV3_REQUIRE(kn >= 1, "mappm: kn must be >= 1 (got %d)", kn);
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(pe1 && pe2, "mappm: NULL array");
    FV3_REQUIRE(fv3::layout_ok(pe1_l, ncol) && fv3::layout_ok(pe2_l, ncol), "mappm: invalid column layout");
    for (int f = 0; f < n_fields; ++f) {
        FV3_REQUIRE(q1[f] && q2[f], "mappm_multi: NULL field %d", f);
        FV3_REQUIRE(fv3::layout_ok(q1_l[f], ncol) && fv3::layout_ok(q2_l[f], ncol),
                    "mappm_multi: invalid column layout of field %d", f);
    }
    FV3_REQUIRE(ncol / 256 < (int64_t)0x7fffffff, "mappm: ncol too large");
    const hipStream_t s = (hipStream_t)stream;
    int f = 0;
    // pairs on the streaming kord <= 7 kernel; the level-parallel (small grids) and
    // cs_profile (kord > 7) paths, and an odd last field, one field per launch
    MappmArgs one{pe1, nullptr, pe2, nullptr, pe1_l, {}, pe2_l, {}, ncol, km, kn, iv, kord, nullptr};
    if (kord <= 7 && !fv3::exact::use_levels_kernel(one, fv3::exact::kLevelsMaxColsPairs)) {
        for (; f + 2 <= n_fields; f += 2) {
            fv3::MappmPairArgs a{pe1, pe2, pe1_l, pe2_l, {q1[f], q1[f + 1]}, {q2[f], q2[f + 1]},
                                 {q1_l[f], q1_l[f + 1]}, {q2_l[f], q2_l[f + 1]}, ncol, km, kn, iv, kord};
            const int st = arith == FV3_ARITH_FAST ? fv3::fast::launch_mappm_pairs(a, s)
                                                   : fv3::exact::launch_mappm_pairs(a, s);
            if (st != FV3_OK) return st;
        }
    }
    for (; f < n_fields; ++f) {
        const int st = fv3_mappm_ex(pe1, pe1_l, q1[f], q1_l[f], pe2, pe2_l, q2[f], q2_l[f], ncol, km, kn, iv, kord,
                                    ptop, arith, stream);
        if (st != FV3_OK) return st;
    }
    return FV3_OK;
}
#endif  // FV3_FAST_ARITH
