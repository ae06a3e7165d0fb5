// fv3net_amd — fused column-wise dense predict on bf16 MFMA with split operands:
// "bf16x3" (2 parts per operand, 3 MFMAs per product) and "bf16x6" (3 parts, 6 MFMAs).
//
// Same graph and boundary as dense.hip (the DenseModel of external/fv3fit/fv3fit/keras/
// _models/dense.py:234-305 and the microphysics emulator's MLP, external/fv3fit/fv3fit/
// emulation/layers/architecture.py:228-345): inputs read in place from [level][column]
// arrays, LogTransform / StandardNorm, n x Dense(relu), one linear Dense per output,
// de-normalisation, OutputLimit, zero mask, residual outputs, written in place.
//
// Arithmetic: every f32 operand x is split into bf16 hi = rne(x) and lo = rne(x - hi),
// and a product a*b is taken as hi_a*hi_b + lo_a*hi_b + hi_a*lo_b on
// v_mfma_f32_16x16x32_bf16 (f32 accumulate).  That keeps ~16 mantissa bits of each
// operand: ~1e-5 rel against the float64 graph on the 2x256 DenseModel and the Zhao-Carr
// emulator (plain bf16: 4.7e-3, outside BASELINE config #5's 1e-3).  Three bf16 MFMAs
// cost 48 cycles per 16x16x32 block against 256 for exact f32, ~5.3x the f32 MFMA rate.
// bf16x6 adds a third part (mid) and takes the six products of order <= 2 (SplitTerms):
// ~24 bits per operand, held to the f32 kernel's 1e-5 per-level bound, 96 cycles per
// block (2.7x the f32 rate); its 48 KiB chunks run a 2-slot LDS-DMA ring.
// Grids with fewer 128-column tiles than CUs run 4-wave blocks of 64 columns (NWV = 4).
//
// Mapping (one 512-thread block per CU, 2 waves per SIMD, persistent over column tiles):
//  * a block tile is 128 columns; wave w owns columns [16w, 16w+16) for the WHOLE network,
//    so activations never leave registers: a layer's 16x16 accumulators (units 4q..4q+3 of
//    each 16-unit tile on lane quarter q, column on lane & 15) are, after bias + relu +
//    split, exactly the B operands of the next layer's 16x16x32 MFMAs (two unit tiles per
//    32-deep k-step, k order permuted; the packed weights carry the permutation);
//  * two waves per SIMD: one wave's epilogue and LDS reads run while the other's MFMAs
//    do; the per-wave state that allows it (<= 256 registers) is what sets 16 columns;
//  * weights stream through LDS in chunks of one 32-deep k-step x all unit tiles x hi/lo
//    (32 KiB at width 256, A-fragment order, one ds_read_b128 per fragment), double-
//    buffered: the chunk after next is loaded into registers while the current one runs
//    (one barrier per chunk); the 8 waves share every chunk, so L2 traffic is 1/128 of a
//    weight per column;
//  * layer-1 inputs are loaded straight into the B-fragment layout (lane = column, 8
//    consecutive levels per lane quarter), two chunks ahead, then log / normalised / split
//    in registers: no LDS staging of inputs;
//  * the output layer runs in chunks of two 16-row tiles (every output variable is padded
//    to 16 rows, so a tile has ONE destination); the epilogue of a chunk (bias, denorm,
//    limits, mask, residual) runs after the next chunk's MFMAs are issued.
// Roofline: bf16 MFMA (3 products per f32 product) — see DESIGN.md §3.5.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "dense_model.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float b3f4 __attribute__((ext_vector_type(4)));

namespace fv3 {

constexpr int kB3Groups = 128;   // 8-feature input groups (<= 1024 padded input features)
constexpr int kB3Cols = 128;     // columns per block tile: 8 waves x 16 (4-wave blocks: 64)
constexpr int kB3OutTiles = 32;  // 16-row output tiles (<= 512 padded output rows)
constexpr int kB3Threads = 512;  // 8-wave blocks (4-wave blocks on small grids: 256)
// the LDS-DMA pipeline by default: emulator C384 2.41 -> 2.29-2.34 ms, 2x256 C384 827 -> 814-820 us
// against the register-staged one on the same box (round 3; a variant holding the output
// chunks' accumulators / residuals in two register sets instead of copying them measured
// the same, within the run-to-run spread)
constexpr bool kB3GldsDefault = true;
// fragment ring: the A fragments of the next (kFR - 2) / 2 tile pairs are in flight while a
// pair's MFMAs issue
#ifndef FV3_B3_FR
#define FV3_B3_FR 4
#endif
constexpr int kFR = FV3_B3_FR;
// instruction order inside a chunk (A/B, same results): 0 = the compiler's; 1 = the next
// pair's fragment reads pinned ahead of this pair's MFMAs (a scheduling barrier between
// them, so the waits before the MFMAs leave the younger reads in flight); 2 = the same
// order as scheduling-group hints (DS reads, then MFMAs, VALU free to fill in)
#ifndef FV3_B3_SCHED
#define FV3_B3_SCHED 0
#endif
__device__ __forceinline__ void b3_sched_pair()
{
#if FV3_B3_SCHED == 1
    __builtin_amdgcn_sched_barrier(0);
#endif
}
template <int NRD, int NMF>
__device__ __forceinline__ void b3_sched_groups()
{
#if FV3_B3_SCHED == 2
    __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);  // DS reads
    __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);  // MFMAs
#endif
}
// weight ring slots: SL (LDS-DMA pipeline: 3, or 2 where three chunks do not fit, e.g.
// bf16x6 at width 256), 0 = the register-staged pipeline (2 slots)
constexpr int b3_slots(int sl) { return sl > 0 ? sl : 2; }
constexpr int b3_in_bytes(bool gl, int nwv) { return gl ? 2 * nwv * 8 * 64 * 4 : 0; }

struct B3Pack {
    void* dbuf = nullptr;
    int ns = 2;  // bf16 parts per weight (2: bf16x3, 3: bf16x6)
    int hu = 0, hp = 0, kp1 = 0, n1 = 0, nhx = 0, n_oc = 0, kop = 0, nch = 0;
    int nconst = 0, wbytes = 0, any_log = 0;  // any_log: 1 every epsilon normal (fast log), 2 some not
    std::vector<int> gmeta;  // per 8-feature group: var | zstart << 4 | nvalid << 24
    std::vector<int> otile;  // per 16-row output tile: var | z0 << 8 | nrow << 24 (var 255: padding)
    size_t consts_off = 0;
};

namespace {

struct B3InVar {
    const float* ptr;
    int64_t ld, bs;
    float leps;  // > 0: LogTransform log(max(x, leps))
    int pad_;
};

struct B3Args {
    const void* wstream;  // [nch][CB]: the packed weight chunks of one column tile
    const float* consts;  // [kp1] mean | [kp1] 1/(sigma+eps) | [nh][HP] bias | [6][kop]
    int wbytes;
    int nch, n1, nhx, n_oc, kp1, kop, nconst, any_log;
    int64_t ncol, ncol_blk, ntiles;
    B3InVar in[kMaxVars];
    int gmeta[kB3Groups];
    // output rows in 16-row tiles, each of ONE variable (every variable is padded to a
    // multiple of 16 rows): tile T = var | z0 << 8 | nrow << 24 (var 255: padding)
    int otile[kB3OutTiles];
    float* out_ptr[kMaxVars];
    int64_t out_ld[kMaxVars], out_bs[kMaxVars];
    const float* res_ptr[kMaxVars];
    int64_t res_ld[kMaxVars], res_bs[kMaxVars];
    int ovec;  // TR: every output / residual row 16-byte aligned (16-byte accesses)
    // profiling hook (fv3_dense_set_trace), NULL normally: per tile [8] int64 =
    // wall clock (100 MHz) at tile start / layer 1 done / hidden done / tile end, CU id,
    // shader clock at tile start / end, shader cycles wave 0 spent in the chunk waits
    // (vmcnt + barrier) of the tile
    long long* trace;
};
static_assert(sizeof(B3Args) <= 4096, "kernel arguments are limited to 4 KiB");

typedef __attribute__((address_space(4))) const B3Args KB3;

// layer-1 input group g (8 levels of one variable), resolved once per block into LDS:
// the lane quarter that reads group g of a k-step takes its address, strides, valid
// level count and LogTransform epsilon with two LDS reads instead of re-deriving them
// from gmeta / in[] (per-lane selects of four 64-bit candidates) every k-step
struct B3Grp {
    const float* ptr;  // level z0 of the group's variable (column 0)
    int64_t bs;        // column-block stride
    int ld;            // level stride (elements)
    int nv;            // valid levels (0..8)
    float leps;        // > 0: LogTransform
    int klog;          // some group of this group's k-step (4 groups) has a LogTransform
};
static_assert(sizeof(B3Grp) == 32, "B3Grp is read as two 16-byte words");
typedef __amdgpu_buffer_rsrc_t Rsrc3;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f)
{
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// this wave's LDS writes done, then the workgroup barrier; global loads in flight (the
// next weight chunk, the next inputs) are NOT drained (a __syncthreads() fence would
// wait vmcnt(0) on gfx9, where loads and stores share the counter)
#ifndef FV3_B3_BUILTIN_BARRIER
#define FV3_B3_BUILTIN_BARRIER 0
#endif
#if FV3_B3_BUILTIN_BARRIER
// the same two instructions as builtins, so the compiler's wait-count pass sees the
// lgkm counter drained here (behind inline asm it assumes scalar loads may still be in
// flight and then drains every later LDS wait to lgkmcnt(0))
__device__ __forceinline__ void b3_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt at their maximum (no wait)
    __builtin_amdgcn_s_barrier();
}
#else
__device__ __forceinline__ void b3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#endif

// LogTransform.forward: log(max(x, eps)).  fast (every LogTransform epsilon of the model
// normal, the host's any_log == 1): v_log_f32 (log2, ~1 ulp) times ln 2, 4 instructions a
// value instead of the library's logf (denormal scaling and an extended-precision product,
// ~14): about 1e-7 rel of the log, far inside the split's own rounding (bf16x3 ~1e-5,
// bf16x6 ~6e-8 per operand, both held to their per-level bounds by the tests); emulator
// C384 2.41-2.42 -> 2.38 ms (profiles/r05ze_b3_fastlog_ab.log).  Otherwise logf.
__device__ __forceinline__ float b3_log(float x, float eps, bool fast)
{
    const float v = x > eps ? x : eps;
    return x != x ? x : (fast ? __builtin_amdgcn_logf(v) * 0.6931471805599453f : logf(v));
}

// y -> NS bf16 parts: part 0 = rne(y), part s = rne(y - parts 0..s-1) (every residual is
// exact in f32).  NS = 2: hi + lo (~16 mantissa bits); NS = 3: hi + mid + lo (~24 bits).
template <int NS>
__device__ __forceinline__ void splitN(const float (&y)[8], bf16x8 (&o)[NS])
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float r = y[j];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const __bf16 h = (__bf16)r;
            o[s][j] = h;
            if (s + 1 < NS) r = r - (float)h;
        }
    }
}

// the split products of one f32 product a*b, in issue order (part of a, part of b):
// NS = 2 (bf16x3): hi*hi, lo*hi, hi*lo; NS = 3 (bf16x6): every pair of order <= 2 in the
// parts' 2^-8 steps (hi*hi; mid*hi, hi*mid; mid*mid, lo*hi, hi*lo), ~2^-24 rel per product
template <int NS>
struct SplitTerms {
    static constexpr int n = NS == 2 ? 3 : 6;
    static constexpr int a[6] = {0, 1, 0, 1, 2, 0};
    static constexpr int b[6] = {0, 0, 1, 1, 0, 2};
};

// two independent accumulations interleaved (c0 <- a0 x b0, c1 <- a1 x b1, each in the
// SplitTerms order): no MFMA waits on the one just issued
template <int NS>
__device__ __forceinline__ void mma_x2(const bf16x8 (&a0)[NS], const bf16x8 (&b0)[NS], b3f4& c0,
                                       const bf16x8 (&a1)[NS], const bf16x8 (&b1)[NS], b3f4& c1)
{
    using T = SplitTerms<NS>;
#pragma unroll
    for (int t = 0; t < T::n; ++t) {
#ifdef FV3_B3_EXP_NOMFMA  // experiment only (results invalid): everything but the MFMAs
        c0[0] += (float)a0[T::a[t]][t] + (float)b0[T::b[t]][t];
        c1[0] += (float)a1[T::a[t]][t] + (float)b1[T::b[t]][t];
#else
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[T::a[t]], b0[T::b[t]], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[T::a[t]], b1[T::b[t]], c1, 0, 0, 0);
#endif
    }
}

// mma_x2 with the operands' roles swapped: the same registers, the same split products
// (SplitTerms is symmetric in a and b), D^T in the accumulator layout: lane l holds
// columns 4 (l >> 4) .. + 3 of row l & 15 (the transposed output layer, TR below)
template <int NS>
__device__ __forceinline__ void mma_x2t(const bf16x8 (&a0)[NS], const bf16x8 (&b0)[NS], b3f4& c0,
                                        const bf16x8 (&a1)[NS], const bf16x8 (&b1)[NS], b3f4& c1)
{
    using T = SplitTerms<NS>;
#pragma unroll
    for (int t = 0; t < T::n; ++t) {
#ifdef FV3_B3_EXP_NOMFMA  // experiment only (results invalid): everything but the MFMAs
        c0[0] += (float)a0[T::a[t]][t] + (float)b0[T::b[t]][t];
        c1[0] += (float)a1[T::a[t]][t] + (float)b1[T::b[t]][t];
#else
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[T::b[t]], a0[T::a[t]], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[T::b[t]], a1[T::a[t]], c1, 0, 0, 0);
#endif
    }
}

// value of lane quarter q from 4 wave-uniform candidates
template <typename T>
__device__ __forceinline__ T sel4(int q, T a0, T a1, T a2, T a3)
{
    const T lo = (q & 1) ? a1 : a0;
    const T hi = (q & 1) ? a3 : a2;
    return (q & 2) ? hi : lo;
}

// s_waitcnt vmcnt(n) for a wave-uniform n (an immediate per value; n >= 47 waits for 47)
__device__ __forceinline__ void vm_wait_le(int n)
{
    switch (n < 47 ? n : 47) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 33: asm volatile("s_waitcnt vmcnt(33)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 35: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
    case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 37: asm volatile("s_waitcnt vmcnt(37)" ::: "memory"); break;
    case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 39: asm volatile("s_waitcnt vmcnt(39)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 41: asm volatile("s_waitcnt vmcnt(41)" ::: "memory"); break;
    case 42: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
    case 43: asm volatile("s_waitcnt vmcnt(43)" ::: "memory"); break;
    case 44: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 45: asm volatile("s_waitcnt vmcnt(45)" ::: "memory"); break;
    case 46: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
    case 47: asm volatile("s_waitcnt vmcnt(47)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

typedef __attribute__((address_space(1))) void* GlobalVoid;
typedef __attribute__((address_space(3))) void* LdsVoid;

// LDS-DMA of 16 B (dwordx4) or 4 B (dword) per lane into the wave-uniform LDS byte address
// `lds` (+ 16 B or 4 B x lane).  FV3_B3_GLDS_ASM: issued from inline asm (M0 saved and
// restored in the same statement) instead of __builtin_amdgcn_global_load_lds.  The
// compiler's wait-count pass files a builtin LDS-DMA as a pending LDS event of another
// kind than the ds_reads and from then on drains every wait before an MFMA to
// lgkmcnt(0), so the fragment reads of the next tile pair never overlap the current
// pair's MFMAs; hidden in asm, it is not counted (it is a VM_CNT operation: the ring's
// own counted vmcnt waits and the chunk barrier cover it) and the ds_read waits stay
// counted.
#ifndef FV3_B3_GLDS_ASM
#define FV3_B3_GLDS_ASM 0
#endif
template <int BYTES>
__device__ __forceinline__ void b3_glds(const void* g, const void* lds)
{
#if FV3_B3_GLDS_ASM
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LdsVoid)lds);
    unsigned keep;
    if constexpr (BYTES == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
#else
    if constexpr (BYTES == 16)
        __builtin_amdgcn_global_load_lds((GlobalVoid)g, (LdsVoid)lds, 16, 0, 0);
    else
        __builtin_amdgcn_global_load_lds((GlobalVoid)g, (LdsVoid)lds, 4, 0, 0);
#endif
}

// GL (default): the weight chunks and the layer-1 inputs go global -> LDS by LDS-DMA
// (global_load_lds), a 3-slot weight ring with two chunks in flight; no staging registers
// and no ds_write pass.  !GL: round 2's pipeline (weights through 16 staging registers and
// ds_write_b128 into a 2-slot ring, inputs into registers), kept for A/B (FV3_B3_STAGE=reg).
// NS: bf16 parts per f32 operand (2: bf16x3, 3: bf16x6, see SplitTerms)
// NWV: waves per block (8; 4 on grids with fewer 128-column tiles than CUs, so every
// CU gets a tile and each SIMD runs one 16-column wave)
// TR: the transposed output layer (operands swapped, mma_x2t): each lane holds 4
// consecutive columns of one output row, so the epilogue reads its constants once per
// row and moves a lane's residuals and results in one 16-byte load / store (p.ovec:
// every output / residual row 16-byte aligned; else 4 dword accesses).  The host picks
// TR when 4-column groups never cross a column block.
template <int HU, int SL, int NS, int NWV, bool TR = false>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NWV == 4 ? 1 : 2, NWV == 4 ? 1 : 2))) void
dense_b3_kernel(B3Args pa)
{
    (void)pa;
    KB3& p = *(KB3*)(__builtin_amdgcn_kernarg_segment_ptr());
    constexpr int HP = 16 * HU;      // padded units
    constexpr int KS = HU / 2;       // 32-deep k-steps over HP units
    constexpr int CB = 1024 * NS * HU;  // chunk: HU A fragments x NS parts x 64 lanes x 16 B
    // 16-B loads per thread per chunk; a chunk that is not a whole number of block-wide
    // loads (HU = 4 at NS = 3: 1.5) has its last load on the first waves only (wave-uniform)
    constexpr int kB3Threads = 64 * NWV, kB3Cols = 16 * NWV;  // this instantiation's block
    constexpr int NST = (CB + 16 * kB3Threads - 1) / (16 * kB3Threads);
    constexpr bool GL = SL > 0;
    constexpr int NSL = b3_slots(SL);            // weight ring slots
    static_assert(HU % 4 == 0 && NST >= 1, "unit tiles per layer must be a multiple of 4");
    extern __shared__ __attribute__((aligned(16))) b3f4 lds3[];
    char* ring = reinterpret_cast<char*>(lds3);
    float* s_in = reinterpret_cast<float*>(ring + NSL * CB);  // GL: [2][8 waves][8 levels][64 lanes]
    float* s_mean = reinterpret_cast<float*>(ring + NSL * CB + b3_in_bytes(GL, NWV));
    float* s_rs = s_mean + p.kp1;
    float* s_bias = s_rs + p.kp1;             // [nh][HP]
    float* s_oc = s_bias + (1 + p.nhx) * HP;  // [6][kop]: bias, sigma, mean, lo, hi, mask
    B3Grp* s_grp = reinterpret_cast<B3Grp*>(reinterpret_cast<char*>(s_mean) + 4 * ((p.nconst + 7) & ~7));  // [4 n1]
    const int kop = p.kop;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hq = lane >> 4;  // lane quarter: k offset 8*hq of a k-step, rows 4*hq of a tile
    const int cl = lane & 15;  // column of this lane inside the wave's 16

    for (int i = tid; i < p.nconst; i += kB3Threads) s_mean[i] = p.consts[i];
    for (int g = tid; g < 4 * p.n1; g += kB3Threads) {
        const int m = p.gmeta[g], v = m & 15;
        B3Grp e;
        e.ptr = p.in[v].ptr + (int64_t)((m >> 4) & 0xfffff) * p.in[v].ld;
        e.bs = p.in[v].bs;
        e.ld = (int)p.in[v].ld;
        e.nv = m >> 24;
        e.leps = p.in[v].leps;
        e.klog = 0;
        for (int i = 4 * (g / 4); i < 4 * (g / 4) + 4; ++i)
            e.klog |= (p.gmeta[i] >> 24) > 0 && p.in[p.gmeta[i] & 15].leps > 0.0f;
        s_grp[g] = e;
    }
    b3_barrier();  // the group table is read by the first tile's input loads below

    // ---- weight stream.  GL: LDS ring of 3 chunks filled by LDS-DMA, two ahead of use.
    //      !GL: LDS ring of 2 chunks, the chunk after next in registers ----
    const Rsrc3 rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.wstream), 0, p.wbytes, 0x00020000);
    auto part_ok = [&](int q) {  // this wave takes part in load q of a chunk
        return CB % (16 * kB3Threads) == 0 || q + 1 < NST || q * 16 * kB3Threads + wave * 1024 < CB;
    };
    int nst_w = 0;  // loads of one chunk this wave issues (the count its vmcnt waits see)
#pragma unroll
    for (int q = 0; q < NST; ++q) nst_w += part_ok(q) ? 1 : 0;
    const char* wsrc = reinterpret_cast<const char*>(p.wstream);
    b3f4 stg[GL ? 1 : NST];
    auto load_stage = [&](int j) {
#pragma unroll
        for (int q = 0; q < NST; ++q)
            if (part_ok(q))
                stg[q] = __builtin_bit_cast(
                    b3f4, __builtin_amdgcn_raw_buffer_load_b128(rw, tid * 16, j * CB + q * 16 * kB3Threads, 0));
    };
    auto write_stage = [&](int slot) {
#pragma unroll
        for (int q = 0; q < NST; ++q)
            if (part_ok(q)) *reinterpret_cast<b3f4*>(ring + slot * CB + q * 16 * kB3Threads + tid * 16) = stg[q];
    };
    // chunk j of the stream into ring slot sl: NST LDS-DMA loads per thread; the LDS side
    // of each is wave-uniform base + 16 B x lane, the chunk image being lane-linear
    auto glds_w = [&](int j, int sl) {
#pragma unroll
        for (int q = 0; q < NST; ++q)
            if (part_ok(q))
                b3_glds<16>(wsrc + (size_t)j * CB + q * 16 * kB3Threads + tid * 16,
                            ring + sl * CB + q * 16 * kB3Threads + wave * 1024);
    };
    int slot = 0;                         // ring slot of the chunk computed next
    // stream index of the chunk staged next (GL: chunk + NSL - 1, !GL: chunk + 2)
    int jn2 = GL && NSL == 2 ? (p.nch > 1 ? 1 : 0) : (p.nch > 2 ? 2 : 2 % p.nch);
    if constexpr (GL) {
        glds_w(0, 0);
        if constexpr (NSL == 3) glds_w(p.nch > 1 ? 1 : 0, 1);
    } else {
        load_stage(0);
        write_stage(0);
        load_stage(p.nch > 1 ? 1 : 0);
    }

    b3f4 acc[HU];
    auto zero_acc = [&]() {
#pragma unroll
        for (int t = 0; t < HU; ++t) acc[t] = b3f4{0.0f, 0.0f, 0.0f, 0.0f};
    };
#ifdef FV3_B3_EXP_NOFRAG
    bf16x8 fconst[2][NS];
    for (int i = 0; i < 2; ++i)
        for (int h = 0; h < NS; ++h) fconst[i][h] = *reinterpret_cast<const bf16x8*>(ring + i * 1024 * NS + h * 1024 + lane * 16);
#endif
    // A fragment i of the chunk in slot sl: part s at (NS i + s) * 1024
    auto frag = [&](int sl, int i, bf16x8 (&f)[NS]) {
#ifdef FV3_B3_EXP_NOFRAG  // experiment only (results invalid): one fragment, no LDS reads per step
        (void)sl;
#pragma unroll
        for (int h = 0; h < NS; ++h) f[h] = fconst[i & 1][h];
#else
        const char* a = ring + sl * CB + i * 1024 * NS + lane * 16;
#pragma unroll
        for (int h = 0; h < NS; ++h) f[h] = *reinterpret_cast<const bf16x8*>(a + h * 1024);
#endif
    };
    auto stage_next = [&]() {
        if constexpr (GL) {
            glds_w(jn2, slot == 0 ? NSL - 1 : slot - 1);  // chunk +NSL-1 into the slot chunk -1 released
        } else {
#ifndef FV3_B3_EXP_NOSTAGE  // experiment only (results invalid): no weight streaming
            write_stage(slot ^ 1);  // chunk +1 (its slot held chunk -1, released by the last barrier)
            load_stage(jn2);        // chunk +2
#endif
        }
    };
    // end of a chunk.  GL: this wave's LDS-DMA of chunk +1 (issued one chunk ago) must have
    // landed before the barrier that publishes it; `younger` = vector-memory operations this
    // chunk issued after its own weight DMA (they, and that DMA, may stay in flight)
#ifdef FV3_B3_TRACE
    long long wait_cyc = 0;  // trace only: wave 0's cycles in the chunk waits of this tile
#endif
    auto advance = [&](int younger) {
#ifdef FV3_B3_TRACE
        const long long tw0 = p.trace ? (long long)__builtin_amdgcn_s_memtime() : 0;
#endif
        // (two slots: the DMA this chunk issued is chunk +1 itself, so none of it may stay)
        if constexpr (GL) vm_wait_le((NSL == 3 ? nst_w : 0) + younger);
        b3_barrier();
#ifdef FV3_B3_TRACE
        if (p.trace) wait_cyc += (long long)__builtin_amdgcn_s_memtime() - tw0;
#endif
        slot = GL ? (slot == NSL - 1 ? 0 : slot + 1) : (slot ^ 1);
        jn2 = jn2 + 1 == p.nch ? 0 : jn2 + 1;
    };
    // layer chunk: unit tile t accumulates A_t x B (one 32-deep k-step); tiles in pairs,
    // their MFMAs interleaved, fragments read one pair ahead
    auto step_layer = [&](const bf16x8 (&bx)[NS], auto&& after_stage) {
        stage_next();
        const int younger = after_stage();  // GL: ops issued after this chunk's weight DMA (vmcnt is in order)
        bf16x8 fa[kFR][NS];
        sfor<kFR - 2>([&](auto ic) { frag(slot, decltype(ic)::value, fa[decltype(ic)::value]); });
        sfor<HU / 2>([&](auto pc) {
            constexpr int t0 = 2 * decltype(pc)::value, t1 = t0 + 1;
            if constexpr (t0 + kFR - 2 < HU) {
                frag(slot, t0 + kFR - 2, fa[(t0 + kFR - 2) % kFR]);
                frag(slot, t1 + kFR - 2, fa[(t1 + kFR - 2) % kFR]);
            }
            b3_sched_pair();
            mma_x2<NS>(fa[t0 % kFR], bx, acc[t0], fa[t1 % kFR], bx, acc[t1]);
            b3_sched_groups<(t0 + kFR - 2 < HU) ? 2 * NS : 0, 2 * SplitTerms<NS>::n>();
            b3_sched_pair();
        });
        advance(younger);
    };

    // ---- layer-1 inputs: B fragments straight from the [level][column] arrays ----
    unsigned lblk = 0, lii = 0;  // column address of the tile being loaded (block, index in block)
    bool lvalid = false;
    auto set_load_tile = [&](int64_t tile) {
        const int64_t c = tile * kB3Cols + wave * 16 + cl;
        lvalid = c < p.ncol;
        const int64_t cc = lvalid ? c : 0;
        const int64_t b = p.ncol_blk < p.ncol ? cc / p.ncol_blk : 0;
        lblk = (unsigned)b;
        lii = (unsigned)(cc - b * p.ncol_blk);
    };
    auto load_in = [&](float (&raw)[8], int c) {  // chunk c: group 4c + hq, 8 levels
        const B3Grp& g = s_grp[4 * c + hq];
        const int ld = g.ld;  // the host checks 8 * ld < 2^31
        const int nv = lvalid ? g.nv : 0;
        typedef const __attribute__((address_space(1))) float* GPtr;
        const GPtr ptr = (GPtr)(g.ptr + (int64_t)lblk * g.bs + lii);
        // all 8 loads issued unconditionally (levels past nv read the group's first level,
        // always in range, and are zeroed after), so none waits behind a branch
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#ifdef FV3_B3_EXP_NOIN  // experiment only (results invalid): no input loads
            const float x = 1.0f + (float)(uintptr_t)(ptr + (j < nv ? j * ld : 0)) * 0.0f;
#else
            // plain (cacheable) loads: the residual outputs re-read T / q / qc one tile
            // later (emulator C384 2.55 -> 2.36 ms against nontemporal loads, round 3)
            const float x = ptr[j < nv ? j * ld : 0];
#endif
            raw[j] = j < nv ? x : 0.0f;
        }
    };
    // GL: chunk c's inputs by LDS-DMA into this wave's rows of buffer `buf`: level j of
    // every lane is one 4-byte LDS-DMA (lane-linear row [buf][wave][j][lane])
    auto glds_in = [&](int buf, int c) {
        const B3Grp& g = s_grp[4 * c + hq];
        const int ld = g.ld;
        const int nv = lvalid ? g.nv : 0;
        const float* ptr = g.ptr + (int64_t)lblk * g.bs + lii;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            b3_glds<4>(ptr + (j < nv ? j * ld : 0), s_in + ((buf * NWV + wave) * 8 + j) * 64);
    };
    auto read_in = [&](int buf, int c, float (&raw)[8]) {  // GL: chunk c's values (landed, see advance)
        const int nv = lvalid ? s_grp[4 * c + hq].nv : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float x = s_in[((buf * NWV + wave) * 8 + j) * 64 + lane];
            raw[j] = j < nv ? x : 0.0f;
        }
    };
    auto stage_in = [&](const float (&raw)[8], int c, bf16x8 (&bx)[NS]) {
        const int f0 = 32 * c + 8 * hq;
        const b3f4 mu0 = *reinterpret_cast<const b3f4*>(s_mean + f0);
        const b3f4 mu1 = *reinterpret_cast<const b3f4*>(s_mean + f0 + 4);
        const b3f4 rs0 = *reinterpret_cast<const b3f4*>(s_rs + f0);
        const b3f4 rs1 = *reinterpret_cast<const b3f4*>(s_rs + f0 + 4);
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = raw[j];
        // the log path only for k-steps that hold a LogTransform group (uniform branch)
        if (p.any_log && __builtin_amdgcn_readfirstlane(s_grp[4 * c].klog)) {
            const float leps = s_grp[4 * c + hq].leps;
#pragma unroll
            for (int j = 0; j < 8; ++j)  // LogTransform.forward (transforms.py:123-124)
                if (leps > 0.0f) y[j] = b3_log(y[j], leps, p.any_log == 1);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (y[j] - (j < 4 ? mu0[j] : mu1[j - 4])) * (j < 4 ? rs0[j] : rs1[j - 4]);
        splitN<NS>(y, bx);
    };

    // ---- activations: B fragments of the next layer (k-step c, element j of quarter q is
    //      unit 32c + 16(j>>2) + 4q + (j&3): registers of unit tiles 2c and 2c+1) ----
    // NS = 2: split as soon as computed (B); NS = 3: kept in f32 (Y, 8 registers per k-step
    // against 12 for the split) and split per chunk as the next hidden layer consumes it;
    // the output layer, whose chunks each read every k-step, splits them all into B first
    bf16x8 B[KS][NS];
    float Y[NS == 3 ? KS : 1][8];
    auto hidden_epi = [&](int l) {  // relu(acc + bias_l) -> B (NS = 2) / Y (NS = 3)
        sfor<KS>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            const b3f4 b0 = *reinterpret_cast<const b3f4*>(s_bias + l * HP + 32 * c + 4 * hq);
            const b3f4 b1 = *reinterpret_cast<const b3f4*>(s_bias + l * HP + 32 * c + 16 + 4 * hq);
            float y[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v0 = acc[2 * c][r] + b0[r];
                const float v1 = acc[2 * c + 1][r] + b1[r];
                y[r] = v0 > 0.0f ? v0 : 0.0f;
                y[4 + r] = v1 > 0.0f ? v1 : 0.0f;
            }
            if constexpr (NS == 2) {
                splitN<NS>(y, B[c]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) Y[c][j] = y[j];
            }
        });
    };
    auto hidden_b = [&](auto cc, bf16x8 (&bx)[NS]) -> const bf16x8(&)[NS] {  // k-step c's B fragments
        constexpr int c = decltype(cc)::value;
        if constexpr (NS == 2) {
            return B[c];
        } else {
            splitN<NS>(Y[c], bx);
            return bx;
        }
    };
    // output chunk: fragment i = 2q + ts accumulates tile ts of the chunk over k-step q
    auto step_out = [&]() {  // fragments 2q, 2q+1: k-step q of tiles 0 and 1, interleaved
        bf16x8 fa[kFR][NS];
        sfor<kFR - 2>([&](auto ic) { frag(slot, decltype(ic)::value, fa[decltype(ic)::value]); });
        sfor<HU / 2>([&](auto qc) {
            constexpr int q = decltype(qc)::value, i0 = 2 * q, i1 = i0 + 1;
            if constexpr (i0 + kFR - 2 < HU) {
                frag(slot, i0 + kFR - 2, fa[(i0 + kFR - 2) % kFR]);
                frag(slot, i1 + kFR - 2, fa[(i1 + kFR - 2) % kFR]);
            }
            b3_sched_pair();
            if constexpr (TR)
                mma_x2t<NS>(fa[i0 % kFR], B[q], acc[0], fa[i1 % kFR], B[q], acc[1]);
            else
                mma_x2<NS>(fa[i0 % kFR], B[q], acc[0], fa[i1 % kFR], B[q], acc[1]);
            b3_sched_groups<(i0 + kFR - 2 < HU) ? 2 * NS : 0, 2 * SplitTerms<NS>::n>();
            b3_sched_pair();
        });
    };

    // ---- output epilogue ----------------------------------------------------------
    // Output tile T's accumulator register r of lane (q, cl) is row 16T + 4q + r of column
    // cl; a tile belongs to ONE output variable (otile), so its destination is one buffer
    // resource plus a 32-bit element offset per lane (the host checks every span < 2^29
    // elements); lanes that must not store (padding rows, columns past the end) get an
    // offset past the range, so no branch per row.  Residual inputs (Difference.backward:
    // after = before + to) are loaded one chunk ahead of their use.
    unsigned oblk = 0, oii = 0;
    bool ovalid = false;
    // TR: this lane's 4-column group (columns 4 hq .. + 3 of the wave's 16): block, index
    // of its first column, valid columns (0..4)
    unsigned o4blk = 0, o4ii = 0;
    int o4n = 0;
    auto res_load_tr = [&](int T, float (&r)[4]) -> int {  // a lower bound of the loads issued
        const int e = p.otile[T];
        const int v = e & 0xff, z0 = (e >> 8) & 0xffff, nrow = e >> 24;
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = 0.0f;
        if (!(v < kMaxVars && p.res_ptr[v])) return 0;  // uniform
        const Rsrc3 rr_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.res_ptr[v]), 0, 0x7ffffffc,
                                                            0x00020000);
        const bool rowok = cl < nrow;
        const unsigned off = (o4blk * (unsigned)p.res_bs[v] + o4ii + (unsigned)(z0 + cl) * (unsigned)p.res_ld[v]) * 4u;
        if (p.ovec && o4n == 4 && rowok) {
            // a plain 16-byte global load: this toolchain's clang lowers
            // __builtin_amdgcn_raw_buffer_load_b128 to ONE dword load splatted over the
            // four lanes of the vector (seen in the ISA), so the buffer form is not used
            const float4 w = *reinterpret_cast<const float4*>(p.res_ptr[v] + off / 4u);
            r[0] = w.x;
            r[1] = w.y;
            r[2] = w.z;
            r[3] = w.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned o = (rowok && q < o4n) ? off + 4u * q : 0x80000000u;
                r[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr_, (int)o, 0, 0));
            }
        }
        return p.ovec ? 1 : 4;
    };
    auto out_tile_tr = [&](const b3f4& a, int T, const float (&r)[4]) -> int {  // a lower bound of the stores
        const int e = p.otile[T];
        const int v = e & 0xff, z0 = (e >> 8) & 0xffff, nrow = e >> 24;
        if (v >= kMaxVars) return 0;  // padding tile (uniform)
        int R0 = 16 * T + cl;
        asm volatile("" : "+v"(R0));  // keep the constant reads next to their use
        const float bo = s_oc[R0], sg = s_oc[kop + R0], mu = s_oc[2 * kop + R0];
        const float lo = s_oc[3 * kop + R0], hi = s_oc[4 * kop + R0], mk = s_oc[5 * kop + R0];
        const Rsrc3 ro = __builtin_amdgcn_make_buffer_rsrc(p.out_ptr[v], 0, 0x7ffffffc, 0x00020000);
        const bool has_res = p.res_ptr[v] != nullptr;  // uniform
        float y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float t = a[q] + bo;
            t = t * sg;
            t = t + mu;
            if (t < lo) t = lo;
            if (t >= hi) t = hi;
            t = t * mk;
            if (has_res) t = r[q] + t;
            y[q] = t;
        }
        const bool rowok = cl < nrow;
        const unsigned off = (o4blk * (unsigned)p.out_bs[v] + o4ii + (unsigned)(z0 + cl) * (unsigned)p.out_ld[v]) * 4u;
#ifdef FV3_B3_EXP_NOOUT  // experiment only (results invalid): store only a value that is never true
        if (y[0] == 1234.5f)
#endif
        {
            if (p.ovec && o4n == 4 && rowok) {
                const v4u w = {__builtin_bit_cast(unsigned, y[0]), __builtin_bit_cast(unsigned, y[1]),
                               __builtin_bit_cast(unsigned, y[2]), __builtin_bit_cast(unsigned, y[3])};
                __builtin_amdgcn_raw_buffer_store_b128(w, ro, (int)off, 0, 0);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned o = (rowok && q < o4n) ? off + 4u * q : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y[q]), ro, (int)o, 0, 0);
                }
            }
        }
        return p.ovec ? 1 : 4;
    };
    auto res_load = [&](int T, float (&r)[4]) -> int {  // returns the loads issued (0 or 4)
        if constexpr (TR) return res_load_tr(T, r);
        const int e = p.otile[T];
        const int v = e & 0xff, z0 = (e >> 8) & 0xffff, nrow = e >> 24;
#ifdef FV3_B3_EXP_NORES  // experiment only (results invalid): no residual loads
        if (false) {
#else
        if (v < kMaxVars && p.res_ptr[v]) {  // uniform
#endif
            const Rsrc3 rr_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.res_ptr[v]), 0, 0x7ffffffc,
                                                                0x00020000);
            const unsigned rb = oblk * (unsigned)p.res_bs[v] + oii;
            const unsigned rld = (unsigned)p.res_ld[v];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 4 * hq + q;
                const unsigned off = (ovalid & (row < nrow)) ? (rb + (unsigned)(z0 + row) * rld) * 4u : 0x80000000u;
                r[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr_, (int)off, 0, 0));
            }
            return 4;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = 0.0f;
        return 0;
    };
    auto out_tile = [&](const b3f4& a, int T, const float (&r)[4]) -> int {  // returns the stores issued
        if constexpr (TR) return out_tile_tr(a, T, r);
        const int e = p.otile[T];
        const int v = e & 0xff, z0 = (e >> 8) & 0xffff, nrow = e >> 24;
        if (v >= kMaxVars) return 0;  // padding tile (uniform)
#ifdef FV3_B3_EXP_NOEPI  // experiment only (results invalid): no epilogue, one conditional store
        {
            const float y = a[0] + a[1] + a[2] + a[3] + r[0];
            if (y == 1234.5f) {
                const Rsrc3 ro = __builtin_amdgcn_make_buffer_rsrc(p.out_ptr[v], 0, 0x7ffffffc, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, 0, 0, 0);
            }
            return 0;
        }
#endif
        int R0 = 16 * T + 4 * hq;
        asm volatile("" : "+v"(R0));  // keep the constant reads next to their use
        const b3f4 bo = *reinterpret_cast<const b3f4*>(s_oc + R0);
        const b3f4 sg = *reinterpret_cast<const b3f4*>(s_oc + kop + R0);
        const b3f4 mu = *reinterpret_cast<const b3f4*>(s_oc + 2 * kop + R0);
        const b3f4 lo = *reinterpret_cast<const b3f4*>(s_oc + 3 * kop + R0);
        const b3f4 hi = *reinterpret_cast<const b3f4*>(s_oc + 4 * kop + R0);
        const b3f4 mk = *reinterpret_cast<const b3f4*>(s_oc + 5 * kop + R0);
        const Rsrc3 ro = __builtin_amdgcn_make_buffer_rsrc(p.out_ptr[v], 0, 0x7ffffffc, 0x00020000);
        const unsigned ob = oblk * (unsigned)p.out_bs[v] + oii;
        const unsigned old_ = (unsigned)p.out_ld[v];
        const bool has_res = p.res_ptr[v] != nullptr;  // uniform
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 4 * hq + q;
            float y = a[q] + bo[q];
            y = y * sg[q];
            y = y + mu[q];
            if (y < lo[q]) y = lo[q];
            if (y >= hi[q]) y = hi[q];
            y = y * mk[q];
            if (has_res) y = r[q] + y;
            const unsigned off = (ovalid & (row < nrow)) ? (ob + (unsigned)(z0 + row) * old_) * 4u : 0x80000000u;
#ifdef FV3_B3_EXP_NOOUT  // experiment only (results invalid): store only a value that is never true
            if (y == 1234.5f)
#endif
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, (int)off, 0, 0);
        }
        return 4;
    };

    float rawA[8], rawB[8];
    int64_t tile = blockIdx.x;
    set_load_tile(tile);
    if (tile < p.ntiles) {
        if constexpr (GL) {
            glds_in(0, 0);
            if (p.n1 > 1) glds_in(1, 1);
        } else {
            load_in(rawA, 0);
            if (p.n1 > 1) load_in(rawB, 1);
        }
    }
    if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    b3_barrier();  // constants and chunk 0 visible

    // trace slot: thread 0 of the block writes tile t's record.  Only in the tools/ trace
    // variant (FV3_B3_TRACE): the clock reads are scheduling barriers that change the
    // product kernel's instruction order even when the pointer is NULL
    auto mark = [&](int slot) {
#ifdef FV3_B3_TRACE
        if (p.trace && tid == 0) {
            long long* r = p.trace + tile * 8;
            if (slot == 0) {
                r[4] = (long long)__smid();
                r[5] = (long long)__builtin_amdgcn_s_memtime();
                wait_cyc = 0;
            }
            if (slot == 3) {
                r[6] = (long long)__builtin_amdgcn_s_memtime();
                r[7] = wait_cyc;
            }
            r[slot] = wall_clock64();
        }
#else
        (void)slot;
#endif
    };
    for (; tile < p.ntiles; tile += gridDim.x) {
        mark(0);
        oblk = lblk;
        oii = lii;
        ovalid = lvalid;
        if constexpr (TR) {
            const int64_t c4 = tile * kB3Cols + wave * 16 + 4 * hq;
            const int64_t nv4 = p.ncol - c4;
            o4n = nv4 <= 0 ? 0 : (nv4 >= 4 ? 4 : (int)nv4);
            const int64_t cc = o4n > 0 ? c4 : 0;
            const int64_t b = p.ncol_blk < p.ncol ? cc / p.ncol_blk : 0;
            o4blk = (unsigned)b;
            o4ii = (unsigned)(cc - b * p.ncol_blk);
        }
        // ---- layer 1 over the padded input features ----
        zero_acc();
        if constexpr (GL) {
            // chunk c: its inputs (buffer c & 1, landed by the wait at the end of chunk c - 1),
            // then the weight DMA of chunk c + 2 and the input DMA of chunk c + 2 into the
            // buffer just read
            for (int c = 0; c < p.n1; ++c) {
                bf16x8 xb[NS];
                read_in(c & 1, c, rawA);
                stage_in(rawA, c, xb);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the reads above before the DMA refills the buffer
                step_layer(xb, [&]() {
                    if (c + 2 < p.n1) {
                        glds_in(c & 1, c + 2);
                        return 8;
                    }
                    return 0;
                });
            }
        } else
        for (int c = 0; c < p.n1; c += 2) {
            bf16x8 xb[NS];
            stage_in(rawA, c, xb);
            if (c + 2 < p.n1) load_in(rawA, c + 2);
            step_layer(xb, [] { return 0; });
            if (c + 1 < p.n1) {
                stage_in(rawB, c + 1, xb);
                if (c + 3 < p.n1) load_in(rawB, c + 3);
                step_layer(xb, [] { return 0; });
            }
        }
        hidden_epi(0);
        mark(1);
        // ---- further hidden layers ----
        for (int l = 0; l < p.nhx; ++l) {
            zero_acc();
            sfor<KS>([&](auto cc) {
                bf16x8 tb[NS];
                step_layer(hidden_b(cc, tb), [] { return 0; });
            });
            hidden_epi(l + 1);
        }
        if constexpr (NS == 3)
            sfor<KS>([&](auto cc) { splitN<NS>(Y[decltype(cc)::value], B[decltype(cc)::value]); });
        mark(2);
        // ---- output layer, two 16-row tiles per chunk; the next tile's inputs start loading ----
        const int64_t nt = tile + gridDim.x;
        if (nt < p.ntiles) {
            set_load_tile(nt);
            if constexpr (!GL) {
                load_in(rawA, 0);
                if (p.n1 > 1) load_in(rawB, 1);
            }
        }
        b3f4 accP[2];
        float resN[2][4], resP[2][4];
        if constexpr (GL) {
            // chunk oc: the weight DMA of chunk +2, this chunk's residual loads (consumed
            // one chunk later), the MFMAs, then the previous chunk's epilogue (8 stores).
            // The next tile's input DMA (16 per thread) goes out with the last chunk.
            for (int oc = 0; oc < p.n_oc; ++oc) {
                acc[0] = acc[1] = b3f4{0.0f, 0.0f, 0.0f, 0.0f};
                stage_next();
                int younger = res_load(2 * oc, resN[0]);
                younger += res_load(2 * oc + 1, resN[1]);
                if (oc + 1 == p.n_oc && nt < p.ntiles) {
                    glds_in(0, 0);
                    younger += 8;
                    if (p.n1 > 1) {
                        glds_in(1, 1);
                        younger += 8;
                    }
                }
                step_out();
                if (oc > 0) {
                    younger += out_tile(accP[0], 2 * oc - 2, resP[0]);
                    younger += out_tile(accP[1], 2 * oc - 1, resP[1]);
                }
                advance(younger);
                accP[0] = acc[0];
                accP[1] = acc[1];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    resP[0][q] = resN[0][q];
                    resP[1][q] = resN[1][q];
                }
            }
            out_tile(accP[0], 2 * p.n_oc - 2, resP[0]);
            out_tile(accP[1], 2 * p.n_oc - 1, resP[1]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's inputs landed
            mark(3);
            continue;
        }
        for (int oc = 0; oc < p.n_oc; ++oc) {
            res_load(2 * oc, resN[0]);  // lands while this chunk and the next run their MFMAs
            res_load(2 * oc + 1, resN[1]);
            acc[0] = acc[1] = b3f4{0.0f, 0.0f, 0.0f, 0.0f};
            stage_next();
            step_out();
            if (oc > 0) {  // finish the previous chunk while these MFMAs run
                out_tile(accP[0], 2 * oc - 2, resP[0]);
                out_tile(accP[1], 2 * oc - 1, resP[1]);
            }
            advance(0);
            accP[0] = acc[0];
            accP[1] = acc[1];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                resP[0][q] = resN[0][q];
                resP[1][q] = resN[1][q];
            }
        }
        out_tile(accP[0], 2 * p.n_oc - 2, resP[0]);
        out_tile(accP[1], 2 * p.n_oc - 1, resP[1]);
        mark(3);
    }
}

uint16_t bf16_rne(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

float bf16_f(uint16_t h)
{
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

}  // namespace

// ------------------------------------------------------------------------------------
// host: pack the model once (fv3_dense_create) into the bf16x3 and bf16x6 chunk streams
// ------------------------------------------------------------------------------------
static int pack_ns(fv3_dense_model* m, const fv3_dense_desc* d, int NS, B3Pack** dst)
{
    auto b = new B3Pack();
    std::unique_ptr<B3Pack> guard(b);
    b->ns = NS;
    const int W = d->width;
    b->hu = W <= 64 ? 4 : (W <= 128 ? 8 : 16);
    b->hp = 16 * b->hu;
    const int HU = b->hu, KS = HU / 2;

    // input feature groups of 8 levels of one variable (chunk = 4 groups = 32 features)
    std::vector<int> fsrc;  // padded feature -> kept feature index or -1
    int kbase = 0;
    for (int v = 0; v < m->n_in; ++v) {
        const int nkeep = m->in_nkeep[v], z0 = m->in_z0[v];
        FV3_REQUIRE(z0 + nkeep < (1 << 20), "dense_create: too many levels for the bf16x3 path");
        for (int g0 = 0; g0 < nkeep; g0 += 8) {
            const int nv = std::min(8, nkeep - g0);
            b->gmeta.push_back(v | ((z0 + g0) << 4) | (nv << 24));
            for (int j = 0; j < 8; ++j) fsrc.push_back(j < nv ? kbase + g0 + j : -1);
        }
        if (m->in_log_eps[v] > 0.0f) b->any_log = std::max(b->any_log, m->in_log_eps[v] >= 0x1p-126f ? 1 : 2);
        kbase += nkeep;
    }
    while (b->gmeta.size() % 4) {
        b->gmeta.push_back(0);
        for (int j = 0; j < 8; ++j) fsrc.push_back(-1);
    }
    FV3_REQUIRE((int)b->gmeta.size() <= kB3Groups, "dense_create: %d input features are too many for bf16x3",
                (int)fsrc.size());
    b->kp1 = (int)fsrc.size();
    b->n1 = b->kp1 / 32;
    b->nhx = d->n_hidden - 1;
    // output rows: each variable padded to a multiple of 16 rows (one variable per 16-row
    // accumulator tile, see the kernel's epilogue), tiles padded to an even count (two per
    // chunk); row R -> (variable, level) or -1
    std::vector<int> ocol_var, ocol_z, okeep;  // okeep: row's index in the model's k_out order
    auto pad_tile = [&]() {
        b->otile.push_back(255);
        for (int j = 0; j < 16; ++j) {
            ocol_var.push_back(-1);
            ocol_z.push_back(0);
            okeep.push_back(-1);
        }
    };
    for (int v = 0, o = 0; v < m->n_out; ++v) {
        const int nz = m->out_nz[v];
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, nz < (1 << 16), "dense_create: output levels too many for bf16x3");
        for (int z0 = 0; z0 < nz; z0 += 16) {
            const int nrow = std::min(16, nz - z0);
            b->otile.push_back(v | (z0 << 8) | (nrow << 24));
            for (int j = 0; j < 16; ++j) {
                ocol_var.push_back(j < nrow ? v : -1);
                ocol_z.push_back(j < nrow ? z0 + j : 0);
                okeep.push_back(j < nrow ? o + z0 + j : -1);
            }
        }
        o += nz;
    }
    if (b->otile.size() % 2) pad_tile();
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, (int)b->otile.size() <= kB3OutTiles,
                     "dense_create: %d padded output rows are too many for bf16x3", (int)ocol_var.size());
    b->n_oc = (int)b->otile.size() / 2;
    b->kop = 16 * (int)b->otile.size();
    b->nch = b->n1 + b->nhx * KS + b->n_oc;
    const size_t cbe = (size_t)512 * NS * HU;  // bf16 elements per chunk
    FV3_REQUIRE((size_t)b->nch * cbe * 2 < (1u << 31), "dense_create: model too large for the bf16x3 stream");

    std::vector<uint16_t> ws((size_t)b->nch * cbe, 0);
    // fragment i of a chunk: lane (q = lane >> 4, r = lane & 15) element j is A[row r][k 8q + j];
    // part s of it (the kernel's splitN: rne of the residual of the parts before) at +512 s
    auto put = [&](int chunk, int i, int lane, int j, float v) {
        const size_t at = (size_t)chunk * cbe + ((size_t)(NS * i) * 64 + lane) * 8 + j;
        float r = v;
        for (int s = 0; s < NS; ++s) {
            const uint16_t h = bf16_rne(r);
            ws[at + 512 * s] = h;
            r = r - bf16_f(h);
        }
    };
    // layer 1: natural feature order, k = 32c + 8q + j; fragment t = unit tile t
    const float* K0 = d->hidden_kernel[0];
    for (int c = 0; c < b->n1; ++c)
        for (int t = 0; t < HU; ++t)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 8; ++j) {
                    const int f = 32 * c + 8 * (lane >> 4) + j;
                    const int unit = 16 * t + (lane & 15);
                    const int src = fsrc[f];
                    put(c, t, lane, j, (src >= 0 && unit < W) ? K0[(size_t)src * W + unit] : 0.0f);
                }
    // hidden and output layers: k-step c, element j of lane quarter q contracts over the
    // previous layer's unit 32c + 16(j>>2) + 4q + (j&3) (its accumulator layout)
    auto in_unit = [](int c, int lane, int j) { return 32 * c + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3); };
    for (int li = 0; li < b->nhx; ++li) {
        const float* K = d->hidden_kernel[li + 1];
        for (int c = 0; c < KS; ++c)
            for (int t = 0; t < HU; ++t)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const int in = in_unit(c, lane, j), unit = 16 * t + (lane & 15);
                        put(b->n1 + li * KS + c, t, lane, j, (in < W && unit < W) ? K[(size_t)in * W + unit] : 0.0f);
                    }
    }
    // output chunk oc, fragment i = 2q + ts: tile 2oc + ts over k-step q
    for (int oc = 0; oc < b->n_oc; ++oc)
        for (int i = 0; i < HU; ++i)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 8; ++j) {
                    const int q = i >> 1, ts = i & 1;
                    const int in = in_unit(q, lane, j);
                    const int R = 16 * (2 * oc + ts) + (lane & 15);
                    float v = 0.0f;
                    if (in < W && ocol_var[R] >= 0) {
                        const int ov = ocol_var[R], oz = ocol_z[R];
                        v = d->out_kernel[ov][(size_t)in * m->out_nz[ov] + oz];
                    }
                    put(b->n1 + b->nhx * KS + oc, i, lane, j, v);
                }

    // constants: [kp1] mean | [kp1] 1/(sigma+eps) | [nh][HP] bias | [6][kop]
    const int nh = 1 + b->nhx, kop = b->kop, HP = b->hp;
    b->nconst = 2 * b->kp1 + nh * HP + 6 * kop;
    std::vector<float> cst((size_t)b->nconst, 0.0f);
    for (int f = 0; f < b->kp1; ++f) {
        const int src = fsrc[f];
        if (src < 0) continue;
        cst[f] = d->in_mean[src];
        volatile float den = d->in_sigma[src] + d->epsilon;  // StandardNormLayer: f32(sigma + eps)
        cst[b->kp1 + f] = 1.0f / den;
    }
    for (int l = 0; l < nh; ++l)
        for (int u = 0; u < W; ++u) cst[2 * b->kp1 + l * HP + u] = d->hidden_bias[l][u];
    float* oc = cst.data() + 2 * b->kp1 + nh * HP;
    for (int R = 0; R < kop; ++R) {
        float v[6] = {0.0f, 1.0f, 0.0f, -INFINITY, INFINITY, 1.0f};
        if (ocol_var[R] >= 0) {
            const int ov = ocol_var[R], oz = ocol_z[R], K = okeep[R];
            v[0] = d->out_bias[ov][oz];
            v[1] = d->out_sigma[K];
            v[2] = d->out_mean[K];
            if (d->out_min) v[3] = d->out_min[K];
            if (d->out_max) v[4] = d->out_max[K];
            if (d->out_mask) v[5] = d->out_mask[K];
        }
        for (int k = 0; k < 6; ++k) oc[(size_t)k * kop + R] = v[k];
    }

    b->wbytes = (int)(ws.size() * 2);
    b->consts_off = ((size_t)b->wbytes + 255) / 256 * 256;
    FV3_HIP(hipMalloc(&b->dbuf, b->consts_off + cst.size() * 4));
    FV3_HIP(hipMemcpy(b->dbuf, ws.data(), ws.size() * 2, hipMemcpyHostToDevice));
    FV3_HIP(hipMemcpy((char*)b->dbuf + b->consts_off, cst.data(), cst.size() * 4, hipMemcpyHostToDevice));
    *dst = guard.release();
    return FV3_OK;
}

// A host copy of the parts of fv3_dense_desc that pack_ns reads (the caller's arrays are
// only valid during fv3_dense_create): the bf16x6 stream, which only bf16x6 callers need,
// is packed from it on the first bf16x6 forward instead of with every model.
struct B3Desc {
    fv3_dense_desc d{};
    std::vector<std::vector<float>> hk, hb, ok, ob;
    std::vector<const float*> hkp, hbp, okp, obp;
    std::vector<float> in_mean, in_sigma, out_mean, out_sigma, out_min, out_max, out_mask;
};

static B3Desc* copy_desc(const fv3_dense_model* m, const fv3_dense_desc* d)
{
    auto c = std::make_unique<B3Desc>();
    const int W = d->width, kin = m->k_in, kout = m->k_out;
    auto vec = [](const float* p, size_t n) { return p ? std::vector<float>(p, p + n) : std::vector<float>(); };
    c->in_mean = vec(d->in_mean, kin);
    c->in_sigma = vec(d->in_sigma, kin);
    c->out_mean = vec(d->out_mean, kout);
    c->out_sigma = vec(d->out_sigma, kout);
    c->out_min = vec(d->out_min, kout);
    c->out_max = vec(d->out_max, kout);
    c->out_mask = vec(d->out_mask, kout);
    for (int l = 0; l < d->n_hidden; ++l) {
        c->hk.push_back(vec(d->hidden_kernel[l], (size_t)(l == 0 ? kin : W) * W));
        c->hb.push_back(vec(d->hidden_bias[l], W));
    }
    for (int v = 0; v < m->n_out; ++v) {
        c->ok.push_back(vec(d->out_kernel[v], (size_t)W * m->out_nz[v]));
        c->ob.push_back(vec(d->out_bias[v], m->out_nz[v]));
    }
    for (auto& x : c->hk) c->hkp.push_back(x.data());
    for (auto& x : c->hb) c->hbp.push_back(x.data());
    for (auto& x : c->ok) c->okp.push_back(x.data());
    for (auto& x : c->ob) c->obp.push_back(x.data());
    c->d = *d;
    c->d.in_mean = c->in_mean.data();
    c->d.in_sigma = c->in_sigma.data();
    c->d.out_mean = c->out_mean.data();
    c->d.out_sigma = c->out_sigma.data();
    c->d.out_min = d->out_min ? c->out_min.data() : nullptr;
    c->d.out_max = d->out_max ? c->out_max.data() : nullptr;
    c->d.out_mask = d->out_mask ? c->out_mask.data() : nullptr;
    c->d.hidden_kernel = c->hkp.data();
    c->d.hidden_bias = c->hbp.data();
    c->d.out_kernel = c->okp.data();
    c->d.out_bias = c->obp.data();
    // pack_ns reads nothing else of the description (the rest is in the model)
    c->d.in_nz = nullptr;
    c->d.in_clip = nullptr;
    c->d.out_nz = nullptr;
    c->d.in_log_eps = nullptr;
    c->d.out_residual = nullptr;
    return c.release();
}

// Each split stream is packed on its own: a model one of them cannot hold (too many
// input features or output rows, a stream past 2 GiB) leaves only that precision
// unsupported (fv3_dense_forward_ex returns FV3_ERR_UNSUPPORTED for it), and the exact-f32
// path is never affected.  Only a HIP failure fails fv3_dense_create.  The bf16x3 stream
// is packed here; the bf16x6 one (1.5x its size) on the first bf16x6 forward.
int b3_pack(fv3_dense_model* m, const fv3_dense_desc* d)
{
    const int st = pack_ns(m, d, 2, &m->b3);
    if (st == FV3_ERR_HIP) return st;
    if (st != FV3_OK) {
        m->b3 = nullptr;
        clear_error();
    }
    m->b6_src = copy_desc(m, d);
    return FV3_OK;
}

// the bf16x6 stream of `m`, packed now if this is its first use (nullptr: unsupported
// for this model, with the reason in fv3_last_error; HIP failures return FV3_ERR_HIP)
static int b6_stream(const fv3_dense_model* cm, const B3Pack** out)
{
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    fv3_dense_model* m = const_cast<fv3_dense_model*>(cm);  // the lazily packed stream only
    if (!m->b6 && m->b6_src) {
        const int st = pack_ns(m, &m->b6_src->d, 3, &m->b6);
        if (st == FV3_ERR_HIP) return st;  // keep the source: a later call may retry
        if (st != FV3_OK) m->b6 = nullptr;
        delete m->b6_src;
        m->b6_src = nullptr;
        if (st != FV3_OK) return st;
    }
    *out = m->b6;
    return FV3_OK;
}

void b3_free(fv3_dense_model* m)
{
    if (!m) return;
    for (B3Pack** pk : {&m->b3, &m->b6}) {
        if (!*pk) continue;
        if ((*pk)->dbuf) (void)hipFree((*pk)->dbuf);
        delete *pk;
        *pk = nullptr;
    }
    delete m->b6_src;
    m->b6_src = nullptr;
}

}  // namespace fv3

extern "C" int fv3_dense_forward_ex(const fv3_dense_model* m, const float* const* inputs, const fv3_layout* in_l,
                                    float* const* outputs, const fv3_layout* out_l, int64_t ncol, int precision,
                                    void* stream)
{
    using namespace fv3;
    if (precision == FV3_DENSE_F32) return fv3_dense_forward(m, inputs, in_l, outputs, out_l, ncol, stream);
    clear_error();
    FV3_REQUIRE(precision == FV3_DENSE_BF16X3 || precision == FV3_DENSE_BF16X6,
                "dense_forward_ex: unknown precision %d", precision);
    FV3_REQUIRE(m, "dense_forward_ex: NULL model");
    const B3Pack* pk = m->b3;
    if (precision == FV3_DENSE_BF16X6) {
        const int st = b6_stream(m, &pk);
        if (st == FV3_ERR_HIP) return st;
        if (st != FV3_OK) pk = nullptr;
    }
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, pk, "dense_forward_ex: this model has no bf16 split pack "
                     "(too many input features or output rows); use FV3_DENSE_F32");
    FV3_REQUIRE(ncol >= 0, "dense_forward_ex: ncol < 0");
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(inputs && in_l && outputs && out_l, "dense_forward_ex: NULL argument");
    const B3Pack& b = *pk;
    B3Args a{};
    const int64_t nb = in_l[0].ncol_blk;
    for (int v = 0; v < m->n_in; ++v) {
        FV3_REQUIRE(inputs[v], "dense_forward_ex: input %d is NULL", v);
        FV3_REQUIRE(layout_ok(in_l[v], ncol) && in_l[v].ncol_blk == nb,
                    "dense_forward_ex: input %d layout invalid or ncol_blk differs", v);
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, in_l[v].ld < ((int64_t)1 << 28),
                         "dense_forward_ex: input %d level stride >= 2^28 elements (bf16x3 path)", v);
        a.in[v] = B3InVar{inputs[v], in_l[v].ld, in_l[v].blk_stride, m->in_log_eps[v], 0};
    }
    for (int v = 0; v < m->n_out; ++v) {
        FV3_REQUIRE(outputs[v], "dense_forward_ex: output %d is NULL", v);
        FV3_REQUIRE(layout_ok(out_l[v], ncol) && out_l[v].ncol_blk == nb,
                    "dense_forward_ex: output %d layout invalid or ncol_blk differs", v);
        a.out_ptr[v] = outputs[v];
        a.out_ld[v] = out_l[v].ld;
        a.out_bs[v] = out_l[v].blk_stride;
        const int r = m->out_residual[v];
        a.res_ptr[v] = r >= 0 ? inputs[r] : nullptr;
        a.res_ld[v] = r >= 0 ? in_l[r].ld : 0;
        a.res_bs[v] = r >= 0 ? in_l[r].blk_stride : 0;
    }
    a.wstream = b.dbuf;
    a.consts = reinterpret_cast<const float*>((const char*)b.dbuf + b.consts_off);
    a.wbytes = b.wbytes;
    a.nch = b.nch;
    a.n1 = b.n1;
    a.nhx = b.nhx;
    a.n_oc = b.n_oc;
    a.kp1 = b.kp1;
    a.kop = b.kop;
    a.nconst = b.nconst;
    a.any_log = b.any_log;
    a.ncol = ncol;
    a.ncol_blk = nb;
    a.trace = m->tmpl.trace;
    for (size_t g = 0; g < b.gmeta.size(); ++g) a.gmeta[g] = b.gmeta[g];
    for (size_t g = 0; g < b.otile.size(); ++g) a.otile[g] = b.otile[g];
    // the epilogue addresses outputs / residual inputs with 32-bit byte offsets
    // ((block * bs + index + z * ld) * 4 < 2^31) and 32-bit block / index values
    FV3_REQUIRE(ncol < (int64_t)1 << 31, "dense_forward_ex: too many columns for bf16x3");
    auto span = [&](const fv3_layout& l, int nz) {
        const int64_t nblk = (ncol + l.ncol_blk - 1) / l.ncol_blk;
        return (nblk - 1) * l.blk_stride + (int64_t)(nz - 1) * l.ld + l.ncol_blk;
    };
    for (int v = 0; v < m->n_out; ++v) {
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, span(out_l[v], m->out_nz[v]) < ((int64_t)1 << 29),
                         "dense_forward_ex: output %d spans too many elements for bf16x3", v);
        const int r = m->out_residual[v];
        if (r >= 0)
            FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, span(in_l[r], m->in_nz[r]) < ((int64_t)1 << 29),
                             "dense_forward_ex: residual input %d spans too many elements for bf16x3", r);
    }

    // FV3_B3_STAGE=glds / reg: the LDS-DMA or the register-staged pipeline (A/B)
    const char* stg_env = fv3::variant_env("FV3_B3_STAGE");
    static std::mutex mu;
    static int n_cu = 0;
    {
        std::lock_guard<std::mutex> lock(mu);
        if (!n_cu) {
            int dev = 0;
            FV3_HIP(hipGetDevice(&dev));
            FV3_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
        }
    }
    // 4-wave blocks of 64 columns where 128-column tiles would leave CUs idle (C48: 108
    // tiles of 128 on 256 CUs -> 216 of 64); FV3_B3_WAVES=4|8 forces one (A/B)
    int nwv = (ncol + kB3Cols - 1) / kB3Cols < n_cu ? 4 : 8;
    if (const char* e = fv3::variant_env("FV3_B3_WAVES")) nwv = atoi(e) == 4 ? 4 : 8;
    const int nthr = 64 * nwv, ncols = 16 * nwv;
    a.ntiles = (ncol + ncols - 1) / ncols;
    auto lds_of = [&](int sl) {
        return (size_t)b3_slots(sl) * 1024 * b.ns * b.hu + (size_t)b3_in_bytes(sl > 0, nwv) +
               (size_t)4 * ((b.nconst + 7) & ~7) + sizeof(B3Grp) * 4 * b.n1;
    };
    // the LDS-DMA pipeline with a 3-slot ring where it fits, else (bf16x6) with 2 slots;
    // a model that only fits the register-staged pipeline's LDS runs on that one
    int sl = 0;
    if (stg_env ? stg_env[0] == 'g' : kB3GldsDefault)
        sl = lds_of(3) <= 160 * 1024 ? 3 : (b.ns == 3 && lds_of(2) <= 160 * 1024 ? 2 : 0);
    if (stg_env && stg_env[0] == 'g' && stg_env[1] == '2' && b.ns == 3 && lds_of(2) <= 160 * 1024) sl = 2;  // A/B
    // the transposed output layer (TR) on the LDS-DMA pipeline when 4-column groups never
    // cross a column block; 16-byte epilogue accesses when every output / residual row is
    // 16-byte aligned.  FV3_B3_TR=0 keeps the row-per-lane epilogue (A/B, tests).
    bool tr = sl > 0 && (nb >= ncol || nb % 4 == 0);
    if (const char* e = fv3::variant_env("FV3_B3_TR")) tr = tr && atoi(e) != 0;
    {
        bool vec = true;
        auto al = [&](const void* ptr, const fv3_layout& l) {
            return ((uintptr_t)ptr % 16) == 0 && l.ld % 4 == 0 && (nb >= ncol || l.blk_stride % 4 == 0);
        };
        for (int v = 0; v < m->n_out; ++v) {
            vec = vec && al(outputs[v], out_l[v]);
            const int r = m->out_residual[v];
            if (r >= 0) vec = vec && al(inputs[r], in_l[r]);
        }
        a.ovec = vec ? 1 : 0;
    }
    auto pick = [&](auto ns) -> const void* {
        constexpr int NS = decltype(ns)::value;
        auto by_hu = [&](auto slc) -> const void* {
            constexpr int S = decltype(slc)::value;
            if constexpr (S > 0) {
                if (tr) {
                    if (nwv == 4)
                        return b.hu == 4 ? (const void*)dense_b3_kernel<4, S, NS, 4, true>
                             : b.hu == 8 ? (const void*)dense_b3_kernel<8, S, NS, 4, true>
                                         : (const void*)dense_b3_kernel<16, S, NS, 4, true>;
                    return b.hu == 4 ? (const void*)dense_b3_kernel<4, S, NS, 8, true>
                         : b.hu == 8 ? (const void*)dense_b3_kernel<8, S, NS, 8, true>
                                     : (const void*)dense_b3_kernel<16, S, NS, 8, true>;
                }
            }
            if (nwv == 4)
                return b.hu == 4 ? (const void*)dense_b3_kernel<4, S, NS, 4>
                     : b.hu == 8 ? (const void*)dense_b3_kernel<8, S, NS, 4>
                                 : (const void*)dense_b3_kernel<16, S, NS, 4>;
            return b.hu == 4 ? (const void*)dense_b3_kernel<4, S, NS, 8>
                 : b.hu == 8 ? (const void*)dense_b3_kernel<8, S, NS, 8>
                             : (const void*)dense_b3_kernel<16, S, NS, 8>;
        };
        if constexpr (NS == 3)
            if (sl == 2) return by_hu(std::integral_constant<int, 2>{});
        return sl == 3 ? by_hu(std::integral_constant<int, 3>{}) : by_hu(std::integral_constant<int, 0>{});
    };
    const void* kfn = b.ns == 3 ? pick(std::integral_constant<int, 3>{}) : pick(std::integral_constant<int, 2>{});
    const size_t lds = lds_of(sl);
    FV3_REQUIRE(lds <= 160 * 1024, "dense_forward_ex: model needs %zu bytes of LDS", lds);
    static std::vector<std::pair<std::pair<const void*, size_t>, int>> resident;
    int res = 0;
    {
        std::lock_guard<std::mutex> lock(mu);
        for (auto& r : resident)
            if (r.first.first == kfn && r.first.second == lds) res = r.second;
        if (!res) {
            FV3_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, kfn, nthr, lds));
            res = std::max(1, res);
            resident.push_back({{kfn, lds}, res});
        }
    }
    int64_t grid = std::min<int64_t>(a.ntiles, (int64_t)res * n_cu);
    if (const char* e = fv3::variant_env("FV3_B3_GRID")) grid = std::min<int64_t>(a.ntiles, std::max(1, atoi(e)));
    void* kargs[] = {&a};
    FV3_HIP(hipLaunchKernel(kfn, dim3((unsigned)grid), dim3(nthr), kargs, lds, (hipStream_t)stream));
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
