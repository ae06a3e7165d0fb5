// fv3net_amd — fused column-wise DenseModel predict on gfx950.
//
// Replaces the Keras `model.predict(inputs)` call in PureKerasModel.predict
// (external/fv3fit/fv3fit/keras/_models/shared/pure_keras.py:112) for the graph
// built by external/fv3fit/fv3fit/keras/_models/dense.py:234-305:
//   clip -> StandardNormLayer (x-mean)/(sigma+eps) -> concat -> [Dense(width, relu)] x n_hidden
//   -> Dense(out_nz) per output -> StandardDenormLayer y*sigma+mean -> OutputLimit -> zero mask
// in ONE kernel: inputs are read straight from the prognostic state's
// [level][column] arrays (fv3fit's stack() is a zero-copy view here) and the
// tendencies are written straight into [level][column] outputs (the unstack).
//
// Mapping (CDNA4, wave64, v_mfma_f32_16x16x4_f32 — exact f32, no xf32 on gfx950):
//  * a block of NW waves (4: one per SIMD; 8: two per SIMD, used when there are few
//    tiles per CU, e.g. C48) owns a tile of NC x 16 columns for the whole network;
//    wave w owns hidden-unit tiles [w*T4, (w+1)*T4) of every hidden layer
//    (T4 = width/(16 NW) tiles of 16 units); lane l holds column (l & 15) and k-slot
//    (l >> 4) of every B operand;
//  * a layer's output is written to LDS in the MFMA accumulator layout
//    ([tile][lane] x 4 regs, register r of tile t = unit 16t + 4(l>>4) + r) and the
//    next layer reads it back with one ds_read_b128 per 4 k-steps: k-step s = 4t + r
//    takes register r of tile t, i.e. the contraction order over hidden units is
//    permuted and the packed weights carry the same permutation (no shuffles);
//  * ONE activation buffer is updated in place (read, barrier, write, barrier) and
//    the staged inputs alias it: ~37 KB of LDS per block -> 3 blocks per CU;
//  * inputs are loaded by "slots" (64 NW threads x one feature row each, the
//    variable uniform per slot), all slots of a tile in flight at once; blocks are
//    persistent over column tiles and load the NEXT tile's inputs into registers
//    while the current tile runs its hidden and output layers;
//  * weights are pre-packed at create time into [k-step][wave][lane][T4] fragment
//    order (every A-operand fetch is one coalesced T4*4 B/lane load) and stream
//    through 3-deep compile-time register rings; each layer's first two groups are
//    loaded before the barrier that precedes it, so no layer starts on a cold ring;
//  * the output layer: whole 16-row output tiles dealt to the waves (one weight fetch
//    feeds both column tiles), the remainder split into (tile, column tile) units so
//    every SIMD gets the same work; the bias/denorm/limit/mask epilogue reads its
//    constants from LDS and writes with range-checked buffer stores;
//  * each input variable's features and each output tile are padded so a k-step
//    (4 features) never straddles two variables.
// Roofline: fp32 MFMA-bound.  2*(k_in*w + (n_hidden-1)*w*w + w*k_out) FLOP per
// column (292,864 for the 2x256 C48 model) against (k_in + k_out) * 4 B of HBM.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "dense_model.h"

// output tiles per wave per pass and output-weight ring depth (A/B: OUT_TILES=2,
// OUT_RING=2 was 0.5% slower at C96-C384, equal at C48)
#ifndef OUT_TILES
#define OUT_TILES 1
#endif
#ifndef OUT_RING
#define OUT_RING 3
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace fv3 {



// phase timestamps of tile t (thread 0): 0 start, 5 prologue done (constants in LDS),
// 1 inputs staged, 2 layer 1 done, 3 hidden layers done, 4 end; slot 7 = hardware CU id
__device__ __forceinline__ void trace_mark(__attribute__((address_space(4))) const DenseArgs& p, int64_t tile,
                                           int slot)
{
    if (p.trace && threadIdx.x == 0) {
        p.trace[tile * 8 + slot] = wall_clock64();
        if (slot == 0) p.trace[tile * 8 + 7] = (long long)__smid();
        // slot 6: shader-clock cycles from tile start (5) to tile end (4)
        if (slot == 5) p.trace[tile * 8 + 6] = (long long)__builtin_amdgcn_s_memtime();
        if (slot == 4) p.trace[tile * 8 + 6] = (long long)__builtin_amdgcn_s_memtime() - p.trace[tile * 8 + 6];
    }
}

// compile-time loop: f(std::integral_constant<int, i>) for i = 0..N-1 (register
// rings indexed by i stay in registers with no copies between iterations)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f)
{
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int T4>
struct Frag;
template <>
struct Frag<1> {
    typedef float type;
};
template <>
struct Frag<2> {
    typedef f32x2 type;
};
template <>
struct Frag<4> {
    typedef f32x4 type;
};

template <int T4>
__device__ __forceinline__ float frag_at(const typename Frag<T4>::type& a, int j)
{
    if constexpr (T4 == 1)
        return a;
    else
        return a[j];
}

// every f32 MFMA of the kernel (FV3_EXP_NOMFMA, experiment only: operands consumed, no MFMA)
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c)
{
#ifdef FV3_EXP_NOMFMA
    asm volatile("" ::"v"(a), "v"(b));
    return c;
#else
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#endif
}

// the tile loop's workgroup barriers
// Only LDS traffic is ordered by these barriers (staged inputs, activations, constants):
// wait for this wave's LDS operations, then s_barrier.  Global loads in flight (the next
// tile's inputs, the weight rings) are NOT drained, as __syncthreads() would (vmcnt(0)).
__device__ __forceinline__ void tile_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// column data: plain loads / stores.  Measured (tools/ab.py): nontemporal input
// loads cost the emulator 4% (its residual outputs re-read the inputs), nontemporal
// stores cost the stepper 8% (its next kernel reads the tendencies); C48 gains < 1%
__device__ __forceinline__ float in_load(const float* p)
{
#ifdef FV3_EXP_NOINLOAD  // experiment only (results invalid): no input loads
    float v;
    asm volatile("v_mov_b32 %0, 1.0" : "=v"(v));
    return v;
#endif
    return *p;
}

// element `off` of an input slot whose base is stored as const float*: IT = double for
// float64 state read in place (the f32 model input is the round-to-nearest cast, as
// Keras's own cast); IT = float is the plain load above
template <typename IT>
__device__ __forceinline__ IT in_at(const float* base, int64_t off)
{
    if constexpr (std::is_same<IT, float>::value) return in_load(base + off);
    else return reinterpret_cast<const IT*>(base)[off];
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.0f, 0.0f, 0.0f, 0.0f}; }

// log(max(x, eps)) with tf.maximum's NaN propagation and a correctly rounded-class log
__device__ __forceinline__ float __logf_exact(float x, float eps) { return x != x ? x : logf(x > eps ? x : eps); }

// relu(acc + bias) for this wave's T4 tiles (x NC column tiles), stored in accumulator layout
template <int T4, int NC, int NW>
__device__ __forceinline__ void bias_relu_store(f32x4 (&acc)[NC][T4], const float* __restrict__ b, int wave,
                                                int lane, int kr, f32x4* __restrict__ dst)
{
    constexpr int HT = NW * T4;
#pragma unroll
    for (int j = 0; j < T4; ++j) {
        const int m = wave * T4 + j;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b + 16 * m + 4 * kr);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float x = acc[c][j][r] + bb[r];
                v[r] = x > 0.0f ? x : 0.0f;
            }
            dst[(c * HT + m) * 64 + lane] = v;
        }
    }
}

// Weights are read with buffer loads from one resource over the model allocation:
// the lane offset is one VGPR and every per-group offset is a scalar, so nothing
// per-address is kept in VGPRs (with 64-bit pointers, the compile-time group offsets
// of every layer become loop-invariant VGPR pairs in the persistent tile loop).
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc make_rsrc(const void* base, int bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

template <typename FT>
__device__ __forceinline__ FT bload(Rsrc r, int voff, int soff)
{
#ifdef FV3_EXP_L1_WEIGHTS  // experiment only: every weight fragment from one 4 KiB window (L1 hits)
    soff &= 0xfff;
#endif
#ifdef FV3_EXP_NOWLOAD  // experiment only (results invalid): no weight loads at all
    FT v;
    if constexpr (sizeof(FT) == 16) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(v[0]) : "s"(soff));
        v[1] = v[0]; v[2] = v[0]; v[3] = v[0];
    } else if constexpr (sizeof(FT) == 8) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(v[0]) : "s"(soff));
        v[1] = v[0];
    } else {
        asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(soff));
    }
    return v;
#endif
    if constexpr (sizeof(FT) == 16)
        return __builtin_bit_cast(FT, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    else if constexpr (sizeof(FT) == 8)
        return __builtin_bit_cast(FT, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    else
        return __builtin_bit_cast(FT, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// first RD-1 groups (4 k-steps each) of a [k-step][wave][lane] fragment stream
// starting at byte offset soff (voff = this lane's (wave * 64 + lane) * sizeof(FT)).
// RD = ring depth: a ring of RD groups is refilled RD-1 groups ahead of use.
template <int RD, int NW, typename FT>
__device__ __forceinline__ void prime_ring(FT (&g)[RD][4], Rsrc r, int voff, int soff)
{
    constexpr int KS = 64 * NW * sizeof(FT);  // bytes per k-step
#pragma unroll
    for (int d = 0; d + 1 < RD; ++d)
#pragma unroll
        for (int q = 0; q < 4; ++q) g[d][q] = bload<FT>(r, voff, soff + (4 * d + q) * KS);
}

// acc[c][j] += W^T h over all HT*4 k-steps, h read from LDS in accumulator layout.
// Weight fragments stream through the RD-group ring g (groups 0..RD-2 primed by the
// caller), RD-1 groups (4*T4*NC MFMAs each) ahead of use.
template <int T4, int NC, int RD, int NW>
__device__ __forceinline__ void gemm_hidden(f32x4 (&acc)[NC][T4], const f32x4* __restrict__ src, Rsrc rw,
                                            int voff, int soff, typename Frag<T4>::type (&g)[RD][4], int lane)
{
    constexpr int HT = NW * T4;
    typedef typename Frag<T4>::type FT;
    constexpr int KS = 64 * NW * sizeof(FT);
    f32x4 bq[2][NC];  // B operands, one group ahead
#pragma unroll
    for (int c = 0; c < NC; ++c) bq[0][c] = src[(c * HT) * 64 + lane];
    static_for<HT>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t + RD - 1 < HT) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                g[(t + RD - 1) % RD][r] = bload<FT>(rw, voff, soff + (4 * (t + RD - 1) + r) * KS);
        }
        if constexpr (t + 1 < HT) {
#pragma unroll
            for (int c = 0; c < NC; ++c) bq[(t + 1) % 2][c] = src[(c * HT + t + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetches ahead of this group's MFMAs
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < T4; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    acc[c][j] = mfma4(frag_at<T4>(g[t % RD][r], j), bq[t % 2][c][r], acc[c][j]);
    });
}

// o[i][c] = W_{m_i}^T h_c for N output tiles over all HT*4 k-steps and NCC column
// tiles: one weight fragment feeds NCC MFMAs (src = column tile c0's activations; the
// next column tile is HT*64 f32x4 further); soff[i] = byte offset of tile i's weights
constexpr int kOutTiles = OUT_TILES;  // output tiles per wave per pass
constexpr int kOutRing = OUT_RING;    // output-weight ring depth (groups held; refilled kOutRing-1 ahead)
template <int HT, int N, int NCC, int RD, int NCA>
__device__ __forceinline__ void gemm_out_tiles(f32x4 (&o)[kOutTiles][NCA], const f32x4* __restrict__ src, Rsrc rw,
                                               int voff, const int (&soff)[kOutTiles],
                                               f32x4 (&g)[RD][kOutTiles])
{
    f32x4 bq[2][NCC];
#pragma unroll
    for (int c = 0; c < NCC; ++c) bq[0][c] = src[(c * HT) * 64];
    static_for<HT>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t + RD - 1 < HT) {
#pragma unroll
            for (int i = 0; i < N; ++i) g[(t + RD - 1) % RD][i] = bload<f32x4>(rw, voff, soff[i] + (t + RD - 1) * 1024);
        }
        if constexpr (t + 1 < HT) {
#pragma unroll
            for (int c = 0; c < NCC; ++c) bq[(t + 1) % 2][c] = src[(c * HT + t + 1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int c = 0; c < NCC; ++c) o[i][c] = mfma4(g[t % RD][i][r], bq[t % 2][c][r], o[i][c]);
    });
}

template <int RD>
__device__ __forceinline__ void prime_out_tiles(f32x4 (&g)[RD][kOutTiles], Rsrc rw, int voff, const int (&soff)[kOutTiles],
                                                int n)
{
#pragma unroll
    for (int i = 0; i < kOutTiles; ++i)
        if (i < n) {
#pragma unroll
            for (int d = 0; d + 1 < RD; ++d) g[d][i] = bload<f32x4>(rw, voff, soff[i] + d * 1024);
        }
}

typedef __attribute__((address_space(4))) const DenseArgs KArgs;

// WPE: waves per SIMD the register allocation targets (2: no limit below 256 VGPRs;
// 3: <= 168, letting three blocks share a CU)
// RD: weight ring depth (groups of 4 k-steps held; refilled RD-1 groups ahead)
// NW: waves per block (4: one per SIMD; 8: two per SIMD sharing a tile, T4 halved)
template <int T4, int NC, int WPE, int RD, int NW, typename IT = float>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void dense_forward_kernel(DenseArgs pa)
{
    // read the arguments in place in the kernarg segment (constant address space):
    // capturing a by-value kernel parameter by reference would copy it to scratch
    (void)pa;
    KArgs& p = *(KArgs*)(__builtin_amdgcn_kernarg_segment_ptr());
    constexpr int NT = 64 * NW;  // threads per block
    constexpr int HT = NW * T4;  // hidden tiles of 16 units
    constexpr int HP = 16 * HT;  // padded width
    constexpr int NCOL = 16 * NC;
    constexpr int FPS = NT / NCOL;  // feature rows per slot
    static_assert(FPS == 8 || FPS == 16, "the staging address split assumes 8 or 16 rows per slot");
    typedef typename Frag<T4>::type FT;
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
    f32x4* hbuf = lds;             // activations [NC][HT][64]
    f32x4* sbuf = lds + p.lds_s;   // staged inputs [NC][kp/16][64], a buffer of their own: the
                                   // next tile's inputs are staged while this tile runs
    float* s_mean = reinterpret_cast<float*>(lds + p.lds_x);  // [kp]
    float* s_denom = s_mean + p.kp;                            // [kp]
    float* s_ep = s_denom + p.kp;                              // [6][kop]
    const int kop = 16 * p.n_otiles;
    // hidden-layer biases [1 + n_hidden_extra][HP], after the dummy f32x4: read from LDS,
    // not memory, so the bias reads after the next tile's input loads are issued do not
    // wait for those HBM loads (vector-memory loads complete in issue order)
    float* s_bias = s_ep + 6 * kop + 4;

    // issue priority over co-resident waves of other kernels (a VALU-bound remap beside
    // this MFMA-bound predict): s_setprio takes an immediate
    // (p.prio 0: the prologue alone at priority 1, so a block that starts beside a
    // computing one is not held back behind the older block's waves: C48, where a CU
    // runs two one-tile blocks, 42.0 -> 41.5 us; C384 unchanged)
    if (p.prio <= 1) __builtin_amdgcn_s_setprio(1);
    else if (p.prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (p.prio >= 3) __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kr = lane >> 4;
    const int cb = threadIdx.x % NCOL;   // column of this thread in the input slots
    const int fq0 = threadIdx.x / NCOL;  // feature row of this thread within a slot

    // ---- input slots: issue every load of a tile at once ----
    // slots prefetched into registers: kRawSlots x 8 feature rows (160) whatever FPS
    constexpr int RS = kRawSlots * 8 / FPS;
    IT raw[RS];  // converted to f32 at staging, after every load of the tile is issued
    auto col_of = [&](int64_t tile, int64_t& blk, int64_t& ii) {
        const int64_t col = tile * NCOL + cb;
        const bool valid = col < p.ncol;
        const int64_t cc = valid ? col : 0;
        if (p.ncol_blk >= p.ncol) {  // one block (uniform): no 64-bit division
            blk = 0;
            ii = cc;
        } else {
            blk = cc / p.ncol_blk;
            ii = cc - blk * p.ncol_blk;
        }
        return valid;
    };
    // slot q's value in this thread's feature row (0 past the variable's kept levels,
    // past the last column, and in unused slots: meta 0).  No branch per slot, so the
    // scalar reads of all slot descriptors can be in flight together.
    auto slot_load = [&](KArgs& pk, int q, int meta, bool valid, int64_t blk, int64_t ii, int fq) {
        return (valid & (fq < ((meta >> 8) & 0xff)))
                   ? (float)in_at<IT>(pk.slot_base[q], blk * pk.slot_bs[q] + ii + (int64_t)fq * pk.slot_ld[q])
                   : 0.0f;
    };
    // the register-prefetched slots: 32-bit element offsets (the host checks every
    // slot's span fits), one branch-free load per slot (a lane that must not read
    // loads the slot's first element instead; unused slots point at a valid array)
    auto load_raw = [&](KArgs& pk, int64_t tile, int fq) {
        int64_t blk, ii;
        const bool valid = col_of(tile, blk, ii);
        const unsigned b32 = (unsigned)blk, i32 = (unsigned)ii;
        static_for<RS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const int meta = pk.slot_meta[q];
            // bitwise, not &&: a short-circuit makes the per-lane `valid` an exec-masked
            // region around the slot's descriptor read, one scalar round trip per slot
            const bool on = valid & (fq < ((meta >> 8) & 0xff));
            const unsigned off = b32 * (unsigned)pk.slot_bs[q] + i32 + (unsigned)fq * (unsigned)pk.slot_ld[q];
            // mask, not a select of pointers: the compiler turns that into a branch per
            // slot, with the descriptor reads and an lgkmcnt(0) wait inside each
            // no select here: consuming the value right away makes the compiler wait for
            // each load in turn; staging zeroes the lanes past a slot's rows anyway
            raw[q] = in_at<IT>(pk.slot_base[q], off & (0u - (unsigned)on));
        });
    };
    // normalise and write the staged inputs in B-operand order: for column tile c,
    // k-step s = 4g + r, k-slot kr, column cl the float index is
    // c*kp*16 + (g*64 + kr*16 + cl)*4 + r (one ds_read_b128 = a group's B operands)
    float* xc = reinterpret_cast<float*>(sbuf) + (cb >> 4) * (p.kp * 16);
    const int cl16 = cb & 15;
    auto xidx = [&](int f) { return ((f >> 4) * 64 + (f & 3) * 16 + cl16) * 4 + ((f >> 2) & 3); };
    float* s_dummy = s_ep + 6 * 16 * p.n_otiles;  // write-only sink
    // branch-free: lanes past the slot's rows store to s_dummy, so the slots of a batch
    // schedule together (no divergent region between them)
    // (x - mean) / denom as (x - mean) * (1 / denom), the reciprocal packed at create time
    // (within 1.5 ulp of the IEEE quotient; the contract is 1e-5)
    auto put = [&](int meta, float x, float leps, float mu, float dn, bool valid, int fq, auto logc) {
        const int f = min(((meta >> 16) & 0x7ff) + fq, p.kp - 1);
        if constexpr (decltype(logc)::value)
            if (leps > 0.0f) x = __logf_exact(x, leps);  // LogTransform.forward (transforms.py:123-124)
        float y = (x - mu) * dn;  // dn = 1 / (sigma + eps)
        asm volatile("" : "+v"(y));  // computed by every lane, then selected: no divergent branch
        y = (valid & (fq < ((meta >> 8) & 0xff))) ? y : 0.0f;
        *(fq < (meta & 0xff) ? xc + xidx(f) : s_dummy) = y;
    };
    auto feat = [&](int meta, int fq) { return min(((meta >> 16) & 0x7ff) + fq, p.kp - 1); };
    // ---- the short staging path (p.fast_stage: every slot FPS-aligned; log inputs and
    // slots past the register prefetch included): the staging address splits into a
    // per-slot scalar part and a per-thread part: with fdst a multiple of FPS,
    //   xidx(fdst + fq) = (fdst >> 4) * 256 + ((fdst >> 2) & 3) + [(fq & 3) * 64 + cl16 * 4 + (fq >> 2)]
    // the short staging path's per-slot store (fdst a multiple of FPS); lanes past a
    // slot's rows are zeroed with a bit mask and write to the dummy word (an index
    // select, not a pointer select: the compiler turns that into a branch per slot)
    float* const L = reinterpret_cast<float*>(lds);
    const int didx = (int)(s_dummy - L);
    auto put_fast = [&](int meta, float x, float le, float mu, float rv, bool valid, int tidx, int fq, auto logc) {
        const int fdst = (meta >> 16) & 0x7ff;
        if constexpr (decltype(logc)::value)
            if (le > 0.0f) x = __logf_exact(x, le);  // LogTransform.forward (transforms.py:123-124); uniform
#ifdef FV3_EXP_NONORM  // experiment only (results invalid): stage the raw values
        const float y = x + 0.0f * (mu + rv);
#else
        const float y = (x - mu) * rv;
#endif
        const unsigned keep = 0u - (unsigned)(valid & (fq < ((meta >> 8) & 0xff)));
        L[fq < (meta & 0xff) ? tidx + ((fdst >> 4) * 256 + ((fdst >> 2) & 3)) : didx] =
            __builtin_bit_cast(float, __builtin_bit_cast(unsigned, y) & keep);
    };
    auto store_x_fast = [&](KArgs& pk, int64_t tile, int fq, auto logc, bool zero_pad) {
        int64_t blk, ii;
        const bool valid = col_of(tile, blk, ii);
        // in batches (descriptors, constants, values) so the scalar and LDS reads of all
        // slots are in flight together
        const int tidx = (int)(xc - L) + (fq & 3) * 64 + cl16 * 4 + (fq >> 2);
        int mt[RS];
        float mu[RS], rv[RS];
        static_for<RS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            mt[q] = pk.slot_meta[q];
        });
        static_for<RS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const int f = min(((mt[q] >> 16) & 0x7ff) + fq, p.kp - 1);
            mu[q] = s_mean[f];
            rv[q] = s_denom[f];
        });
        static_for<RS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            put_fast(mt[q], raw[q], decltype(logc)::value ? pk.slot_leps[q] : 0.0f, mu[q], rv[q], valid, tidx, fq,
                     logc);
        });
        // slots past the register prefetch (wide inputs, e.g. the emulator's 736
        // features): batches of 8, every load of a batch in flight before any use
        const unsigned b32 = (unsigned)blk, i32 = (unsigned)ii;
        for (int q0 = RS; q0 < pk.nslots; q0 += 8) {
            int mw[8];
            IT xw[8];
            float mw_mu[8], mw_rv[8];
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                mw[i] = q0 + i < pk.nslots ? pk.slot_meta[q0 + i] : 0;  // uniform
            });
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const int q = min(q0 + i, kMaxSlots - 1);  // past nslots: meta 0, any valid base
                const bool on = valid & (fq < ((mw[i] >> 8) & 0xff));
                const unsigned off = b32 * (unsigned)pk.slot_bs[q] + i32 + (unsigned)fq * (unsigned)pk.slot_ld[q];
                xw[i] = in_at<IT>(pk.slot_base[q], off & (0u - (unsigned)on));
            });
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const int f = min(((mw[i] >> 16) & 0x7ff) + fq, p.kp - 1);
                mw_mu[i] = s_mean[f];
                mw_rv[i] = s_denom[f];
            });
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                put_fast(mw[i], xw[i], decltype(logc)::value ? pk.slot_leps[min(q0 + i, kMaxSlots - 1)] : 0.0f, mw_mu[i], mw_rv[i],
                         valid, tidx, fq, logc);
            });
        }
        if (zero_pad)  // the padding features: once, the buffer holds nothing else
            for (int f = 4 * p.in_steps_total + fq; f < p.kp; f += FPS) xc[xidx(f)] = 0.0f;
    };
    auto store_x = [&](KArgs& pk, int64_t tile, int fq, auto logc, bool zero_pad) {
        int64_t blk, ii;
        const bool valid = col_of(tile, blk, ii);
        constexpr int B = 5;  // slots per batch: descriptors and constants read before any use
        static_assert(RS % B == 0, "");
        static_for<RS / B>([&](auto bc) {
            constexpr int b = decltype(bc)::value;
            int mt[B];
            float le[B], mu[B], dn[B];
            static_for<B>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                mt[i] = pk.slot_meta[b * B + i];
                le[i] = pk.slot_leps[b * B + i];
            });
            static_for<B>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                mu[i] = s_mean[feat(mt[i], fq)];
                dn[i] = s_denom[feat(mt[i], fq)];
            });
            static_for<B>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                put(mt[i], raw[b * B + i], le[i], mu[i], dn[i], valid, fq, logc);
            });
        });
        // inputs wider than the register prefetch: batches of 8 loads in flight
        for (int q0 = RS; q0 < pk.nslots; q0 += 8) {
            float xt[8];
            int mt[8];
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                mt[i] = q0 + i < pk.nslots ? pk.slot_meta[q0 + i] : 0;
                xt[i] = slot_load(pk, q0 + i, mt[i], valid, blk, ii, fq);
            });
            static_for<8>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                put(mt[i], xt[i], mt[i] ? pk.slot_leps[q0 + i] : 0.0f, s_mean[feat(mt[i], fq)],
                    s_denom[feat(mt[i], fq)], valid, fq, logc);
            });
        }
        if (zero_pad)  // the padding features: once, the buffer holds nothing else
            for (int f = 4 * p.in_steps_total + fq; f < p.kp; f += FPS) xc[xidx(f)] = 0.0f;
    };

    // ---- prologue: this tile's inputs and the layer-1 ring in flight, constants to LDS ----
    int64_t tile = blockIdx.x;
    trace_mark(p, tile, 0);
    const Rsrc rw = make_rsrc(p.wbase, p.wbytes);
    const int voff = (wave * 64 + lane) * (int)sizeof(FT);  // hidden-layer fragments
    const int voff_o = lane * 16;                           // output-layer fragments
    constexpr int KS = NT * sizeof(FT);
    FT g1[RD][4];
    // loads complete in issue order (one vmcnt counter): the constants and the layer-1
    // ring go first, so writing the constants to LDS and the first MFMAs do not wait
    // for the tile's inputs (HBM), which are issued last
    {
        constexpr int NM = 1024 / NT, NE = 3072 / NT;  // constants held in registers: kp <= 1024, 6*kop <= 3072
        float cm[NM], cd[NM], ce[NE];
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            const int i = threadIdx.x + NT * j;
            cm[j] = i < p.kp ? p.in_mean[i] : 0.0f;
            cd[j] = i < p.kp ? p.in_denom[i] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < NE; ++j) {
            const int i = threadIdx.x + NT * j;
            ce[j] = i < 6 * kop ? p.oep[i] : 0.0f;
        }
        prime_ring<RD, NW, FT>(g1, rw, voff, p.w1_off);
        if (tile < p.ntiles) load_raw(p, tile, fq0);
#pragma unroll
        for (int j = 0; j < NM; ++j) {
            const int i = threadIdx.x + NT * j;
            if (i < p.kp) {
                s_mean[i] = cm[j];
                s_denom[i] = cd[j];
            }
        }
#pragma unroll
        for (int j = 0; j < NE; ++j) {
            const int i = threadIdx.x + NT * j;
            if (i < 6 * kop) s_ep[i] = ce[j];
        }
        for (int i = threadIdx.x + NT * NM; i < p.kp; i += NT) {
            s_mean[i] = p.in_mean[i];
            s_denom[i] = p.in_denom[i];
        }
        for (int i = threadIdx.x + NT * NE; i < 6 * kop; i += NT) s_ep[i] = p.oep[i];
    }
    for (int i = threadIdx.x; i < (1 + p.n_hidden_extra) * HP; i += NT) s_bias[i] = i < HP ? p.b1[i] : p.bh[i - HP];

    // output plan of this wave.  The first (n_otiles / NW) * NW output tiles go whole to
    // the waves (tile m to wave m % NW): one weight fetch feeds both column tiles.  The
    // rest are split into (tile, column tile) units dealt round-robin, so every SIMD
    // still gets the same number of units (C48's 10 tiles on 8 waves: one whole tile
    // per wave plus one unit on waves 0-3)
    const int n_whole = p.n_otiles / NW;           // whole tiles per wave (every wave the same)
    const int m_split = n_whole * NW;              // first split tile
    const int n_units = (p.n_otiles - m_split) * NC;
    const int n_split = n_units > wave ? (n_units - wave + NW - 1) / NW : 0;  // split units of this wave
    auto whole_soff = [&](int j0, int (&so)[kOutTiles]) {  // tiles wave + NW*(j0+i); returns how many
        const int n = min(kOutTiles, n_whole - j0);
#pragma unroll
        for (int i = 0; i < kOutTiles; ++i) so[i] = p.wo_off + (wave + NW * (j0 + min(i, n - 1))) * (HP / 16) * 1024;
        return n;
    };
    auto split_unit = [&](int k, int& m, int& c) {
        const int u = wave + NW * k;
        m = m_split + u / NC;
        c = u % NC;
    };
    // prime the ring of the layer that follows hidden layer l.  The rings (gh, go) are
    // declared per tile, not across the tile loop: loop-carried ring registers made the
    // compiler copy them at the merge after the next tile's input loads are issued, behind
    // an s_waitcnt vmcnt(0) that waited for those HBM loads (vector-memory loads complete
    // in issue order)
    auto prime_after = [&](int l, auto& gh, auto& go) {
        if (l + 1 < p.n_hidden_extra) {
            prime_ring<RD, NW, FT>(gh, rw, voff, p.wh_off + (l + 1) * (HP / 4) * KS);
        } else if (n_whole > 0) {
            int so[kOutTiles];
            const int n = whole_soff(0, so);
            prime_out_tiles<kOutRing>(go, rw, voff_o, so, n);
        } else if (n_split > 0) {
            int m, c;
            split_unit(0, m, c);
            int so[kOutTiles];
#pragma unroll
            for (int i = 0; i < kOutTiles; ++i) so[i] = p.wo_off + m * (HP / 16) * 1024;
            prime_out_tiles<kOutRing>(go, rw, voff_o, so, 1);
        }
    };
    // stage this tile's inputs (into their own buffer: the stages of later tiles run
    // inside the previous tile, before its output layer)
    auto stage = [&](int64_t t, bool zero_pad) {
        // opaque per stage: addresses derived from the thread's feature row are rebuilt
        // each tile instead of being hoisted out of the loop as 20 live 64-bit values
        int fq = fq0;
        asm volatile("" : "+v"(fq));
        // likewise the slot descriptors: reloaded per tile (scalar-cache hits) rather than
        // ~100 loop-invariant scalars spilled into VGPRs for the whole loop
        KArgs* pt = &p;
        asm volatile("" : "+s"(pt));
#ifndef FV3_EXP_NOSTAGE  // experiment only (results invalid): no input staging
        if (p.fast_stage && p.has_log)
            store_x_fast(*pt, t, fq, std::true_type{}, zero_pad);
        else if (p.fast_stage)
            store_x_fast(*pt, t, fq, std::false_type{}, zero_pad);
        else if (p.has_log)
            store_x(*pt, t, fq, std::true_type{}, zero_pad);
        else
            store_x(*pt, t, fq, std::false_type{}, zero_pad);
#endif
    };
    // the staging reads every feature's normalisation constants, which other waves wrote
    // to LDS above: without this barrier a wave whose constants had not yet been written
    // read what an earlier kernel left in the LDS (the first tile of a block: inf outputs
    // after a bf16x6 launch, tests/test_stepper.py::test_two_model_stepper_matches_oracle)
    tile_sync();
    if (tile < p.ntiles) stage(tile, true);
    tile_sync();
    if (p.prio == 0) __builtin_amdgcn_s_setprio(0);

    for (; tile < p.ntiles; tile += gridDim.x) {  // persistent over column tiles
        trace_mark(p, tile, 5);
        trace_mark(p, tile, 1);
        const bool has_next = tile + gridDim.x < p.ntiles;

        // ---- layer 1: Dense(width) over the padded input features ----
        f32x4 go[kOutRing][kOutTiles];
        FT gh[RD][4];
        f32x4 acc[NC][T4];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < T4; ++j) acc[c][j] = zero4();
        {
            const f32x4* xq = sbuf + lane;  // + c*kp*4 + g*64
            const int ngroups = p.kp / 16;
            f32x4 xb[RD][NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) xb[0][c] = xq[c * p.kp * 4];
            for (int gi = 0; gi < ngroups; gi += RD) {
                static_for<RD>([&](auto hc) {
                    constexpr int h = decltype(hc)::value;
                    const int grp = gi + h;
                    // RD == 2: kp is a multiple of 32, so every pair is whole and the
                    // loads past the last group read (in-bounds) padding never used
                    if (RD == 2 || grp < ngroups) {
                        if (RD == 2 || grp + RD - 1 < ngroups) {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                g1[(h + RD - 1) % RD][r] = bload<FT>(rw, voff, p.w1_off + (4 * (grp + RD - 1) + r) * KS);
                        }
                        if (RD == 2 || grp + 1 < ngroups) {
#pragma unroll
                            for (int c = 0; c < NC; ++c)
                                xb[(h + 1) % RD][c] = xq[c * p.kp * 4 + min(grp + 1, ngroups - 1) * 64];
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int r = 0; r < 4; ++r)
#pragma unroll
                            for (int j = 0; j < T4; ++j)
#pragma unroll
                                for (int c = 0; c < NC; ++c)
                                    acc[c][j] = mfma4(frag_at<T4>(g1[h][r], j), xb[h][c][r], acc[c][j]);
                    }
                });
            }
        }
        prime_after(-1, gh, go);
        // no barrier before: the activations are free since the end of the last tile,
        // and the staged inputs are not overwritten until after the next barrier
        bias_relu_store<T4, NC, NW>(acc, s_bias, wave, lane, kr, hbuf);
        // the next tile's inputs travel while this tile runs its remaining layers.  Issued
        // after layer 1's weight loads and the next ring's: loads complete in issue order,
        // so every weight wait after this point also waits for these HBM loads (measured:
        // issued before the ring, C384 2.10 ms; here, 2.07 ms)
        if (has_next) {
            KArgs* pn = &p;
            asm volatile("" : "+s"(pn));
            int fq = fq0;
            asm volatile("" : "+v"(fq));
            load_raw(*pn, tile + gridDim.x, fq);
        }
        tile_sync();  // the activations are written; every wave is done with the staged inputs
        trace_mark(p, tile, 2);

        // ---- further hidden layers, in place ----
        for (int l = 0; l < p.n_hidden_extra; ++l) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int j = 0; j < T4; ++j) acc[c][j] = zero4();
            gemm_hidden<T4, NC, RD, NW>(acc, hbuf, rw, voff, p.wh_off + l * (HP / 4) * KS, gh, lane);
            prime_after(l, gh, go);
            tile_sync();  // every wave is done reading this layer's input
            bias_relu_store<T4, NC, NW>(acc, s_bias + (l + 1) * HP, wave, lane, kr, hbuf);
            tile_sync();
        }
        trace_mark(p, tile, 3);

        // ---- output Dense layers + bias/denorm/limit/mask epilogue ----
        unsigned ob_c[NC], oi_c[NC];  // per column tile: block and in-block index of this lane's column
        bool cv_c[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int64_t colw = tile * NCOL + 16 * c + (lane & 15);
            cv_c[c] = colw < p.ncol;
            const int64_t cc = cv_c[c] ? colw : 0;
            const int64_t oblk = p.ncol_blk >= p.ncol ? 0 : cc / p.ncol_blk;
            ob_c[c] = (unsigned)oblk;
            oi_c[c] = (unsigned)(cc - oblk * p.ncol_blk);
        }
        // bias / denorm / OutputLimit / mask of output tile m, column tile c, then the store
        auto epilogue = [&](int m, int c, const f32x4& acc) {
            const int ovar = p.otile[m].var, oz0 = p.otile[m].z0, onrow = p.otile[m].nrow;
            if (ovar < 0) return;
            // buffer stores at 32-bit byte offsets (the host checks the spans): a lane that
            // must not store (padding rows, columns past the end) gets an offset past the
            // range and its store is dropped, so no branch per row
            const Rsrc ro = make_rsrc(p.out_ptr[ovar], 0x7ffffffc);
            const unsigned ob = ob_c[c] * (unsigned)p.out_bs[ovar] + oi_c[c];
            const unsigned old_ = (unsigned)p.out_ld[ovar];
            const bool has_res = p.res_ptr[ovar] != nullptr;  // uniform
            const Rsrc rres = make_rsrc(has_res ? p.res_ptr[ovar] : p.out_ptr[ovar], 0x7ffffffc);
            const unsigned rb = ob_c[c] * (unsigned)p.res_bs[ovar] + oi_c[c];
            const unsigned rld = (unsigned)p.res_ld[ovar];
            int fo = 16 * m + 4 * kr;
            asm volatile("" : "+v"(fo));  // keep this tile's constant reads here, not hoisted above the GEMM
            const f32x4 bo = *reinterpret_cast<const f32x4*>(s_ep + fo);
            const f32x4 sg = *reinterpret_cast<const f32x4*>(s_ep + kop + fo);
            const f32x4 mu = *reinterpret_cast<const f32x4*>(s_ep + 2 * kop + fo);
            const f32x4 lo = *reinterpret_cast<const f32x4*>(s_ep + 3 * kop + fo);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(s_ep + 4 * kop + fo);
            const f32x4 mk = *reinterpret_cast<const f32x4*>(s_ep + 5 * kop + fo);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * kr + r;
                float y = acc[r] + bo[r];
                y = y * sg[r];
                y = y + mu[r];
                if (y < lo[r]) y = lo[r];
                if (y >= hi[r]) y = hi[r];
                y = y * mk[r];
                const bool ok = cv_c[c] && row < onrow;  // padding rows of the last tile: no reads either
                if (has_res) {  // after = before + to (Difference.backward)
                    const unsigned roff = ok ? (rb + (unsigned)(oz0 + row) * rld) * 4u : 0x80000000u;
                    y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rres, (int)roff, 0, 0)) + y;
                }
                const unsigned off = ok ? (ob + (unsigned)(oz0 + row) * old_) * 4u : 0x80000000u;
#ifdef FV3_EXP_NOSTORE  // experiment only (results invalid): keep the value, skip the store
                asm volatile("" ::"v"(y), "v"(off));
#else
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, (int)off, 0, 0);
#endif
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        // whole output tiles: both column tiles per weight fetch
        for (int j0 = 0; j0 < n_whole; j0 += kOutTiles) {
            int so[kOutTiles];
            const int n = whole_soff(j0, so);
            if (j0 > 0) prime_out_tiles<kOutRing>(go, rw, voff_o, so, n);
            f32x4 o[kOutTiles][NC];
#pragma unroll
            for (int i = 0; i < kOutTiles; ++i)
#pragma unroll
                for (int c = 0; c < NC; ++c) o[i][c] = zero4();
            if (n == 1)
                gemm_out_tiles<HT, 1, NC, kOutRing>(o, hbuf + lane, rw, voff_o, so, go);
            else
                gemm_out_tiles<HT, kOutTiles, NC, kOutRing>(o, hbuf + lane, rw, voff_o, so, go);
#pragma unroll
            for (int i = 0; i < kOutTiles; ++i) {
                if (i >= n) break;
#pragma unroll
                for (int c = 0; c < NC; ++c) epilogue(wave + NW * (j0 + i), c, o[i][c]);
            }
        }
        // the remaining tiles, split into (tile, column tile) units
        for (int k = 0; k < n_split; ++k) {
            int m, c;
            split_unit(k, m, c);
            int so[kOutTiles];
#pragma unroll
            for (int i = 0; i < kOutTiles; ++i) so[i] = p.wo_off + m * (HP / 16) * 1024;
            if (k > 0 || n_whole > 0) prime_out_tiles<kOutRing>(go, rw, voff_o, so, 1);
            f32x4 o[kOutTiles][NC];
            o[0][0] = zero4();
            gemm_out_tiles<HT, 1, 1, kOutRing>(o, hbuf + c * HT * 64 + lane, rw, voff_o, so, go);
            epilogue(m, c, o[0][0]);
        }
        // the next tile's inputs to their buffer (free since the barrier after layer 1),
        // ordered before the next tile's layer 1 by the barrier below.  Here, after the
        // output layer, rather than before it: C384 2,056 -> 2,044 us, C48 unchanged
        if (has_next) stage(tile + gridDim.x, false);
        prime_ring<RD, NW, FT>(g1, rw, voff, p.w1_off);  // the next tile's layer 1
        tile_sync();         // the activations are free for the next tile's inputs
        trace_mark(p, tile, 4);
    }
}

}  // namespace fv3

// ------------------------------------------------------------------------------------
// host side: model creation (validation + fragment packing), forward launch
// ------------------------------------------------------------------------------------

namespace {

int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace

extern "C" int fv3_dense_create(const fv3_dense_desc* d, fv3_dense_model** out)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(d && out, "dense_create: NULL argument");
    *out = nullptr;
    FV3_REQUIRE(d->n_in >= 1 && d->n_in <= kMaxVars, "dense_create: n_in must be in [1, %d]", kMaxVars);
    FV3_REQUIRE(d->n_out >= 1 && d->n_out <= kMaxVars, "dense_create: n_out must be in [1, %d]", kMaxVars);
    FV3_REQUIRE(d->width >= 1 && d->width <= 256, "dense_create: width must be in [1, 256] (got %d)", d->width);
    FV3_REQUIRE(d->n_hidden >= 1, "dense_create: need at least one hidden layer (depth >= 2)");
    FV3_REQUIRE(d->in_nz && d->out_nz && d->in_mean && d->in_sigma && d->out_mean && d->out_sigma,
                "dense_create: NULL array in descriptor");
    FV3_REQUIRE(d->hidden_kernel && d->hidden_bias && d->out_kernel && d->out_bias,
                "dense_create: NULL weights");

    auto m = new fv3_dense_model();
    std::unique_ptr<fv3_dense_model> guard(m);
    m->n_in = d->n_in;
    m->n_out = d->n_out;
    m->width = d->width;
    m->n_hidden = d->n_hidden;
    m->hp = d->width <= 64 ? 64 : (d->width <= 128 ? 128 : 256);
    m->ht = m->hp / 16;

    // inputs: clip + per-variable padding to whole k-steps
    int step = 0, k_in = 0;
    std::vector<int> feat_src;  // padded feature -> kept-feature index or -1
    for (int v = 0; v < d->n_in; ++v) {
        const int nz = d->in_nz[v];
        FV3_REQUIRE(nz >= 1, "dense_create: input %d has no levels", v);
        int z0 = 0, z1 = nz;
        if (d->in_clip) {
            z0 = d->in_clip[2 * v];
            z1 = d->in_clip[2 * v + 1];
            FV3_REQUIRE(0 <= z0 && z0 < z1 && z1 <= nz, "dense_create: bad clip for input %d", v);
        }
        const int nkeep = z1 - z0;
        const int nsteps = (nkeep + 3) / 4;
        m->in_nz.push_back(nz);
        m->in_log_eps.push_back(d->in_log_eps ? d->in_log_eps[v] : 0.0f);
        m->in_z0.push_back(z0);
        m->in_nkeep.push_back(nkeep);
        m->in_step0.push_back(step);
        m->in_nsteps.push_back(nsteps);
        for (int i = 0; i < 4 * nsteps; ++i) feat_src.push_back(i < nkeep ? k_in + i : -1);
        k_in += nkeep;
        step += nsteps;
    }
    m->k_in = k_in;
    m->steps_total = step;
    while (step % 8) {  // whole pairs of groups of 4 k-steps: the layer-1 loop has no tail
        for (int i = 0; i < 4; ++i) feat_src.push_back(-1);
        ++step;
    }
    m->kp = 4 * step;

    // outputs: per-variable padding to whole 16-row tiles, tiles paired into chunks
    int k_out = 0;
    std::vector<int> ofeat_src;  // padded output row -> original output column or -1
    for (int v = 0; v < d->n_out; ++v) {
        const int nz = d->out_nz[v];
        FV3_REQUIRE(nz >= 1, "dense_create: output %d has no levels", v);
        m->out_nz.push_back(nz);
        const int res = d->out_residual ? d->out_residual[v] : -1;
        FV3_REQUIRE(res < d->n_in, "dense_create: output %d residual input %d out of range", v, res);
        if (res >= 0)
            FV3_REQUIRE(d->in_nz[res] >= nz, "dense_create: residual input %d has fewer levels than output %d", res, v);
        m->out_residual.push_back(res < 0 ? -1 : res);
        for (int z0 = 0; z0 < nz; z0 += 16) {
            DenseOutTile t{v, z0, std::min(16, nz - z0)};
            m->otiles.push_back(t);
            for (int r = 0; r < 16; ++r) ofeat_src.push_back(r < t.nrow ? k_out + z0 + r : -1);
        }
        k_out += nz;
    }
    FV3_REQUIRE((int)m->otiles.size() <= kMaxOutTiles, "dense_create: too many output rows (%d tiles)",
                (int)m->otiles.size());
    m->k_out = k_out;
    m->n_otiles = (int)m->otiles.size();
    const int kop = 16 * m->n_otiles;
    const int HP = m->hp, HT = m->ht, W = d->width;

    // ---- pack host buffer ----
    std::vector<float> in_mean(m->kp, 0.0f), in_denom(m->kp, 1.0f);
    for (int f = 0; f < m->kp; ++f) {
        const int src = feat_src[f];
        if (src < 0) continue;
        in_mean[f] = d->in_mean[src];
        volatile float s = d->in_sigma[src];
        volatile float den = s + d->epsilon;  // StandardNormLayer computes sigma + epsilon in f32
        in_denom[f] = 1.0f / den;             // the kernel multiplies: <= 1.5 ulp from the quotient
    }
    // layer 1: W1[k_in][W] -> [KP/4][wave][64][T4]; tile m = wave*T4 + j, T4 = HT / NW
    // (packed for NW = 4 waves per block, and for NW = 8 when HT >= 8)
    const int nhx = d->n_hidden - 1;
    auto pack_w1 = [&](int NW) {
        const int T4 = HT / NW;
        std::vector<float> w1((size_t)m->kp * HP, 0.0f);
        for (int s = 0; s < m->kp / 4; ++s)
            for (int wv = 0; wv < NW; ++wv)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < T4; ++j) {
                        const int f = 4 * s + (l >> 4);
                        const int unit = 16 * (wv * T4 + j) + (l & 15);
                        const int src = feat_src[f];
                        float v = 0.0f;
                        if (src >= 0 && unit < W) v = d->hidden_kernel[0][(size_t)src * W + unit];
                        w1[(((size_t)s * NW + wv) * 64 + l) * T4 + j] = v;
                    }
        return w1;
    };
    // hidden layers 2..n: W[W][W] -> [HP/4][wave][64][T4]; k-step s = 4t + r reads
    // input unit 16t + 4(l>>4) + r (the accumulator-layout permutation)
    auto pack_wh = [&](int NW) {
        const int T4 = HT / NW;
        std::vector<float> wh((size_t)std::max(nhx, 1) * HP * HP, 0.0f);
        for (int li = 0; li < nhx; ++li) {
            const float* K = d->hidden_kernel[li + 1];
            for (int s = 0; s < HP / 4; ++s) {
                const int t = s / 4, r = s % 4;
                for (int wv = 0; wv < NW; ++wv)
                    for (int l = 0; l < 64; ++l)
                        for (int j = 0; j < T4; ++j) {
                            const int in = 16 * t + 4 * (l >> 4) + r;
                            const int unit = 16 * (wv * T4 + j) + (l & 15);
                            float v = 0.0f;
                            if (in < W && unit < W) v = K[(size_t)in * W + unit];
                            wh[(size_t)li * HP * HP + (((size_t)s * NW + wv) * 64 + l) * T4 + j] = v;
                        }
            }
        }
        return wh;
    };
    const bool nw8 = HT >= 8;
    std::vector<float> w1 = pack_w1(4), wh = pack_wh(4);
    std::vector<float> w1_8, wh_8;
    if (nw8) {
        w1_8 = pack_w1(8);
        wh_8 = pack_wh(8);
    }
    std::vector<float> b1(HP, 0.0f);
    for (int u = 0; u < W; ++u) b1[u] = d->hidden_bias[0][u];
    std::vector<float> bh((size_t)std::max(nhx, 1) * HP, 0.0f);
    for (int li = 0; li < nhx; ++li)
        for (int u = 0; u < W; ++u) bh[(size_t)li * HP + u] = d->hidden_bias[li + 1][u];
    // output layer: concat of out kernels [W][out_nz] -> [otile][HP/16][64][4 k-steps]
    std::vector<int> ocol_var(k_out), ocol_z(k_out);
    {
        int o = 0;
        for (int v = 0; v < d->n_out; ++v)
            for (int z = 0; z < d->out_nz[v]; ++z, ++o) {
                ocol_var[o] = v;
                ocol_z[o] = z;
            }
    }
    std::vector<float> wo((size_t)m->n_otiles * (HP / 4) * 64, 0.0f);
    for (int mt = 0; mt < m->n_otiles; ++mt)
        for (int s = 0; s < HP / 4; ++s) {
            const int t = s / 4, r = s % 4;
            for (int l = 0; l < 64; ++l) {
                const int in = 16 * t + 4 * (l >> 4) + r;
                const int row = 16 * mt + (l & 15);
                const int src = ofeat_src[row];
                float v = 0.0f;
                if (src >= 0 && in < W) {
                    const int ov = ocol_var[src], oz = ocol_z[src];
                    v = d->out_kernel[ov][(size_t)in * d->out_nz[ov] + oz];
                }
                wo[(((size_t)mt * (HP / 16) + t) * 64 + l) * 4 + r] = v;
            }
        }
    // epilogue constants [6][KOP]: bias, sigma, mean, lo, hi, mask
    std::vector<float> oep((size_t)6 * kop);
    for (int row = 0; row < kop; ++row) {
        float v[6] = {0.0f, 1.0f, 0.0f, -INFINITY, INFINITY, 1.0f};
        const int src = ofeat_src[row];
        if (src >= 0) {
            const int ov = ocol_var[src], oz = ocol_z[src];
            v[0] = d->out_bias[ov][oz];
            v[1] = d->out_sigma[src];
            v[2] = d->out_mean[src];
            if (d->out_min) v[3] = d->out_min[src];
            if (d->out_max) v[4] = d->out_max[src];
            if (d->out_mask) v[5] = d->out_mask[src];
        }
        for (int k = 0; k < 6; ++k) oep[(size_t)k * kop + row] = v[k];
    }

    // ---- one device allocation ----
    struct Piece {
        const void* src;
        size_t bytes;
        size_t off;
    };
    std::vector<Piece> pcs = {
        {in_mean.data(), in_mean.size() * 4, 0}, {in_denom.data(), in_denom.size() * 4, 0},
        {w1.data(), w1.size() * 4, 0},           {b1.data(), b1.size() * 4, 0},
        {wh.data(), wh.size() * 4, 0},           {bh.data(), bh.size() * 4, 0},
        {wo.data(), wo.size() * 4, 0},           {oep.data(), oep.size() * 4, 0},
        {w1_8.data(), w1_8.size() * 4, 0},       {wh_8.data(), wh_8.size() * 4, 0},
    };
    size_t total = 0;
    for (auto& p : pcs) {
        p.off = total;
        total += (p.bytes + 255) / 256 * 256;
    }
    size_t alloc = total;
    if (const char* e = fv3::variant_env("FV3_DENSE_PAD_MB")) alloc = std::max(alloc, (size_t)atoi(e) << 20);
    FV3_HIP(hipMalloc(&m->dbuf, alloc));
    for (auto& p : pcs)
        if (p.bytes) FV3_HIP(hipMemcpy((char*)m->dbuf + p.off, p.src, p.bytes, hipMemcpyHostToDevice));
    auto at = [&](int i) { return (char*)m->dbuf + pcs[i].off; };
    DenseArgs& a = m->tmpl;
    a.in_mean = (const float*)at(0);
    a.in_denom = (const float*)at(1);
    a.w1 = (const float*)at(2);
    a.b1 = (const float*)at(3);
    a.wh = (const float*)at(4);
    a.bh = (const float*)at(5);
    a.wo = (const float*)at(6);
    a.oep = (const float*)at(7);
    FV3_REQUIRE(total < (1u << 31), "dense_create: model too large for 32-bit buffer offsets");
    a.wbase = (const float*)m->dbuf;
    a.w1_off = (int)pcs[2].off;
    a.wh_off = (int)pcs[4].off;
    a.wo_off = (int)pcs[6].off;
    a.wbytes = (int)total;
    m->w1_off8 = nw8 ? (int)pcs[8].off : -1;
    m->wh_off8 = nw8 ? (int)pcs[9].off : -1;
    for (int t = 0; t < m->n_otiles; ++t) a.otile[t] = m->otiles[t];
    a.n_in = m->n_in;
    a.n_hidden_extra = nhx;
    a.n_otiles = m->n_otiles;
    a.kp = m->kp;
    a.in_steps_total = m->steps_total;
    // the bf16x3 / bf16x6 weight streams (fv3_dense_forward_ex); a model a split stream
    // cannot hold still runs in exact f32 (b3_pack leaves that precision unsupported)
    if (const int st = b3_pack(m, d)) {
        b3_free(m);
        (void)hipFree(m->dbuf);
        return st;
    }
    *out = guard.release();
    return FV3_OK;
}

extern "C" int fv3_dense_set_trace(fv3_dense_model* m, long long* trace)
{
    fv3::clear_error();
    FV3_REQUIRE(m, "dense_set_trace: NULL model");
    m->tmpl.trace = trace;
    return FV3_OK;
}

extern "C" int fv3_dense_destroy(fv3_dense_model* m)
{
    fv3::clear_error();
    if (!m) return FV3_OK;
    fv3::b3_free(m);
    if (m->dbuf) FV3_HIP(hipFree(m->dbuf));
    delete m;
    return FV3_OK;
}

extern "C" int fv3_dense_k_in(const fv3_dense_model* m) { return m ? m->k_in : -1; }
extern "C" int fv3_dense_k_out(const fv3_dense_model* m) { return m ? m->k_out : -1; }

// in64: inputs are float64 (read in place, cast to f32 in the staging)
static int dense_forward_impl(const fv3_dense_model* m, const void* const* inputs, bool in64, const fv3_layout* in_l,
                              float* const* outputs, const fv3_layout* out_l, int64_t ncol, void* stream)
{
    using namespace fv3;
    clear_error();
    // element `off` of input v, as the const float* the slot descriptors carry
    auto in_ptr = [&](int v, int64_t off) -> const float* {
        return in64 ? reinterpret_cast<const float*>(static_cast<const double*>(inputs[v]) + off)
                    : static_cast<const float*>(inputs[v]) + off;
    };
    FV3_REQUIRE(m, "dense_forward: NULL model");
    FV3_REQUIRE(ncol >= 0, "dense_forward: ncol < 0");
    if (ncol == 0) return FV3_OK;
    FV3_REQUIRE(inputs && in_l && outputs && out_l, "dense_forward: NULL argument");
    DenseArgs a = m->tmpl;
    const int64_t nb = in_l[0].ncol_blk;
    for (int v = 0; v < m->n_in; ++v) {
        FV3_REQUIRE(inputs[v], "dense_forward: input %d is NULL", v);
        FV3_REQUIRE(layout_ok(in_l[v], ncol) && in_l[v].ncol_blk == nb,
                    "dense_forward: input %d layout invalid or ncol_blk differs", v);
        FV3_REQUIRE(in_l[v].ld < (1LL << 31) && in_l[v].blk_stride < (1LL << 31),
                    "dense_forward: input %d strides exceed 2^31 elements", v);
    }
    for (int v = 0; v < m->n_out; ++v) {
        FV3_REQUIRE(outputs[v], "dense_forward: output %d is NULL", v);
        FV3_REQUIRE(layout_ok(out_l[v], ncol) && out_l[v].ncol_blk == nb,
                    "dense_forward: output %d layout invalid or ncol_blk differs", v);
        {  // the epilogue stores (and residual reads) at 32-bit byte offsets below 2^31
            const int64_t nblk = (ncol + nb - 1) / nb;
            auto span = [&](const fv3_layout& l, int nz) {
                return (nblk > 1 ? (nblk - 1) * l.blk_stride : 0) + (std::min<int64_t>(nb, ncol) - 1) +
                       (int64_t)(nz - 1) * l.ld;
            };
            const int r = m->out_residual[v];
            FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED,
                             span(out_l[v], m->out_nz[v]) < ((int64_t)1 << 29) &&
                                 (r < 0 || span(in_l[r], m->out_nz[v]) < ((int64_t)1 << 29)),
                             "dense_forward: output %d spans more than 2^29 elements", v);
        }
        a.out_ptr[v] = outputs[v];
        a.out_ld[v] = out_l[v].ld;
        a.out_bs[v] = out_l[v].blk_stride;
        const int r = m->out_residual[v];
        FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, !in64 || r < 0,
                         "dense_forward: residual outputs need float32 inputs");
        a.res_ptr[v] = r >= 0 ? in_ptr(r, 0) : nullptr;
        a.res_ld[v] = r >= 0 ? (int)in_l[r].ld : 0;
        a.res_bs[v] = r >= 0 ? (int)in_l[r].blk_stride : 0;
    }
    a.ncol = ncol;
    a.ncol_blk = nb;
    // columns per tile: two 16-column tiles (halves weight traffic per FLOP; measured
    // fastest at C48 and C384); FV3_DENSE_NC=1 for A/B
    // wide-input models (the microphysics emulator: 736 padded features) stage 32
    // columns in > 64 KiB of LDS, i.e. one block per CU: use 16-column tiles there
    // (with 8-wave blocks, wide inputs keep 32-column tiles at one block per CU: the
    // emulator 7.12 -> 6.66 ms; 16-column tiles remain for widths < 128)
    const bool wide = (size_t)2 * 16 * 4 * m->kp > 64 * 1024;
    // LDS of a block: activations (NC x HT tiles x 64 lanes x 16 B), the staged inputs
    // (NC x kp features x 16 columns), then the constants, one
    // dummy f32x4 (the staging stores of lanes past a slot's rows land there) and the
    // hidden-layer biases
    auto lds_of = [&](int c) {
        const size_t hb = (size_t)c * 16 * 64 * (size_t)m->ht, xb = (size_t)c * sizeof(float) * 16 * (size_t)m->kp;
        return hb + xb + sizeof(float) * (2 * (size_t)m->kp + 6 * 16 * (size_t)m->n_otiles) + 16 +
               sizeof(float) * (1 + (size_t)m->tmpl.n_hidden_extra) * 16 * (size_t)m->ht;
    };
    // any model whose 32-column tiles do not fit the LDS (deep models hold ~1 KiB of
    // biases per hidden layer at width 256) runs 16-column tiles
    const bool fits2 = lds_of(2) <= 160 * 1024;
    int nc = (wide && m->w1_off8 < 0) || !fits2 ? 1 : 2;
    if (const char* e = fv3::variant_env("FV3_DENSE_NC")) nc = atoi(e) == 1 || !fits2 ? 1 : 2;
    // waves per block: 8, two per SIMD on one tile and each wave half the hidden units,
    // measured faster than 4 at every size after the staging work (C48 42.8 vs 47.9 us,
    // C96 141 vs 147 us, C384 2.15 vs 2.18 ms).  Needs 32-column tiles and width >= 128.
    // FV3_DENSE_NW=4|8 for A/B
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
    int nw = 8;
    if (const char* e = fv3::variant_env("FV3_DENSE_NW")) nw = atoi(e) == 8 ? 8 : 4;
    if (nc == 1 || m->w1_off8 < 0) nw = 4;
    const int nt = 64 * nw;
    if (nw == 8) {
        a.w1_off = m->w1_off8;
        a.wh_off = m->wh_off8;
    }
    const int ncol_tile = 16 * nc;
    a.ntiles = (ncol + ncol_tile - 1) / ncol_tile;
    // input slots: nt threads read nt / ncol_tile feature rows of one variable
    const int fps = nt / ncol_tile;
    a.nslots = 0;
    for (int v = 0; v < m->n_in; ++v) {
        const int nf_v = 4 * m->in_nsteps[v], nk_v = m->in_nkeep[v];
        for (int f0 = 0; f0 < nf_v; f0 += fps) {
            FV3_REQUIRE(a.nslots < kMaxSlots, "dense_forward: %d input features are too many", m->kp);
            const int q = a.nslots++;
            const int zf = std::min(m->in_z0[v] + f0, m->in_nz[v] - 1);  // never dereferenced past nk
            a.slot_base[q] = in_ptr(v, (int64_t)zf * in_l[v].ld);
            a.slot_bs[q] = (int)in_l[v].blk_stride;
            a.slot_ld[q] = (int)in_l[v].ld;
            const int nk = std::max(0, std::min(nk_v - f0, 255));
            const int nf = std::min(nf_v - f0, 255);
            a.slot_meta[q] = (v << 27) | ((4 * m->in_step0[v] + f0) << 16) | (nk << 8) | nf;
            a.slot_leps[q] = m->in_log_eps[v];
            a.has_log |= m->in_log_eps[v] > 0.0f;
        }
    }
    for (int q = a.nslots; q < kMaxSlots; ++q) {  // unused slots: meta 0 (no rows), a valid base
        a.slot_base[q] = in_ptr(0, 0);
        a.slot_bs[q] = a.slot_ld[q] = a.slot_meta[q] = 0;
        a.slot_leps[q] = 0.0f;
    }
    {
        bool fast = true;
        const int64_t nblk = (ncol + nb - 1) / nb;
        for (int q = 0; q < a.nslots; ++q) {
            const int fdst = (a.slot_meta[q] >> 16) & 0x7ff;
            const int64_t bs = nblk > 1 ? (int64_t)a.slot_bs[q] : 0;
            const int64_t span = (nblk - 1) * bs + (std::min<int64_t>(nb, ncol) - 1) + (int64_t)(fps - 1) * a.slot_ld[q];
            // the kernel addresses a slot's rows with 32-bit unsigned element offsets
            FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, bs >= 0 && a.slot_ld[q] >= 0 && span < ((int64_t)1 << 32),
                             "dense_forward: input %d spans more than 2^32 elements", a.slot_meta[q] >> 27);
            fast = fast && fdst % fps == 0;
        }
        if (fv3::variant_env("FV3_DENSE_SLOWSTAGE")) fast = false;  // A/B
        a.fast_stage = fast;
    }
    hipStream_t s = (hipStream_t)stream;
    const size_t hbytes = (size_t)nc * 16 * 64 * (size_t)m->ht, xbytes = (size_t)nc * sizeof(float) * 16 * (size_t)m->kp;
    a.lds_s = (int)(hbytes / 16);
    a.lds_x = (int)((hbytes + xbytes) / 16);
    const size_t lds = lds_of(nc);
    FV3_REQUIRE(lds <= 160 * 1024, "dense_forward: %d input features need too much LDS", m->kp);
    // (waves per SIMD targeted by register allocation, weight ring depth):
    // FV3_DENSE_CFG = "3,2" (default) | "2,3" | "4,2" (A/B)
    int wpe = 3, rd = 2;  // measured best at C48 and C384
#if FV3_VARIANT_KERNELS
    if (const char* e = fv3::variant_env("FV3_DENSE_CFG")) {
        if (!strcmp(e, "2,3")) wpe = 2, rd = 3;
        else if (!strcmp(e, "4,2")) wpe = 4, rd = 2;
    }
#endif
    auto kernel_of = [&](int t4) -> const void* {
#define FV3_K(T4, NC, W, R) (const void*)dense_forward_kernel<T4, NC, W, R, 4>
        if (nw == 8) return t4 == 1 ? (const void*)dense_forward_kernel<1, 2, 4, 2, 8> : (const void*)dense_forward_kernel<2, 2, 4, 2, 8>;
#if FV3_VARIANT_KERNELS  // the other register targets / ring depths (A/B)
        if (wpe == 4 && nc == 1) return t4 == 1 ? FV3_K(1, 1, 4, 2) : t4 == 2 ? FV3_K(2, 1, 4, 2) : FV3_K(4, 1, 4, 2);
        if (wpe == 2 && nc == 1) return t4 == 1 ? FV3_K(1, 1, 2, 3) : t4 == 2 ? FV3_K(2, 1, 2, 3) : FV3_K(4, 1, 2, 3);
        if (wpe == 4) return t4 == 1 ? FV3_K(1, 2, 4, 2) : t4 == 2 ? FV3_K(2, 2, 4, 2) : FV3_K(4, 2, 4, 2);
        if (wpe == 2) return t4 == 1 ? FV3_K(1, 2, 2, 3) : t4 == 2 ? FV3_K(2, 2, 2, 3) : FV3_K(4, 2, 2, 3);
#endif
        (void)wpe, (void)rd;
        if (nc == 1) return t4 == 1 ? FV3_K(1, 1, 3, 2) : t4 == 2 ? FV3_K(2, 1, 3, 2) : FV3_K(4, 1, 3, 2);
        return t4 == 1 ? FV3_K(1, 2, 3, 2) : t4 == 2 ? FV3_K(2, 2, 3, 2) : FV3_K(4, 2, 3, 2);
#undef FV3_K
    };
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, !in64 || nw == 8,
                     "dense_forward: float64 inputs need the 8-wave kernel (32-column tiles, width >= 128)");
    const void* kfn = in64 ? (m->ht / nw == 1 ? (const void*)dense_forward_kernel<1, 2, 4, 2, 8, double>
                                              : (const void*)dense_forward_kernel<2, 2, 4, 2, 8, double>)
                           : kernel_of(m->ht / nw);
    // persistent blocks: resident blocks per CU x CUs (queried once per kernel);
    // FV3_DENSE_GRID overrides (A/B)
    struct Resident {
        const void* fn;
        size_t lds;
        int blocks;
    };
    static std::vector<Resident> resident;  // keyed by kernel and LDS size (models differ in LDS)
    std::lock_guard<std::mutex> lock(mu);
    int res = 0;
    for (auto& r : resident)
        if (r.fn == kfn && r.lds == lds) res = r.blocks;
    if (!res) {
        FV3_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, kfn, nt, lds));
        res = std::max(1, res);
        resident.push_back({kfn, lds, res});
    }
    int64_t grid = std::min<int64_t>(a.ntiles, (int64_t)res * n_cu);
    if (const char* e = fv3::variant_env("FV3_DENSE_GRID")) grid = std::min<int64_t>(a.ntiles, std::max(1, atoi(e)));
    a.prio = 0;
    if (const char* e = fv3::variant_env("FV3_DENSE_PRIO")) a.prio = std::max(0, std::min(3, atoi(e)));
    void* kargs[] = {&a};
    FV3_HIP(hipLaunchKernel(kfn, dim3((unsigned)grid), dim3(nt), kargs, lds, s));
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}

extern "C" int fv3_dense_forward(const fv3_dense_model* m, const float* const* inputs, const fv3_layout* in_l,
                                 float* const* outputs, const fv3_layout* out_l, int64_t ncol, void* stream)
{
    return dense_forward_impl(m, reinterpret_cast<const void* const*>(inputs), false, in_l, outputs, out_l, ncol,
                              stream);
}

extern "C" int fv3_dense_forward_f64in(const fv3_dense_model* m, const double* const* inputs, const fv3_layout* in_l,
                                       float* const* outputs, const fv3_layout* out_l, int64_t ncol, void* stream)
{
    return dense_forward_impl(m, reinterpret_cast<const void* const*>(inputs), true, in_l, outputs, out_l, ncol,
                              stream);
}
