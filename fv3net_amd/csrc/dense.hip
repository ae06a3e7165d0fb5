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
//  * one 256-thread block (4 waves, one per SIMD) owns a 16-column tile for the
//    whole network; wave w owns hidden-unit tiles [w*T4, (w+1)*T4) of every hidden
//    layer (T4 = width/64 tiles of 16 units) and every 4th output tile, so four
//    independent accumulators per wave keep the MFMA pipe busy and a C48 step
//    (864 tiles) puts ~3.4 waves on every SIMD;
//  * lane l holds column (l & 15) and k-slot (l >> 4) of every B operand;
//  * a layer's output is written to LDS in the MFMA accumulator layout
//    ([tile][lane] x 4 regs, register r of tile t = unit 16t + 4(l>>4) + r) and the
//    next layer reads it back with one ds_read_b128 per 4 k-steps: k-step s = 4t + r
//    takes register r of tile t, i.e. the contraction order over hidden units is
//    permuted and the packed weights carry the same permutation (no shuffles);
//  * two 16 KiB LDS buffers ping-pong between layers (one barrier per layer);
//    the normalised inputs are staged once per block in the second buffer;
//  * weights are pre-packed at create time into [k-step][wave][lane][T4] fragment
//    order: every A-operand fetch is one T4*4 B/lane fully coalesced load;
//  * each input variable's features and each output tile are padded so a k-step
//    (4 features) never straddles two variables: the source pointer is uniform.
// Roofline: fp32 MFMA-bound.  2*(k_in*w + (n_hidden-1)*w*w + w*k_out) FLOP per
// column (292,864 for the 2x256 C48 model) against (k_in + k_out) * 4 B of HBM.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>

#include "common.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace fv3 {

constexpr int kMaxVars = 16;
constexpr int kMaxOutTiles = 64;

struct DenseInVar {
    const float* ptr;
    int64_t ld, bs;
    int step0;    // first padded k-step of this variable
    int nsteps;   // padded k-steps (4 features each)
    int z0;       // first kept level (clip start)
    int nkeep;    // kept levels
};

struct DenseOutTile {
    int var;  // output variable or -1 (padding tile)
    int z0;   // level of the tile's first row
    int nrow; // valid rows in this tile (<= 16)
    int pad;
};

struct DenseArgs {
    const float* in_mean;   // [KP] padded feature order
    const float* in_denom;  // [KP] f32(sigma + eps)
    const float* w1;        // [KP/4][4 waves][64][T4]
    const float* b1;        // [HP]
    const float* wh;        // [n_hidden-1][HP/4][4 waves][64][T4]
    const float* bh;        // [n_hidden-1][HP]
    const float* wo;        // [n_otiles][HP/16][64][4]: 4 k-steps per lane
    const float* bo;        // [KOP]
    const float* o_sigma;   // [KOP]
    const float* o_mean;    // [KOP]
    const float* o_lo;      // [KOP]
    const float* o_hi;      // [KOP]
    const float* o_mask;    // [KOP]
    DenseInVar in[kMaxVars];
    float* out_ptr[kMaxVars];
    int64_t out_ld[kMaxVars];
    int64_t out_bs[kMaxVars];
    DenseOutTile otile[kMaxOutTiles];
    int64_t ncol, ncol_blk;
    int n_in, n_hidden_extra, n_otiles, kp;
    int in_steps_total, pad_;
};

typedef float f32x1 __attribute__((ext_vector_type(1)));

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

// relu(acc + bias) for this wave's T4 tiles (x NC column tiles), stored in accumulator layout
template <int T4, int NC>
__device__ __forceinline__ void bias_relu_store(f32x4 (&acc)[NC][T4], const float* __restrict__ b, int wave,
                                                int lane, int kr, f32x4* __restrict__ dst)
{
    constexpr int HT = 4 * T4;
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

// acc[c][j] += W^T h over all HT*4 k-steps, h read from LDS in accumulator layout.
// Weight fragments stream through a 3-group register ring (groups of 4 k-steps),
// two groups (8 k-steps, 8*T4*NC MFMAs) ahead of use, so the L2 latency of a
// fragment is covered by this wave's own MFMAs.  The ring is indexed at compile
// time (static_for): no register copies, hence no premature vmcnt(0).
template <int T4, int NC>
__device__ __forceinline__ void gemm_from_lds(f32x4 (&acc)[NC][T4], const f32x4* __restrict__ src,
                                              const typename Frag<T4>::type* __restrict__ w, int wave,
                                              int lane)
{
    constexpr int HT = 4 * T4;
    typedef typename Frag<T4>::type FT;
    const FT* wp = w + (size_t)wave * 64 + lane;  // k-step s at wp[s * 256]
    FT g[3][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        g[0][r] = wp[(size_t)r * 256];
        g[1][r] = wp[(size_t)(4 + r) * 256];
    }
    f32x4 bq[2][NC];  // B operands, one group ahead
#pragma unroll
    for (int c = 0; c < NC; ++c) bq[0][c] = src[(c * HT) * 64 + lane];
    static_for<HT>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t + 2 < HT) {
#pragma unroll
            for (int r = 0; r < 4; ++r) g[(t + 2) % 3][r] = wp[(size_t)(4 * (t + 2) + r) * 256];
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
                    acc[c][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(frag_at<T4>(g[t % 3][r], j), bq[t % 2][c][r],
                                                                     acc[c][j], 0, 0, 0);
    });
}

// one or two output units (16 output rows x one 16-column tile each) over all
// k-steps; unit u reads weight rows w[u] and the B operands of column tile cs[u];
// weights pipelined two groups ahead as in gemm_from_lds
template <int T4, int NC, int NT>
__device__ __forceinline__ void out_units(f32x4 (&o)[2], const f32x4* __restrict__ cur, const f32x4* __restrict__ w0,
                                          const f32x4* __restrict__ w1, int c0, int c1)
{
    constexpr int HT = 4 * T4;
    f32x4 g[3][NT];  // weight fragments of 4 k-steps per unit
    const f32x4* wt[2] = {w0, w1};
    const int cs[2] = {c0, c1};
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        g[0][u] = wt[u][0];
        g[1][u] = wt[u][64];
    }
    f32x4 bq[2][NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) bq[0][c] = cur[(c * HT) * 64];
    static_for<HT>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t + 2 < HT) {
#pragma unroll
            for (int u = 0; u < NT; ++u) g[(t + 2) % 3][u] = wt[u][(t + 2) * 64];
        }
        if constexpr (t + 1 < HT) {
#pragma unroll
            for (int c = 0; c < NC; ++c) bq[(t + 1) % 2][c] = cur[(c * HT + t + 1) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x4 bu[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            bu[u] = bq[t % 2][0];
#pragma unroll
            for (int c = 1; c < NC; ++c)
                if (cs[u] == c) bu[u] = bq[t % 2][c];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int u = 0; u < NT; ++u)
                o[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(g[t % 3][u][r], bu[u][r], o[u], 0, 0, 0);
    });
}

// T4: hidden tiles per wave (width/64); NC: 16-column tiles per block
template <int T4, int NC>
__global__ __launch_bounds__(256) void dense_forward_kernel(DenseArgs p)
{
    constexpr int HT = 4 * T4;  // hidden tiles of 16 units
    constexpr int HP = 16 * HT; // padded width
    constexpr int NCOL = 16 * NC;
    typedef typename Frag<T4>::type FT;
    extern __shared__ __attribute__((aligned(16))) f32x4 lds[];  // buf0 [NC][HT][64], buf1 >= same
    f32x4* buf0 = lds;
    f32x4* buf1 = lds + NC * HT * 64;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cl = lane & 15;
    const int kr = lane >> 4;
    const int64_t col0 = (int64_t)blockIdx.x * NCOL;

    // ---- stage normalised inputs into buf1 in MFMA B-operand order ----
    // x for column tile c, k-step s = 4g + r, k-slot kr, column cl lives at float
    // index c*kp*16 + (g*64 + kr*16 + cl)*4 + r: one ds_read_b128 per lane yields the
    // B operands of a whole group of 4 k-steps.
    {
        float* xs = reinterpret_cast<float*>(buf1);
        const int cb = threadIdx.x % NCOL;  // column within the block
        const int64_t col = col0 + cb;
        const bool valid = col < p.ncol;
        const int64_t cc = valid ? col : col0;
        const int64_t blk = cc / p.ncol_blk;
        const int64_t ii = cc - blk * p.ncol_blk;
        float* xc = xs + (cb >> 4) * (p.kp * 16);
        const int cl16 = cb & 15;
        constexpr int FSTRIDE = 256 / NCOL;
        auto xidx = [&](int f) { return ((f >> 4) * 64 + (f & 3) * 16 + cl16) * 4 + ((f >> 2) & 3); };
        for (int v = 0; v < p.n_in; ++v) {
            const DenseInVar iv = p.in[v];
            const float* src = iv.ptr + blk * iv.bs + ii;
            const int nf = 4 * iv.nsteps;
            for (int f0 = threadIdx.x / NCOL; f0 < nf; f0 += 16 * FSTRIDE) {
                float raw[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {  // sixteen HBM loads in flight per thread
                    const int fz = f0 + q * FSTRIDE;
                    raw[q] = (fz < iv.nkeep && valid) ? src[(int64_t)(iv.z0 + fz) * iv.ld] : 0.0f;
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int fz = f0 + q * FSTRIDE;
                    if (fz < nf) {
                        const int f = 4 * iv.step0 + fz;
                        xc[xidx(f)] = (fz < iv.nkeep && valid) ? (raw[q] - p.in_mean[f]) / p.in_denom[f] : 0.0f;
                    }
                }
            }
        }
        for (int f = 4 * p.in_steps_total + threadIdx.x / NCOL; f < p.kp; f += FSTRIDE) xc[xidx(f)] = 0.0f;
    }
    __syncthreads();

    // ---- layer 1: Dense(width) over the padded input features ----
    f32x4 acc[NC][T4];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < T4; ++j) acc[c][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    {
        const f32x4* xq = buf1 + lane;  // + c*kp*4 + g*64
        const FT* w1 = reinterpret_cast<const FT*>(p.w1) + (size_t)wave * 64 + lane;
        const int ngroups = p.kp / 16;
        // weights of the next group and B operands of the next group in flight
        FT g[2][4];
        f32x4 xb[2][NC];
#pragma unroll
        for (int r = 0; r < 4; ++r) g[0][r] = w1[(size_t)r * 256];
#pragma unroll
        for (int c = 0; c < NC; ++c) xb[0][c] = xq[c * p.kp * 4];
        for (int gi = 0; gi < ngroups; gi += 2) {
            static_for<2>([&](auto hc) {
                constexpr int h = decltype(hc)::value;
                const int grp = gi + h;
                if (grp < ngroups) {
                    if (grp + 1 < ngroups) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) g[1 - h][r] = w1[(size_t)(4 * (grp + 1) + r) * 256];
#pragma unroll
                        for (int c = 0; c < NC; ++c) xb[1 - h][c] = xq[c * p.kp * 4 + (grp + 1) * 64];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int j = 0; j < T4; ++j)
#pragma unroll
                            for (int c = 0; c < NC; ++c)
                                acc[c][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(frag_at<T4>(g[h][r], j), xb[h][c][r],
                                                                                 acc[c][j], 0, 0, 0);
                }
            });
        }
    }
    __syncthreads();  // every wave is done with the staged inputs (buf1)
    bias_relu_store<T4, NC>(acc, p.b1, wave, lane, kr, buf0);
    __syncthreads();

    // ---- further hidden layers (ping-pong) ----
    f32x4* cur = buf0;
    f32x4* nxt = buf1;
    for (int l = 0; l < p.n_hidden_extra; ++l) {
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < T4; ++j) acc[c][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        gemm_from_lds<T4, NC>(acc, cur, reinterpret_cast<const FT*>(p.wh) + (size_t)l * (HP / 4) * 4 * 64, wave,
                              lane);
        bias_relu_store<T4, NC>(acc, p.bh + (size_t)l * HP, wave, lane, kr, nxt);
        __syncthreads();
        f32x4* t = cur;
        cur = nxt;
        nxt = t;
    }

    // ---- output Dense layers + denorm/limit/mask epilogue ----
    // units u = (tile m = u / NC, column tile c = u % NC); wave w takes u = w, w+4, ...
    // two at a time, so the 4 waves share the n_otiles*NC units evenly
    const int nunits = p.n_otiles * NC;
    for (int u0 = wave; u0 < nunits; u0 += 8) {
        const int u1 = u0 + 4;
        const bool two = u1 < nunits;
        const int m0 = u0 / NC, c0 = u0 % NC;
        const int m1 = two ? u1 / NC : m0, c1 = two ? u1 % NC : c0;
        f32x4 o[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
        const f32x4* w0 = reinterpret_cast<const f32x4*>(p.wo) + (size_t)m0 * (HP / 16) * 64 + lane;
        const f32x4* w1p = reinterpret_cast<const f32x4*>(p.wo) + (size_t)m1 * (HP / 16) * 64 + lane;
        if (two)
            out_units<T4, NC, 2>(o, cur + lane, w0, w1p, c0, c1);
        else
            out_units<T4, NC, 1>(o, cur + lane, w0, w1p, c0, c1);
#pragma unroll
        for (int uu = 0; uu < 2; ++uu) {
            if (uu == 1 && !two) break;
            const int m = uu == 0 ? m0 : m1;
            const int c = uu == 0 ? c0 : c1;
            const DenseOutTile ot = p.otile[m];
            if (ot.var < 0) continue;
            const int64_t col = col0 + 16 * c + cl;
            const bool valid = col < p.ncol;
            const int64_t cc = valid ? col : col0;
            const int64_t blk = cc / p.ncol_blk;
            const int64_t ii = cc - blk * p.ncol_blk;
            const f32x4 ov = o[uu];
            float* dst = p.out_ptr[ot.var] + blk * p.out_bs[ot.var] + ii;
            const int64_t ld = p.out_ld[ot.var];
            const int fo = 16 * m + 4 * kr;
            const f32x4 bo = *reinterpret_cast<const f32x4*>(p.bo + fo);
            const f32x4 sg = *reinterpret_cast<const f32x4*>(p.o_sigma + fo);
            const f32x4 mu = *reinterpret_cast<const f32x4*>(p.o_mean + fo);
            const f32x4 lo = *reinterpret_cast<const f32x4*>(p.o_lo + fo);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(p.o_hi + fo);
            const f32x4 mk = *reinterpret_cast<const f32x4*>(p.o_mask + fo);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * kr + r;
                float y = ov[r] + bo[r];
                y = y * sg[r];
                y = y + mu[r];
                if (y < lo[r]) y = lo[r];
                if (y >= hi[r]) y = hi[r];
                y = y * mk[r];
                if (valid && row < ot.nrow) dst[(int64_t)(ot.z0 + row) * ld] = y;
            }
        }
    }
}

}  // namespace fv3

// ------------------------------------------------------------------------------------
// host side: model creation (validation + fragment packing), forward launch
// ------------------------------------------------------------------------------------
struct fv3_dense_model {
    int n_in = 0, n_out = 0, k_in = 0, k_out = 0, width = 0, ht = 0, hp = 0, n_hidden = 0;
    int kp = 0, n_otiles = 0, steps_total = 0;
    std::vector<int> in_nz, out_nz, in_z0, in_nkeep, in_step0, in_nsteps;
    std::vector<fv3::DenseOutTile> otiles;
    void* dbuf = nullptr;
    fv3::DenseArgs tmpl{};  // device pointers filled, per-call fields empty
};

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
    while (step % 4) {  // whole groups of 4 k-steps for the layer-1 pipeline
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
        for (int z0 = 0; z0 < nz; z0 += 16) {
            DenseOutTile t{v, z0, std::min(16, nz - z0), 0};
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
        in_denom[f] = s + d->epsilon;  // StandardNormLayer computes sigma + epsilon in f32
    }
    const int T4 = HT / 4;
    // layer 1: W1[k_in][W] -> [KP/4][wave][64][T4]; tile m = wave*T4 + j
    std::vector<float> w1((size_t)m->kp * HP, 0.0f);
    for (int s = 0; s < m->kp / 4; ++s)
        for (int wv = 0; wv < 4; ++wv)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < T4; ++j) {
                    const int f = 4 * s + (l >> 4);
                    const int unit = 16 * (wv * T4 + j) + (l & 15);
                    const int src = feat_src[f];
                    float v = 0.0f;
                    if (src >= 0 && unit < W) v = d->hidden_kernel[0][(size_t)src * W + unit];
                    w1[(((size_t)s * 4 + wv) * 64 + l) * T4 + j] = v;
                }
    std::vector<float> b1(HP, 0.0f);
    for (int u = 0; u < W; ++u) b1[u] = d->hidden_bias[0][u];
    // hidden layers 2..n: W[W][W] -> [HP/4][wave][64][T4]; k-step s = 4t + r reads
    // input unit 16t + 4(l>>4) + r (the accumulator-layout permutation)
    const int nhx = d->n_hidden - 1;
    std::vector<float> wh((size_t)std::max(nhx, 1) * HP * HP, 0.0f), bh((size_t)std::max(nhx, 1) * HP, 0.0f);
    for (int li = 0; li < nhx; ++li) {
        const float* K = d->hidden_kernel[li + 1];
        for (int s = 0; s < HP / 4; ++s) {
            const int t = s / 4, r = s % 4;
            for (int wv = 0; wv < 4; ++wv)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < T4; ++j) {
                        const int in = 16 * t + 4 * (l >> 4) + r;
                        const int unit = 16 * (wv * T4 + j) + (l & 15);
                        float v = 0.0f;
                        if (in < W && unit < W) v = K[(size_t)in * W + unit];
                        wh[(size_t)li * HP * HP + (((size_t)s * 4 + wv) * 64 + l) * T4 + j] = v;
                    }
        }
        for (int u = 0; u < W; ++u) bh[(size_t)li * HP + u] = d->hidden_bias[li + 1][u];
    }
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
    std::vector<float> bo(kop, 0.0f), osig(kop, 1.0f), omean(kop, 0.0f), olo(kop, -INFINITY),
        ohi(kop, INFINITY), omask(kop, 1.0f);
    for (int row = 0; row < kop; ++row) {
        const int src = ofeat_src[row];
        if (src < 0) continue;
        const int ov = ocol_var[src], oz = ocol_z[src];
        bo[row] = d->out_bias[ov][oz];
        osig[row] = d->out_sigma[src];
        omean[row] = d->out_mean[src];
        if (d->out_min) olo[row] = d->out_min[src];
        if (d->out_max) ohi[row] = d->out_max[src];
        if (d->out_mask) omask[row] = d->out_mask[src];
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
        {wo.data(), wo.size() * 4, 0},           {bo.data(), bo.size() * 4, 0},
        {osig.data(), osig.size() * 4, 0},       {omean.data(), omean.size() * 4, 0},
        {olo.data(), olo.size() * 4, 0},         {ohi.data(), ohi.size() * 4, 0},
        {omask.data(), omask.size() * 4, 0},
    };
    size_t total = 0;
    for (auto& p : pcs) {
        p.off = total;
        total += (p.bytes + 255) / 256 * 256;
    }
    FV3_HIP(hipMalloc(&m->dbuf, total));
    for (auto& p : pcs) FV3_HIP(hipMemcpy((char*)m->dbuf + p.off, p.src, p.bytes, hipMemcpyHostToDevice));
    auto at = [&](int i) { return (char*)m->dbuf + pcs[i].off; };
    DenseArgs& a = m->tmpl;
    a.in_mean = (const float*)at(0);
    a.in_denom = (const float*)at(1);
    a.w1 = (const float*)at(2);
    a.b1 = (const float*)at(3);
    a.wh = (const float*)at(4);
    a.bh = (const float*)at(5);
    a.wo = (const float*)at(6);
    a.bo = (const float*)at(7);
    a.o_sigma = (const float*)at(8);
    a.o_mean = (const float*)at(9);
    a.o_lo = (const float*)at(10);
    a.o_hi = (const float*)at(11);
    a.o_mask = (const float*)at(12);
    for (int v = 0; v < m->n_in; ++v) {
        a.in[v].step0 = m->in_step0[v];
        a.in[v].nsteps = m->in_nsteps[v];
        a.in[v].z0 = m->in_z0[v];
        a.in[v].nkeep = m->in_nkeep[v];
    }
    for (int t = 0; t < m->n_otiles; ++t) a.otile[t] = m->otiles[t];
    a.n_in = m->n_in;
    a.n_hidden_extra = nhx;
    a.n_otiles = m->n_otiles;
    a.kp = m->kp;
    a.in_steps_total = m->steps_total;
    *out = guard.release();
    return FV3_OK;
}

extern "C" int fv3_dense_destroy(fv3_dense_model* m)
{
    fv3::clear_error();
    if (!m) return FV3_OK;
    if (m->dbuf) FV3_HIP(hipFree(m->dbuf));
    delete m;
    return FV3_OK;
}

extern "C" int fv3_dense_k_in(const fv3_dense_model* m) { return m ? m->k_in : -1; }
extern "C" int fv3_dense_k_out(const fv3_dense_model* m) { return m ? m->k_out : -1; }

extern "C" int fv3_dense_forward(const fv3_dense_model* m, const float* const* inputs, const fv3_layout* in_l,
                                 float* const* outputs, const fv3_layout* out_l, int64_t ncol, void* stream)
{
    using namespace fv3;
    clear_error();
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
        a.in[v].ptr = inputs[v];
        a.in[v].ld = in_l[v].ld;
        a.in[v].bs = in_l[v].blk_stride;
    }
    for (int v = 0; v < m->n_out; ++v) {
        FV3_REQUIRE(outputs[v], "dense_forward: output %d is NULL", v);
        FV3_REQUIRE(layout_ok(out_l[v], ncol) && out_l[v].ncol_blk == nb,
                    "dense_forward: output %d layout invalid or ncol_blk differs", v);
        a.out_ptr[v] = outputs[v];
        a.out_ld[v] = out_l[v].ld;
        a.out_bs[v] = out_l[v].blk_stride;
    }
    a.ncol = ncol;
    a.ncol_blk = nb;
    // columns per block: two 16-column tiles (measured fastest at C48/C96/C384:
    // halves weight traffic per FLOP; 2 blocks/CU by LDS)
    int nc = 2;
    if (const char* e = getenv("FV3_DENSE_NC")) {
        nc = atoi(e) == 1 ? 1 : 2;  // A/B switch; 2 is fastest at C48, C96 and C384
    }
    const int64_t grid = (ncol + 16 * nc - 1) / (16 * nc);
    FV3_REQUIRE(grid < (int64_t)0x7fffffff, "dense_forward: ncol too large");
    hipStream_t s = (hipStream_t)stream;
    // buf0: one layer of activations (NC x HT tiles x 64 lanes x 16 B); buf1: the other
    // layer, or the staged inputs (NC x kp features x 16 columns) if those are larger
    const size_t hbytes = (size_t)nc * 16 * 64 * (size_t)m->ht;
    const size_t xbytes = (size_t)nc * sizeof(float) * 16 * (size_t)m->kp;
    const size_t lds = hbytes + std::max(hbytes, xbytes);
    FV3_REQUIRE(lds <= 160 * 1024, "dense_forward: %d input features need too much LDS", m->kp);
#define FV3_DENSE_LAUNCH(T4, NC) \
    hipLaunchKernelGGL((dense_forward_kernel<T4, NC>), dim3((unsigned)grid), dim3(256), lds, s, a)
    if (nc == 1) {
        if (m->ht == 4) FV3_DENSE_LAUNCH(1, 1);
        else if (m->ht == 8) FV3_DENSE_LAUNCH(2, 1);
        else FV3_DENSE_LAUNCH(4, 1);
    } else {
        if (m->ht == 4) FV3_DENSE_LAUNCH(1, 2);
        else if (m->ht == 8) FV3_DENSE_LAUNCH(2, 2);
        else FV3_DENSE_LAUNCH(4, 2);
    }
#undef FV3_DENSE_LAUNCH
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
