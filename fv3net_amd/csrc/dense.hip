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
//  * one wave owns a 16-column tile for the whole network; four waves per block;
//  * lane l holds column (l & 15) and k-slot (l >> 4) of every B operand;
//  * layer activations live in the MFMA accumulators (unit 16m + 4(l>>4) + r in
//    register r of tile m) and are fed AS-IS as the B operand of the next layer:
//    k-step s = 4t + r takes register r of tile t, so the contraction order over
//    hidden units is permuted and the packed weights carry the same permutation;
//  * weights are pre-packed at create time into per-lane fragment order, so every
//    A-operand fetch is one 16 B/lane (1 KiB per wave) fully coalesced load that
//    the 4 waves of a block (and neighbouring blocks on the CU) share through L1/L2;
//  * each input variable's features and each output tile are padded so a k-step
//    (4 features) never straddles two variables: the source pointer is uniform.
// Roofline: fp32 MFMA-bound.  2*(k_in*w + (n_hidden-1)*w*w + w*k_out) FLOP per
// column (292,864 for the 2x256 C48 model) against (k_in + k_out) * 4 B of HBM.
#include <cmath>
#include <cstring>
#include <memory>
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
    const f32x4* w1;        // [KP/4][HT/4][64]
    const float* b1;        // [HP]
    const f32x4* wh;        // [n_hidden-1][HP/4][HT/4][64]
    const float* bh;        // [n_hidden-1][HP]
    const f32x2* wo;        // [n_chunks][HP/4][64]
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
    int n_in, n_hidden_extra, n_chunks, pad_;
};

template <int HT>
__device__ __forceinline__ void bias_relu(f32x4 (&h)[HT], const float* __restrict__ b, int kr)
{
#pragma unroll
    for (int m = 0; m < HT; ++m) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b + 16 * m + 4 * kr);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = h[m][r] + bb[r];
            h[m][r] = v > 0.0f ? v : 0.0f;
        }
    }
}

// one hidden Dense(width, relu): g = relu(W^T h + b), h in accumulator layout
template <int HT>
__device__ __forceinline__ void hidden_layer(const f32x4 (&h)[HT], f32x4 (&g)[HT],
                                             const f32x4* __restrict__ w, const float* __restrict__ b,
                                             int lane, int kr)
{
#pragma unroll
    for (int m = 0; m < HT; ++m) g[m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int s = 4 * t + r;
            const f32x4* ws = w + (size_t)s * (HT / 4) * 64 + lane;
            const float bop = h[t][r];
#pragma unroll
            for (int mq = 0; mq < HT / 4; ++mq) {
                const f32x4 a = ws[mq * 64];
                g[4 * mq + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bop, g[4 * mq + 0], 0, 0, 0);
                g[4 * mq + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bop, g[4 * mq + 1], 0, 0, 0);
                g[4 * mq + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bop, g[4 * mq + 2], 0, 0, 0);
                g[4 * mq + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bop, g[4 * mq + 3], 0, 0, 0);
            }
        }
    }
    bias_relu<HT>(g, b, kr);
}

template <int HT>
__global__ __launch_bounds__(256) void dense_forward_kernel(DenseArgs p)
{
    constexpr int HP = HT * 16;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t col0 = ((int64_t)blockIdx.x * 4 + wave) * 16;
    if (col0 >= p.ncol) return;  // wave-uniform
    const int cl = lane & 15;
    const int kr = lane >> 4;
    const int64_t col = col0 + cl;
    const bool valid = col < p.ncol;
    const int64_t cc = valid ? col : col0;
    const int64_t blk = cc / p.ncol_blk;
    const int64_t ii = cc - blk * p.ncol_blk;

    // ---- layer 1: normalize + Dense(width) over the padded input features ----
    f32x4 h[HT];
#pragma unroll
    for (int m = 0; m < HT; ++m) h[m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int v = 0; v < p.n_in; ++v) {
        const DenseInVar iv = p.in[v];
        const float* src = iv.ptr + blk * iv.bs + ii;
        for (int s = 0; s < iv.nsteps; ++s) {
            const int zrel = 4 * s + kr;
            const int f = 4 * (iv.step0 + s) + kr;
            float x = 0.0f;
            if (zrel < iv.nkeep && valid) {
                const float raw = src[(int64_t)(iv.z0 + zrel) * iv.ld];
                x = (raw - p.in_mean[f]) / p.in_denom[f];
            }
            const f32x4* ws = p.w1 + (size_t)(iv.step0 + s) * (HT / 4) * 64 + lane;
#pragma unroll
            for (int mq = 0; mq < HT / 4; ++mq) {
                const f32x4 a = ws[mq * 64];
                h[4 * mq + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], x, h[4 * mq + 0], 0, 0, 0);
                h[4 * mq + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], x, h[4 * mq + 1], 0, 0, 0);
                h[4 * mq + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], x, h[4 * mq + 2], 0, 0, 0);
                h[4 * mq + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], x, h[4 * mq + 3], 0, 0, 0);
            }
        }
    }
    bias_relu<HT>(h, p.b1, kr);

    // ---- further hidden layers ----
    for (int l = 0; l < p.n_hidden_extra; ++l) {
        f32x4 g[HT];
        hidden_layer<HT>(h, g, p.wh + (size_t)l * (HP / 4) * (HT / 4) * 64, p.bh + (size_t)l * HP, lane, kr);
#pragma unroll
        for (int m = 0; m < HT; ++m) h[m] = g[m];
    }

    // ---- output Dense layers (32 output rows per chunk) + denorm/limit/mask epilogue ----
    for (int ch = 0; ch < p.n_chunks; ++ch) {
        f32x4 o0 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        f32x4 o1 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const f32x2* wc = p.wo + (size_t)ch * (HP / 4) * 64 + lane;
#pragma unroll
        for (int t = 0; t < HT; ++t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f32x2 a = wc[(size_t)(4 * t + r) * 64];
                o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], h[t][r], o0, 0, 0, 0);
                o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], h[t][r], o1, 0, 0, 0);
            }
        }
#pragma unroll
        for (int mm = 0; mm < 2; ++mm) {
            const int m = 2 * ch + mm;
            const DenseOutTile ot = p.otile[m];
            if (ot.var < 0) continue;
            const f32x4 acc = mm == 0 ? o0 : o1;
            float* dst = p.out_ptr[ot.var] + blk * p.out_bs[ot.var] + ii;
            const int64_t ld = p.out_ld[ot.var];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * kr + r;
                const int fo = 16 * m + row;
                float y = acc[r] + p.bo[fo];
                y = y * p.o_sigma[fo];
                y = y + p.o_mean[fo];
                const float lo = p.o_lo[fo], hi = p.o_hi[fo];
                if (y < lo) y = lo;
                if (y >= hi) y = hi;
                y = y * p.o_mask[fo];
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
    int kp = 0, n_chunks = 0, n_otiles = 0;
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
    if (m->otiles.size() % 2) {
        m->otiles.push_back(DenseOutTile{-1, 0, 0, 0});
        for (int r = 0; r < 16; ++r) ofeat_src.push_back(-1);
    }
    FV3_REQUIRE((int)m->otiles.size() <= kMaxOutTiles, "dense_create: too many output rows (%d tiles)",
                (int)m->otiles.size());
    m->k_out = k_out;
    m->n_otiles = (int)m->otiles.size();
    m->n_chunks = m->n_otiles / 2;
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
    // layer 1: W1[k_in][W] -> [KP/4][HT/4][64][4]
    std::vector<float> w1((size_t)m->kp * HP, 0.0f);
    for (int s = 0; s < m->kp / 4; ++s)
        for (int mq = 0; mq < HT / 4; ++mq)
            for (int l = 0; l < 64; ++l)
                for (int c = 0; c < 4; ++c) {
                    const int f = 4 * s + (l >> 4);
                    const int unit = 16 * (4 * mq + c) + (l & 15);
                    const int src = feat_src[f];
                    float v = 0.0f;
                    if (src >= 0 && unit < W) v = d->hidden_kernel[0][(size_t)src * W + unit];
                    w1[(((size_t)s * (HT / 4) + mq) * 64 + l) * 4 + c] = v;
                }
    std::vector<float> b1(HP, 0.0f);
    for (int u = 0; u < W; ++u) b1[u] = d->hidden_bias[0][u];
    // hidden layers 2..n: W[W][W] -> [HP/4][HT/4][64][4] with permuted k
    const int nhx = d->n_hidden - 1;
    std::vector<float> wh((size_t)std::max(nhx, 1) * HP * HP, 0.0f), bh((size_t)std::max(nhx, 1) * HP, 0.0f);
    for (int li = 0; li < nhx; ++li) {
        const float* K = d->hidden_kernel[li + 1];
        for (int s = 0; s < HP / 4; ++s) {
            const int t = s / 4, r = s % 4;
            for (int mq = 0; mq < HT / 4; ++mq)
                for (int l = 0; l < 64; ++l)
                    for (int c = 0; c < 4; ++c) {
                        const int in = 16 * t + 4 * (l >> 4) + r;
                        const int unit = 16 * (4 * mq + c) + (l & 15);
                        float v = 0.0f;
                        if (in < W && unit < W) v = K[(size_t)in * W + unit];
                        wh[(size_t)li * HP * HP + (((size_t)s * (HT / 4) + mq) * 64 + l) * 4 + c] = v;
                    }
        }
        for (int u = 0; u < W; ++u) bh[(size_t)li * HP + u] = d->hidden_bias[li + 1][u];
    }
    // output layer: concat of out kernels [W][out_nz] -> [n_chunks][HP/4][64][2]
    std::vector<int> ocol_var(k_out), ocol_z(k_out);
    {
        int o = 0;
        for (int v = 0; v < d->n_out; ++v)
            for (int z = 0; z < d->out_nz[v]; ++z, ++o) {
                ocol_var[o] = v;
                ocol_z[o] = z;
            }
    }
    std::vector<float> wo((size_t)m->n_chunks * (HP / 4) * 64 * 2, 0.0f);
    for (int ch = 0; ch < m->n_chunks; ++ch)
        for (int s = 0; s < HP / 4; ++s) {
            const int t = s / 4, r = s % 4;
            for (int l = 0; l < 64; ++l)
                for (int mm = 0; mm < 2; ++mm) {
                    const int in = 16 * t + 4 * (l >> 4) + r;
                    const int row = 32 * ch + 16 * mm + (l & 15);
                    const int src = ofeat_src[row];
                    float v = 0.0f;
                    if (src >= 0 && in < W) {
                        const int ov = ocol_var[src], oz = ocol_z[src];
                        v = d->out_kernel[ov][(size_t)in * d->out_nz[ov] + oz];
                    }
                    wo[(((size_t)ch * (HP / 4) + s) * 64 + l) * 2 + mm] = v;
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
    a.w1 = (const f32x4*)at(2);
    a.b1 = (const float*)at(3);
    a.wh = (const f32x4*)at(4);
    a.bh = (const float*)at(5);
    a.wo = (const f32x2*)at(6);
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
    a.n_chunks = m->n_chunks;
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
    const int64_t tiles = (ncol + 15) / 16;
    const int64_t grid = (tiles + 3) / 4;
    FV3_REQUIRE(grid < (int64_t)0x7fffffff, "dense_forward: ncol too large");
    hipStream_t s = (hipStream_t)stream;
    switch (m->ht) {
    case 4:
        hipLaunchKernelGGL(dense_forward_kernel<4>, dim3((unsigned)grid), dim3(256), 0, s, a);
        break;
    case 8:
        hipLaunchKernelGGL(dense_forward_kernel<8>, dim3((unsigned)grid), dim3(256), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(dense_forward_kernel<16>, dim3((unsigned)grid), dim3(256), 0, s, a);
        break;
    }
    FV3_LAUNCH_CHECK();
    return FV3_OK;
}
