// TEST-ONLY host build of the product's streaming mappm (fv3net_amd/csrc/mappm_core.h).
// Lets the CPU test suite check the one-pass algorithm bit-for-bit against the
// oracle without a GPU.  Not part of the product library and never loaded by it.
#include <cstdint>
#include <vector>
#include "../../fv3net_amd/csrc/mappm_core.h"

namespace {
struct Col {
    const float *pe1_, *q1_, *pe2_;
    float* q2_;
    int64_t ncol, i;
    int kn;
    float q1(int k) const { return q1_[(int64_t)(k - 1) * ncol + i]; }
    float pe1(int k) const { return pe1_[(int64_t)(k - 1) * ncol + i]; }
    float pe2(int k) const { return pe2_[(int64_t)(k - 1) * ncol + i]; }
    void emit(int k, float v) { q2_[(int64_t)(k - 1) * ncol + i] = v; }
    float next_edge(int k) const { return (k + 1 <= kn + 1) ? pe2(k + 1) : 0.0f; }
};
struct Scr {
    std::vector<float> ev, gv;
    float& e(int k) { return ev[k]; }
    float& g(int k) { return gv[k]; }
};
}  // namespace

extern "C" int host_mappm(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                          float* q2, int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1) return -1;
    Scr scr{std::vector<float>(km + 3), std::vector<float>(km + 3)};
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        if (kord > 7)
            fv3::mappm_cs_column(c, scr, km, kn, iv, kord);
        else
            fv3::mappm_ppm_column(c, km, kn, iv, kord);
    }
    return 0;
}

// kord > 7 with the bottom `nt` edges in registers (mappm_cs_column<..., NT>), as the
// device kernel runs it: the same bits as host_mappm's all-scratch column
extern "C" int host_mappm_cs_tail(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                  float* q2, int64_t ncol, int iv, int kord, int nt)
{
    if (km < 4 || kn < 1 || kord <= 7) return -1;
    Scr scr{std::vector<float>(km + 3), std::vector<float>(km + 3)};
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        switch (nt) {
        case 8: fv3::mappm_cs_column<Col, Scr, 8>(c, scr, km, kn, iv, kord); break;
        case 16: fv3::mappm_cs_column<Col, Scr, 16>(c, scr, km, kn, iv, kord); break;
        case 32: fv3::mappm_cs_column<Col, Scr, 32>(c, scr, km, kn, iv, kord); break;
        case 48: fv3::mappm_cs_column<Col, Scr, 48>(c, scr, km, kn, iv, kord); break;
        default: return -1;
        }
    }
    return 0;
}

// kord > 7 with the loads run `pf` levels ahead (mappm_cs_column<..., NT, PF>) and the
// bottom `nt` edges in registers, as the device kernel runs it
template <int NT>
static int cs_pf(Col& c, Scr& scr, int km, int kn, int iv, int kord, int pf)
{
    switch (pf) {
    case 2: fv3::mappm_cs_column<Col, Scr, NT, 2>(c, scr, km, kn, iv, kord); return 0;
    case 4: fv3::mappm_cs_column<Col, Scr, NT, 4>(c, scr, km, kn, iv, kord); return 0;
    case 8: fv3::mappm_cs_column<Col, Scr, NT, 8>(c, scr, km, kn, iv, kord); return 0;
    default: return -1;
    }
}
extern "C" int host_mappm_cs_prefetch(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                      float* q2, int64_t ncol, int iv, int kord, int nt, int pf)
{
    if (km < 4 || kn < 1 || kord <= 7) return -1;
    Scr scr{std::vector<float>(km + 3), std::vector<float>(km + 3)};
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        const int st = nt == 0 ? cs_pf<0>(c, scr, km, kn, iv, kord, pf) : cs_pf<16>(c, scr, km, kn, iv, kord, pf);
        if (st) return st;
    }
    return 0;
}

// same through the output-driven cursor (kord <= 7), as the fused coarsen kernel uses it
extern "C" int host_mappm_cursor(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                 float* q2, int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        fv3::mappm_ppm_column_by_output(c, km, kn, iv, kord);
    }
    return 0;
}

// the streaming column with the reference-shaped event loop (remap_layer) instead of
// remap_layer_fast: the two must agree bit for bit on every input, sorted or not
extern "C" int host_mappm_generic(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                  float* q2, int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        fv3::mappm_ppm_column<Col, false>(c, km, kn, iv, kord);
    }
    return 0;
}

// the same column with level L + 4's loads carried one iteration ahead (CARRY: the
// device mappm kernel's build)
extern "C" int host_mappm_carry(int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                float* q2, int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        fv3::mappm_ppm_column<Col, true, true>(c, km, kn, iv, kord);
    }
    return 0;
}

// the window in register rings (RING: the fast single-field kernel's column), with CARRY
extern "C" int host_mappm_ring(int km, const float* pe1, const float* q1, int kn, const float* pe2, float* q2,
                               int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    for (int64_t i = 0; i < ncol; ++i) {
        Col c{pe1, q1, pe2, q2, ncol, i, kn};
        fv3::mappm_ppm_column<Col, true, true, true>(c, km, kn, iv, kord);
    }
    return 0;
}

// NF fields on one pressure column in one pass (mappm_multi.h), as the fused coarsen
// kernel runs them: q1 / q2 hold NF arrays [km][ncol] / [kn][ncol] back to back
#include "../../fv3net_amd/csrc/mappm_multi.h"
namespace {
struct ColN {
    const float *pe1_, *q1_, *pe2_;
    float* q2_;
    int64_t ncol, i;
    int km, kn;
    float q1(int f, int k) const { return q1_[((int64_t)f * km + (k - 1)) * ncol + i]; }
    float pe1(int k) const { return pe1_[(int64_t)(k - 1) * ncol + i]; }
    float pe2(int k) const { return pe2_[(int64_t)(k - 1) * ncol + i]; }
    void emit(int f, int k, float v) { q2_[((int64_t)f * kn + (k - 1)) * ncol + i] = v; }
    float next_edge(int k) const { return (k + 1 <= kn + 1) ? pe2(k + 1) : 0.0f; }
};
template <int NF, bool CARRY = false>
void run_n(int km, const float* pe1, const float* q1, int kn, const float* pe2, float* q2, int64_t ncol, int iv,
           int kord)
{
    for (int64_t i = 0; i < ncol; ++i) {
        ColN c{pe1, q1, pe2, q2, ncol, i, km, kn};
        fv3::mappm_ppm_columns<NF, ColN, CARRY>(c, km, kn, iv, kord);
    }
}
}  // namespace

// two fields with level L + 4's loads carried one iteration ahead (the device pair kernel)
extern "C" int host_mappm_pair_carry(int km, const float* pe1, const float* q1, int kn, const float* pe2, float* q2,
                                     int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    run_n<2, true>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord);
    return 0;
}

extern "C" int host_mappm_multi(int nf, int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                float* q2, int64_t ncol, int iv, int kord)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    switch (nf) {
        case 1: run_n<1>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord); return 0;
        case 2: run_n<2>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord); return 0;
        case 3: run_n<3>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord); return 0;
        case 4: run_n<4>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord); return 0;
    }
    return -1;
}

// a column on two lanes (mappm_ppm_columns<NF, .., SPLIT>, the small-grid pair kernel):
// the two halves one after the other, with the kernel's start-layer search, streamed
// sortedness checks and single-pass fix-up; kb = 0: the kernel's split point kn / 2 + 1;
// walk = 1: the second half always from layer 1
template <int NF>
static void run_split(int km, const float* pe1, const float* q1, int kn, const float* pe2, float* q2, int64_t ncol,
                      int iv, int kord, int kb, int walk)
{
    for (int64_t i = 0; i < ncol; ++i) {
        ColN c{pe1, q1, pe2, q2, ncol, i, km, kn};
        if (kn < 2) {  // the host runs the single-lane kernel
            fv3::mappm_ppm_columns<NF, ColN, true>(c, km, kn, iv, kord);
            continue;
        }
        const int kB = kb > 0 ? kb : kn / 2 + 1;
        const float t = c.pe2(kB);
        const int L0 = walk ? 1 : fv3::split_first_layer(c, km, t, fv3::split_count_sorted(c, km, t));
        fv3::SplitCheck a{1, km}, b{1, km};
        fv3::mappm_ppm_columns<NF, ColN, true, true>(c, km, kn, iv, kord, 1, kB - 1, 1, &a);
        fv3::mappm_ppm_columns<NF, ColN, true, true>(c, km, kn, iv, kord, kB, kn, L0, &b);
        if (!fv3::split_exact(a, b, L0, km)) fv3::mappm_ppm_columns<NF, ColN, true>(c, km, kn, iv, kord);
    }
}
// a column on three lanes (the kernel's split points kn / 3 + 1 and 2 kn / 3 + 1, kn >= 3)
template <int NF>
static void run_split3(int km, const float* pe1, const float* q1, int kn, const float* pe2, float* q2, int64_t ncol,
                       int iv, int kord, int walk)
{
    for (int64_t i = 0; i < ncol; ++i) {
        ColN c{pe1, q1, pe2, q2, ncol, i, km, kn};
        if (kn < 3) {
            fv3::mappm_ppm_columns<NF, ColN, true>(c, km, kn, iv, kord);
            continue;
        }
        const int kB1 = kn / 3 + 1, kB2 = 2 * kn / 3 + 1;
        const float t1 = c.pe2(kB1), t2 = c.pe2(kB2);
        const int L1 = walk ? 1 : fv3::split_first_layer(c, km, t1, fv3::split_count_sorted(c, km, t1));
        const int L2 = walk ? 1 : fv3::split_first_layer(c, km, t2, fv3::split_count_sorted(c, km, t2));
        fv3::SplitCheck a{1, km}, b{1, km}, d{1, km};
        fv3::mappm_ppm_columns<NF, ColN, true, true>(c, km, kn, iv, kord, 1, kB1 - 1, 1, &a);
        fv3::mappm_ppm_columns<NF, ColN, true, true>(c, km, kn, iv, kord, kB1, kB2 - 1, L1, &b);
        fv3::mappm_ppm_columns<NF, ColN, true, true>(c, km, kn, iv, kord, kB2, kn, L2, &d);
        if (!fv3::split3_exact(a, b, d, L1, L2, km)) fv3::mappm_ppm_columns<NF, ColN, true>(c, km, kn, iv, kord);
    }
}
extern "C" int host_mappm_split3(int nf, int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                 float* q2, int64_t ncol, int iv, int kord, int walk)
{
    if (km < 4 || kn < 1 || kord > 7) return -1;
    switch (nf) {
        case 1: run_split3<1>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord, walk); return 0;
        case 2: run_split3<2>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord, walk); return 0;
    }
    return -1;
}
extern "C" int host_mappm_split(int nf, int km, const float* pe1, const float* q1, int kn, const float* pe2,
                                float* q2, int64_t ncol, int iv, int kord, int kb, int walk)
{
    if (km < 4 || kn < 1 || kord > 7 || kb > kn || kb == 1) return -1;
    switch (nf) {
        case 1: run_split<1>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord, kb, walk); return 0;
        case 2: run_split<2>(km, pe1, q1, kn, pe2, q2, ncol, iv, kord, kb, walk); return 0;
    }
    return -1;
}
