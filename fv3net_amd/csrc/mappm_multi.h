// fv3net_amd — the streaming PPM remap (mappm_core.h, kord <= 7) for NF fields that
// share one column's pressure edges, in ONE pass.
//
// coarsen_restarts_on_pressure remaps every masked variable of a restart file onto the
// same coarse pressure edges (external/vcm/vcm/cubedsphere/coarsen_restarts.py:411-516,
// 840-887; one regrid_vertical -> mappm call per variable, regridz.py:164-279).  In
// mappm (external/mappm/mappm/mappm.f90:10-126, ppm_profile :614-851) a large part of
// the work depends on the pressures alone:
//   * ppm_profile: of the 7 divisions per level in dc(k) and the provisional edge
//     a4(2,k), 5 divide pressure thicknesses only (c1, c2 of dc; a1, a2 and
//     2/(d4(k-1)+d4(k+1)) of the edge), the 6th denominator (d4(k)+delp(k+1)) too;
//   * the remap: every decision (which output edge falls in which input layer) and
//     every position PL / PR / ESL, and dpsum.
// Here those are computed once per column and level, and only the field-dependent
// parts (differences of q, the limiters, the pieces' values, qsum / dpsum) per field.
// Each shared value is the same expression on the same operands as in the
// single-field code, so every field's result carries exactly the bits of
// mappm_ppm_column (and of the reference) for that field alone.
//
// `Col` provides (1-based levels, f = 0..NF-1):
//   float q1(int f, int k)      float pe1(int k)      float pe2(int k)
//   void emit(int f, int k, float v)                  float next_edge(int k)
//   optionally void layer_done() (called after every input layer, as layer_hook)
#pragma once

#include "mappm_core.h"

namespace fv3 {
namespace FV3_ARITH_NS {  // the arithmetic policy of mappm_core.h
#ifdef FV3_FAST_ARITH
#pragma clang fp contract(on)
#endif

// ---- pressure-only / field parts of ppm_dc, ppm_al, ppm_h2 (mappm.f90:658-683, 784-795) ----

struct DcShared {
    float c1, c2, den;
};
FV3_HD inline DcShared ppm_dc_shared(float dm1, float d0, float dp1)
{
    const float d4k = dm1 + d0;    // d4(k)
    const float d4kp = d0 + dp1;   // d4(k+1)
    return DcShared{FV3_DIV(dm1 + 0.5f * d0, d4kp), FV3_DIV(dp1 + 0.5f * d0, d4k), d4k + dp1};
}
FV3_HD inline float ppm_dc_field(const DcShared& p, float qm1, float q0, float qp1, float d0)
{
    const float delq_k = qp1 - q0;
    const float delq_km = q0 - qm1;
    const float df2 = FV3_DIV(d0 * (p.c1 * delq_k + p.c2 * delq_km), p.den);
    return fsign(fmin3(fabsf(df2), fmax3(qm1, q0, qp1) - q0, q0 - fmin3(qm1, q0, qp1)), df2);
}

struct AlShared {
    float d4k, s2, amd, a2, dm1a1;
};
FV3_HD inline AlShared ppm_al_shared(float dm2, float dm1, float d0, float dp1)
{
    const float d4km = dm2 + dm1;  // d4(k-1)
    const float d4k = dm1 + d0;    // d4(k)
    const float d4kp = d0 + dp1;   // d4(k+1)
    const float a1 = FV3_DIV(d4km, d4k + dm1);
    const float a2 = FV3_DIV(d4kp, d4k + d0);
    return AlShared{d4k, FV3_DIV(2.0f, d4km + d4kp), a1 - a2, a2, dm1 * a1};
}
FV3_HD inline float ppm_al_field(const AlShared& p, float dm1, float d0, float qm1, float q0, float dcm1, float dc0)
{
    const float c1 = FV3_DIV((q0 - qm1) * dm1, p.d4k);
    return qm1 + c1 + p.s2 * (d0 * (c1 * p.amd + p.a2 * dcm1) - p.dm1a1 * dc0);
}

// ---- remap consumer for NF fields (remap_layer_fast / remap_finish semantics) ----

template <int NF>
struct RemapStateN {
    int k;
    bool accum;
    float dpsum, t, b, xt;
    bool xv;
    float qsum[NF];
};

template <int NF>
struct LayerViewN {
    float pl0, pl1, dp;
    float q1[NF], al[NF], ar[NF], a6[NF];
};

template <int NF>
struct ColumnEndsN {
    float pe_top, pe_bot;
    float q_top[NF], q_bot[NF];
};

template <int NF, class Out>
FV3_HD inline void remap_layer_n(RemapStateN<NF>& s, const LayerViewN<NF>& v, const ColumnEndsN<NF>& e, int kn,
                                 Out& out)
{
    const float r3 = 1.0f / 3.0f, r23 = 2.0f / 3.0f;
    s.xv = false;
    if (s.k > kn) return;
    if (s.accum) {
        if (s.b > v.pl1) {
            // whole layer (mappm.f90:99-104)
            for (int f = 0; f < NF; ++f) s.qsum[f] = s.qsum[f] + v.dp * v.q1[f];
            s.dpsum = s.dpsum + v.dp;
            return;
        }
        // bottom piece (mappm.f90:105-112)
        const float delp = s.b - v.pl0;
        const float esl = FV3_DIVQ(delp, v.dp);
        const float h = 0.5f * esl;
        const float w = 1.0f - r23 * esl;
        for (int f = 0; f < NF; ++f)
            s.qsum[f] = s.qsum[f] + delp * (v.al[f] + h * (v.ar[f] - v.al[f] + v.a6[f] * w));
        s.dpsum = s.dpsum + delp;
        for (int f = 0; f < NF; ++f) out.emit(f, s.k, FV3_DIVQ(s.qsum[f], s.dpsum));
        s.accum = false;
        s.k += 1;
        s.t = s.b;
        s.b = out.next_edge(s.k);
        s.xt = esl;
        s.xv = true;
    }
    while (s.k <= kn) {
        bool above = s.t <= e.pe_top;
        bool bnd = above || s.t >= e.pe_bot;
        bool inl = !bnd && s.t >= v.pl0 && s.t <= v.pl1;
        if (!bnd && !inl) return;
        if (bnd) {
            for (int f = 0; f < NF; ++f) out.emit(f, s.k, above ? e.q_top[f] : e.q_bot[f]);
            s.k += 1;
            s.t = s.b;
            s.b = out.next_edge(s.k);
            s.xv = false;
            continue;
        }
        if (!s.xv) s.xt = FV3_DIVQ(s.t - v.pl0, v.dp);
        if (s.b <= v.pl1) {
            // entire new layer inside input layer L (mappm.f90:76-83)
            const float pl = s.xt;
            const float pr = FV3_DIVQ(s.b - v.pl0, v.dp);
            const float tt = r3 * (pr * (pr + pl) + pl * pl);
            const float x = pr + pl;
            for (int f = 0; f < NF; ++f)
                out.emit(f, s.k, v.al[f] + 0.5f * (v.a6[f] + v.ar[f] - v.al[f]) * x - v.a6[f] * tt);
            s.k += 1;
            s.t = s.b;
            s.b = out.next_edge(s.k);
            s.xt = pr;
            s.xv = true;
            if (s.k > kn) return;
            above = s.t <= e.pe_top;
            bnd = above || s.t >= e.pe_bot;
            inl = !bnd && s.t >= v.pl0 && s.t <= v.pl1;
            if (!inl || s.b <= v.pl1) continue;
        }
        // fractional top piece (mappm.f90:85-92)
        const float pl = s.xt;
        const float tt = r3 * (1.0f + pl * (1.0f + pl));
        const float x = 1.0f + pl;
        const float delp = v.pl1 - s.t;
        for (int f = 0; f < NF; ++f)
            s.qsum[f] = delp * (v.al[f] + 0.5f * (v.a6[f] + v.ar[f] - v.al[f]) * x - v.a6[f] * tt);
        s.dpsum = delp;
        s.accum = true;
        return;
    }
}

template <int NF, class Out>
FV3_HD inline void remap_finish_n(RemapStateN<NF>& s, const ColumnEndsN<NF>& e, int kn, Out& out)
{
    while (s.k <= kn) {
        if (s.accum) {
            const float delp = s.b - e.pe_bot;
            if (delp > 0.0f) {
                for (int f = 0; f < NF; ++f) s.qsum[f] = s.qsum[f] + delp * e.q_bot[f];
                s.dpsum = s.dpsum + delp;
            }
            for (int f = 0; f < NF; ++f) out.emit(f, s.k, FV3_DIVQ(s.qsum[f], s.dpsum));
            s.accum = false;
        } else if (s.t <= e.pe_top) {
            for (int f = 0; f < NF; ++f) out.emit(f, s.k, e.q_top[f]);
        } else if (s.t >= e.pe_bot) {
            for (int f = 0; f < NF; ++f) out.emit(f, s.k, e.q_bot[f]);
        } else {
            for (int f = 0; f < NF; ++f) out.emit(f, s.k, __builtin_nanf(""));  // search failed: reference UB
        }
        s.k += 1;
        s.t = s.b;
        s.b = out.next_edge(s.k);
    }
}

// ---- two lanes per column (small grids): where the second lane starts ----
// A column's outputs split at kB: one lane streams outputs 1 .. kB - 1 from input layer
// 1, the other outputs kB .. kn from the input layer L0 where the single streaming pass
// begins output kB.  With non-decreasing pe1 and pe2 that is the first L with
// pe2(kB) <= pe1(L + 1) (pe1(1) < pe2(kB) < pe1(km + 1); an output's top edge lies in the
// layer where the previous output ended, and no earlier layer reaches it), i.e.
// L0 = 1 + #{L : pe1(L + 1) < pe2(kB)}, found by split_count_sorted in two rounds of
// loads.  Whether pe1 and pe2 are in fact non-decreasing is checked on the values the
// lanes stream anyway (SplitCheck, in mappm_ppm_columns): the first lane's pe1 pairs run
// from the top to its last window, the second lane's from its start window to the bottom
// (a tail it did not stream is read at its exit), and the two ranges must meet; every
// output edge pair is checked by the lane that consumes it.  A column that fails (or
// holds NaNs) is run again by the single pass (the kernel's fix-up).
struct SplitCheck {
    int mono;    // every pe1 / pe2 pair this lane checked is non-decreasing (NaN: 0)
    int l_exit;  // the input layer after which the lane stopped (km: it ran to the end)
};

// #{L in 1..km : pe1(L + 1) < t} for non-decreasing pe1 in two rounds of loads: every 8th
// edge, then the 8 edges of the block where the count stops (any value in 0..km for
// unsorted pe1, which the checks then reject)
template <class Col>
FV3_HD inline int split_count_sorted(Col& c, int km, float t)
{
    int c1 = 0;  // sampled edges j = 2 + 8m below t
    for (int m = 0; 2 + 8 * m <= km + 1; ++m) c1 += c.pe1(2 + 8 * m) < t;
    if (c1 == 0) return 0;
    const int j0 = 2 + 8 * (c1 - 1);
    int n = 0;
    for (int i = 0; i < 8; ++i) n += (j0 + i <= km + 1) && c.pe1(j0 + i <= km + 1 ? j0 + i : km + 1) < t;
    return j0 - 2 + n;
}

// the split's two ranges of checked pe1 pairs meet: the first lane (from layer 1) checked
// the pairs (j, j + 1) for j <= l_exit + 3, the second (its window built at L0, when
// 4 <= L0 <= km - 3; else it walked from layer 1 itself) those from j = L0 - 3
FV3_HD inline bool split_meets(const SplitCheck& a, int L0, int km)
{
    return L0 < 4 || L0 > km - 3 || a.l_exit + 7 >= L0;
}
FV3_HD inline bool split_exact(const SplitCheck& a, const SplitCheck& b, int L0, int km)
{
    return a.mono && b.mono && split_meets(a, L0, km);
}
// three lanes (outputs split at kB1 and kB2; L0b / L0c the second and third lanes'
// start layers): every lane's checks passed and each lane's range meets the next one's
FV3_HD inline bool split3_exact(const SplitCheck& a, const SplitCheck& b, const SplitCheck& c, int L0b, int L0c,
                                int km)
{
    return a.mono && b.mono && c.mono && split_meets(a, L0b, km) && split_meets(b, L0c, km);
}

// SPLIT: the remap consumer's view of the column with every output edge it takes checked
// against the one before (the split's pe2 sortedness, on the edges it streams)
template <class Col>
struct EdgeCheckOut {
    Col& c;
    int kn;
    float last;
    int& mono;
    FV3_HD void emit(int f, int k, float v) { c.emit(f, k, v); }
    FV3_HD float next_edge(int k)
    {
        const float r = c.next_edge(k);
        if (k + 1 <= kn + 1) {
            mono &= last <= r;
            last = r;
        }
        return r;
    }
};

// the second lane's first input layer from the pe1 count (pe2(kB) outside (pe1(1),
// pe1(km + 1)): the boundary outputs, emitted from layer 1 on as the single pass does)
template <class Col>
FV3_HD inline int split_first_layer(Col& c, int km, float t, int cnt)
{
    return (t <= c.pe1(1) || t >= c.pe1(km + 1)) ? 1 : 1 + cnt;
}

// ---- NF columns on one pressure column, kord <= 7, fully streaming ----
// CARRY: as mappm_ppm_column's (level L + 4's loads one iteration ahead, carried across
// the back edge, or at the iteration's start); same loads, same bits.
// SPLIT: this lane emits outputs k_first .. k_last only (a column on two lanes, above),
// and records in *chk whether the pe1 / pe2 pairs it streams are non-decreasing.
// k_first > 1 starts the remap fresh at output k_first: from input layer L_first with
// the window E_{L_first} built directly from its local stencil (every entry the same
// expression on the same operands as the streaming advance computes it) when
// 4 <= L_first <= km - 3, else from layer 1 (the layers above output k_first's top edge
// pass without a remap event).  A lane stops once it has emitted k_last.
template <int NF, class Col, bool CARRY = false, bool SPLIT = false>
FV3_HD inline void mappm_ppm_columns(Col& c, int km, int kn, int iv, int kord, int k_first = 1, int k_last = 0,
                                     int L_first = 1, SplitCheck* chk = nullptr)
{
    int mono = 1;  // SPLIT: the pairs checked so far are non-decreasing
    // window state E_L as in mappm_ppm_column, the q-dependent parts per field
    float qv[NF][4], dcv[NF][3], alv[NF][3], h2v[NF][3], ar_km[NF];
    float dpv[4], pev[5];
    const bool huynh = kord >= 7;
    int L_start = 1;
    if constexpr (SPLIT) {
        if (k_first > 1 && L_first >= 4 && L_first <= km - 3) L_start = L_first;
    }
    const int kn_out = SPLIT ? k_last : kn;  // the last output this lane emits

    ColumnEndsN<NF> ends;
    ends.pe_bot = c.pe1(km + 1);
    for (int f = 0; f < NF; ++f) ends.q_bot[f] = c.q1(f, km);
    if (SPLIT && L_start > 1) {
        ends.pe_top = c.pe1(1);
        for (int f = 0; f < NF; ++f) ends.q_top[f] = c.q1(f, 1);
        // E_{L0} from levels L0 - 3 .. L0 + 4: index i <-> level L0 - 3 + i
        const int l0 = L_start - 3;
        float pw[8], dw[7];
        for (int i = 0; i < 8; ++i) pw[i] = c.pe1(l0 + i);
        for (int i = 0; i < 7; ++i) dw[i] = pw[i + 1] - pw[i];
        for (int i = 0; i < 7; ++i) mono &= pw[i] <= pw[i + 1];
        DcShared pd[6];
        for (int i = 1; i <= 5; ++i) pd[i] = ppm_dc_shared(dw[i - 1], dw[i], dw[i + 1]);  // dc(L0-2 .. L0+2)
        AlShared pa[6];
        for (int i = 3; i <= 5; ++i) pa[i] = ppm_al_shared(dw[i - 2], dw[i - 1], dw[i], dw[i + 1]);  // AL(L0 .. L0+2)
        for (int f = 0; f < NF; ++f) {
            float qw[7], dcw[6];
            for (int i = 0; i < 7; ++i) qw[i] = c.q1(f, l0 + i);
            for (int i = 1; i <= 5; ++i) dcw[i] = ppm_dc_field(pd[i], qw[i - 1], qw[i], qw[i + 1], dw[i]);
            for (int i = 0; i < 4; ++i) qv[f][i] = qw[3 + i];
            for (int i = 0; i < 3; ++i) {
                dcv[f][i] = dcw[3 + i];
                alv[f][i] = ppm_al_field(pa[3 + i], dw[2 + i], dw[3 + i], qw[2 + i], qw[3 + i], dcw[2 + i], dcw[3 + i]);
                // h2(k), k = L0 - 1 + i: the streaming advance's expression (k >= 3 here)
                const int j = 2 + i;
                const int k = L_start - 1 + i;
                if (huynh && k <= km - 1) {
                    const float hden = dw[j] + 0.5f * (dw[j - 1] + dw[j + 1]);
                    const float d0sq = dw[j] * dw[j];
                    h2v[f][i] = FV3_DIV(2.0f * (FV3_DIV(dcw[j + 1], dw[j + 1]) - FV3_DIV(dcw[j - 1], dw[j - 1])), hden) * d0sq;
                } else {
                    h2v[f][i] = 0.0f;
                }
            }
            ar_km[f] = 0.0f;
        }
        for (int i = 0; i < 5; ++i) pev[i] = pw[3 + i];
        for (int i = 0; i < 4; ++i) dpv[i] = dw[3 + i];
    } else {
    for (int f = 0; f < NF; ++f)
        for (int i = 0; i < 4; ++i) qv[f][i] = c.q1(f, 1 + i);
    for (int i = 0; i < 5; ++i) pev[i] = c.pe1(1 + i);
    for (int i = 0; i < 4; ++i) dpv[i] = pev[i + 1] - pev[i];
    if constexpr (SPLIT)
        for (int i = 0; i < 4; ++i) mono &= pev[i] <= pev[i + 1];

    ends.pe_top = pev[0];
    for (int f = 0; f < NF; ++f) ends.q_top[f] = qv[f][0];

    {
        const DcShared p2 = ppm_dc_shared(dpv[0], dpv[1], dpv[2]);
        const DcShared p3 = ppm_dc_shared(dpv[1], dpv[2], dpv[3]);
        const AlShared a3 = ppm_al_shared(dpv[0], dpv[1], dpv[2], dpv[3]);
        const float hden = dpv[1] + 0.5f * (dpv[0] + dpv[2]);
        const float d0sq = dpv[1] * dpv[1];
        for (int f = 0; f < NF; ++f) {
            const float dc2 = ppm_dc_field(p2, qv[f][0], qv[f][1], qv[f][2], dpv[1]);
            const float dc3 = ppm_dc_field(p3, qv[f][1], qv[f][2], qv[f][3], dpv[2]);  // 3 <= km-1
            const float al3 = ppm_al_field(a3, dpv[1], dpv[2], qv[f][1], qv[f][2], dc2, dc3);
            float al1, al2, dc1;
            ppm_top_cubic(qv[f][0], qv[f][1], dpv[0], dpv[1], al3, iv, al1, al2, dc1);
            dcv[f][0] = dc1; dcv[f][1] = dc2; dcv[f][2] = dc3;
            alv[f][0] = al1; alv[f][1] = al2; alv[f][2] = al3;
            h2v[f][0] = 0.0f; h2v[f][1] = 0.0f;
            // h2(2) = ppm_h2(dc1, dc3, dp(1), dp(2), dp(3))
            h2v[f][2] = huynh ? FV3_DIV(2.0f * (FV3_DIV(dc3, dpv[2]) - FV3_DIV(dc1, dpv[0])), hden) * d0sq : 0.0f;
            ar_km[f] = 0.0f;
        }
    }
    }

    int lmt = kord - 3;
    lmt = lmt > 0 ? lmt : 0;
    if (iv == 0) lmt = lmt < 2 ? lmt : 2;

    RemapStateN<NF> s;
    s.k = SPLIT ? k_first : 1;
    s.accum = false;
    s.dpsum = 0.0f;
    s.t = c.pe2(s.k);
    s.b = c.pe2(s.k + 1);
    if constexpr (SPLIT) mono &= s.t <= s.b;
    EdgeCheckOut<Col> eo{c, kn, s.b, mono};
    s.xt = 0.0f;
    s.xv = false;
    for (int f = 0; f < NF; ++f) s.qsum[f] = 0.0f;

    float qc_pf[NF], pec_pf = 0.0f;
    for (int f = 0; f < NF; ++f) qc_pf[f] = 0.0f;
    if constexpr (CARRY) {
        if (L_start + 4 <= km) {
            for (int f = 0; f < NF; ++f) qc_pf[f] = c.q1(f, L_start + 4);
            pec_pf = c.pe1(L_start + 5);
        }
    }
    for (int L = L_start; L <= km; ++L) {
        // level L + 4's q1 / pe1: carried from the previous iteration (CARRY) or read at
        // this iteration's start, as in mappm_ppm_column
        float q_pf[NF], pe_pf = pec_pf;
        for (int f = 0; f < NF; ++f) q_pf[f] = qc_pf[f];
        if constexpr (!CARRY) {
            if (L + 4 <= km) {
                for (int f = 0; f < NF; ++f) q_pf[f] = c.q1(f, L + 4);
                pe_pf = c.pe1(L + 5);
            }
        }
        // ---- the final coefficients of layer L, per field ----
        LayerViewN<NF> v;
        v.pl0 = pev[0];
        v.pl1 = pev[1];
        v.dp = dpv[0];
        for (int f = 0; f < NF; ++f) {
            Ppm a{qv[f][0], alv[f][0], (L < km) ? alv[f][1] : ar_km[f], 0.0f};
            const float dcL = dcv[f][0];
            if (L <= 2 || L >= km - 1) {
                a.a6 = a6_of(a);
                ppm_limit(dcL, a, 0);
            } else if (huynh) {
                ppm_huynh(a, dcL, h2v[f][0], h2v[f][2]);
                if (iv == 0) ppm_limit(dcL, a, 2);
            } else {
                if (kord != 4) a.a6 = a6_of(a);
                if (kord != 6) ppm_limit(dcL, a, lmt);
            }
            v.q1[f] = qv[f][0];
            v.al[f] = a.al;
            v.ar[f] = a.ar;
            v.a6[f] = a.a6;
        }
        if constexpr (SPLIT)
            remap_layer_n<NF>(s, v, ends, kn_out, eo);
        else
            remap_layer_n<NF>(s, v, ends, kn_out, c);
        layer_hook(c, 0);

        if (L == km) break;
        if constexpr (SPLIT) {
            if (s.k > kn_out) {  // this lane's outputs are done
                if (k_last == kn) {  // the column's last lane: the pe1 pairs below its window
                    float prev = pev[4];
                    for (int jj = L + 5; jj <= km + 1; ++jj) {
                        const float x = c.pe1(jj);
                        mono &= prev <= x;
                        prev = x;
                    }
                }
                chk->mono = mono;
                chk->l_exit = L;
                return;
            }
        }
        // ---- advance the window E_L -> E_{L+1} ----
        const int j = L + 4;
        float qn[NF], pen = 0.0f, dpn = 0.0f;
        for (int f = 0; f < NF; ++f) qn[f] = 0.0f;
        if (j <= km) {
            for (int f = 0; f < NF; ++f) qn[f] = q_pf[f];
            pen = pe_pf;
            dpn = pen - pev[4];
            if constexpr (SPLIT) mono &= pev[4] <= pen;
        }
        if constexpr (CARRY) {
            if (j + 1 <= km) {  // level j + 1, for the next iteration
                for (int f = 0; f < NF; ++f) qc_pf[f] = c.q1(f, j + 1);
                pec_pf = c.pe1(j + 2);
            }
        }
        const int m = L + 3;
        float dcm[NF], alm[NF];
        for (int f = 0; f < NF; ++f) {
            dcm[f] = 0.0f;
            alm[f] = 0.0f;
        }
        if (m <= km - 1) {
            const DcShared pd = ppm_dc_shared(dpv[2], dpv[3], dpn);
            const AlShared pa = ppm_al_shared(dpv[1], dpv[2], dpv[3], dpn);
            for (int f = 0; f < NF; ++f) {
                dcm[f] = ppm_dc_field(pd, qv[f][2], qv[f][3], qn[f], dpv[3]);
                alm[f] = ppm_al_field(pa, dpv[2], dpv[3], qv[f][2], qv[f][3], dcv[f][2], dcm[f]);
            }
        } else if (m == km) {
            for (int f = 0; f < NF; ++f) {
                float ar;
                ppm_bottom_cubic(qv[f][3], qv[f][2], dpv[3], dpv[2], alv[f][2], iv, alm[f], ar, dcm[f]);
                ar_km[f] = ar;
            }
        }
        if (huynh && L + 2 <= km - 1) {  // h2(L+2) = ppm_h2(dc(L+1), dc(L+3), dp(L+1..L+3))
            const float hden = dpv[2] + 0.5f * (dpv[1] + dpv[3]);
            const float d0sq = dpv[2] * dpv[2];
            for (int f = 0; f < NF; ++f) {
                const float h2n = FV3_DIV(2.0f * (FV3_DIV(dcm[f], dpv[3]) - FV3_DIV(dcv[f][1], dpv[1])), hden) * d0sq;
                h2v[f][0] = h2v[f][1]; h2v[f][1] = h2v[f][2]; h2v[f][2] = h2n;
            }
        } else {
            for (int f = 0; f < NF; ++f) {
                h2v[f][0] = h2v[f][1]; h2v[f][1] = h2v[f][2]; h2v[f][2] = 0.0f;
            }
        }
        for (int f = 0; f < NF; ++f) {
            qv[f][0] = qv[f][1]; qv[f][1] = qv[f][2]; qv[f][2] = qv[f][3]; qv[f][3] = qn[f];
            dcv[f][0] = dcv[f][1]; dcv[f][1] = dcv[f][2]; dcv[f][2] = dcm[f];
            alv[f][0] = alv[f][1]; alv[f][1] = alv[f][2]; alv[f][2] = alm[f];
        }
        dpv[0] = dpv[1]; dpv[1] = dpv[2]; dpv[2] = dpv[3]; dpv[3] = dpn;
        pev[0] = pev[1]; pev[1] = pev[2]; pev[2] = pev[3]; pev[3] = pev[4]; pev[4] = pen;
    }
    if constexpr (SPLIT) {
        remap_finish_n<NF>(s, ends, kn_out, eo);
        chk->mono = mono;
        chk->l_exit = km;
    } else {
        remap_finish_n<NF>(s, ends, kn_out, c);
    }
}

// A one-field view of an NF-interface column, so NF = 1 runs the single-field
// streaming code (mappm_ppm_column) on it.
template <class Col>
struct FirstField {
    Col& c;
    FV3_HD float q1(int k) { return c.q1(0, k); }
    FV3_HD float pe1(int k) { return c.pe1(k); }
    FV3_HD float pe2(int k) { return c.pe2(k); }
    FV3_HD void emit(int k, float v) { c.emit(0, k, v); }
    FV3_HD float next_edge(int k) { return c.next_edge(k); }
    FV3_HD void layer_done() { layer_hook(c, 0); }
};

#ifdef FV3_FAST_ARITH
#pragma clang fp contract(off)
#endif
}  // namespace FV3_ARITH_NS
}  // namespace fv3
