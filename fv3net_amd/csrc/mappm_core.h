// fv3net_amd — streaming, one-pass formulation of FV3's vertical remap `mappm`.
//
// Reference semantics: /root/reference/external/mappm/mappm/mappm.f90
//   mappm :10-126, cs_profile :132-532, cs_limiters :535-611,
//   ppm_profile :614-851, ppm_limiters :854-931.
//
// The reference builds whole-column arrays (a4(4,km), dc, h2, delq, df2, d4)
// and then walks output layers.  That needs ~2 KB of scratch per column, which
// on gfx950 would either sink occupancy (LDS) or double HBM traffic (scratch).
// Here one thread owns one column and walks the INPUT layers L = 1..km exactly
// once ("lockstep over L"): a rolling register window produces the final PPM
// coefficients of layer L (every value computed by the reference's own
// expression tree, so results are bit-identical), and a small per-thread state
// machine consumes the output layers whose edges fall in layer L.  Because the
// reference's layer search only ever moves forward (k0 is carried,
// mappm.f90:59,70-74,111), every output layer is finished from layers >= the
// current one, so one forward sweep reproduces it.
//
// Arithmetic rules for bit parity with the x86 reference build:
//   * compile with -ffp-contract=off (no FMA contraction), IEEE f32 division;
//   * Fortran MAX/MIN as AMD flang emits them: a>b?a:b / a<b?a:b, left fold;
//   * SIGN(a,b) = copysign(|a|, b).
// Excluded from parity (reference UB): non-monotone pe1 where
// the layer search fails (NaN here), qs for iv=-2 with kord>7 (0 here), and a
// non-monotone pe2 that leaves the column below the old surface and re-enters.
#pragma once
#include <type_traits>

#ifndef FV3_HD
#define FV3_HD
#endif

#if !defined(__HIPCC__)
#include <cmath>
#include <cstdint>
#endif

// ---- arithmetic policy (one per translation unit) ----
// Default (namespace fv3::exact): the reference build's arithmetic, bit for bit (the rules
// above).  With FV3_FAST_ARITH defined before the include (namespace fv3::fast, compiled
// in csrc/*_fast.hip): north_star's floating-point tolerance contract (1e-5 rel; the
// reference's own test accepts cross-platform differences in mappm,
// external/vcm/tests/test_coarsen_restarts.py:115-122) instead of bit parity:
//   * every division a / b as a * rcp(b) (v_rcp_f32, 1 ulp: 2 instructions for the 11 of
//     a correctly rounded division), identical denominators sharing one reciprocal;
//   * a * b + c contracted to one FMA within an expression (fp contract(on));
//   * MAX / MIN as the hardware's v_max_f32 / v_min_f32 (v_max3 / v_min3 for three
//     operands).  These equal the reference's a > b ? a : b for finite operands; a NaN
//     operand is dropped instead of propagated by position, so non-finite inputs need the
//     exact path.
// Same algorithm, same order of operations, same limiter branches (a comparison near its
// switching point may take the other branch; the PPM limiters are continuous there).
#ifdef FV3_FAST_ARITH
#define FV3_ARITH_NS fast
#if defined(__HIP_DEVICE_COMPILE__)
#define FV3_RCP(b) __builtin_amdgcn_rcpf(b)
#else
#define FV3_RCP(b) (1.0f / (b))
#endif
namespace fv3 {
// a / b from the 1-ulp reciprocal plus one Newton step on the quotient (4 instructions):
// within ~1 ulp of the correctly rounded quotient.  The profile's divisions (dc, the
// edge estimates, h2, the end cubics) feed differences that cancel on irregular
// thicknesses; with the bare a * rcp(b) a rough 79-level column (delp over 3 decades)
// reached 1.35e-5 per level, with this step 2.8e-6 (tools/remap_fast_random.py).
FV3_HD inline float div_refined(float a, float b)
{
    const float r = FV3_RCP(b);
    const float q = a * r;
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
#else
    return a / b;
#endif
}
}  // namespace fv3
#define FV3_DIV(a, b) (::fv3::div_refined((a), (b)))
// the remap consumer's quotients: a position inside a layer ((t - pe1) / dp, in [0, 1])
// and the final mean qsum / dpsum, where a 1-ulp quotient stays a 1-ulp result
#define FV3_DIVQ(a, b) ((a) * FV3_RCP(b))
#define FV3_DIVX(a, b) ((a) / (b))  // the reference's division in either policy
#else
#define FV3_ARITH_NS exact
#define FV3_DIV(a, b) ((a) / (b))
#define FV3_DIVQ(a, b) ((a) / (b))
#define FV3_DIVX(a, b) ((a) / (b))
#endif

namespace fv3 {
namespace FV3_ARITH_NS {
#ifdef FV3_FAST_ARITH
#pragma clang fp contract(on)
FV3_HD inline float fmax2(float a, float b) { return __builtin_fmaxf(a, b); }
FV3_HD inline float fmin2(float a, float b) { return __builtin_fminf(a, b); }
#else
FV3_HD inline float fmax2(float a, float b) { return a > b ? a : b; }
FV3_HD inline float fmin2(float a, float b) { return a < b ? a : b; }
#endif
FV3_HD inline int imin2(int a, int b) { return a < b ? a : b; }
FV3_HD inline int imax2(int a, int b) { return a > b ? a : b; }
FV3_HD inline float fmax3(float a, float b, float c) { return fmax2(fmax2(a, b), c); }
FV3_HD inline float fmin3(float a, float b, float c) { return fmin2(fmin2(a, b), c); }
FV3_HD inline float fsign(float a, float b) { return copysignf(fabsf(a), b); }

// PPM coefficients of one layer: a1 = mean, al/ar = edges, a6 = curvature.
struct Ppm {
    float a1, al, ar, a6;
};

// ppm_limiters (mappm.f90:854-931) applied to one layer.
FV3_HD inline void ppm_limit(float dm, Ppm& a, int lmt)
{
    const float r12 = 1.0f / 12.0f;
    if (lmt == 3) return;
    if (lmt == 0) {
        if (dm == 0.0f) {
            a.al = a.a1; a.ar = a.a1; a.a6 = 0.0f;
        } else {
            const float da1 = a.ar - a.al;
            const float da2 = da1 * da1;
            const float a6da = a.a6 * da1;
            if (a6da < -da2) {
                a.a6 = 3.0f * (a.al - a.a1);
                a.ar = a.al - a.a6;
            } else if (a6da > da2) {
                a.a6 = 3.0f * (a.ar - a.a1);
                a.al = a.ar - a.a6;
            }
        }
    } else if (lmt == 1) {
        const float qmp = 2.0f * dm;
        a.al = a.a1 - fsign(fmin2(fabsf(qmp), fabsf(a.al - a.a1)), qmp);
        a.ar = a.a1 + fsign(fmin2(fabsf(qmp), fabsf(a.ar - a.a1)), qmp);
        a.a6 = 3.0f * (2.0f * a.a1 - (a.al + a.ar));
    } else if (lmt == 2) {
        if (fabsf(a.ar - a.al) < -a.a6) {
            const float d = a.ar - a.al;
            const float fmin = a.a1 + FV3_DIV(0.25f * (d * d), a.a6) + a.a6 * r12;
            if (fmin < 0.0f) {
                if (a.a1 < a.ar && a.a1 < a.al) {
                    a.ar = a.a1; a.al = a.a1; a.a6 = 0.0f;
                } else if (a.ar > a.al) {
                    a.a6 = 3.0f * (a.al - a.a1);
                    a.ar = a.al - a.a6;
                } else {
                    a.a6 = 3.0f * (a.ar - a.a1);
                    a.al = a.ar - a.a6;
                }
            }
        }
    }
}

// cs_limiters (mappm.f90:535-611) applied to one layer.
FV3_HD inline void cs_limit(bool extm, Ppm& a, int iv)
{
    const float r12 = 1.0f / 12.0f;
    if (iv == 0) {
        if (a.a1 <= 0.0f) {
            a.al = a.a1; a.ar = a.a1; a.a6 = 0.0f;
        } else if (fabsf(a.ar - a.al) < -a.a6) {
            const float d = a.ar - a.al;
            if ((a.a1 + FV3_DIV(0.25f * (d * d), a.a6) + a.a6 * r12) < 0.0f) {
                if (a.a1 < a.ar && a.a1 < a.al) {
                    a.ar = a.a1; a.al = a.a1; a.a6 = 0.0f;
                } else if (a.ar > a.al) {
                    a.a6 = 3.0f * (a.al - a.a1);
                    a.ar = a.al - a.a6;
                } else {
                    a.a6 = 3.0f * (a.ar - a.a1);
                    a.al = a.ar - a.a6;
                }
            }
        }
        return;
    }
    bool flat = (iv == 1) ? ((a.a1 - a.al) * (a.a1 - a.ar) >= 0.0f) : extm;
    if (flat) {
        a.al = a.a1; a.ar = a.a1; a.a6 = 0.0f;
    } else {
        const float da1 = a.ar - a.al;
        const float da2 = da1 * da1;
        const float a6da = a.a6 * da1;
        if (a6da < -da2) {
            a.a6 = 3.0f * (a.al - a.a1);
            a.ar = a.al - a.a6;
        } else if (a6da > da2) {
            a.a6 = 3.0f * (a.ar - a.a1);
            a.al = a.ar - a.a6;
        }
    }
}

FV3_HD inline float a6_of(const Ppm& a) { return 3.0f * (2.0f * a.a1 - (a.al + a.ar)); }

// ---- ppm_profile pieces (mappm.f90:651-747), each the reference's expression ----

// dc(k), interior k = 2..km-1 (mappm.f90:658-668); qm1,q0,qp1 = q(k-1..k+1),
// dm1,d0,dp1 = delp(k-1..k+1).
FV3_HD inline float ppm_dc(float qm1, float q0, float qp1, float dm1, float d0, float dp1)
{
    const float d4k = dm1 + d0;    // d4(k)
    const float d4kp = d0 + dp1;   // d4(k+1)
    const float c1 = FV3_DIV(dm1 + 0.5f * d0, d4kp);
    const float c2 = FV3_DIV(dp1 + 0.5f * d0, d4k);
    const float delq_k = qp1 - q0;   // delq(k)
    const float delq_km = q0 - qm1;  // delq(k-1)
    const float df2 = FV3_DIV(d0 * (c1 * delq_k + c2 * delq_km), d4k + dp1);
    return fsign(fmin3(fabsf(df2), fmax3(qm1, q0, qp1) - q0, q0 - fmin3(qm1, q0, qp1)), df2);
}

// provisional left edge a4(2,k), interior k = 3..km-1 (mappm.f90:674-683);
// d(-2..1) = delp(k-2..k+1), qm1,q0 = q(k-1), q(k); dcm1,dc0 = dc(k-1), dc(k).
FV3_HD inline float ppm_al(float dm2, float dm1, float d0, float dp1, float qm1, float q0,
                           float dcm1, float dc0)
{
    const float d4km = dm2 + dm1;  // d4(k-1)
    const float d4k = dm1 + d0;    // d4(k)
    const float d4kp = d0 + dp1;   // d4(k+1)
    const float c1 = FV3_DIV((q0 - qm1) * dm1, d4k);
    const float a1 = FV3_DIV(d4km, d4k + dm1);
    const float a2 = FV3_DIV(d4kp, d4k + d0);
    return qm1 + c1 + FV3_DIV(2.0f, d4km + d4kp) * (d0 * (c1 * (a1 - a2) + a2 * dcm1) - dm1 * a1 * dc0);
}

// h2(k) (mappm.f90:784-795), k = 2..km-1.
FV3_HD inline float ppm_h2(float dcm1, float dcp1, float dm1, float d0, float dp1)
{
    return FV3_DIV(2.0f * (FV3_DIV(dcp1, dp1) - FV3_DIV(dcm1, dm1)), d0 + 0.5f * (dm1 + dp1)) * (d0 * d0);
}

// Huynh's 2nd constraint for an interior PPM layer (mappm.f90:799-821).
FV3_HD inline void ppm_huynh(Ppm& a, float dc, float h2m, float h2p)
{
    const float fac = 1.5f;
    const float pmp = 2.0f * dc;
    float qmp = a.a1 + pmp;
    float lac = a.a1 + fac * h2m + dc;
    a.ar = fmin2(fmax2(a.ar, fmin3(a.a1, qmp, lac)), fmax3(a.a1, qmp, lac));
    qmp = a.a1 - pmp;
    lac = a.a1 + fac * h2p - dc;
    a.al = fmin2(fmax2(a.al, fmin3(a.a1, qmp, lac)), fmax3(a.a1, qmp, lac));
    a.a6 = a6_of(a);
}

// ---- the area-preserving end cubics, one field (mappm.f90:689-725, 729-761) ----
// Always the reference's arithmetic (IEEE division, no contraction), in both policies:
// they run once per column, and their clamps (al2 onto [min, max](q1, q2), and likewise
// at the bottom) decide whether dc of an end layer is exactly 0, which flattens that
// layer (ppm_limiters lmt 0, `dm == 0`).  Computed in the fast arithmetic, an edge value
// within an ulp of its clamp bound could land on the other side and flip the layer.

FV3_HD inline void ppm_top_cubic(float q1, float q2, float d1, float d2, float al3, int iv, float& al1,
                                 float& al2, float& dc1)
{
#pragma clang fp contract(off)
    const float qm = FV3_DIVX(d2 * q1 + d1 * q2, d1 + d2);
    const float dq = FV3_DIVX(2.0f * (q2 - q1), d1 + d2);
    const float c1 = FV3_DIVX(4.0f * (al3 - qm - d2 * dq), d2 * (2.0f * d2 * d2 + d1 * (d2 + 3.0f * d1)));
    const float c3 = dq - 0.5f * c1 * (d2 * (5.0f * d1 + d2) - 3.0f * d1 * d1);
    al2 = qm - 0.25f * c1 * d1 * d2 * (d2 + 3.0f * d1);
    al1 = d1 * (2.0f * c1 * (d1 * d1) - c3) + al2;
    al2 = fmax2(al2, fmin2(q1, q2));
    al2 = fmin2(al2, fmax2(q1, q2));
    dc1 = 0.5f * (al2 - q1);
    if (iv == 0) {
        al1 = fmax2(0.0f, al1);
        al2 = fmax2(0.0f, al2);
    } else if (iv == -1) {
        if (al1 * q1 <= 0.0f) al1 = 0.0f;
    } else if (iv == 2 || iv == -2) {
        al1 = q1;
    }
}

// d1 = dp(km), d2 = dp(km-1), qk = q(km), qk1 = q(km-1), alk1 = ALraw(km-1)
FV3_HD inline void ppm_bottom_cubic(float qk, float qk1, float d1, float d2, float alk1, int iv, float& alm,
                                    float& ar, float& dcm)
{
#pragma clang fp contract(off)
    const float qm = FV3_DIVX(d2 * qk + d1 * qk1, d1 + d2);
    const float dq = FV3_DIVX(2.0f * (qk1 - qk), d1 + d2);
    const float c1 = FV3_DIVX(alk1 - qm - d2 * dq, d2 * (2.0f * d2 * d2 + d1 * (d2 + 3.0f * d1)));
    const float c3 = dq - 2.0f * c1 * (d2 * (5.0f * d1 + d2) - 3.0f * d1 * d1);
    alm = qm - c1 * d1 * d2 * (d2 + 3.0f * d1);
    ar = d1 * (8.0f * c1 * (d1 * d1) - c3) + alm;
    alm = fmax2(alm, fmin2(qk, qk1));
    alm = fmin2(alm, fmax2(qk, qk1));
    dcm = 0.5f * (qk - alm);
    if (iv == 0) {
        alm = fmax2(0.0f, alm);
        ar = fmax2(0.0f, ar);
    } else if (iv < 0) {
        if (qk * ar <= 0.0f) ar = 0.0f;
    }
}

// ---- remap consumer: the output-layer loop of mappm.f90:58-124, lockstep over L ----

struct RemapState {
    int k;          // current output layer (1-based)
    bool accum;     // true: accumulating whole layers below the top edge (label 111 loop)
    float qsum, dpsum;
    float t, b;     // pe2(k), pe2(k+1)
    float xt = 0.0f;  // remap_layer_fast: (t - pe1(L)) / dp1(L) of the current layer L, valid if xv
    bool xv = false;
};

// The column's input layer L as the consumer sees it.
struct LayerView {
    float pl0, pl1, dp, q1;  // pe1(L), pe1(L+1), dp1(L), q1(L)
    Ppm a;
};

// Column-wide constants for the boundary branches (mappm.f90:62-67).
struct ColumnEnds {
    float pe_top, pe_bot, q_top, q_bot;  // pe1(1), pe1(km+1), q1(1), q1(km)
};

// Consume every output-layer event inside layer L.  `Out` provides
// emit(k, value) and next_edge() -> pe2(k+2) for the layer after the current.
template <class Out>
FV3_HD inline void remap_layer(RemapState& s, const LayerView& v, const ColumnEnds& e, int kn, Out& out)
{
    const float r3 = 1.0f / 3.0f, r23 = 2.0f / 3.0f;
    while (s.k <= kn) {
        if (!s.accum) {
            if (s.t <= e.pe_top) {
                out.emit(s.k, e.q_top);
            } else if (s.t >= e.pe_bot) {
                out.emit(s.k, e.q_bot);
            } else if (s.t >= v.pl0 && s.t <= v.pl1) {
                const float pl = FV3_DIVQ(s.t - v.pl0, v.dp);
                if (s.b <= v.pl1) {
                    // entire new layer inside input layer L (mappm.f90:76-83)
                    const float pr = FV3_DIVQ(s.b - v.pl0, v.dp);
                    const float tt = r3 * (pr * (pr + pl) + pl * pl);
                    out.emit(s.k, v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (pr + pl) - v.a.a6 * tt);
                } else {
                    // fractional top piece (mappm.f90:85-92); continue in layers below
                    const float delp = v.pl1 - s.t;
                    const float tt = r3 * (1.0f + pl * (1.0f + pl));
                    s.qsum = delp * (v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (1.0f + pl) - v.a.a6 * tt);
                    s.dpsum = delp;
                    s.accum = true;
                    return;
                }
            } else {
                return;  // top edge lies further down: search continues at L+1
            }
        } else {
            if (s.b > v.pl1) {
                // whole layer (mappm.f90:99-104)
                s.qsum = s.qsum + v.dp * v.q1;
                s.dpsum = s.dpsum + v.dp;
                return;
            }
            // bottom piece (mappm.f90:105-112)
            const float delp = s.b - v.pl0;
            const float esl = FV3_DIVQ(delp, v.dp);
            s.qsum = s.qsum + delp * (v.a.al + 0.5f * esl * (v.a.ar - v.a.al + v.a.a6 * (1.0f - r23 * esl)));
            s.dpsum = s.dpsum + delp;
            out.emit(s.k, FV3_DIVQ(s.qsum, s.dpsum));
            s.accum = false;
        }
        // advance to the next output layer; its search restarts at this L (k0 = L)
        s.k += 1;
        s.t = s.b;
        s.b = out.next_edge(s.k);
    }
}

// remap_layer with the same events, values and bits, arranged for a wave of columns
// whose lanes sit at different points of the event sequence (mappm.f90:58-124):
//  * an accumulating output meets at most one event per layer and only as the layer's
//    first (whole layer, or the bottom piece that ends it), so it runs once up front;
//  * every edge's normalised position (pe2(e) - pe1(L)) / dp1(L) is the same
//    expression whether the edge is the bottom of one output (ESL, PR) or the top of
//    the next (PL), so it is divided once and carried in xt;
//  * an inside-layer output (mappm.f90:76-83) is followed, in the same pass, by the
//    next output's fractional top piece (mappm.f90:85-92) when that is the next event,
//    so a wave needs one pass per layer unless a lane has several inside outputs.
// Holds for every input (no ordering assumption): each value is computed by the
// reference's expression on the same operands.
template <class Out>
FV3_HD inline void remap_layer_fast(RemapState& s, const LayerView& v, const ColumnEnds& e, int kn, Out& out)
{
    const float r3 = 1.0f / 3.0f, r23 = 2.0f / 3.0f;
    s.xv = false;
    if (s.k > kn) return;
    if (s.accum) {
        if (s.b > v.pl1) {
            // whole layer (mappm.f90:99-104)
            s.qsum = s.qsum + v.dp * v.q1;
            s.dpsum = s.dpsum + v.dp;
            return;
        }
        // bottom piece (mappm.f90:105-112)
        const float delp = s.b - v.pl0;
        const float esl = FV3_DIVQ(delp, v.dp);
        s.qsum = s.qsum + delp * (v.a.al + 0.5f * esl * (v.a.ar - v.a.al + v.a.a6 * (1.0f - r23 * esl)));
        s.dpsum = s.dpsum + delp;
        out.emit(s.k, FV3_DIVQ(s.qsum, s.dpsum));
        s.accum = false;
        s.k += 1;
        s.t = s.b;
        s.b = out.next_edge(s.k);
        s.xt = esl;  // = (t - pe1(L)) / dp1(L) for the new top edge
        s.xv = true;
    }
    while (s.k <= kn) {
        bool above = s.t <= e.pe_top;
        bool bnd = above || s.t >= e.pe_bot;
        bool inl = !bnd && s.t >= v.pl0 && s.t <= v.pl1;
        if (!bnd && !inl) return;  // top edge further down: next layer
        if (bnd) {
            out.emit(s.k, above ? e.q_top : e.q_bot);
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
            out.emit(s.k, v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (pr + pl) - v.a.a6 * tt);
            s.k += 1;
            s.t = s.b;
            s.b = out.next_edge(s.k);
            s.xt = pr;
            s.xv = true;
            if (s.k > kn) return;
            // the usual next event is this output's top piece in the same layer: run it
            // here rather than in another pass of the loop
            above = s.t <= e.pe_top;
            bnd = above || s.t >= e.pe_bot;
            inl = !bnd && s.t >= v.pl0 && s.t <= v.pl1;
            if (!inl || s.b <= v.pl1) continue;  // anything else: the loop head
        }
        // fractional top piece (mappm.f90:85-92); continue in the layers below
        const float pl = s.xt;
        const float tt = r3 * (1.0f + pl * (1.0f + pl));
        const float delp = v.pl1 - s.t;
        s.qsum = delp * (v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (1.0f + pl) - v.a.a6 * tt);
        s.dpsum = delp;
        s.accum = true;
        return;
    }
}

// After the last input layer: extension below the old surface and the
// boundary branches for what is left (mappm.f90:115-121, 62-67).
template <class Out>
FV3_HD inline void remap_finish(RemapState& s, const ColumnEnds& e, int kn, Out& out)
{
    while (s.k <= kn) {
        if (s.accum) {
            const float delp = s.b - e.pe_bot;
            if (delp > 0.0f) {
                s.qsum = s.qsum + delp * e.q_bot;
                s.dpsum = s.dpsum + delp;
            }
            out.emit(s.k, FV3_DIVQ(s.qsum, s.dpsum));
            s.accum = false;
        } else if (s.t <= e.pe_top) {
            out.emit(s.k, e.q_top);
        } else if (s.t >= e.pe_bot) {
            out.emit(s.k, e.q_bot);
        } else {
            out.emit(s.k, __builtin_nanf(""));  // search failed: reference UB
        }
        s.k += 1;
        s.t = s.b;
        s.b = out.next_edge(s.k);
    }
}

// Optional per-layer hook: a `Col` with layer_done() has it called after every input
// layer's outputs (lockstep over L, so a wave can act on its lanes' emits together).
template <class C>
FV3_HD inline auto layer_hook(C& c, int) -> decltype(c.layer_done(), void())
{
    c.layer_done();
}
template <class C>
FV3_HD inline void layer_hook(C&, long) {}

// ---- one column, kord <= 7 (ppm_profile path), fully streaming ----
//
// `Col` provides (1-based levels):
//   float q1(int k)   k = 1..km          float pe1(int k)  k = 1..km+1
//   float pe2(int k)  k = 1..kn+1        void emit(int k, float v)
//   float next_edge(int k) -> pe2(k+1) or 0 when k+1 > kn+1
// FAST selects remap_layer_fast (default) or the reference-shaped remap_layer (host A/B).
// CARRY: level L + 4's loads issued one iteration ahead and carried across the loop's
// back edge (the mappm kernel: measured faster there, 0.527 vs 0.535 ms at C384 kord 1)
// or at the iteration's start (the coarsen kernels: 1 field 0.767 -> 0.753 ms,
// profiles/r04o_remap_ab.log).  Same loads, same bits.
// RING: the window E_L in rings of 5 registers -- element i of the window at layer L in
// slot (L - 1 + i) % 5, so advancing it writes the one new element and moves nothing --
// with the layer loop run in groups of 5 (one per ring phase, every slot index a
// compile-time constant).  Shifting the arrays (RING = false) costs ~14 v_mov_b32 per
// layer.  Same operations on the same values: the same bits.  Measured (one box,
// interleaved): the fast single-field mappm kernel 0.384 -> 0.367 ms at C384 kord 1
// (profiles/r06zk_ring_ab.log); with it the exact kernel went 0.499 -> 0.533 and the
// one-field coarsen 0.577 -> 0.662 ms (five copies of their larger layer bodies; the
// coarsen's rings spill at its 6 waves per SIMD and lose at 5 too, coarsen.hip
// FV3_COARSEN_RING, profiles/r06zi_ring_ab.log, r06zo_coarsen_ring_ab.log), so only the
// former takes it.  The same rings in the
// multi-field column (mappm_multi.h) measured no faster on the C384 pair kernel and 9 %
// slower on one rank's split-lane kernels (profiles/r06zl_ring_ab.log): not kept.
template <class Col, bool FAST = true, bool CARRY = false, bool RING = false>
FV3_HD inline void mappm_ppm_column(Col& c, int km, int kn, int iv, int kord)
{
    // window state E_L: q(L..L+3), dp(L..L+3), pe1(L..L+4), dc(L..L+2), ALraw(L..L+2),
    // h2(L-1..L+1) (RING: in their ring slots; else element i at index i)
    constexpr int R = 5;
    constexpr int RQ = RING ? R : 4, RD = RING ? R : 3;  // the shifting window's own sizes otherwise
    float qv[RQ], dpv[RQ], pev[R], dcv[RD], alv[RD], h2v[RD];
    float ar_km = 0.0f;
    const bool huynh = kord >= 7;

    // prologue (levels 1..4 exist because km >= 4): phase 0, element i in slot i
    for (int i = 0; i < 4; ++i) qv[i] = c.q1(1 + i);
    for (int i = 0; i < 5; ++i) pev[i] = c.pe1(1 + i);
    for (int i = 0; i < 4; ++i) dpv[i] = pev[i + 1] - pev[i];
    if constexpr (RING) {
        qv[RQ - 1] = dpv[RQ - 1] = 0.0f;
        for (int i = 3; i < RD; ++i) dcv[i] = alv[i] = h2v[i] = 0.0f;
    }

    const ColumnEnds ends{pev[0], c.pe1(km + 1), qv[0], c.q1(km)};

    float dc1, dc2, dc3, al1, al2, al3;
    dc2 = ppm_dc(qv[0], qv[1], qv[2], dpv[0], dpv[1], dpv[2]);
    dc3 = ppm_dc(qv[1], qv[2], qv[3], dpv[1], dpv[2], dpv[3]);  // 3 <= km-1
    al3 = ppm_al(dpv[0], dpv[1], dpv[2], dpv[3], qv[1], qv[2], dc2, dc3);
    // top: area-preserving cubic (mappm.f90:689-725)
    ppm_top_cubic(qv[0], qv[1], dpv[0], dpv[1], al3, iv, al1, al2, dc1);
    dcv[0] = dc1; dcv[1] = dc2; dcv[2] = dc3;
    alv[0] = al1; alv[1] = al2; alv[2] = al3;
    h2v[0] = 0.0f; h2v[1] = 0.0f;
    h2v[2] = huynh ? ppm_h2(dc1, dc3, dpv[0], dpv[1], dpv[2]) : 0.0f;  // h2(2)

    int lmt = kord - 3;
    lmt = lmt > 0 ? lmt : 0;
    if (iv == 0) lmt = lmt < 2 ? lmt : 2;

    RemapState s{1, false, 0.0f, 0.0f, c.pe2(1), c.pe2(2)};

    // level j = L + 4 is ingested at the end of iteration L; its q1 / pe1 are read one
    // iteration earlier (CARRY) or at the iteration's start (ahead of its stores, so the
    // compiler keeps them there), so each load has arithmetic to arrive behind
    float qc_pf = 0.0f, pec_pf = 0.0f;
    if constexpr (CARRY) {
        if (5 <= km) {
            qc_pf = c.q1(5);
            pec_pf = c.pe1(6);
        }
    }
    // layer L at ring phase P = (L - 1) % 5 (RING; else 0); returns true after the last layer
    auto layer = [&](int L, auto phase) -> bool {
        constexpr int P = RING ? decltype(phase)::value : 0;
#define FV3_W(arr, i) arr[(P + (i)) % R]  // RING: slot of element i; else (P = 0) index i
        float q_pf = qc_pf, pe_pf = pec_pf;
        if constexpr (!CARRY) {
            if (L + 4 <= km) {
                q_pf = c.q1(L + 4);
                pe_pf = c.pe1(L + 5);
            }
        }
        // ---- emit the final coefficients of layer L ----
        Ppm a{FV3_W(qv, 0), FV3_W(alv, 0), (L < km) ? FV3_W(alv, 1) : ar_km, 0.0f};
        const float dcL = FV3_W(dcv, 0);
        if (L <= 2 || L >= km - 1) {
            a.a6 = a6_of(a);
            ppm_limit(dcL, a, 0);
        } else if (huynh) {
            ppm_huynh(a, dcL, FV3_W(h2v, 0), FV3_W(h2v, 2));
            if (iv == 0) ppm_limit(dcL, a, 2);
        } else {
            if (kord != 4) a.a6 = a6_of(a);
            if (kord != 6) ppm_limit(dcL, a, lmt);
        }
        const LayerView v{FV3_W(pev, 0), FV3_W(pev, 1), FV3_W(dpv, 0), FV3_W(qv, 0), a};
#ifdef FV3_EXP_NOREMAP  // experiment only (results invalid): profile cost without the consumer
        if (L <= kn) c.emit(L, v.a.al + v.a.ar + v.a.a6);
#else
        if constexpr (FAST)
            remap_layer_fast(s, v, ends, kn, c);
        else
            remap_layer(s, v, ends, kn, c);
#endif
        // RING: once per group of R layers (a hook is free to lag: the coarsen's takes
        // whatever whole levels every lane has emitted, and drains the rest at the end)
        if constexpr (!RING || P == R - 1) layer_hook(c, 0);

        if (L == km) return true;
        // ---- advance the window E_L -> E_{L+1}: one new element per ring ----
        const int j = L + 4;  // level to ingest
        float qn = 0.0f, pen = 0.0f, dpn = 0.0f;
        if (j <= km) {
            qn = q_pf;
            pen = pe_pf;
            dpn = pen - FV3_W(pev, 4);
        }
        if constexpr (CARRY) {
            if (j + 1 <= km) {  // level j + 1, for the next iteration
                qc_pf = c.q1(j + 1);
                pec_pf = c.pe1(j + 2);
            }
        }
        const int m = L + 3;  // dc(m), ALraw(m)
        float dcm = 0.0f, alm = 0.0f;
        if (m <= km - 1) {
#ifdef FV3_EXP_NOPROFILE  // experiment only (results invalid): consumer cost without dc/al
            dcm = qn - FV3_W(qv, 3);
            alm = 0.5f * (FV3_W(qv, 2) + FV3_W(qv, 3));
#else
            dcm = ppm_dc(FV3_W(qv, 2), FV3_W(qv, 3), qn, FV3_W(dpv, 2), FV3_W(dpv, 3), dpn);
            alm = ppm_al(FV3_W(dpv, 1), FV3_W(dpv, 2), FV3_W(dpv, 3), dpn, FV3_W(qv, 2), FV3_W(qv, 3),
                         FV3_W(dcv, 2), dcm);
#endif
        } else if (m == km) {
            // bottom: area-preserving cubic (mappm.f90:729-761)
            ppm_bottom_cubic(FV3_W(qv, 3), FV3_W(qv, 2), FV3_W(dpv, 3), FV3_W(dpv, 2), FV3_W(alv, 2), iv, alm, ar_km,
                             dcm);
        }
        float h2n = 0.0f;  // h2(L+2)
        if (huynh && L + 2 <= km - 1) h2n = ppm_h2(FV3_W(dcv, 1), dcm, FV3_W(dpv, 1), FV3_W(dpv, 2), FV3_W(dpv, 3));

        if constexpr (RING) {
            // window at L + 1: element i in slot (P + 1 + i) % 5; the new last elements
            FV3_W(qv, 4) = qn;    // q(L+4)   = element 3 at L + 1
            FV3_W(dpv, 4) = dpn;  // dp(L+4)
            FV3_W(pev, 5) = pen;  // pe1(L+5) = element 4 at L + 1 (pe1(L)'s slot, now dead)
            FV3_W(dcv, 3) = dcm;  // dc(L+3)  = element 2 at L + 1
            FV3_W(alv, 3) = alm;
            FV3_W(h2v, 3) = h2n;  // h2(L+2)  = element 2 at L + 1
        } else {
            qv[0] = qv[1]; qv[1] = qv[2]; qv[2] = qv[3]; qv[3] = qn;
            dpv[0] = dpv[1]; dpv[1] = dpv[2]; dpv[2] = dpv[3]; dpv[3] = dpn;
            pev[0] = pev[1]; pev[1] = pev[2]; pev[2] = pev[3]; pev[3] = pev[4]; pev[4] = pen;
            dcv[0] = dcv[1]; dcv[1] = dcv[2]; dcv[2] = dcm;
            alv[0] = alv[1]; alv[1] = alv[2]; alv[2] = alm;
            h2v[0] = h2v[1]; h2v[1] = h2v[2]; h2v[2] = h2n;
        }
#undef FV3_W
        return false;
    };
    using std::integral_constant;
    if constexpr (RING) {
        for (int L = 1;; L += R) {
            if (layer(L, integral_constant<int, 0>{})) break;
            if (layer(L + 1, integral_constant<int, 1>{})) break;
            if (layer(L + 2, integral_constant<int, 2>{})) break;
            if (layer(L + 3, integral_constant<int, 3>{})) break;
            if (layer(L + 4, integral_constant<int, 4>{})) break;
        }
    } else {
        for (int L = 1; L <= km; ++L)
            if (layer(L, integral_constant<int, 0>{})) break;
    }
#ifndef FV3_EXP_NOREMAP
    remap_finish(s, ends, kn, c);
#endif
}

// ---- resumable PPM column (kord <= 7): one OUTPUT level per call ----
//
// The arithmetic of mappm_ppm_column, in the same order, restructured so that the
// caller drives it by output level: next() returns q2(k) for k = 1, 2, ... kn.
// Each call ingests as many input layers as this column needs (a per-lane,
// data-dependent loop); between calls every lane of a wave is reconverged, which the
// fused coarse-graining kernel uses to combine neighbouring columns level by level
// with cross-lane shuffles instead of staging whole columns in LDS.
// `Col` as for mappm_ppm_column (emit() unused).

// One output-layer event of remap_layer: true (value in `val`, state advanced to the
// next output layer) or false (this input layer is exhausted: move to L+1).
template <class Out>
FV3_HD inline bool remap_one(RemapState& s, const LayerView& v, const ColumnEnds& e, Out& out, float& val)
{
    const float r3 = 1.0f / 3.0f, r23 = 2.0f / 3.0f;
    if (!s.accum) {
        if (s.t <= e.pe_top) {
            val = e.q_top;
        } else if (s.t >= e.pe_bot) {
            val = e.q_bot;
        } else if (s.t >= v.pl0 && s.t <= v.pl1) {
            const float pl = FV3_DIVQ(s.t - v.pl0, v.dp);
            if (s.b <= v.pl1) {
                const float pr = FV3_DIVQ(s.b - v.pl0, v.dp);
                const float tt = r3 * (pr * (pr + pl) + pl * pl);
                val = v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (pr + pl) - v.a.a6 * tt;
            } else {
                const float delp = v.pl1 - s.t;
                const float tt = r3 * (1.0f + pl * (1.0f + pl));
                s.qsum = delp * (v.a.al + 0.5f * (v.a.a6 + v.a.ar - v.a.al) * (1.0f + pl) - v.a.a6 * tt);
                s.dpsum = delp;
                s.accum = true;
                return false;
            }
        } else {
            return false;
        }
    } else {
        if (s.b > v.pl1) {
            s.qsum = s.qsum + v.dp * v.q1;
            s.dpsum = s.dpsum + v.dp;
            return false;
        }
        const float delp = s.b - v.pl0;
        const float esl = FV3_DIVQ(delp, v.dp);
        s.qsum = s.qsum + delp * (v.a.al + 0.5f * esl * (v.a.ar - v.a.al + v.a.a6 * (1.0f - r23 * esl)));
        s.dpsum = s.dpsum + delp;
        val = FV3_DIVQ(s.qsum, s.dpsum);
        s.accum = false;
    }
    s.k += 1;
    s.t = s.b;
    s.b = out.next_edge(s.k);
    return true;
}

template <class Col>
struct PpmCursor {
    Col& c;
    int km, kn, iv, kord, lmt;
    bool huynh;
    float qv[4], dpv[4], pev[5], dcv[3], alv[3], h2v[3];
    float ar_km;
    ColumnEnds ends;
    RemapState s;
    LayerView v;
    int L;      // current input layer (1-based); km + 1 once all are consumed
    bool have;  // v holds layer L's final coefficients

    FV3_HD PpmCursor(Col& col, int km_, int kn_, int iv_, int kord_)
        : c(col), km(km_), kn(kn_), iv(iv_), kord(kord_), ar_km(0.0f), L(1), have(false)
    {
        huynh = kord >= 7;
        for (int i = 0; i < 4; ++i) qv[i] = c.q1(1 + i);
        for (int i = 0; i < 5; ++i) pev[i] = c.pe1(1 + i);
        for (int i = 0; i < 4; ++i) dpv[i] = pev[i + 1] - pev[i];
        ends = ColumnEnds{pev[0], c.pe1(km + 1), qv[0], c.q1(km)};
        float dc1, dc2, dc3, al1, al2, al3;
        dc2 = ppm_dc(qv[0], qv[1], qv[2], dpv[0], dpv[1], dpv[2]);
        dc3 = ppm_dc(qv[1], qv[2], qv[3], dpv[1], dpv[2], dpv[3]);
        al3 = ppm_al(dpv[0], dpv[1], dpv[2], dpv[3], qv[1], qv[2], dc2, dc3);
        // top: area-preserving cubic (mappm.f90:689-725)
        ppm_top_cubic(qv[0], qv[1], dpv[0], dpv[1], al3, iv, al1, al2, dc1);
        dcv[0] = dc1; dcv[1] = dc2; dcv[2] = dc3;
        alv[0] = al1; alv[1] = al2; alv[2] = al3;
        h2v[0] = 0.0f; h2v[1] = 0.0f;
        h2v[2] = huynh ? ppm_h2(dc1, dc3, dpv[0], dpv[1], dpv[2]) : 0.0f;
        lmt = kord - 3;
        lmt = lmt > 0 ? lmt : 0;
        if (iv == 0) lmt = lmt < 2 ? lmt : 2;
        s = RemapState{1, false, 0.0f, 0.0f, c.pe2(1), c.pe2(2)};
    }

    // final coefficients of layer L (the top of mappm_ppm_column's L loop)
    FV3_HD void load_layer()
    {
        Ppm a{qv[0], alv[0], (L < km) ? alv[1] : ar_km, 0.0f};
        const float dcL = dcv[0];
        if (L <= 2 || L >= km - 1) {
            a.a6 = a6_of(a);
            ppm_limit(dcL, a, 0);
        } else if (huynh) {
            ppm_huynh(a, dcL, h2v[0], h2v[2]);
            if (iv == 0) ppm_limit(dcL, a, 2);
        } else {
            if (kord != 4) a.a6 = a6_of(a);
            if (kord != 6) ppm_limit(dcL, a, lmt);
        }
        v = LayerView{pev[0], pev[1], dpv[0], qv[0], a};
        have = true;
    }

    // window E_L -> E_{L+1} (the bottom of mappm_ppm_column's L loop)
    FV3_HD void advance()
    {
        have = false;
        if (L == km) {
            L = km + 1;
            return;
        }
        const int j = L + 4;
        float qn = 0.0f, pen = 0.0f, dpn = 0.0f;
        if (j <= km) {
            qn = c.q1(j);
            pen = c.pe1(j + 1);
            dpn = pen - pev[4];
        }
        const int m = L + 3;
        float dcm = 0.0f, alm = 0.0f;
        if (m <= km - 1) {
            dcm = ppm_dc(qv[2], qv[3], qn, dpv[2], dpv[3], dpn);
            alm = ppm_al(dpv[1], dpv[2], dpv[3], dpn, qv[2], qv[3], dcv[2], dcm);
        } else if (m == km) {
            ppm_bottom_cubic(qv[3], qv[2], dpv[3], dpv[2], alv[2], iv, alm, ar_km, dcm);
        }
        float h2n = 0.0f;
        if (huynh && L + 2 <= km - 1) h2n = ppm_h2(dcv[1], dcm, dpv[1], dpv[2], dpv[3]);
        qv[0] = qv[1]; qv[1] = qv[2]; qv[2] = qv[3]; qv[3] = qn;
        dpv[0] = dpv[1]; dpv[1] = dpv[2]; dpv[2] = dpv[3]; dpv[3] = dpn;
        pev[0] = pev[1]; pev[1] = pev[2]; pev[2] = pev[3]; pev[3] = pev[4]; pev[4] = pen;
        dcv[0] = dcv[1]; dcv[1] = dcv[2]; dcv[2] = dcm;
        alv[0] = alv[1]; alv[1] = alv[2]; alv[2] = alm;
        h2v[0] = h2v[1]; h2v[1] = h2v[2]; h2v[2] = h2n;
        L += 1;
    }

    // q2(k) for the next output layer k = s.k (remap_layer / remap_finish semantics)
    FV3_HD float next()
    {
        float val = 0.0f;
        while (L <= km) {
            if (!have) load_layer();
            if (remap_one(s, v, ends, c, val)) return val;
            advance();
        }
        // below the last input layer (mappm.f90:115-121, 62-67)
        if (s.accum) {
            const float delp = s.b - ends.pe_bot;
            if (delp > 0.0f) {
                s.qsum = s.qsum + delp * ends.q_bot;
                s.dpsum = s.dpsum + delp;
            }
            val = FV3_DIVQ(s.qsum, s.dpsum);
            s.accum = false;
        } else if (s.t <= ends.pe_top) {
            val = ends.q_top;
        } else if (s.t >= ends.pe_bot) {
            val = ends.q_bot;
        } else {
            val = __builtin_nanf("");  // search failed: reference UB
        }
        s.k += 1;
        s.t = s.b;
        s.b = c.next_edge(s.k);
        return val;
    }
};

// mappm_ppm_column driven through the cursor (host test of the cursor's equivalence)
template <class Col>
FV3_HD inline void mappm_ppm_column_by_output(Col& c, int km, int kn, int iv, int kord)
{
    PpmCursor<Col> cur(c, km, kn, iv, kord);
    for (int k = 1; k <= kn; ++k) c.emit(k, cur.next());
}

// ---- one column, kord > 7 (cs_profile path) ----
//
// `Scr` is per-column scratch of 2*(km+2) floats: edge(k) for k = 1..km+1 and
// gam(k), addressed by scr.e(k) / scr.g(k) (global memory or LDS on the device).
//
// NT > 0 (iv != -2, km >= NT + 1): the bottom NT edges never touch the scratch.  The
// forward sweep keeps the last NT - 1 levels' (edge, gam) in registers, the
// back-substitution runs over them first (fully unrolled, static register indices) and
// leaves the solved edges kt..km+1 (kt = km + 2 - NT) in registers, and the main loop,
// which reads every edge exactly once in increasing k, takes them from the front of that
// register queue.  Same operations in the same order on the same values: the bits are
// those of the all-scratch path, with 6 NT fewer scratch accesses per column (the
// scratch round trips are most of kord > 7's HBM traffic).
//
// PF > 0: the loads run ahead of their use.  The scratch stores of each level may alias
// the next level's loads as far as the compiler can tell, so as written every level of
// the forward sweep and of the back-substitution waits out one full memory round trip
// (load, wait, compute, store).  With PF, the sweep's q1 / pe1 and the
// back-substitution's edge / gam are loaded PF levels ahead into a register ring (loop
// unrolled by PF, static ring indices), and the main loop's q1 / edge / pe1 one layer
// ahead.  Loads only move earlier, past stores to other addresses: the same values, the
// same bits.
//
// KORD > 0: the column for |kord| = KORD only (the host dispatches it for that kord): the
// kord switch and the flags that kord never reads fold away at compile time.
template <class Col, class Scr, int NT = 0, int PF = 0, int KORD = 0>
FV3_HD inline void mappm_cs_column(Col& c, Scr& scr, int km, int kn, int iv, int kord)
{
    const int akord = KORD > 0 ? KORD : (kord < 0 ? -kord : kord);
    const float qs = 0.0f;  // mappm passes an uninitialised qs (mappm.f90:33,49)
    constexpr int NTR = NT > 0 ? NT : 1;
    const bool tail = NT > 0 && iv != -2 && km >= NT + 1;
    const int kt = tail ? km + 2 - NT : km + 2;  // first edge held in registers
    float te[NTR], tg[NTR];                      // edge / gam of levels kt + j

    // ---- tridiagonal edge solve (mappm.f90:153-205): forward sweep into scratch ----
    {
        float qm1 = c.q1(1), pe0 = c.pe1(1), pe1v = c.pe1(2);
        float dpm1 = pe1v - pe0;
        if (iv == -2) {
            scr.g(2) = 0.5f;
            float qprev = 1.5f * qm1;
            scr.e(1) = qprev;
            float gk = 0.5f;  // gam(k)
            float pek = pe1v;
            for (int k = 2; k <= km - 1; ++k) {
                const float qk = c.q1(k);
                const float pen = c.pe1(k + 1);
                const float dpk = pen - pek;
                const float grat = FV3_DIV(dpm1, dpk);
                const float bet = 2.0f + grat + grat - gk;
                qprev = FV3_DIV(3.0f * (qm1 + qk) - qprev, bet);
                scr.e(k) = qprev;
                gk = FV3_DIV(grat, bet);
                scr.g(k + 1) = gk;
                qm1 = qk; dpm1 = dpk; pek = pen;
            }
            const float qkm = c.q1(km);
            const float dpkm = c.pe1(km + 1) - pek;
            const float grat = FV3_DIV(dpm1, dpkm);
            qprev = FV3_DIV(3.0f * (qm1 + qkm) - grat * qs - qprev, 2.0f + grat + grat - gk);
            scr.e(km) = qprev;
            scr.e(km + 1) = qs;
            float qn = qprev;
            for (int k = km - 1; k >= 1; --k) {
                qn = scr.e(k) - scr.g(k + 1) * qn;
                scr.e(k) = qn;
            }
        } else {
            float q2v = c.q1(2);
            float pe2v = c.pe1(3);
            float dp2 = pe2v - pe1v;
            float grat = FV3_DIV(dp2, dpm1);
            float bet = grat * (grat + 0.5f);
            float qprev = FV3_DIV((grat + grat) * (grat + 1.0f) * qm1 + q2v, bet);
            float gprev = FV3_DIV(1.0f + grat * (grat + 1.5f), bet);
            scr.e(1) = qprev;
            scr.g(1) = gprev;
            float d4 = 0.0f;
            float pek = pe1v;
            float qkm1 = qm1;
            float qk = qm1;
            auto sweep_v = [&](float qkv, float pen, auto&& e_out, auto&& g_out) {
                qk = qkv;
                const float dpk = pen - pek;
                d4 = FV3_DIV(dpm1, dpk);
                bet = 2.0f + d4 + d4 - gprev;
                qprev = FV3_DIV(3.0f * (qkm1 + d4 * qk) - qprev, bet);
                gprev = FV3_DIV(d4, bet);
                e_out = qprev;
                g_out = gprev;
                qkm1 = qk; dpm1 = dpk; pek = pen;
            };
            auto sweep = [&](int k, auto&& e_out, auto&& g_out) { sweep_v(c.q1(k), c.pe1(k + 1), e_out, g_out); };
            const int kend = tail ? kt - 1 : km;
            if constexpr (PF > 0) {
                // blocks of PF levels in two register sets: block b + 1's loads are issued
                // when block b starts, so they have a whole block to land.  (The compiler
                // runs a block's independent divisions ahead, so it waits for the whole
                // block's loads at its start.)  Two static sets, the loop unrolled by two
                // blocks: no register copies across the back edge, which would wait for
                // the loads in flight.  Loads past kend are clamped to km: spare loads.
                float qa[PF], pa[PF], qb[PF], pb[PF];
                auto load_blk = [&](float (&q)[PF], float (&p)[PF], int k0) {
#pragma unroll
                    for (int j = 0; j < PF; ++j) {
                        const int kk = imin2(k0 + j, km);
                        q[j] = c.q1(kk);
                        p[j] = c.pe1(kk + 1);
                    }
                };
                auto run_blk = [&](const float (&q)[PF], const float (&p)[PF], int k0, int n) {
#pragma unroll
                    for (int j = 0; j < PF; ++j)
                        if (j < n) sweep_v(q[j], p[j], scr.e(k0 + j), scr.g(k0 + j));
                };
                load_blk(qa, pa, 2);
                int k = 2;
                for (; k + 2 * PF - 1 <= kend; k += 2 * PF) {
                    load_blk(qb, pb, k + PF);
                    run_blk(qa, pa, k, PF);
                    load_blk(qa, pa, k + 2 * PF);
                    run_blk(qb, pb, k + PF, PF);
                }
                if (k + PF - 1 <= kend) {  // one whole block left (qa), then < PF levels (qb)
                    load_blk(qb, pb, k + PF);
                    run_blk(qa, pa, k, PF);
                    run_blk(qb, pb, k + PF, kend - (k + PF) + 1);
                } else {
                    run_blk(qa, pa, k, kend - k + 1);
                }
            } else {
                for (int k = 2; k <= kend; ++k) sweep(k, scr.e(k), scr.g(k));
            }
            if constexpr (NT > 0) {
                if (tail) {
#pragma unroll
                    for (int j = 0; j < NT - 1; ++j) sweep(kt + j, te[j], tg[j]);  // k = kt .. km
                }
            }
            // qkm1 == qk == q(km) here; need q(km-1)
            const float a_bot = 1.0f + d4 * (d4 + 1.5f);
            const float qkmm1 = c.q1(km - 1);
            float qn = FV3_DIV(2.0f * d4 * (d4 + 1.0f) * qk + qkmm1 - a_bot * qprev, d4 * (d4 + 0.5f) - a_bot * gprev);
            int kb = km;  // back-substitution continues in the scratch from here
            if constexpr (NT > 0) {
                if (tail) {
                    te[NT - 1] = qn;  // e(km+1)
#pragma unroll
                    for (int j = NT - 2; j >= 0; --j) {
                        qn = te[j] - tg[j] * qn;
                        te[j] = qn;
                    }
                    kb = kt - 1;
                }
            }
            if (!tail) scr.e(km + 1) = qn;
            if constexpr (PF > 0) {
                // descending blocks of PF levels in two register sets, as in the sweep;
                // loads below level 1 are clamped to 1 (spare loads, never used), and a
                // block's loads precede the stores of the block before it in program order
                float ea[PF], ga[PF], eb[PF], gb[PF];
                auto load_blk = [&](float (&e)[PF], float (&g)[PF], int k0) {
#pragma unroll
                    for (int j = 0; j < PF; ++j) {
                        const int kk = imax2(k0 - j, 1);
                        e[j] = scr.e(kk);
                        g[j] = scr.g(kk);
                    }
                };
                auto run_blk = [&](const float (&e)[PF], const float (&g)[PF], int k0, int n) {
#pragma unroll
                    for (int j = 0; j < PF; ++j) {
                        if (j < n) {
                            qn = e[j] - g[j] * qn;
                            scr.e(k0 - j) = qn;
                        }
                    }
                };
                load_blk(ea, ga, kb);
                int k = kb;
                for (; k - (2 * PF - 1) >= 1; k -= 2 * PF) {
                    load_blk(eb, gb, k - PF);
                    run_blk(ea, ga, k, PF);
                    load_blk(ea, ga, k - 2 * PF);
                    run_blk(eb, gb, k - PF, PF);
                }
                if (k - (PF - 1) >= 1) {
                    load_blk(eb, gb, k - PF);
                    run_blk(ea, ga, k, PF);
                    run_blk(eb, gb, k - PF, k - PF);
                } else {
                    run_blk(ea, ga, k, k);
                }
            } else {
                for (int k = kb; k >= 1; --k) {
                    qn = scr.e(k) - scr.g(k) * qn;
                    scr.e(k) = qn;
                }
            }
        }
    }
    // solved edge e(k), read once per k in increasing k by edge_c below: the register
    // queue's front from kt on
    auto e_at = [&](int k) -> float {
        if constexpr (NT > 0) {
            if (tail && k >= kt) {
                const float v = te[0];
#pragma unroll
                for (int j = 0; j + 1 < NT; ++j) te[j] = te[j + 1];
                return v;
            }
        }
        return scr.e(k);
    };

    const ColumnEnds ends{c.pe1(1), c.pe1(km + 1), c.q1(1), c.q1(km)};
    RemapState s{1, false, 0.0f, 0.0f, c.pe2(1), c.pe2(2)};

    // constrained edge qc(k) (mappm.f90:207-260) from the solved edge e(k) and
    // q1(k-2..k+1); the large-scale constraints use gam(k) = q1(k) - q1(k-1).
    auto edge_cv = [&](int k, float q, float qkm2, float qkm1, float qk0, float qkp1) -> float {
        if (akord > 16 || k <= 1 || k >= km + 1) return q;
        if (k == 2 || k == km) {
            q = fmin2(q, fmax2(qkm1, qk0));
            q = fmax2(q, fmin2(qkm1, qk0));
        } else {
            const float gm = qkm1 - qkm2;  // gam(k-1)
            const float gp = qkp1 - qk0;   // gam(k+1)
            if (gm * gp > 0.0f) {
                q = fmin2(q, fmax2(qkm1, qk0));
                q = fmax2(q, fmin2(qkm1, qk0));
            } else if (gm > 0.0f) {
                q = fmax2(q, fmin2(qkm1, qk0));
            } else {
                q = fmin2(q, fmax2(qkm1, qk0));
                if (iv == 0) q = fmax2(0.0f, q);
            }
        }
        return q;
    };
    auto edge_c = [&](int k, float qkm2, float qkm1, float qk0, float qkp1) -> float {
        return edge_cv(k, e_at(k), qkm2, qkm1, qk0, qkp1);
    };
    auto q1_or0 = [&](int k) -> float { return (k >= 1 && k <= km) ? c.q1(k) : 0.0f; };

    // rolling windows at layer L: qw[i] = q1(L-2+i) (i=0..5), qcw[i] = qc(L-1+i) (i=0..3)
    float qw[6], qcw[4];
    for (int i = 0; i < 6; ++i) qw[i] = q1_or0(i - 1);
    qcw[0] = 0.0f;
    qcw[1] = edge_c(1, 0.0f, 0.0f, qw[2], qw[3]);
    qcw[2] = edge_c(2, 0.0f, qw[2], qw[3], qw[4]);
    qcw[3] = edge_c(3, qw[2], qw[3], qw[4], qw[5]);
    float pl0 = c.pe1(1), pl1 = c.pe1(2);

    // subgrid flags of layers L-1, L, L+1 (mappm.f90:269-288), index i = 0, 1, 2 of the
    // window: each layer's flags are computed once, as index 2, and shift with the window
    bool extm[3] = {false, false, false}, ext5[3] = {false, false, false}, ext6[3] = {false, false, false};
    auto flags = [&](int i, int k) {
        const float qkm = qw[i], qk = qw[i + 1], qkp = qw[i + 2];
        const float ql = qcw[i], qr = qcw[i + 1];
        if (k == 1 || k == km)
            extm[i] = (ql - qk) * (qr - qk) > 0.0f;
        else
            extm[i] = (qk - qkm) * (qkp - qk) < 0.0f;
        const float x0 = 2.0f * qk - (ql + qr);
        const float x1 = fabsf(ql - qr);
        ext5[i] = fabsf(x0) > x1;
        ext6[i] = fabsf(3.0f * x0) > x1;
    };
    if (akord <= 16) {
        flags(0, 0);  // layer 0: never read
        flags(1, 1);
    }

    for (int L = 1; L <= km; ++L) {
        // PF: q1(L + 4), edge(L + 3), pe1(L + 2), which the end of layer L takes into the
        // windows, are loaded at its start (ahead of the layer's stores, so the compiler
        // keeps them there): the layer's arithmetic covers their latency.  Locals, not
        // loop-carried registers: a register copy at the loop's back edge would wait for
        // a load in flight.
        float nq = 0.0f, ne = 0.0f, np = 0.0f;
        if constexpr (PF > 0) {
            if (L < km) {
                nq = q1_or0(L + 4);
                if (L + 3 <= km + 1) ne = e_at(L + 3);
                np = c.pe1(L + 2);
            }
        }
        Ppm a{qw[2], qcw[1], qcw[2], 0.0f};
        if (akord > 16) {
            a.a6 = a6_of(a);  // perfectly linear scheme (mappm.f90:207-216)
        } else {
            flags(2, L + 1);
            const float g_m1 = qw[1] - qw[0];  // gam(L-1)
            const float g_0 = qw[2] - qw[1];   // gam(L)
            const float g_p1 = qw[3] - qw[2];  // gam(L+1)
            const float g_p2 = qw[4] - qw[3];  // gam(L+2)
            auto huynh_l = [&]() {
                const float pmp_1 = a.a1 - 2.0f * g_p1;
                const float lac_1 = pmp_1 + 1.5f * g_p2;
                a.al = fmin2(fmax2(a.al, fmin3(a.a1, pmp_1, lac_1)), fmax3(a.a1, pmp_1, lac_1));
            };
            auto huynh_r = [&]() {
                const float pmp_2 = a.a1 + 2.0f * g_0;
                const float lac_2 = pmp_2 - 1.5f * g_m1;
                a.ar = fmin2(fmax2(a.ar, fmin3(a.a1, pmp_2, lac_2)), fmax3(a.a1, pmp_2, lac_2));
            };
            auto a6_alt = [&]() { a.a6 = 6.0f * a.a1 - 3.0f * (a.al + a.ar); };
            auto flat = [&]() { a.al = a.a1; a.ar = a.a1; };

            if (L == 1) {
                if (iv == 0) {
                    a.al = fmax2(0.0f, a.al);
                } else if (iv == -1) {
                    if (a.al * a.a1 <= 0.0f) a.al = 0.0f;
                } else if (iv == 2) {
                    a.al = a.a1; a.ar = a.a1; a.a6 = 0.0f;
                }
                if (iv != 2) {
                    a.a6 = a6_of(a);
                    cs_limit(extm[1], a, 1);
                }
            } else if (L == 2) {
                a.a6 = a6_of(a);
                cs_limit(extm[1], a, 2);
            } else if (L <= km - 2) {
                // Huynh's 2nd constraint for the interior (mappm.f90:328-504)
                if (akord < 9) {
                    huynh_l(); huynh_r(); a.a6 = a6_of(a);
                } else if (akord == 9) {
                    if ((extm[1] && extm[0]) || (extm[1] && extm[2])) {
                        flat(); a.a6 = 0.0f;
                    } else {
                        a6_alt();
                        if (fabsf(a.a6) > fabsf(a.al - a.ar)) { huynh_l(); huynh_r(); a6_alt(); }
                    }
                } else if (akord == 10) {
                    if (ext5[1]) {
                        if (ext5[0] || ext5[2]) flat();
                        else if (ext6[0] || ext6[2]) { huynh_l(); huynh_r(); }
                    } else if (ext6[1]) {
                        if (ext5[0] || ext5[2]) { huynh_l(); huynh_r(); }
                    }
                    a.a6 = a6_of(a);
                } else if (akord == 12) {
                    if (extm[1]) {
                        flat(); a.a6 = 0.0f;
                    } else {
                        a6_alt();
                        if (fabsf(a.a6) > fabsf(a.al - a.ar)) { huynh_l(); huynh_r(); a6_alt(); }
                    }
                } else if (akord == 13) {
                    if (ext6[1] && ext6[0] && ext6[2]) flat();
                    a.a6 = a6_of(a);
                } else if (akord == 14) {
                    a.a6 = a6_of(a);
                } else if (akord == 15) {
                    if (ext5[1]) {
                        if (ext5[0] || ext5[2]) flat();
                    } else if (ext6[1]) {
                        huynh_l(); huynh_r();
                    }
                    a.a6 = a6_of(a);
                } else if (akord == 16) {
                    if (ext5[1]) {
                        if (ext5[0] || ext5[2]) flat();
                        else if (ext6[0] || ext6[2]) { huynh_l(); huynh_r(); }
                    }
                    a.a6 = a6_of(a);
                } else {  // kord = 11
                    if (ext5[1] && (ext5[0] || ext5[2])) {
                        flat(); a.a6 = 0.0f;
                    } else {
                        a.a6 = a6_of(a);
                    }
                }
                if (iv == 0) cs_limit(extm[1], a, 0);
            } else if (L == km - 1) {
                a.a6 = a6_of(a);
                cs_limit(extm[1], a, 2);
            } else {  // L == km (mappm.f90:514-530)
                if (iv == 0) {
                    a.ar = fmax2(0.0f, a.ar);
                } else if (iv == -1) {
                    if (a.ar * a.a1 <= 0.0f) a.ar = 0.0f;
                }
                a.a6 = a6_of(a);
                cs_limit(extm[1], a, 1);
            }
        }
        const LayerView v{pl0, pl1, pl1 - pl0, qw[2], a};
        remap_layer_fast(s, v, ends, kn, c);
        if (L == km) break;
        for (int i = 0; i < 5; ++i) qw[i] = qw[i + 1];
        for (int i = 0; i < 3; ++i) qcw[i] = qcw[i + 1];
        for (int i = 0; i < 2; ++i) {
            extm[i] = extm[i + 1];
            ext5[i] = ext5[i + 1];
            ext6[i] = ext6[i + 1];
        }
        pl0 = pl1;
        if constexpr (PF > 0) {
            qw[5] = nq;
            qcw[3] = (L + 3 <= km + 1) ? edge_cv(L + 3, ne, qw[2], qw[3], qw[4], qw[5]) : 0.0f;
            pl1 = np;
        } else {
            qw[5] = q1_or0(L + 4);
            qcw[3] = (L + 3 <= km + 1) ? edge_c(L + 3, qw[2], qw[3], qw[4], qw[5]) : 0.0f;
            pl1 = c.pe1(L + 2);
        }
    }
    remap_finish(s, ends, kn, c);
}

#ifdef FV3_FAST_ARITH
#pragma clang fp contract(off)
#endif
}  // namespace FV3_ARITH_NS
using namespace FV3_ARITH_NS;
}  // namespace fv3
