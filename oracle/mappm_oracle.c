/*
 * ORACLE — test infrastructure only.  Never linked into, loaded by, or called
 * from the fv3net_amd product path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Plain-C restatement of fv3net's vertical remap `mappm` (FV3 fv_mapz):
 *   /root/reference/external/mappm/mappm/mappm.f90
 *     mappm        :10-126    remap loop over output layers
 *     cs_profile   :132-532   kord > 7  (tridiagonal edge solve + Huynh limits)
 *     cs_limiters  :535-611
 *     ppm_profile  :614-851   kord <= 7 (4th-order edges + PPM limiters)
 *     ppm_limiters :854-931
 * Arithmetic is real*4 (float) throughout, evaluated in the Fortran source's
 * left-to-right order, one rounding per operation (compile with
 * -ffp-contract=off).  Fortran intrinsics follow what AMD flang emits on x86:
 *   max(a,b) = a > b ? a : b,   min(a,b) = a < b ? a : b   (left fold for 3 args)
 *   sign(a,b) = copysign(|a|, b)
 * The structure deliberately mirrors the Fortran (whole-column arrays, one
 * pass per stage) so the two can be read side by side; the product kernel in
 * fv3net_amd/csrc is a different (streaming, one-pass) formulation that is
 * checked against this file and against the flang build in oracle/_ref.
 *
 * Layout: Fortran column-major, i.e. element (col i, level k) at [k*ncol + i],
 * levels 0-based here (Fortran k = kf is index kf-1).
 *
 * Undefined behaviour in the reference that is NOT reproduced (excluded from
 * parity): uninitialised qs for iv=-2 with kord>7 (we use 0),
 * and stale k1/qsum/dpsum when the layer search fails on a non-monotone pe1
 * (we return NaN for that output layer).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define FMAX(a, b) ((a) > (b) ? (a) : (b))
#define FMIN(a, b) ((a) < (b) ? (a) : (b))
static inline float fmax3(float a, float b, float c) { float m = FMAX(a, b); return FMAX(m, c); }
static inline float fmin3(float a, float b, float c) { float m = FMIN(a, b); return FMIN(m, c); }
static inline float fsign(float a, float b) { return copysignf(fabsf(a), b); }

/* 1-based accessors for one column: A4(n,k) n=1..4, k=1..km */
#define A4(n, k) a4[((k) - 1) * 4 + ((n) - 1)]

static void ppm_limiters_col(float dm, float *a /* a4(1..4) of one level */, int lmt)
{
    const float r12 = 1.0f / 12.0f;
    float *a1 = &a[0], *a2 = &a[1], *a3 = &a[2], *a6 = &a[3];
    if (lmt == 3) return;
    if (lmt == 0) {
        if (dm == 0.0f) {
            *a2 = *a1; *a3 = *a1; *a6 = 0.0f;
        } else {
            float da1 = *a3 - *a2;
            float da2 = da1 * da1;
            float a6da = *a6 * da1;
            if (a6da < -da2) {
                *a6 = 3.0f * (*a2 - *a1);
                *a3 = *a2 - *a6;
            } else if (a6da > da2) {
                *a6 = 3.0f * (*a3 - *a1);
                *a2 = *a3 - *a6;
            }
        }
    } else if (lmt == 1) {
        float qmp = 2.0f * dm;
        *a2 = *a1 - fsign(FMIN(fabsf(qmp), fabsf(*a2 - *a1)), qmp);
        *a3 = *a1 + fsign(FMIN(fabsf(qmp), fabsf(*a3 - *a1)), qmp);
        *a6 = 3.0f * (2.0f * *a1 - (*a2 + *a3));
    } else if (lmt == 2) {
        if (fabsf(*a3 - *a2) < -*a6) {
            float d = *a3 - *a2;
            float fmin = *a1 + 0.25f * (d * d) / *a6 + *a6 * r12;
            if (fmin < 0.0f) {
                if (*a1 < *a3 && *a1 < *a2) {
                    *a3 = *a1; *a2 = *a1; *a6 = 0.0f;
                } else if (*a3 > *a2) {
                    *a6 = 3.0f * (*a2 - *a1);
                    *a3 = *a2 - *a6;
                } else {
                    *a6 = 3.0f * (*a3 - *a1);
                    *a2 = *a3 - *a6;
                }
            }
        }
    }
}

static void cs_limiters_col(int extm, float *a, int iv)
{
    const float r12 = 1.0f / 12.0f;
    float *a1 = &a[0], *a2 = &a[1], *a3 = &a[2], *a6 = &a[3];
    if (iv == 0) {
        if (*a1 <= 0.0f) {
            *a2 = *a1; *a3 = *a1; *a6 = 0.0f;
        } else if (fabsf(*a3 - *a2) < -*a6) {
            float d = *a3 - *a2;
            if ((*a1 + 0.25f * (d * d) / *a6 + *a6 * r12) < 0.0f) {
                if (*a1 < *a3 && *a1 < *a2) {
                    *a3 = *a1; *a2 = *a1; *a6 = 0.0f;
                } else if (*a3 > *a2) {
                    *a6 = 3.0f * (*a2 - *a1);
                    *a3 = *a2 - *a6;
                } else {
                    *a6 = 3.0f * (*a3 - *a1);
                    *a2 = *a3 - *a6;
                }
            }
        }
    } else if (iv == 1) {
        if ((*a1 - *a2) * (*a1 - *a3) >= 0.0f) {
            *a2 = *a1; *a3 = *a1; *a6 = 0.0f;
        } else {
            float da1 = *a3 - *a2;
            float da2 = da1 * da1;
            float a6da = *a6 * da1;
            if (a6da < -da2) {
                *a6 = 3.0f * (*a2 - *a1);
                *a3 = *a2 - *a6;
            } else if (a6da > da2) {
                *a6 = 3.0f * (*a3 - *a1);
                *a2 = *a3 - *a6;
            }
        }
    } else {
        if (extm) {
            *a2 = *a1; *a3 = *a1; *a6 = 0.0f;
        } else {
            float da1 = *a3 - *a2;
            float da2 = da1 * da1;
            float a6da = *a6 * da1;
            if (a6da < -da2) {
                *a6 = 3.0f * (*a2 - *a1);
                *a3 = *a2 - *a6;
            } else if (a6da > da2) {
                *a6 = 3.0f * (*a3 - *a1);
                *a2 = *a3 - *a6;
            }
        }
    }
}

/* ppm_profile (mappm.f90:614-851) for one column; delp(1..km) */
static void ppm_profile_col(float *a4, const float *delp_, int km, int iv, int kord)
{
#define DELP(k) delp_[(k) - 1]
    float *dc = calloc((size_t)km + 2, sizeof(float));
    float *h2 = calloc((size_t)km + 2, sizeof(float));
    float *delq = calloc((size_t)km + 2, sizeof(float));
    float *df2 = calloc((size_t)km + 2, sizeof(float));
    float *d4 = calloc((size_t)km + 2, sizeof(float));
    const int km1 = km - 1;
    int k;

    for (k = 2; k <= km; k++) {
        delq[k - 1] = A4(1, k) - A4(1, k - 1);
        d4[k] = DELP(k - 1) + DELP(k);
    }
    for (k = 2; k <= km1; k++) {
        float c1 = (DELP(k - 1) + 0.5f * DELP(k)) / d4[k + 1];
        float c2 = (DELP(k + 1) + 0.5f * DELP(k)) / d4[k];
        df2[k] = DELP(k) * (c1 * delq[k] + c2 * delq[k - 1]) / (d4[k] + DELP(k + 1));
        dc[k] = fsign(fmin3(fabsf(df2[k]),
                            fmax3(A4(1, k - 1), A4(1, k), A4(1, k + 1)) - A4(1, k),
                            A4(1, k) - fmin3(A4(1, k - 1), A4(1, k), A4(1, k + 1))),
                      df2[k]);
    }
    for (k = 3; k <= km1; k++) {
        float c1 = delq[k - 1] * DELP(k - 1) / d4[k];
        float a1 = d4[k - 1] / (d4[k] + DELP(k - 1));
        float a2 = d4[k + 1] / (d4[k] + DELP(k));
        A4(2, k) = A4(1, k - 1) + c1 + 2.0f / (d4[k - 1] + d4[k + 1]) *
                   (DELP(k) * (c1 * (a1 - a2) + a2 * dc[k - 1]) - DELP(k - 1) * a1 * dc[k]);
    }
    {   /* top */
        float d1 = DELP(1), d2 = DELP(2);
        float qm = (d2 * A4(1, 1) + d1 * A4(1, 2)) / (d1 + d2);
        float dq = 2.0f * (A4(1, 2) - A4(1, 1)) / (d1 + d2);
        float c1 = 4.0f * (A4(2, 3) - qm - d2 * dq) / (d2 * (2.0f * d2 * d2 + d1 * (d2 + 3.0f * d1)));
        float c3 = dq - 0.5f * c1 * (d2 * (5.0f * d1 + d2) - 3.0f * d1 * d1);
        A4(2, 2) = qm - 0.25f * c1 * d1 * d2 * (d2 + 3.0f * d1);
        A4(2, 1) = d1 * (2.0f * c1 * (d1 * d1) - c3) + A4(2, 2);
        A4(2, 2) = FMAX(A4(2, 2), FMIN(A4(1, 1), A4(1, 2)));
        A4(2, 2) = FMIN(A4(2, 2), FMAX(A4(1, 1), A4(1, 2)));
        dc[1] = 0.5f * (A4(2, 2) - A4(1, 1));
    }
    if (iv == 0) {
        A4(2, 1) = FMAX(0.0f, A4(2, 1));
        A4(2, 2) = FMAX(0.0f, A4(2, 2));
    } else if (iv == -1) {
        if (A4(2, 1) * A4(1, 1) <= 0.0f) A4(2, 1) = 0.0f;
    } else if (abs(iv) == 2) {
        A4(2, 1) = A4(1, 1);
        A4(3, 1) = A4(1, 1);
    }
    {   /* bottom */
        float d1 = DELP(km), d2 = DELP(km1);
        float qm = (d2 * A4(1, km) + d1 * A4(1, km1)) / (d1 + d2);
        float dq = 2.0f * (A4(1, km1) - A4(1, km)) / (d1 + d2);
        float c1 = (A4(2, km1) - qm - d2 * dq) / (d2 * (2.0f * d2 * d2 + d1 * (d2 + 3.0f * d1)));
        float c3 = dq - 2.0f * c1 * (d2 * (5.0f * d1 + d2) - 3.0f * d1 * d1);
        A4(2, km) = qm - c1 * d1 * d2 * (d2 + 3.0f * d1);
        A4(3, km) = d1 * (8.0f * c1 * (d1 * d1) - c3) + A4(2, km);
        A4(2, km) = FMAX(A4(2, km), FMIN(A4(1, km), A4(1, km1)));
        A4(2, km) = FMIN(A4(2, km), FMAX(A4(1, km), A4(1, km1)));
        dc[km] = 0.5f * (A4(1, km) - A4(2, km));
    }
    if (iv == 0) {
        A4(2, km) = FMAX(0.0f, A4(2, km));
        A4(3, km) = FMAX(0.0f, A4(3, km));
    } else if (iv < 0) {
        if (A4(1, km) * A4(3, km) <= 0.0f) A4(3, km) = 0.0f;
    }
    for (k = 1; k <= km1; k++) A4(3, k) = A4(2, k + 1);

    for (k = 1; k <= 2; k++) {
        A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k)));
        ppm_limiters_col(dc[k], &A4(1, k), 0);
    }
    if (kord >= 7) {
        const float fac = 1.5f;
        for (k = 2; k <= km1; k++) {
            h2[k] = 2.0f * (dc[k + 1] / DELP(k + 1) - dc[k - 1] / DELP(k - 1)) /
                    (DELP(k) + 0.5f * (DELP(k - 1) + DELP(k + 1))) * (DELP(k) * DELP(k));
        }
        for (k = 3; k <= km - 2; k++) {
            float pmp = 2.0f * dc[k];
            float qmp = A4(1, k) + pmp;
            float lac = A4(1, k) + fac * h2[k - 1] + dc[k];
            A4(3, k) = FMIN(FMAX(A4(3, k), fmin3(A4(1, k), qmp, lac)), fmax3(A4(1, k), qmp, lac));
            qmp = A4(1, k) - pmp;
            lac = A4(1, k) + fac * h2[k + 1] - dc[k];
            A4(2, k) = FMIN(FMAX(A4(2, k), fmin3(A4(1, k), qmp, lac)), fmax3(A4(1, k), qmp, lac));
            A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k)));
            if (iv == 0 && kord >= 6) ppm_limiters_col(dc[k], &A4(1, k), 2);
        }
    } else {
        int lmt = kord - 3;
        lmt = lmt > 0 ? lmt : 0;
        if (iv == 0) lmt = lmt < 2 ? lmt : 2;
        for (k = 3; k <= km - 2; k++) {
            if (kord != 4) A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k)));
            if (kord != 6) ppm_limiters_col(dc[k], &A4(1, k), lmt);
        }
    }
    for (k = km1; k <= km; k++) {
        A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k)));
        ppm_limiters_col(dc[k], &A4(1, k), 0);
    }
    free(dc); free(h2); free(delq); free(df2); free(d4);
#undef DELP
}

/* cs_profile (mappm.f90:132-532) for one column */
static void cs_profile_col(float qs, float *a4, const float *delp_, int km, int iv, int kord)
{
#define DELP(k) delp_[(k) - 1]
    float *gam = calloc((size_t)km + 3, sizeof(float));
    float *q = calloc((size_t)km + 3, sizeof(float));
    unsigned char *extm = calloc((size_t)km + 3, 1);
    unsigned char *ext5 = calloc((size_t)km + 3, 1);
    unsigned char *ext6 = calloc((size_t)km + 3, 1);
    float d4 = 0.0f;
    int k;
    const int akord = abs(kord);

    if (iv == -2) {
        gam[2] = 0.5f;
        q[1] = 1.5f * A4(1, 1);
        for (k = 2; k <= km - 1; k++) {
            float grat = DELP(k - 1) / DELP(k);
            float bet = 2.0f + grat + grat - gam[k];
            q[k] = (3.0f * (A4(1, k - 1) + A4(1, k)) - q[k - 1]) / bet;
            gam[k + 1] = grat / bet;
        }
        {
            float grat = DELP(km - 1) / DELP(km);
            q[km] = (3.0f * (A4(1, km - 1) + A4(1, km)) - grat * qs - q[km - 1]) /
                    (2.0f + grat + grat - gam[km]);
            q[km + 1] = qs;
        }
        for (k = km - 1; k >= 1; k--) q[k] = q[k] - gam[k + 1] * q[k + 1];
    } else {
        {
            float grat = DELP(2) / DELP(1);
            float bet = grat * (grat + 0.5f);
            q[1] = ((grat + grat) * (grat + 1.0f) * A4(1, 1) + A4(1, 2)) / bet;
            gam[1] = (1.0f + grat * (grat + 1.5f)) / bet;
        }
        for (k = 2; k <= km; k++) {
            d4 = DELP(k - 1) / DELP(k);
            float bet = 2.0f + d4 + d4 - gam[k - 1];
            q[k] = (3.0f * (A4(1, k - 1) + d4 * A4(1, k)) - q[k - 1]) / bet;
            gam[k] = d4 / bet;
        }
        {
            float a_bot = 1.0f + d4 * (d4 + 1.5f);
            q[km + 1] = (2.0f * d4 * (d4 + 1.0f) * A4(1, km) + A4(1, km - 1) - a_bot * q[km]) /
                        (d4 * (d4 + 0.5f) - a_bot * gam[km]);
        }
        for (k = km; k >= 1; k--) q[k] = q[k] - gam[k] * q[k + 1];
    }

    if (akord > 16) {
        for (k = 1; k <= km; k++) {
            A4(2, k) = q[k];
            A4(3, k) = q[k + 1];
            A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k)));
        }
        goto done;
    }

    q[2] = FMIN(q[2], FMAX(A4(1, 1), A4(1, 2)));
    q[2] = FMAX(q[2], FMIN(A4(1, 1), A4(1, 2)));
    for (k = 2; k <= km; k++) gam[k] = A4(1, k) - A4(1, k - 1);
    for (k = 3; k <= km - 1; k++) {
        if (gam[k - 1] * gam[k + 1] > 0.0f) {
            q[k] = FMIN(q[k], FMAX(A4(1, k - 1), A4(1, k)));
            q[k] = FMAX(q[k], FMIN(A4(1, k - 1), A4(1, k)));
        } else if (gam[k - 1] > 0.0f) {
            q[k] = FMAX(q[k], FMIN(A4(1, k - 1), A4(1, k)));
        } else {
            q[k] = FMIN(q[k], FMAX(A4(1, k - 1), A4(1, k)));
            if (iv == 0) q[k] = FMAX(0.0f, q[k]);
        }
    }
    q[km] = FMIN(q[km], FMAX(A4(1, km - 1), A4(1, km)));
    q[km] = FMAX(q[km], FMIN(A4(1, km - 1), A4(1, km)));
    for (k = 1; k <= km; k++) {
        A4(2, k) = q[k];
        A4(3, k) = q[k + 1];
    }
    for (k = 1; k <= km; k++) {
        if (k == 1 || k == km)
            extm[k] = (A4(2, k) - A4(1, k)) * (A4(3, k) - A4(1, k)) > 0.0f;
        else
            extm[k] = gam[k] * gam[k + 1] < 0.0f;
        if (akord > 9) {
            float x0 = 2.0f * A4(1, k) - (A4(2, k) + A4(3, k));
            float x1 = fabsf(A4(2, k) - A4(3, k));
            A4(4, k) = 3.0f * x0;
            ext5[k] = fabsf(x0) > x1;
            ext6[k] = fabsf(A4(4, k)) > x1;
        }
    }

    if (iv == 0) {
        A4(2, 1) = FMAX(0.0f, A4(2, 1));
    } else if (iv == -1) {
        if (A4(2, 1) * A4(1, 1) <= 0.0f) A4(2, 1) = 0.0f;
    } else if (iv == 2) {
        A4(2, 1) = A4(1, 1);
        A4(3, 1) = A4(1, 1);
        A4(4, 1) = 0.0f;
    }
    if (iv != 2) {
        A4(4, 1) = 3.0f * (2.0f * A4(1, 1) - (A4(2, 1) + A4(3, 1)));
        cs_limiters_col(extm[1], &A4(1, 1), 1);
    }
    A4(4, 2) = 3.0f * (2.0f * A4(1, 2) - (A4(2, 2) + A4(3, 2)));
    cs_limiters_col(extm[2], &A4(1, 2), 2);

#define HUYNH_L(k) do { \
        float pmp_1 = A4(1, k) - 2.0f * gam[(k) + 1]; \
        float lac_1 = pmp_1 + 1.5f * gam[(k) + 2]; \
        A4(2, k) = FMIN(FMAX(A4(2, k), fmin3(A4(1, k), pmp_1, lac_1)), fmax3(A4(1, k), pmp_1, lac_1)); \
    } while (0)
#define HUYNH_R(k) do { \
        float pmp_2 = A4(1, k) + 2.0f * gam[k]; \
        float lac_2 = pmp_2 - 1.5f * gam[(k) - 1]; \
        A4(3, k) = FMIN(FMAX(A4(3, k), fmin3(A4(1, k), pmp_2, lac_2)), fmax3(A4(1, k), pmp_2, lac_2)); \
    } while (0)
#define SET_A6(k) (A4(4, k) = 3.0f * (2.0f * A4(1, k) - (A4(2, k) + A4(3, k))))
#define SET_A6_ALT(k) (A4(4, k) = 6.0f * A4(1, k) - 3.0f * (A4(2, k) + A4(3, k)))
#define FLAT(k) do { A4(2, k) = A4(1, k); A4(3, k) = A4(1, k); } while (0)

    for (k = 3; k <= km - 2; k++) {
        if (akord < 9) {
            HUYNH_L(k);
            HUYNH_R(k);
            SET_A6(k);
        } else if (akord == 9) {
            if (extm[k] && extm[k - 1]) {
                FLAT(k); A4(4, k) = 0.0f;
            } else if (extm[k] && extm[k + 1]) {
                FLAT(k); A4(4, k) = 0.0f;
            } else {
                SET_A6_ALT(k);
                if (fabsf(A4(4, k)) > fabsf(A4(2, k) - A4(3, k))) {
                    HUYNH_L(k);
                    HUYNH_R(k);
                    SET_A6_ALT(k);
                }
            }
        } else if (akord == 10) {
            if (ext5[k]) {
                if (ext5[k - 1] || ext5[k + 1]) {
                    FLAT(k);
                } else if (ext6[k - 1] || ext6[k + 1]) {
                    HUYNH_L(k);
                    HUYNH_R(k);
                }
            } else if (ext6[k]) {
                if (ext5[k - 1] || ext5[k + 1]) {
                    HUYNH_L(k);
                    HUYNH_R(k);
                }
            }
            SET_A6(k);
        } else if (akord == 12) {
            if (extm[k]) {
                FLAT(k); A4(4, k) = 0.0f;
            } else {
                SET_A6_ALT(k);
                if (fabsf(A4(4, k)) > fabsf(A4(2, k) - A4(3, k))) {
                    HUYNH_L(k);
                    HUYNH_R(k);
                    SET_A6_ALT(k);
                }
            }
        } else if (akord == 13) {
            if (ext6[k]) {
                if (ext6[k - 1] && ext6[k + 1]) FLAT(k);
            }
            SET_A6(k);
        } else if (akord == 14) {
            SET_A6(k);
        } else if (akord == 15) {
            if (ext5[k]) {
                if (ext5[k - 1] || ext5[k + 1]) FLAT(k);
            } else if (ext6[k]) {
                HUYNH_L(k);
                HUYNH_R(k);
            }
            SET_A6(k);
        } else if (akord == 16) {
            if (ext5[k]) {
                if (ext5[k - 1] || ext5[k + 1]) {
                    FLAT(k);
                } else if (ext6[k - 1] || ext6[k + 1]) {
                    HUYNH_L(k);
                    HUYNH_R(k);
                }
            }
            SET_A6(k);
        } else { /* kord = 11 */
            if (ext5[k] && (ext5[k - 1] || ext5[k + 1])) {
                FLAT(k); A4(4, k) = 0.0f;
            } else {
                SET_A6(k);
            }
        }
        if (iv == 0) cs_limiters_col(extm[k], &A4(1, k), 0);
    }
    if (iv == 0) {
        A4(3, km) = FMAX(0.0f, A4(3, km));
    } else if (iv == -1) {
        if (A4(3, km) * A4(1, km) <= 0.0f) A4(3, km) = 0.0f;
    }
    for (k = km - 1; k <= km; k++) {
        SET_A6(k);
        if (k == km - 1) cs_limiters_col(extm[k], &A4(1, k), 2);
        if (k == km) cs_limiters_col(extm[k], &A4(1, k), 1);
    }
done:
    free(gam); free(q); free(extm); free(ext5); free(ext6);
#undef DELP
}

/*
 * mappm (mappm.f90:10-126).  pe1[(km+1)*ncol], q1[km*ncol], pe2[(kn+1)*ncol],
 * q2[kn*ncol], all column-fastest.  Returns 0, or -1 for unsupported sizes.
 */
int oracle_mappm(int km, const float *pe1, const float *q1, int kn, const float *pe2,
                 float *q2, long ncol, int iv, int kord)
{
    const float r3 = 1.0f / 3.0f, r23 = 2.0f / 3.0f;
    if (km < 4 || kn < 1 || ncol < 0) return -1;
    float *a4 = malloc(sizeof(float) * 4 * (size_t)km);
    float *dp1 = malloc(sizeof(float) * (size_t)km);
    float *p1 = malloc(sizeof(float) * ((size_t)km + 1));
    float *p2 = malloc(sizeof(float) * ((size_t)kn + 1));
    for (long i = 0; i < ncol; i++) {
#define PE1(k) p1[(k) - 1]
#define PE2(k) p2[(k) - 1]
#define DP1(k) dp1[(k) - 1]
#define Q1(k) A4(1, k)
        for (int k = 0; k <= km; k++) p1[k] = pe1[(size_t)k * ncol + i];
        for (int k = 0; k <= kn; k++) p2[k] = pe2[(size_t)k * ncol + i];
        for (int k = 1; k <= km; k++) {
            DP1(k) = PE1(k + 1) - PE1(k);
            A4(1, k) = q1[(size_t)(k - 1) * ncol + i];
            A4(2, k) = A4(3, k) = A4(4, k) = 0.0f;
        }
        if (kord > 7)
            cs_profile_col(0.0f, a4, dp1, km, iv, kord);
        else
            ppm_profile_col(a4, dp1, km, iv, kord);

        int k0 = 1;
        for (int k = 1; k <= kn; k++) {
            float out;
            if (PE2(k) <= PE1(1)) {
                out = Q1(1);
            } else if (PE2(k) >= PE1(km + 1)) {
                out = Q1(km);
            } else {
                int L, found = 0, k1 = 0;
                float qsum = 0.0f, dpsum = 0.0f;
                out = NAN;
                for (L = k0; L <= km; L++) {
                    if (PE2(k) >= PE1(L) && PE2(k) <= PE1(L + 1)) {
                        k0 = L;
                        float pl = (PE2(k) - PE1(L)) / DP1(L);
                        if (PE2(k + 1) <= PE1(L + 1)) {
                            float pr = (PE2(k + 1) - PE1(L)) / DP1(L);
                            float tt = r3 * (pr * (pr + pl) + pl * pl);
                            out = A4(2, L) + 0.5f * (A4(4, L) + A4(3, L) - A4(2, L)) * (pr + pl) -
                                  A4(4, L) * tt;
                            found = 2;
                        } else {
                            float delp = PE1(L + 1) - PE2(k);
                            float tt = r3 * (1.0f + pl * (1.0f + pl));
                            qsum = delp * (A4(2, L) + 0.5f * (A4(4, L) + A4(3, L) - A4(2, L)) * (1.0f + pl) -
                                           A4(4, L) * tt);
                            dpsum = delp;
                            k1 = L + 1;
                            found = 1;
                        }
                        break;
                    }
                }
                if (found == 1) {
                    int done = 0;
                    for (L = k1; L <= km; L++) {
                        if (PE2(k + 1) > PE1(L + 1)) {
                            qsum = qsum + DP1(L) * Q1(L);
                            dpsum = dpsum + DP1(L);
                        } else {
                            float delp = PE2(k + 1) - PE1(L);
                            float esl = delp / DP1(L);
                            qsum = qsum + delp * (A4(2, L) + 0.5f * esl *
                                                  (A4(3, L) - A4(2, L) + A4(4, L) * (1.0f - r23 * esl)));
                            dpsum = dpsum + delp;
                            k0 = L;
                            done = 1;
                            break;
                        }
                    }
                    if (!done) {
                        float delp = PE2(k + 1) - PE1(km + 1);
                        if (delp > 0.0f) {
                            qsum = qsum + delp * Q1(km);
                            dpsum = dpsum + delp;
                        }
                    }
                    out = qsum / dpsum;
                }
                /* found == 0: search failed (non-monotone pe1) -> UB upstream; NaN here */
            }
            q2[(size_t)(k - 1) * ncol + i] = out;
        }
#undef PE1
#undef PE2
#undef DP1
#undef Q1
    }
    free(a4); free(dp1); free(p1); free(p2);
    return 0;
}
