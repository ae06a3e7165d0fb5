// fv3net_amd — shared plumbing for the HIP sources: error capture for the C ABI,
// column-layout addressing, launch checks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/fv3net_amd.h"

// Experiment knobs (FV3_EXP_* / FV3_B3_EXP_*) replace parts of a kernel to price them
// (no MFMAs, no loads, ...): their results are invalid by construction.  They compile
// only in the tools/ variant builds (tools/build_*variant.sh, which define
// FV3_EXPERIMENT_BUILD and write tools/variants/, never fv3net_amd/_lib/).  The product
// library is built by fv3net_amd/build.py with FV3_PRODUCT_BUILD, and any knob there is
// a compile error.  tests/test_build_flags.py checks that every knob named in csrc/ is
// listed here.
#if defined(FV3_EXP_L1_WEIGHTS) || defined(FV3_EXP_NOINLOAD) || defined(FV3_EXP_NOMFMA) ||         \
    defined(FV3_EXP_NONORM) || defined(FV3_EXP_NOPPM) || defined(FV3_EXP_NOPROFILE) ||             \
    defined(FV3_EXP_NOREMAP) || defined(FV3_EXP_NOSTAGE) || defined(FV3_EXP_NOSTORE) ||            \
    defined(FV3_EXP_NOWLOAD) || defined(FV3_B3_EXP_NOFRAG) || defined(FV3_B3_EXP_NOIN) ||          \
    defined(FV3_B3_EXP_NOMFMA) || defined(FV3_B3_EXP_NOOUT) || defined(FV3_B3_EXP_NOSTAGE) ||      \
    defined(FV3_B3_EXP_NORES) || defined(FV3_B3_EXP_NOEPI) || defined(FV3_B3_TRACE) ||             \
    defined(FV3_EXPERIMENT_BUILD)
#define FV3_EXPERIMENT_KNOBS 1
#ifdef FV3_PRODUCT_BUILD
#error "experiment knobs (results invalid) in the product build"
#endif
#endif

// Variant kernels: alternatives that only an A/B knob selects (FV3_VARIANTS=1 plus the
// knob), never the product's own heuristics -- other register targets, load distances,
// register-tail depths, LDS scratch.  Every one gives the product kernel's bits; they
// are instantiated in the tools/ variant builds only, so the product library holds the
// kernels its host code can pick and nothing else (a knob naming an absent variant is
// ignored there; tests that pin a variant skip on the product build).
#ifdef FV3_PRODUCT_BUILD
#define FV3_VARIANT_KERNELS 0
#else
#define FV3_VARIANT_KERNELS 1
#endif

namespace fv3 {

void set_error(const char* fmt, ...);
void clear_error();

// A kernel-variant selector (A/B builds' knobs and the tests that pin every variant
// bit-identical): the value of environment variable `name`, but only while FV3_VARIANTS=1
// is set; otherwise NULL, so the product path is the same under any environment.
const char* variant_env(const char* name);

#define FV3_REQUIRE(cond, ...)                     \
    do {                                           \
        if (!(cond)) {                             \
            ::fv3::set_error(__VA_ARGS__);         \
            return FV3_ERR_INVALID;                \
        }                                          \
    } while (0)

#define FV3_REQUIRE_CODE(code, cond, ...)          \
    do {                                           \
        if (!(cond)) {                             \
            ::fv3::set_error(__VA_ARGS__);         \
            return (code);                         \
        }                                          \
    } while (0)

#define FV3_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::fv3::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),    \
                             __FILE__, __LINE__);                                      \
            return FV3_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

#define FV3_LAUNCH_CHECK() FV3_HIP(hipGetLastError())

// Device-side view of one column of one array under an fv3_layout.
struct ColAddr {
    int64_t ld;
    int64_t off;  // (c / ncol_blk) * blk_stride + (c % ncol_blk)
};

__device__ __forceinline__ int64_t col_offset(const fv3_layout& l, int64_t c)
{
    if (l.ncol_blk <= 0 || c < l.ncol_blk) return c;  // single block: no division
    const int64_t b = c / l.ncol_blk;
    return b * l.blk_stride + (c - b * l.ncol_blk);
}

inline bool layout_ok(const fv3_layout& l, int64_t ncol)
{
    if (l.ld <= 0) return false;
    if (l.ncol_blk <= 0) return false;
    if (ncol > l.ncol_blk && l.blk_stride <= 0) return false;
    return l.ld >= l.ncol_blk || l.ld == 0;
}

inline fv3_layout plain_layout(int64_t ncol) { return fv3_layout{ncol, ncol, 0}; }

// Workgroups are dealt round-robin over the 8 XCDs (each with its own L2): block b runs
// on XCD b % 8.  This bijection of [0, nblocks) gives the blocks of one XCD consecutive
// logical ids, so neighbouring tiles that share cache lines land in the same L2.
constexpr unsigned kNumXcd = 8;
__device__ __forceinline__ unsigned xcd_swizzle(unsigned b, unsigned nblocks)
{
    const unsigned r = b % kNumXcd, q = b / kNumXcd;
    const unsigned per = nblocks / kNumXcd, rem = nblocks % kNumXcd;
    return r * per + (r < rem ? r : rem) + q;
}

}  // namespace fv3
