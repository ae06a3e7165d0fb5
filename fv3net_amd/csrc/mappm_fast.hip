// fv3net_amd — mappm's kernels under the tolerance-contract arithmetic (mappm_core.h,
// FV3_FAST_ARITH: reciprocal divisions, FMA contraction, hardware MAX / MIN), as
// namespace fv3::fast.  The C ABI in mappm.hip dispatches here for FV3_ARITH_FAST.
#define FV3_FAST_ARITH 1
#include "mappm.hip"
