// fv3net_amd — the fused pressure-level coarsen kernels under the tolerance-contract
// arithmetic (mappm_core.h, FV3_FAST_ARITH), as namespace fv3::fast.  The C ABI in
// coarsen.hip dispatches here for FV3_ARITH_FAST.
#define FV3_FAST_ARITH 1
#include "coarsen.hip"
