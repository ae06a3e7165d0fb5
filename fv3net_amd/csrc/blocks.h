// fv3net_amd — f x f block sums in numpy's order (shared by the coarse-graining kernels).
//
// xarray's coarsen().sum() (skipna) on a (.., Y, f, X, f) C-order reshape is numpy's
// nansum over the two f axes: each x-row of f values is reduced on its own (sequential
// for f < 8, numpy's 8-way pairwise kernel for f == 8), the rows are then added in y
// order; NaN terms count as 0.  Used by csrc/coarsen.hip (masked and delp sums) and
// csrc/restarts.hip (plain weighted_block_average, coarsen.py:183-218).
#pragma once

#include <hip/hip_runtime.h>

namespace fv3 {

template <typename T>
__device__ __forceinline__ T nan0(T x) { return x != x ? T(0) : x; }  // nansum: NaN terms count as 0

// val(j) is element j = dy*f + dx of the block
template <typename T, typename V>
__device__ __forceinline__ T block_sum(int f, V val)
{
    auto row = [&](int r) -> T {
        const int b = r * f;
        if (f == 8)
            return ((val(b) + val(b + 1)) + (val(b + 2) + val(b + 3))) +
                   ((val(b + 4) + val(b + 5)) + (val(b + 6) + val(b + 7)));
        T s = val(b);
        for (int c = 1; c < f; ++c) s = s + val(b + c);
        return s;
    };
    T acc = row(0);
    for (int r = 1; r < f; ++r) acc = acc + row(r);
    return acc;
}

}  // namespace fv3
