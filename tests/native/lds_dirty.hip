// Test-only (tests/test_lds_handoff.py): fill every CU's LDS with a chosen 32-bit pattern,
// so that a kernel launched next which read LDS before writing it (a missing barrier on a
// cross-wave hand-off) would pick the pattern up.  Built by __graft_entry__.build() into
// tests/_build/liblds_dirty.so; never part of the product library.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void lds_fill_kernel(uint32_t pattern, int words, uint32_t* sink)
{
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < words; i += kThreads) lds[i] = pattern ^ (uint32_t)(i & 0);
    __syncthreads();
    // one read back, so the stores are not optimised away; the sink is written only if
    // the pattern did not land (never, in practice)
    if (lds[(threadIdx.x * 97) % words] != pattern) sink[blockIdx.x] = 1u;
}

}  // namespace

// every CU's LDS (160 KiB on gfx950) filled with `pattern`: 8 blocks per CU of the
// largest dynamic LDS one block may hold, on `stream`; 0 on success
extern "C" int lds_dirty(uint32_t pattern, void* sink, void* stream)
{
    const int bytes = 160 * 1024;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(lds_fill_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
        return 1;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 2;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 3;
    hipLaunchKernelGGL(lds_fill_kernel, dim3(8 * cus), dim3(kThreads), bytes, (hipStream_t)stream, pattern,
                       bytes / 4, static_cast<uint32_t*>(sink));
    return hipGetLastError() == hipSuccess ? 0 : 4;
}
