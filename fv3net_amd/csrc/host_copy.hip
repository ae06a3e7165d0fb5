// fv3net_amd — host <-> device copies of the drop-in call, and device-to-host copies as a
// kernel storing into the library's page-locked arena (host_memory.cpp).
//
// The pipelined host call (DenseColumnModel.forward_host) overlaps the
// inputs' host-to-device copies with the outputs' device-to-host copies.  Issued as two
// copy-engine streams, the two directions overlapped in some runs and ran nearly in
// sequence in others (the runtime's engine choice).  Here the out-copy is a kernel on the
// compute stream that stores straight into the arena's page-locked pages over PCIe (16-byte
// vector stores), leaving the copy engines to the in-copies.
#include <algorithm>

#include "common.h"
#include "host_memory.h"

namespace fv3 {
namespace {

__global__ __launch_bounds__(256) void copy_to_host_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                           int64_t n16)
{
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void copy_tail_kernel(const unsigned char* __restrict__ src,
                                                       unsigned char* __restrict__ dst, int n)
{
    if ((int)threadIdx.x < n) dst[threadIdx.x] = src[threadIdx.x];
}

// Host memory page-locked by someone other than the library (torch pin_memory, a
// hipHostRegister'ed buffer): the runtime's copy from / to it is a true asynchronous DMA,
// unlike the staged pageable copy.  The copies below promise completion on return for
// every non-arena host buffer, so those are waited for explicitly.
bool foreign_page_locked(const void* host, size_t bytes)
{
    if (hostmem::inside((uintptr_t)host, bytes)) return false;  // the arena: asynchronous by contract
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, host) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory is unknown to the runtime
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

}  // namespace
}  // namespace fv3

extern "C" int fv3_host_copy(void* dst, const void* src, size_t bytes, int kind, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(dst && src, "host_copy: NULL pointer");
    FV3_REQUIRE(kind == 1 || kind == 2, "host_copy: kind %d (1: host to device, 2: device to host)", kind);
    if (!bytes) return FV3_OK;
    // arena memory: asynchronous DMA; pageable memory: the runtime's staged copy, which it
    // completes before returning; memory page-locked elsewhere: waited for here, so the
    // caller's buffer is free on return in both of the latter cases
    FV3_HIP(hipMemcpyAsync(dst, src, bytes, kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    if (foreign_page_locked(kind == 1 ? src : dst, bytes)) FV3_HIP(hipStreamSynchronize((hipStream_t)stream));
    return FV3_OK;
}

extern "C" int fv3_copy_to_host(void* host_dst, const void* dev_src, size_t bytes, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(host_dst && dev_src, "copy_to_host: NULL pointer");
    if (!bytes) return FV3_OK;
    // only the library's own page-locked memory, which outlives the kernel (an arena block
    // returns to the cache only when no array refers to it)
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, hostmem::inside((uintptr_t)host_dst, bytes),
                     "copy_to_host: host range not inside one fv3_host_alloc block");
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, host_dst, 0);
    if (e != hipSuccess || !d) {
        (void)hipGetLastError();
        set_error("copy_to_host: host memory not mapped (%s)", hipGetErrorString(e));
        return FV3_ERR_UNSUPPORTED;
    }
    FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, ((uintptr_t)d % 16) == 0 && ((uintptr_t)dev_src % 16) == 0,
                     "copy_to_host: 16-byte aligned buffers only");
    hipStream_t s = (hipStream_t)stream;
    const int64_t n16 = (int64_t)(bytes / 16);
    if (n16) {
        const int64_t blocks = std::min<int64_t>((n16 + 255) / 256, 4096);
        hipLaunchKernelGGL(copy_to_host_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                           reinterpret_cast<const uint4*>(dev_src), reinterpret_cast<uint4*>(d), n16);
        FV3_LAUNCH_CHECK();
    }
    const int tail = (int)(bytes % 16);
    if (tail) {
        hipLaunchKernelGGL(copy_tail_kernel, dim3(1), dim3(64), 0, s,
                           reinterpret_cast<const unsigned char*>(dev_src) + 16 * n16,
                           reinterpret_cast<unsigned char*>(d) + 16 * n16, tail);
        FV3_LAUNCH_CHECK();
    }
    return FV3_OK;
}

// A pitched (2-D) copy between host and device on `stream`: `height` rows of `width`
// bytes, rows `spitch` / `dpitch` bytes apart.  A band of columns of a level-leading
// [level][column] array is such a copy, one row per level (the pipelined host call over
// column bands, bench.py predict + mappm host-to-host).  kind 1: host to device, 2:
// device to host.  Asynchronous when the host rows are arena memory (fv3_host_alloc);
// otherwise complete on return (the runtime's pageable copy, or waited for when the rows
// are page-locked by someone else).
extern "C" int fv3_copy_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                           int kind, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(dst && src, "copy_2d: NULL pointer");
    FV3_REQUIRE(kind == 1 || kind == 2, "copy_2d: kind %d (1: host to device, 2: device to host)", kind);
    FV3_REQUIRE(width <= dpitch && width <= spitch, "copy_2d: row wider than its pitch");
    if (!width || !height) return FV3_OK;
    FV3_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height,
                             kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, (hipStream_t)stream));
    const size_t span = (height - 1) * (kind == 1 ? spitch : dpitch) + width;
    if (foreign_page_locked(kind == 1 ? src : dst, span)) FV3_HIP(hipStreamSynchronize((hipStream_t)stream));
    return FV3_OK;
}
