// fv3net_amd — page-locking the caller's host arrays for the drop-in call's DMA.
//
// The reference predicts on host arrays (external/fv3fit/fv3fit/keras/_models/shared/
// pure_keras.py:98-118): every call crosses PCIe both ways.  Copies from pageable memory
// go through the runtime's bounce buffer, or through our pinned staging plus a host
// memcpy (fv3net_amd/transfer.py).  Registering the caller's own pages instead lets the
// copy engines read and write them directly; on MI355X registering and unregistering the
// four arrays of one rank's (79, 48, 48) call costs ~14 us against ~50 us of host memcpy
// (tools/h2h_register.py).
#include "common.h"

extern "C" int fv3_host_register(void* ptr, size_t bytes)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ptr && bytes, "host_register: NULL pointer or zero size");
    // Already page-locked (hipHostMalloc, or registered by the caller or an enclosing
    // call): leave it to its owner.  The runtime accepts a second registration of the
    // same range, and releasing it here could unpin memory the owner still relies on.
    hipPointerAttribute_t at{};
    const hipError_t q = hipPointerGetAttributes(&at, ptr);
    if (q != hipSuccess) (void)hipGetLastError();
    if (q == hipSuccess && at.type != hipMemoryTypeUnregistered) {
        set_error("host_register: memory already page-locked or not host memory");
        return FV3_ERR_UNSUPPORTED;
    }
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
        // already registered (by the caller, or pages shared with another array) or not
        // lockable: the caller copies through staging instead.  The runtime's sticky
        // last-error is cleared so that a later launch check does not report it.
        (void)hipGetLastError();
        set_error("hipHostRegister: %s", hipGetErrorString(e));
        return FV3_ERR_UNSUPPORTED;
    }
    return FV3_OK;
}

extern "C" int fv3_host_unregister(void* ptr)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ptr, "host_unregister: NULL pointer");
    FV3_HIP(hipHostUnregister(ptr));
    return FV3_OK;
}
