// What the HIP runtime reports for overlapping host registrations: the
// round-4 registration pattern (whole arrays, start-address check only) on two arrays that
// share a page, and the runtime's view of memory after a pageable copy.  Queries only:
// no copy touches memory after any part of it was unregistered.
//   hipcc --offload-arch=gfx950 -O1 tools/host_pin_probe.cpp -o tools/host_pin_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

static const char* kind(const void* p)
{
    hipPointerAttribute_t at{};
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return "error(unregistered)";
    }
    switch (at.type) {
    case hipMemoryTypeUnregistered: return "unregistered";
    case hipMemoryTypeHost: return "host(page-locked)";
    case hipMemoryTypeDevice: return "device";
    default: return "other";
    }
}

static void q(const char* what, const void* p)
{
    void* d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, const_cast<void*>(p), 0);
    if (e != hipSuccess) (void)hipGetLastError();
    printf("%-58s %-20s devptr=%s\n", what, kind(p), e == hipSuccess ? "yes" : "no");
}

int main()
{
    const size_t MB = 1 << 20;
    char* raw = (char*)malloc(8 * MB);
    memset(raw, 1, 8 * MB);
    char* a = raw + 4096 - ((uintptr_t)raw % 4096) + 100;  // an array starting 100 B into a page
    char* b = a + MB;                                       // its neighbour: shares a's last page
    void* dev = nullptr;
    if (hipMalloc(&dev, 4 * MB) != hipSuccess) return 1;

    q("fresh heap memory, a", a);
    hipMemcpy(dev, a, 2 * MB, hipMemcpyHostToDevice);  // pageable: the runtime's own path
    q("after a pageable 2 MB H2D from a: a", a);
    q("  a + 1 MB", a + MB);

    int ra = (int)hipHostRegister(a, MB, hipHostRegisterDefault);
    (void)hipGetLastError();
    printf("hipHostRegister(a, 1 MB) = %d\n", ra);
    q("  a", a);
    q("  a + 1 MB - 1 (a's last byte)", a + MB - 1);
    q("  b (first byte of b, in a's last page)", b);
    q("  b + 4096 (b's next page)", b + 4096);

    int rb = (int)hipHostRegister(b, MB, hipHostRegisterDefault);
    (void)hipGetLastError();
    printf("hipHostRegister(b, 1 MB) [shares a's last page] = %d\n", rb);
    q("  b", b);

    int ra2 = (int)hipHostRegister(a, MB, hipHostRegisterDefault);
    (void)hipGetLastError();
    printf("hipHostRegister(a, 1 MB) again = %d\n", ra2);

    int ua = (int)hipHostUnregister(a);
    (void)hipGetLastError();
    printf("hipHostUnregister(a) = %d\n", ua);
    q("  a", a);
    q("  b (its registration still there?)", b);
    if (ra2 == 0) {
        int ua2 = (int)hipHostUnregister(a);
        (void)hipGetLastError();
        printf("hipHostUnregister(a) second = %d\n", ua2);
        q("  a", a);
    }
    if (rb == 0) {
        int ub = (int)hipHostUnregister(b);
        (void)hipGetLastError();
        printf("hipHostUnregister(b) = %d\n", ub);
        q("  b", b);
    }
    // the page-exclusive interior (csrc/host_memory.cpp) of a and of b
    char* sa = (char*)(((uintptr_t)a / 4096 + 1) * 4096);
    char* ea = (char*)(((uintptr_t)(a + MB)) / 4096 * 4096);
    char* sb = (char*)(((uintptr_t)b / 4096 + 1) * 4096);
    char* eb = (char*)(((uintptr_t)(b + MB)) / 4096 * 4096);
    printf("interiors: a [%+ld, %+ld) b [%+ld, %+ld) relative to a; disjoint=%d\n", (long)(sa - a), (long)(ea - a),
           (long)(sb - a), (long)(eb - a), (int)(ea <= sb));
    int ia = (int)hipHostRegister(sa, ea - sa, hipHostRegisterDefault);
    int ib = (int)hipHostRegister(sb, eb - sb, hipHostRegisterDefault);
    (void)hipGetLastError();
    printf("hipHostRegister(interior a) = %d, (interior b) = %d\n", ia, ib);
    q("  a (pageable head)", a);
    q("  a's first interior byte", sa);
    q("  b (in the shared page, outside both)", b);
    if (ia == 0) hipHostUnregister(sa);
    if (ib == 0) hipHostUnregister(sb);
    (void)hipGetLastError();
    hipFree(dev);
    free(raw);
    printf("probe done\n");
    return 0;
}
