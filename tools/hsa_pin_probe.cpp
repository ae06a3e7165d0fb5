// Whether the HIP runtime keeps host pages it pinned for a pageable copy, and what a
// hipHostRegister / hipHostUnregister of some of those pages does to that pin (DESIGN.md
// §3.7).  ROCr's own view of each address (hsa_amd_pointer_info): queries only, and no
// copy is issued after any registration was released.
//   hipcc --offload-arch=gfx950 -O1 tools/hsa_pin_probe.cpp -o tools/hsa_pin_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

static char* g_ref = nullptr;

static void info(const char* what, const void* p)
{
    hsa_amd_pointer_info_t in{};
    in.size = sizeof(in);
    const hsa_status_t s = hsa_amd_pointer_info(const_cast<void*>(p), &in, nullptr, nullptr, nullptr);
    const char* t = in.type == HSA_EXT_POINTER_TYPE_UNKNOWN ? "unknown"
                    : in.type == HSA_EXT_POINTER_TYPE_LOCKED ? "LOCKED"
                    : in.type == HSA_EXT_POINTER_TYPE_HSA    ? "hsa"
                                                              : "other";
    if (in.type == HSA_EXT_POINTER_TYPE_UNKNOWN)
        printf("%-52s st=%d %-8s\n", what, (int)s, t);
    else
        printf("%-52s st=%d %-8s host_base=ref%+ld size=%zu agent_base=%p registered=%d\n", what, (int)s, t,
               (long)((char*)in.hostBaseAddress - g_ref), in.sizeInBytes, in.agentBaseAddress, (int)in.registered);
}

int main()
{
    hipSetDevice(0);
    hsa_init();
    const size_t MB = 1 << 20;
    void* dev = nullptr;
    if (hipMalloc(&dev, 64 * MB) != hipSuccess) return 1;
    char* raw = (char*)malloc(200 * MB);
    memset(raw, 3, 200 * MB);
    g_ref = raw;
    printf("ref = %p (malloc, 200 MB)\n", raw);
    // pageable copies of several sizes, each from its own region
    const size_t sizes[] = {64 << 10, 256 << 10, MB, 8 * MB, 48 * MB};
    char* regions[5];
    char* cur = raw + 100;
    for (int i = 0; i < 5; ++i) {
        regions[i] = cur;
        cur += sizes[i] + 3 * MB;
        char what[96];
        snprintf(what, sizeof(what), "before any copy: region %d (%zu KiB)", i, sizes[i] >> 10);
        info(what, regions[i]);
        hipMemcpy(dev, regions[i], sizes[i], hipMemcpyHostToDevice);
        snprintf(what, sizeof(what), "after pageable H2D of region %d", i);
        info(what, regions[i]);
        snprintf(what, sizeof(what), "  its middle byte");
        info(what, regions[i] + sizes[i] / 2);
    }
    hipDeviceSynchronize();
    printf("-- after hipDeviceSynchronize\n");
    for (int i = 0; i < 5; ++i) {
        char what[96];
        snprintf(what, sizeof(what), "region %d", i);
        info(what, regions[i]);
    }
    // a D2H pageable copy into region 3
    hipMemcpy(regions[3], dev, sizes[3], hipMemcpyDeviceToHost);
    info("after pageable D2H into region 3", regions[3]);
    // register the page-exclusive interior of region 3 and of region 4
    for (int i = 3; i < 5; ++i) {
        char* s = (char*)(((uintptr_t)regions[i] / 4096 + 1) * 4096);
        char* e = (char*)(((uintptr_t)(regions[i] + sizes[i])) / 4096 * 4096);
        const int r = (int)hipHostRegister(s, e - s, hipHostRegisterDefault);
        (void)hipGetLastError();
        printf("hipHostRegister(interior of region %d, %zu B) = %d\n", i, (size_t)(e - s), r);
        info("  the interior's first byte", s);
        info("  the region's first byte (pageable head)", regions[i]);
        const int u = (int)hipHostUnregister(s);
        (void)hipGetLastError();
        printf("hipHostUnregister(interior of region %d) = %d\n", i, u);
        info("  the interior's first byte", s);
        info("  the region's first byte", regions[i]);
    }
    // the same with the round-4 pattern: the whole region
    {
        const int r = (int)hipHostRegister(regions[2], sizes[2], hipHostRegisterDefault);
        (void)hipGetLastError();
        printf("hipHostRegister(whole region 2) = %d\n", r);
        info("  region 2", regions[2]);
        const int u = (int)hipHostUnregister(regions[2]);
        (void)hipGetLastError();
        printf("hipHostUnregister(whole region 2) = %d\n", u);
        info("  region 2", regions[2]);
    }
    hipFree(dev);
    printf("probe done\n");
    return 0;
}
