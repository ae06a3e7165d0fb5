// fv3net_amd — page-locked host memory for the drop-in call's PCIe crossings: an arena of
// blocks this library allocates itself, and nothing else.
//
// The reference predicts on host arrays (external/fv3fit/fv3fit/keras/_models/shared/
// pure_keras.py:98-118): every call crosses PCIe both ways.  Copies from pageable memory
// go through the runtime's own path (a bounce buffer, or pages it pins for the copy);
// copies from page-locked memory are DMA straight from / to it.
//
// Round 4 page-locked the caller's own arrays per call (hipHostRegister /
// hipHostUnregister) and hit intermittent illegal-address faults on later pageable
// copies.  What the runtime does (tools/host_pin_probe.cpp, profiles/r05b_probe.log):
// it accepts a second registration of the same range (one unregister then removes it),
// accepts a neighbour's registration of a shared page, and reports a shared page's bytes
// outside the first array as unregistered, so no start-address check can see an
// overlap.  Registering only page-exclusive interiors, refcounted process-wide, removed
// every overlap this library could create, and a full GPU-test run still faulted on a
// later pageable torch copy of freshly allocated memory (profiles/r05b_gpu_tests.log):
// the runtime's own pins for pageable copies are not visible through any query
// (hipPointerGetAttributes, hsa_amd_pointer_info: profiles/r05c_hsaprobe.log), so no
// registration of memory the caller owns can be proven disjoint from them.  So the
// library never registers memory it does not own.  The arrays a host call hands back
// come from here instead: hipHostMalloc blocks, page-aligned, registered once by the
// runtime's own allocator and reused from a cache after the caller drops them (no
// registration and no first-touch page faults per call); inputs cross as pageable copies
// or through staging blocks of this arena (fv3net_amd/transfer.py).
#include <unistd.h>

#include <algorithm>
#include <iterator>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "host_memory.h"

namespace fv3 {
namespace hostmem {
namespace {

struct Seg {
    uintptr_t end;
    uint64_t id;
    bool live;  // handed out (false: in the cache)
};

std::mutex g_mu;
std::map<uintptr_t, Seg> g_segs;  // start -> block; blocks never overlap
uint64_t g_next_id = 1;
std::multimap<size_t, uintptr_t> g_free;  // cached arena blocks by size
size_t g_cached = 0, g_live = 0;
size_t g_limit = size_t(2) << 30;  // cached arena bytes kept registered
// live + cached bytes of page-locked memory this library holds at most: arrays a caller
// keeps (diagnostics across steps) stay pinned, so the total is bounded; past it
// fv3_host_alloc fails and the caller uses pageable memory (transfer.empty_host)
size_t g_cap = size_t(32) << 30;

size_t page_size()
{
    static const size_t p = (size_t)sysconf(_SC_PAGESIZE);
    return p;
}

// the first segment ending after p (segments are disjoint and sorted)
std::map<uintptr_t, Seg>::iterator first_after(uintptr_t p)
{
    auto it = g_segs.upper_bound(p);
    if (it != g_segs.begin()) {
        auto pr = std::prev(it);
        if (pr->second.end > p) return pr;
    }
    return it;
}

bool inside_locked(uintptr_t p, size_t n)
{
    auto it = first_after(p);
    return it != g_segs.end() && it->first <= p && p + n <= it->second.end;
}

void free_block(uintptr_t p) { (void)hipHostFree((void*)p); }

// drop cached blocks until at most `keep` bytes stay cached; returns the blocks to free
// (freed outside the lock: hipHostFree may wait for the device)
void trim_locked(size_t keep, std::vector<uintptr_t>& out)
{
    while (g_cached > keep && !g_free.empty()) {
        auto it = std::prev(g_free.end());  // largest first
        g_cached -= it->first;
        g_segs.erase(it->second);
        out.push_back(it->second);
        g_free.erase(it);
    }
}

}  // namespace

bool inside(uintptr_t p, size_t n)
{
    std::lock_guard<std::mutex> g(g_mu);
    return inside_locked(p, n);
}

}  // namespace hostmem
}  // namespace fv3

using namespace fv3;
using namespace fv3::hostmem;

extern "C" int fv3_host_alloc(size_t bytes, void** out)
{
    clear_error();
    FV3_REQUIRE(out, "host_alloc: NULL out");
    *out = nullptr;
    const size_t P = page_size();
    const size_t n = std::max(P, (bytes + P - 1) / P * P);
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_free.find(n);
        if (it != g_free.end()) {
            const uintptr_t p = it->second;
            g_free.erase(it);
            g_cached -= n;
            g_live += n;
            g_segs.at(p).live = true;
            *out = (void*)p;
            return FV3_OK;
        }
    }
    {
        std::vector<uintptr_t> drop;
        {
            std::lock_guard<std::mutex> g(g_mu);
            FV3_REQUIRE_CODE(FV3_ERR_UNSUPPORTED, g_live + n <= g_cap,
                             "host_alloc: %zu live page-locked bytes + %zu exceed the arena cap %zu "
                             "(fv3_host_arena_cap)", g_live, n, g_cap);
            trim_locked(g_cap - g_live - n, drop);  // make room from the cache first
        }
        for (uintptr_t q : drop) free_block(q);
    }
    void* p = nullptr;
    FV3_HIP(hipHostMalloc(&p, n, hipHostMallocDefault));
    std::lock_guard<std::mutex> g(g_mu);
    g_segs.emplace((uintptr_t)p, Seg{(uintptr_t)p + n, g_next_id++, true});
    g_live += n;
    *out = p;
    return FV3_OK;
}

extern "C" int fv3_host_free(void* ptr)
{
    clear_error();
    if (!ptr) return FV3_OK;
    std::vector<uintptr_t> drop;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_segs.find((uintptr_t)ptr);
        FV3_REQUIRE(it != g_segs.end() && it->second.live,
                    "host_free: %p is not a live fv3_host_alloc block", ptr);
        const size_t n = it->second.end - it->first;
        it->second.live = false;
        g_live -= n;
        g_free.emplace(n, it->first);
        g_cached += n;
        trim_locked(g_limit, drop);
    }
    for (uintptr_t p : drop) free_block(p);
    return FV3_OK;
}

extern "C" int fv3_host_arena_limit(size_t cached_bytes)
{
    clear_error();
    std::vector<uintptr_t> drop;
    {
        std::lock_guard<std::mutex> g(g_mu);
        g_limit = cached_bytes;
        trim_locked(g_limit, drop);
    }
    for (uintptr_t p : drop) free_block(p);
    return FV3_OK;
}

extern "C" int fv3_host_arena_cap(size_t total_bytes)
{
    clear_error();
    std::vector<uintptr_t> drop;
    {
        std::lock_guard<std::mutex> g(g_mu);
        g_cap = total_bytes;
        trim_locked(g_cap > g_live ? g_cap - g_live : 0, drop);
    }
    for (uintptr_t p : drop) free_block(p);
    return FV3_OK;
}

extern "C" int fv3_host_memory_stats(uint64_t* stats)
{
    clear_error();
    FV3_REQUIRE(stats, "host_memory_stats: NULL out");
    std::lock_guard<std::mutex> g(g_mu);
    stats[0] = g_live;
    stats[1] = g_cached;
    stats[2] = g_segs.size();
    return FV3_OK;
}
