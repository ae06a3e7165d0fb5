// fv3net_amd — the process-wide registry of the page-locked arena blocks this library
// allocated (host_memory.cpp), shared with the copy entry points (host_copy.hip).
#pragma once

#include <cstddef>
#include <cstdint>

namespace fv3 {
namespace hostmem {

// Whether [p, p + n) lies wholly inside one arena block (fv3_host_alloc).
bool inside(uintptr_t p, size_t n);

}  // namespace hostmem
}  // namespace fv3
