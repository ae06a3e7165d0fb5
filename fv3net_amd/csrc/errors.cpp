// fv3net_amd — thread-local error text for the C ABI (never throws across it).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace {
thread_local char g_err[1024] = {0};
}

namespace fv3 {
void set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
void clear_error() { g_err[0] = 0; }
const char* variant_env(const char* name)
{
    const char* on = getenv("FV3_VARIANTS");
    return (on && on[0] == '1' && on[1] == 0) ? getenv(name) : nullptr;
}
}  // namespace fv3

extern "C" const char* fv3_last_error(void) { return g_err; }
extern "C" int fv3_abi_version(void) { return 11; }

// "product": built by fv3net_amd/build.py with FV3_PRODUCT_BUILD and no experiment knob
// (common.h refuses one); anything else is a tools/ variant.
#if defined(FV3_PRODUCT_BUILD) && !defined(FV3_EXPERIMENT_KNOBS)
extern "C" const char* fv3_build_kind(void) { return "product"; }
#else
extern "C" const char* fv3_build_kind(void) { return "experiment"; }
#endif
