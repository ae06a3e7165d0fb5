// fv3net_amd — thread-local error text for the C ABI (never throws across it).
#include <cstdarg>
#include <cstdio>

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
}  // namespace fv3

extern "C" const char* fv3_last_error(void) { return g_err; }
extern "C" int fv3_abi_version(void) { return 4; }
