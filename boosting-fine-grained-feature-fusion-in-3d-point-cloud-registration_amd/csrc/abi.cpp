// Error reporting and version of the libfgreg C ABI.
#include <cstdarg>
#include <cstdio>

#include "../../include/fgreg.h"

namespace fgr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace fgr

extern "C" int fgr_abi_version(void) { return FGR_ABI_VERSION; }

extern "C" const char* fgr_last_error(void) { return fgr::g_err; }
