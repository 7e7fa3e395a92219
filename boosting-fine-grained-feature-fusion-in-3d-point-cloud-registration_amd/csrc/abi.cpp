// Error reporting and version of the libfgreg C ABI.
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace fgr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

static thread_local hipEvent_t g_t_start = nullptr, g_t_end = nullptr;

void timing_arm_take(hipEvent_t* start, hipEvent_t* end) {
    *start = g_t_start;
    *end = g_t_end;
    g_t_start = g_t_end = nullptr;
}

}  // namespace fgr

extern "C" int fgr_time_next_call(void* start_event, void* end_event) {
    fgr::g_t_start = reinterpret_cast<hipEvent_t>(start_event);
    fgr::g_t_end = reinterpret_cast<hipEvent_t>(end_event);
    return FGR_OK;
}

extern "C" int fgr_abi_version(void) { return FGR_ABI_VERSION; }

extern "C" const char* fgr_last_error(void) { return fgr::g_err; }
