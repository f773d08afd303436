// Error reporting and identification for the librg_hip.so C-ABI.
#include <hip/hip_runtime.h>

#include <string>

#include "rg_common.h"

namespace rg {

static thread_local std::string g_last_error;
static thread_local LaunchEvents g_launch_events;

LaunchEvents &launch_events() { return g_launch_events; }

void set_error(const std::string &msg) { g_last_error = msg; }

int fail_arg(const std::string &msg) {
    set_error(msg);
    return RG_E_ARG;
}

int check_launch(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return RG_E_LAUNCH;
    }
    return RG_OK;
}

}  // namespace rg

extern "C" const char *rg_last_error(void) { return rg::g_last_error.c_str(); }

extern "C" int rg_event_elapsed_ms(void *ev_begin, void *ev_end, float *ms) {
    if (!ev_begin || !ev_end || !ms) return rg::fail_arg("rg_event_elapsed_ms: null argument");
    hipError_t e = hipEventSynchronize((hipEvent_t)ev_end);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, (hipEvent_t)ev_begin, (hipEvent_t)ev_end);
    if (e != hipSuccess) {
        rg::set_error(std::string("rg_event_elapsed_ms: ") + hipGetErrorString(e));
        return RG_E_LAUNCH;
    }
    return RG_OK;
}

extern "C" const char *rg_version(void) { return "librg_hip 0.2 gfx950 abi=2"; }

extern "C" int32_t rg_build_flags(void) { return RG_AB ? RG_BUILD_AB : 0; }
