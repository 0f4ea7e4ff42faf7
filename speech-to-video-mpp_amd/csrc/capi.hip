// Error reporting and device queries shared by every entry point of libs2v.
#include "common.hpp"

#include <cstring>

namespace s2v {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return S2V_E_LAUNCH;
    }
    return S2V_OK;
}

int device_cus() {
    static int cached = -1;
    if (cached < 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
        cached = cus;
    }
    return cached;
}

}  // namespace s2v

extern "C" const char *s2v_last_error(void) { return s2v::g_err; }
extern "C" int s2v_device_cus(void) { return s2v::device_cus(); }
extern "C" const char *s2v_version(void) { return "s2v 0.1.0 gfx950"; }
