// C ABI plumbing: error strings, version, device query.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "fm_common.h"

namespace fm {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return FM_EHIP;
    }
    return FM_OK;
}
}  // namespace fm

extern "C" const char* fm_version(void) { return "libfm_hip 0.1.0 (gfx950)"; }

extern "C" const char* fm_last_error(void) { return fm::g_err; }

extern "C" int fm_abi_sizes(int32_t* gram_args, int32_t* solve_args) {
    *gram_args = (int32_t)sizeof(fm_gram_args);
    *solve_args = (int32_t)sizeof(fm_solve_args);
    return FM_OK;
}

extern "C" int64_t fm_struct_size(const char* name) {
    if (name == nullptr) return -1;
    const std::string n(name);
    if (n == "fm_gram_args") return (int64_t)sizeof(fm_gram_args);
    if (n == "fm_solve_args") return (int64_t)sizeof(fm_solve_args);
    if (n == "fm_select_args") return (int64_t)sizeof(fm_select_args);
    if (n == "fm_universe_args") return (int64_t)sizeof(fm_universe_args);
    if (n == "fm_ts_args") return (int64_t)sizeof(fm_ts_args);
    if (n == "fm_chars_args") return (int64_t)sizeof(fm_chars_args);
    return -1;
}

extern "C" int fm_device_arch(char* buf, int32_t len) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        fm::set_error("hipGetDevice: %s", hipGetErrorString(e));
        return FM_EHIP;
    }
    hipDeviceProp_t p;
    e = hipGetDeviceProperties(&p, dev);
    if (e != hipSuccess) {
        fm::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
        return FM_EHIP;
    }
    snprintf(buf, (size_t)len, "%s", p.gcnArchName);
    return FM_OK;
}
