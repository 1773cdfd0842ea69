// Library-wide host utilities: thread-local error text, device selection, version.
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace yta {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int select_device(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        set_error("no HIP device available (%s)", e == hipSuccess ? "0 devices" : hipGetErrorString(e));
        return YTA_ERR_HIP;
    }
    if (device < 0 || device >= n) {
        set_error("device %d out of range (%d devices)", device, n);
        return YTA_ERR_INVALID;
    }
    YTA_HIP(hipSetDevice(device));
    return YTA_OK;
}

hipError_t host_wait(hipStream_t s) {
    constexpr int MAX_DEV = 64;
    thread_local hipEvent_t ev[MAX_DEV] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (s) {
        hipDevice_t sd;
        if (hipStreamGetDevice(s, &sd) == hipSuccess) dev = (int)sd;
    }
    if (dev < 0 || dev >= MAX_DEV) return hipStreamSynchronize(s);
    if (!ev[dev]) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        e = hipEventCreateWithFlags(&ev[dev], hipEventBlockingSync | hipEventDisableTiming);
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            ev[dev] = nullptr;
            return hipStreamSynchronize(s);
        }
    }
    e = hipEventRecord(ev[dev], s);
    if (e != hipSuccess) return e;
    return hipEventSynchronize(ev[dev]);
}

}  // namespace yta

extern "C" {

int yta_version(void) { return 1; }

const char *yta_last_error(void) { return yta::g_err; }

int yta_device_count(int *count) {
    YTA_CHECK(count, YTA_ERR_INVALID, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return YTA_OK;
}

}  // extern "C"
