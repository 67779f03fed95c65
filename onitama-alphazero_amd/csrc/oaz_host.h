// oaz_host.h — host-side helpers shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/onitama_az.h"

// Records the thread-local error message returned by oaz_last_error(); returns `code`.
int oaz_set_err(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return oaz_set_err(OAZ_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                               __FILE__, __LINE__);                                             \
    } while (0)

// An entry point's device: `device` is current for the call and the calling thread's current device is
// restored on return (every C-ABI entry point that touches the GPU; include/onitama_az.h, Threading).
struct DeviceScope {
    int prev = -1;
    hipError_t rc;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        rc = hipSetDevice(device);
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
#define OAZ_ON_DEVICE(dev)       \
    DeviceScope dev_scope_(dev); \
    HIP_TRY(dev_scope_.rc)

// Engine internals used by the communicator (oaz_comm.cpp).
int oaz_engine_samples_peek(oaz_engine* e, const oaz_sample** dev, size_t* n, int* device);
int oaz_engine_samples_consume(oaz_engine* e, size_t n);
