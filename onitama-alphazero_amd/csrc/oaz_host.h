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

// Engine internals used by the communicator (oaz_comm.cpp).
int oaz_engine_samples_peek(oaz_engine* e, const oaz_sample** dev, size_t* n, int* device);
int oaz_engine_samples_consume(oaz_engine* e, size_t n);
