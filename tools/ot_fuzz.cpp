// ot_fuzz.cpp — libFuzzer + AddressSanitizer/UBSan harness for the C .ot reader
// (csrc/oaz_weights_io.cpp, oaz_ot_read): the reader takes untrusted files, so every input must end
// in an error code or a well-formed blob, with no out-of-bounds access, overflow or leak on the way.
// Host code only (no GPU): the engine entry points the reader's translation unit links against are
// stubbed below. Build and run: tools/ot_fuzz.sh.
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <vector>

#include "../include/onitama_az.h"

// ---- stubs for the symbols oaz_weights_io.cpp takes from oaz_engine.cpp ----------------------
int oaz_set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return code;
}
// same formula as oaz_engine.cpp (the reader checks its own canonical table against it)
extern "C" size_t oaz_weight_count(int blocks, int channels, int in_planes) {
    const size_t C = (size_t)channels, I = (size_t)in_planes;
    size_t n = C * I * 9 + C + 4 * C;
    n += (size_t)blocks * 2 * (C * C * 9 + C + 4 * C);
    n += C + 1 + 4 + C * 25 + C + C + 1;
    n += 2 * C + 2 + 8 + 50 * 50 + 50;
    return n;
}
extern "C" int oaz_get_config(const oaz_engine*, oaz_config*) { return OAZ_ERR_ARG; }
extern "C" int oaz_load_weights(oaz_engine*, const float*, size_t) { return OAZ_ERR_ARG; }

static char g_path[64];

extern "C" int LLVMFuzzerInitialize(int*, char***) {
    snprintf(g_path, sizeof(g_path), "/tmp/ot_fuzz_%d.ot", (int)getpid());
    return 0;
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    FILE* f = fopen(g_path, "wb");
    if (!f) abort();
    if (size && fwrite(data, 1, size, f) != size) abort();
    fclose(f);
    size_t n = 0;
    int blocks = -1;
    if (oaz_ot_read(g_path, nullptr, 0, &n, &blocks) == 0) {
        // accepted: the blob must be exactly a canonical network of the reported block count
        if (blocks < 0 || blocks > 64 || n != oaz_weight_count(blocks, 64, 21)) abort();
        std::vector<float> out(n);
        size_t n2 = 0;
        if (oaz_ot_read(g_path, out.data(), out.size(), &n2, nullptr) != 0 || n2 != n) abort();
    }
    return 0;
}
