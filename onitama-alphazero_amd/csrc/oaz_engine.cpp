// oaz_engine.cpp — host side of the C ABI (include/onitama_az.h).
//
// Owns the device buffers of one engine (one GPU), orchestrates the per-simulation kernel
// sequence  select -> evaluate -> expand/backup  for all G games in lock step, and the
// per-move finalisation (search result or self-play ply). No compute happens on the host
// except weight folding/packing, deck dealing for host helpers and sqrt tables.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stddef.h>
#include <time.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_device.h"
#include "oaz_host.h"
#include "oaz_kernels.h"

using namespace oaz;

static_assert(offsetof(oaz_config, search_time_ns) == 104 && sizeof(oaz_config) == 120, "oaz_config layout (ABI 4)");

// ---- errors ---------------------------------------------------------------------------------
static thread_local std::string g_err;

int oaz_set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" int oaz_abi_version(void) { return OAZ_ABI_VERSION; }
extern "C" const char* oaz_last_error(void) { return g_err.c_str(); }

extern "C" void oaz_config_default(oaz_config* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->blocks = 5;          // bin/train.rs:57-61
    c->channels = 64;
    c->in_planes = 21;
    c->sims = 400;          // bin/train.rs:53
    c->c_puct = 5.0;        // bin/train.rs:54
    c->train_noise = 1;     // bin/train.rs:55
    c->max_plies = 150;     // train.rs:152
    c->dirichlet_alpha = 0.03;
    c->dirichlet_eps = 0.25;
    c->games = 4096;
    c->evaluator = OAZ_EVAL_NN;
    // the fp32 network by the fp16x3 split (within 1e-5 of fp32, tests/test_gpu.py): the precision the
    // one-launch Agent search (k_search_lat) and the C3 headline run; OAZ_FP32 is the exact-fp32 MFMA kernel
    c->precision = OAZ_FP32_SPLIT16;
    c->fixed_deck = 0;
    for (int i = 0; i < 5; ++i) c->deck[i] = (uint8_t)i;  // ORIGINAL_CARDS[0..5]
    c->seed = 20260101ull;
    c->rank = 0;
    c->world = 1;
}

extern "C" int oaz_device_count(int* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (n) *n = (e == hipSuccess) ? c : 0;
    if (e != hipSuccess) return oaz_set_err(OAZ_ERR_NO_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    return 0;
}

static double now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e9 + (double)ts.tv_nsec;
}

// ---- host helpers -----------------------------------------------------------------------------
extern "C" void oaz_attack_maps(uint32_t out[2 * 16 * 25]) {
    memcpy(out, kAttackHost.m, sizeof(kAttackHost.m));
}

extern "C" size_t oaz_nn_device_bytes(int blocks, int precision) {
    if (blocks < 0 || blocks > 64 || precision < OAZ_FP32 || precision > OAZ_FP32_SPLIT16) return 0;
    return nn_packed_floats(blocks, precision) * sizeof(float);
}

extern "C" size_t oaz_weight_count(int blocks, int channels, int in_planes) {
    const size_t C = (size_t)channels, I = (size_t)in_planes;
    size_t n = C * I * 9 + C + 4 * C;
    n += (size_t)blocks * 2 * (C * C * 9 + C + 4 * C);
    n += C + 1 + 4 + C * 25 + C + C + 1;
    n += 2 * C + 2 + 8 + 50 * 50 + 50;
    return n;
}

extern "C" int oaz_random_weights(uint64_t seed, int blocks, float* out, size_t n) {
    const size_t need = oaz_weight_count(blocks, 64, 21);
    if (!out || n != need || blocks < 0) return oaz_set_err(OAZ_ERR_ARG, "random_weights: need %zu floats", need);
    uint64_t ctr = 0;
    auto uni = [&](float bound) {
        const uint64_t r = splitmix64(seed ^ splitmix64(ctr++));
        const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
        return (float)((2.0 * u - 1.0) * bound);
    };
    float* p = out;
    auto conv = [&](size_t wn, int cout, size_t fan_in) {  // weight + bias U(+-1/sqrt(fan_in))
        const float b = (float)(1.0 / sqrt((double)fan_in));
        for (size_t i = 0; i < wn; ++i) *p++ = uni(b);
        for (int i = 0; i < cout; ++i) *p++ = uni(b);
    };
    auto bn = [&](int c) {  // gamma 1, beta 0, mean 0, var 1
        for (int i = 0; i < c; ++i) *p++ = 1.0f;
        for (int i = 0; i < c; ++i) *p++ = 0.0f;
        for (int i = 0; i < c; ++i) *p++ = 0.0f;
        for (int i = 0; i < c; ++i) *p++ = 1.0f;
    };
    conv(64 * 21 * 9, 64, 21 * 9);
    bn(64);
    for (int b = 0; b < blocks; ++b)
        for (int j = 0; j < 2; ++j) {
            conv(64 * 64 * 9, 64, 64 * 9);
            bn(64);
        }
    conv(64, 1, 64);
    bn(1);
    conv(64 * 25, 64, 25);
    conv(64, 1, 64);
    conv(128, 2, 64);
    bn(2);
    conv(2500, 50, 50);
    if ((size_t)(p - out) != need) return oaz_set_err(OAZ_ERR_STATE, "random_weights: layout mismatch");
    return 0;
}

extern "C" void oaz_deal_deck(uint64_t seed, uint64_t game_id, uint8_t out[5]) {
    deal_deck(seed, game_id, out);
}

extern "C" int oaz_slot_game_ids(int rank, int world, int games, uint64_t seq, uint64_t* out) {
    if (!out || games < 1 || world < 1 || rank < 0 || rank >= world)
        return oaz_set_err(OAZ_ERR_ARG, "slot_game_ids: rank %d of %d, %d games", rank, world, games);
    for (int g = 0; g < games; ++g) out[g] = slot_game_id(seq, (uint32_t)world, (uint32_t)rank, (uint32_t)games, (uint32_t)g);
    return 0;
}

extern "C" void oaz_initial_state(const uint8_t deck[5], oaz_state* out) {
    if (!deck || !out) return;
    initial_state(deck, *out);
}

extern "C" double oaz_root_noise(uint64_t seed, uint64_t game_id, uint32_t ply, uint32_t sim, uint32_t draw,
                                double alpha, int nchild) {
    return (double)root_noise(seed, game_id, (ply << 16) | (sim & 0xFFFFu), draw, alpha, nchild);
}

extern "C" void oaz_hash_eval(const oaz_state* s, float policy[50], float* value) {
    const uint64_t h = hash_state(*s);
    for (int i = 0; i < 50; ++i) policy[i] = hash_policy(h, i);
    *value = hash_value(h);
}

// ---- weights: canonical (tch VarStore order) -> BN-folded -> MFMA-packed ----------------------
// Canonical order (DESIGN.md "Weights"): conv_init_1.{weight,bias}, bn1.{weight,bias,
// running_mean,running_var}, for each block i, j in {1,2}: resnet_i.resnet_small_block{j}.
// {small_block_conv.{weight,bias}, small_block_bn.{4}}, vh_conv.{w,b}, vh_bn.{4},
// vh_linear1.{w,b}, vh_linear2.{w,b}, policy_conv.{w,b}, policy_bn.{4}, ph_linear2.{w,b}.
struct FoldedConv {
    std::vector<float> w;  // [cout][cin][taps]
    std::vector<float> b;  // [cout]
};

static FoldedConv fold(const float*& p, int cout, int cin, int taps) {
    FoldedConv f;
    const float* w = p;
    p += (size_t)cout * cin * taps;
    const float* b = p;
    p += cout;
    const float *g = p, *beta = p + cout, *mean = p + 2 * cout, *var = p + 3 * cout;
    p += 4 * cout;
    f.w.resize((size_t)cout * cin * taps);
    f.b.resize(cout);
    for (int o = 0; o < cout; ++o) {
        const double s = (double)g[o] / sqrt((double)var[o] + 1e-5);  // BN eval, eps 1e-5
        for (size_t k = 0; k < (size_t)cin * taps; ++k)
            f.w[(size_t)o * cin * taps + k] = (float)((double)w[(size_t)o * cin * taps + k] * s);
        f.b[o] = (float)(((double)b[o] - (double)mean[o]) * s + (double)beta[o]);
    }
    return f;
}

// B fragments of v_mfma_f32_16x16x4f32 for a 64->64 conv: lane l supplies B[k=l>>4][col=l&15];
// k-group g of tap t covers channels ci = 16g + 4(l>>4) + q, q = 0..3; N-tile nt = 16 columns.
static void pack_conv64(const FoldedConv& f, std::vector<float>& out) {
    for (int t = 0; t < 9; ++t)
        for (int g = 0; g < 4; ++g)
            for (int nt = 0; nt < 4; ++nt)
                for (int l = 0; l < 64; ++l)
                    for (int q = 0; q < 4; ++q) {
                        const int co = nt * 16 + (l & 15);
                        const int ci = 16 * g + 4 * (l >> 4) + q;
                        out.push_back(f.w[((size_t)co * 64 + ci) * 9 + t]);
                    }
    for (int o = 0; o < 64; ++o) out.push_back(f.b[o]);
}

// bf16 B fragments of v_mfma_f32_16x16x32_bf16: for K-half m, lane l supplies
// B[k = 8(l>>4) + e][col l&15] = W[co = 16nt + (l&15)][ci = 32m + 8(l>>4) + e][tap t].
static uint16_t f32_to_bf16(float f) {  // round to nearest even
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static void pack_conv64_bf16(const FoldedConv& f, std::vector<float>& out) {
    std::vector<uint16_t> h;
    h.reserve(9 * 2 * 4 * 64 * 8);
    for (int t = 0; t < 9; ++t)
        for (int m = 0; m < 2; ++m)
            for (int nt = 0; nt < 4; ++nt)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e) {
                        const int co = nt * 16 + (l & 15);
                        const int ci = 32 * m + 8 * (l >> 4) + e;
                        h.push_back(f32_to_bf16(f.w[((size_t)co * 64 + ci) * 9 + t]));
                    }
    const size_t base = out.size();
    out.resize(base + h.size() / 2);
    memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
    for (int o = 0; o < 64; ++o) out.push_back(f.b[o]);
}

// fp32 split (OAZ_FP32_SPLIT): w = hi + mid + lo exactly, each term the top 16 bits of an fp32
// (8 significant bits: bf16). hi = trunc(w), mid = trunc(w - hi), lo = w - hi - mid (both
// subtractions exact, lo has <= 8 significant bits). Same split as split3() in oaz_nn.hip.
static void split3_host(float w, uint16_t out[3]) {
    auto bits = [](float f) { uint32_t u; memcpy(&u, &f, 4); return u; };
    auto from = [](uint32_t u) { float f; memcpy(&f, &u, 4); return f; };
    const uint32_t h = bits(w) & 0xffff0000u;
    const float r = w - from(h);
    const uint32_t m = bits(r) & 0xffff0000u;
    const float l = r - from(m);
    out[0] = (uint16_t)(h >> 16);
    out[1] = (uint16_t)(m >> 16);
    out[2] = (uint16_t)(bits(l) >> 16);
}

// Split B fragments: [tap][K-half m][piece p][N-tile][lane] bf16x8, lane l supplying
// B[k = 8(l>>4) + e][col l&15] = piece p of W[co = 16nt + (l&15)][ci = 32m + 8(l>>4) + e][tap].
static void pack_conv64_split(const FoldedConv& f, std::vector<float>& out) {
    std::vector<uint16_t> h;
    h.reserve(9 * 2 * 3 * 4 * 64 * 8);
    for (int t = 0; t < 9; ++t)
        for (int m = 0; m < 2; ++m)
            for (int pc = 0; pc < 3; ++pc)
                for (int nt = 0; nt < 4; ++nt)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e) {
                            const int co = nt * 16 + (l & 15);
                            const int ci = 32 * m + 8 * (l >> 4) + e;
                            uint16_t s[3];
                            split3_host(f.w[((size_t)co * 64 + ci) * 9 + t], s);
                            h.push_back(s[pc]);
                        }
    const size_t base = out.size();
    out.resize(base + h.size() / 2);
    memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
    for (int o = 0; o < 64; ++o) out.push_back(f.b[o]);
}

// fp16 split (OAZ_FP32_SPLIT16): hi = fp16(x) (round to nearest even), lo = fp16(x - hi); the same
// split as epilogue_h3_pack in oaz_nn.hip. Weights are first scaled by s = 2^k per output channel so
// that max |w s| lies in [2^14, 2^15): the top of fp16's range (products with activations < 65504
// stay far inside fp32), which keeps hi normal for weights down to 2^-28 of the channel's largest and
// bounds each weight's representation error by 2^-25 / s = 2^-39 max|w| (a channel with one huge
// weight no longer pushes its ordinary weights into fp16 subnormals). 1/s is stored for the epilogue.
static void split16_host(float x, uint16_t out[2]) {
    const _Float16 h = (_Float16)x;
    const _Float16 l = (_Float16)(x - (float)h);
    memcpy(&out[0], &h, 2);
    memcpy(&out[1], &l, 2);
}
static float pow2_scale(const float* w, size_t n, size_t stride, float* inv) {
    float mx = 0.0f;
    for (size_t k = 0; k < n; ++k) mx = fmaxf(mx, fabsf(w[k * stride]));
    if (!(mx > 0.0f) || !std::isfinite(mx)) {
        *inv = 1.0f;
        return 1.0f;
    }
    int e = 0;
    (void)frexpf(mx, &e);  // mx = f 2^e, f in [0.5, 1)
    if (e < -100) e = -100;  // keep s and 1/s normal floats
    *inv = ldexpf(1.0f, e - 15);
    return ldexpf(1.0f, 15 - e);
}

// Split16 B fragments: [tap][K-half m][piece p][N-tile][lane] f16x8, lane l supplying
// B[k = 8(l>>4) + e][col l&15] = piece p of s_co W[co = 16nt + (l&15)][ci = 32m + 8(l>>4) + e][tap];
// then bias[64], 1/s[64].
static void pack_conv64_split16(const FoldedConv& f, std::vector<float>& out) {
    float sc[64], inv[64];
    for (int co = 0; co < 64; ++co) sc[co] = pow2_scale(&f.w[(size_t)co * 64 * 9], 64 * 9, 1, &inv[co]);
    std::vector<uint16_t> h;
    h.reserve(9 * 2 * 2 * 4 * 64 * 8);
    for (int t = 0; t < 9; ++t)
        for (int m = 0; m < 2; ++m)
            for (int pc = 0; pc < 2; ++pc)
                for (int nt = 0; nt < 4; ++nt)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e) {
                            const int co = nt * 16 + (l & 15);
                            const int ci = 32 * m + 8 * (l >> 4) + e;
                            uint16_t s2[2];
                            split16_host(f.w[((size_t)co * 64 + ci) * 9 + t] * sc[co], s2);  // exact scaling
                            h.push_back(s2[pc]);
                        }
    const size_t base = out.size();
    out.resize(base + h.size() / 2);
    memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
    for (int o = 0; o < 64; ++o) out.push_back(f.b[o]);
    for (int o = 0; o < 64; ++o) out.push_back(inv[o]);
}

// First layer (k_nn_sq16): the 4 bitboard planes go through MFMA (lane l supplies
// W[co = 16nt + (l&15)][plane l>>4][tap t]); the 16 card planes and the blue-to-move plane
// (constant over the board, common.rs:68-77,32-37) become T[square][c][co] = sum over the
// on-board taps of W[co][plane][tap], with c = card index or 16 for the colour plane.
static void pack_first_layer(const FoldedConv& f, std::vector<float>& out) {
    for (int t = 0; t < 9; ++t)
        for (int nt = 0; nt < 4; ++nt)
            for (int l = 0; l < 64; ++l) out.push_back(f.w[((size_t)(nt * 16 + (l & 15)) * 21 + (l >> 4)) * 9 + t]);
    for (int o = 0; o < 64; ++o) out.push_back(f.b[o]);
    for (int sq = 0; sq < 25; ++sq)
        for (int c = 0; c < 17; ++c) {
            const int plane = c < 16 ? 4 + c : 20;
            for (int co = 0; co < 64; ++co) {
                double acc = 0.0;
                for (int t = 0; t < 9; ++t) {
                    const int r = sq / 5 + t / 3 - 1, cc = sq % 5 + t % 3 - 1;
                    if (r < 0 || r > 4 || cc < 0 || cc > 4) continue;
                    acc += (double)f.w[((size_t)co * 21 + plane) * 9 + t];
                }
                out.push_back((float)acc);
            }
        }
}

static int pack_weights(const float* raw, int blocks, int precision, std::vector<float>& out) {
    out.clear();
    out.reserve(nn_packed_floats(blocks, precision));
    const float* p = raw;
    pack_first_layer(fold(p, 64, 21, 9), out);
    for (int b = 0; b < blocks; ++b)
        for (int j = 0; j < 2; ++j) {
            if (precision == OAZ_BF16) pack_conv64_bf16(fold(p, 64, 64, 9), out);
            else if (precision == OAZ_FP32_SPLIT) pack_conv64_split(fold(p, 64, 64, 9), out);
            else if (precision == OAZ_FP32_SPLIT16) pack_conv64_split16(fold(p, 64, 64, 9), out);
            else pack_conv64(fold(p, 64, 64, 9), out);
        }
    // value head: vh_conv + vh_bn folded, vh_linear1, vh_linear2
    FoldedConv vc = fold(p, 1, 64, 1);
    for (int c = 0; c < 64; ++c) out.push_back(vc.w[c]);
    out.push_back(vc.b[0]);
    for (int i = 0; i < 3; ++i) out.push_back(0.0f);
    for (int q = 0; q < 25; ++q)  // vh_linear1.weight [64][25], stored transposed [25][64] (coalesced per lane)
        for (int o = 0; o < 64; ++o) out.push_back(p[o * 25 + q]);
    p += 64 * 25;
    for (int i = 0; i < 64; ++i) out.push_back(*p++);       // vh_linear1.bias
    for (int i = 0; i < 64; ++i) out.push_back(*p++);       // vh_linear2.weight [1][64]
    out.push_back(*p++);                                    // vh_linear2.bias
    for (int i = 0; i < 3; ++i) out.push_back(0.0f);
    // policy head: policy_conv + policy_bn folded, ph_linear2
    FoldedConv pc = fold(p, 2, 64, 1);
    for (int i = 0; i < 128; ++i) out.push_back(pc.w[i]);
    out.push_back(pc.b[0]);
    out.push_back(pc.b[1]);
    out.push_back(0.0f);
    out.push_back(0.0f);
    for (int f = 0; f < 50; ++f)  // ph_linear2.weight [50 out][50 in], stored transposed [in][out]
        for (int o = 0; o < 50; ++o) out.push_back(p[o * 50 + f]);
    p += 2500;
    for (int i = 0; i < 50; ++i) out.push_back(*p++);    // ph_linear2.bias
    out.push_back(0.0f);
    out.push_back(0.0f);
    if (precision == OAZ_FP32_SPLIT) {
        // k_nn_x6 head 1x1 convs on MFMA: split B pieces [K-half m][piece][lane] bf16x8, lane l
        // supplying B[k = 8(l>>4) + e][col n = l&15] for channel 32m + 8(l>>4) + e, columns
        // n = 0 value conv, 1 / 2 policy conv planes, 3..15 zero
        std::vector<uint16_t> h;
        for (int m = 0; m < 2; ++m)
            for (int pcs = 0; pcs < 3; ++pcs)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e) {
                        const int c = 32 * m + 8 * (l >> 4) + e, n = l & 15;
                        const float w = n == 0 ? vc.w[c] : n <= 2 ? pc.w[(n - 1) * 64 + c] : 0.0f;
                        uint16_t sp[3];
                        split3_host(w, sp);
                        h.push_back(sp[pcs]);
                    }
        const size_t base = out.size();
        out.resize(base + h.size() / 2);
        memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
    }
    if (precision == OAZ_BF16) {
        // k_nn_h3 in bf16 mode (k_nn_h1): head 1x1 convs as [K-half m][lane] bf16x8, lane l supplying
        // B[k = 8(l>>4) + e][col n = l&15] for channel 32m + 8(l>>4) + e, columns n = 0 value conv,
        // 1 / 2 policy conv planes, 3..15 zero
        std::vector<uint16_t> h;
        for (int m = 0; m < 2; ++m)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 8; ++e) {
                    const int c = 32 * m + 8 * (l >> 4) + e, n = l & 15;
                    h.push_back(f32_to_bf16(n == 0 ? vc.w[c] : n <= 2 ? pc.w[(n - 1) * 64 + c] : 0.0f));
                }
        const size_t base = out.size();
        out.resize(base + h.size() / 2);
        memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
    }
    if (precision == OAZ_FP32_SPLIT16) {
        // k_nn_h3 head 1x1 convs: [K-half m][piece][lane] f16x8 of the column-scaled weights
        // (column n = 0 value conv, 1 / 2 policy conv planes, 3..15 zero), then 1/s per column (+pad)
        float sc[3], inv[4] = {1.0f, 1.0f, 1.0f, 0.0f};
        sc[0] = pow2_scale(vc.w.data(), 64, 1, &inv[0]);
        sc[1] = pow2_scale(pc.w.data(), 64, 1, &inv[1]);
        sc[2] = pow2_scale(pc.w.data() + 64, 64, 1, &inv[2]);
        std::vector<uint16_t> h;
        for (int m = 0; m < 2; ++m)
            for (int pcs = 0; pcs < 2; ++pcs)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e) {
                        const int c = 32 * m + 8 * (l >> 4) + e, n = l & 15;
                        const float w = n == 0 ? vc.w[c] * sc[0] : n <= 2 ? pc.w[(n - 1) * 64 + c] * sc[n] : 0.0f;
                        uint16_t sp[2];
                        split16_host(w, sp);
                        h.push_back(sp[pcs]);
                    }
        const size_t base = out.size();
        out.resize(base + h.size() / 2);
        memcpy(out.data() + base, h.data(), h.size() * sizeof(uint16_t));
        for (int k = 0; k < 4; ++k) out.push_back(inv[k]);
    }
    if (precision == OAZ_FP32_SPLIT16 || precision == OAZ_BF16) {
        // k_nn_h3 first layer on fp16 MFMA (both modes): K block 0 = [piece][N-tile][lane] f16x8, lane
        // l supplying A[row co = 16nt + (l&15)][k = 8q + e] (q = l>>4) = piece of s_co W[co][plane q][tap e];
        // K block 1 per square = [square][piece][N-tile][lane] f16x8 with k = 8q + e: e = 0 tap 8 of
        // plane q, e >= 1 the table T[sq][c = 7q + e - 1][co] (c < 17: the 16 card planes and the
        // colour plane summed over the square's on-board taps); then 1/s[64]. s = 2^k per output
        // channel over all of them (max |s w| in [2^14, 2^15)).
        const float* r1 = raw;  // (fold advances its pointer)
        FoldedConv f1 = fold(r1, 64, 21, 9);
        std::vector<float> T((size_t)25 * 17 * 64);
        for (int sq = 0; sq < 25; ++sq)
            for (int c = 0; c < 17; ++c) {
                const int plane = c < 16 ? 4 + c : 20;
                for (int co = 0; co < 64; ++co) {
                    double acc = 0.0;
                    for (int t = 0; t < 9; ++t) {
                        const int r = sq / 5 + t / 3 - 1, cc = sq % 5 + t % 3 - 1;
                        if (r < 0 || r > 4 || cc < 0 || cc > 4) continue;
                        acc += (double)f1.w[((size_t)co * 21 + plane) * 9 + t];
                    }
                    T[((size_t)sq * 17 + c) * 64 + co] = (float)acc;
                }
            }
        float s1[64], inv1[64];
        for (int co = 0; co < 64; ++co) {
            float mx = 0.0f;
            for (int pl = 0; pl < 4; ++pl)
                for (int t = 0; t < 9; ++t) mx = fmaxf(mx, fabsf(f1.w[((size_t)co * 21 + pl) * 9 + t]));
            for (int sq = 0; sq < 25; ++sq)
                for (int c = 0; c < 17; ++c) mx = fmaxf(mx, fabsf(T[((size_t)sq * 17 + c) * 64 + co]));
            s1[co] = pow2_scale(&mx, 1, 1, &inv1[co]);
        }
        auto frag = [&](int blk, int sq, std::vector<uint16_t>& h1) {  // blk 0 (sq unused) or 1
            for (int pcs = 0; pcs < 2; ++pcs)
                for (int nt = 0; nt < 4; ++nt)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e) {
                            const int co = nt * 16 + (l & 15), q = l >> 4;
                            float w = 0.0f;
                            if (blk == 0) w = f1.w[((size_t)co * 21 + q) * 9 + e];
                            else if (e == 0) w = f1.w[((size_t)co * 21 + q) * 9 + 8];
                            else if (7 * q + e - 1 < 17) w = T[((size_t)sq * 17 + 7 * q + e - 1) * 64 + co];
                            uint16_t sp[2];
                            split16_host(w * s1[co], sp);  // exact scaling
                            h1.push_back(sp[pcs]);
                        }
        };
        std::vector<uint16_t> h1;
        frag(0, 0, h1);
        for (int sq = 0; sq < 25; ++sq) frag(1, sq, h1);
        const size_t b1 = out.size();
        out.resize(b1 + h1.size() / 2);
        memcpy(out.data() + b1, h1.data(), h1.size() * sizeof(uint16_t));
        for (int co = 0; co < 64; ++co) out.push_back(inv1[co]);
    }
    if (out.size() != nn_packed_floats(blocks, precision)) return oaz_set_err(OAZ_ERR_STATE, "pack: size mismatch");
    if ((size_t)(p - raw) != oaz_weight_count(blocks, 64, 21)) return oaz_set_err(OAZ_ERR_STATE, "pack: raw size mismatch");
    if (precision == OAZ_FP32_SPLIT16) {
        // k_nn_h3 recomputes fp16-range tiles with the k_nn_x6 body: the OAZ_FP32_SPLIT blob follows
        std::vector<float> x6;
        if (int rc = pack_weights(raw, blocks, OAZ_FP32_SPLIT, x6)) return rc;
        out.insert(out.end(), x6.begin(), x6.end());
    }
    return 0;
}

// Device floats of an engine's packed weights (SPLIT16 carries the SPLIT blob for its fallback).
static size_t weights_floats(int blocks, int precision) {
    return nn_packed_floats(blocks, precision) +
           (precision == OAZ_FP32_SPLIT16 ? nn_packed_floats(blocks, OAZ_FP32_SPLIT) : 0);
}

// ---- rules context (no engine needed) ----------------------------------------------------------
struct Scratch {
    void* p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        HIP_TRY(hipMalloc(&p, bytes));
        n = bytes;
        return 0;
    }
};

// One context per device (stream + scratch buffers allocated on that device): the rules entry points run
// on the calling thread's current device, so calls from threads on different GPUs never share buffers.
struct RulesCtx {
    std::mutex mu;
    bool init = false;
    hipStream_t stream = nullptr;
    Scratch a, b, c, d;
};
constexpr int kRulesMaxDevices = 64;
static RulesCtx g_rules_dev[kRulesMaxDevices];

// The current device's context, locked for the caller (lk), its stream created on first use.
static int rules_begin(RulesCtx** out, std::unique_lock<std::mutex>& lk) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return oaz_set_err(OAZ_ERR_NO_DEVICE, "no HIP device visible (the rules run on the GPU)");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= kRulesMaxDevices) return oaz_set_err(OAZ_ERR_ARG, "rules: device %d unsupported", dev);
    RulesCtx& r = g_rules_dev[dev];
    lk = std::unique_lock<std::mutex>(r.mu);
    if (!r.init) {
        HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
        r.init = true;
    }
    *out = &r;
    return 0;
}

extern "C" int oaz_movegen(const oaz_state* s, int n, uint32_t* masks, oaz_move* moves, uint8_t* counts) {
    if (!s || n < 0) return oaz_set_err(OAZ_ERR_ARG, "movegen: bad arguments");
    if (n == 0) return 0;
    RulesCtx* R = nullptr;
    std::unique_lock<std::mutex> lk;
    if (int rc = rules_begin(&R, lk)) return rc;
    hipStream_t st = R->stream;
    if (int rc = R->a.ensure((size_t)n * sizeof(oaz_state))) return rc;
    if (int rc = R->b.ensure((size_t)n * 50 * 4)) return rc;
    if (int rc = R->c.ensure((size_t)n * OAZ_MAX_MOVES * sizeof(oaz_move))) return rc;
    if (int rc = R->d.ensure((size_t)n)) return rc;
    HIP_TRY(hipMemcpyAsync(R->a.p, s, (size_t)n * sizeof(oaz_state), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_movegen((oaz_state*)R->a.p, n, masks ? (uint32_t*)R->b.p : nullptr,
                           moves ? (oaz_move*)R->c.p : nullptr, counts ? (uint8_t*)R->d.p : nullptr, st));
    if (masks) HIP_TRY(hipMemcpyAsync(masks, R->b.p, (size_t)n * 50 * 4, hipMemcpyDeviceToHost, st));
    if (moves) HIP_TRY(hipMemcpyAsync(moves, R->c.p, (size_t)n * OAZ_MAX_MOVES * sizeof(oaz_move), hipMemcpyDeviceToHost, st));
    if (counts) HIP_TRY(hipMemcpyAsync(counts, R->d.p, (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

extern "C" int oaz_step(oaz_state* s, const oaz_move* mv, int n, uint8_t* results) {
    if (!s || !mv || n < 0) return oaz_set_err(OAZ_ERR_ARG, "step: bad arguments");
    if (n == 0) return 0;
    for (int i = 0; i < n; ++i)
        if (mv[i].from > 24 || mv[i].to > 24 || mv[i].slot > 3 || mv[i].piece > 1)
            return oaz_set_err(OAZ_ERR_ARG, "step: move %d out of range", i);  // deck.rs:88 assert
    RulesCtx* R = nullptr;
    std::unique_lock<std::mutex> lk;
    if (int rc = rules_begin(&R, lk)) return rc;
    hipStream_t st = R->stream;
    if (int rc = R->a.ensure((size_t)n * sizeof(oaz_state))) return rc;
    if (int rc = R->c.ensure((size_t)n * sizeof(oaz_move))) return rc;
    if (int rc = R->d.ensure((size_t)n)) return rc;
    HIP_TRY(hipMemcpyAsync(R->a.p, s, (size_t)n * sizeof(oaz_state), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(R->c.p, mv, (size_t)n * sizeof(oaz_move), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_step((oaz_state*)R->a.p, (const oaz_move*)R->c.p, n, (uint8_t*)R->d.p, st));
    HIP_TRY(hipMemcpyAsync(s, R->a.p, (size_t)n * sizeof(oaz_state), hipMemcpyDeviceToHost, st));
    if (results) HIP_TRY(hipMemcpyAsync(results, R->d.p, (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

extern "C" int oaz_current_state(const oaz_state* s, int n, uint8_t* results) {
    if (!s || !results || n < 0) return oaz_set_err(OAZ_ERR_ARG, "current_state: bad arguments");
    if (n == 0) return 0;
    RulesCtx* R = nullptr;
    std::unique_lock<std::mutex> lk;
    if (int rc = rules_begin(&R, lk)) return rc;
    hipStream_t st = R->stream;
    if (int rc = R->a.ensure((size_t)n * sizeof(oaz_state))) return rc;
    if (int rc = R->d.ensure((size_t)n)) return rc;
    HIP_TRY(hipMemcpyAsync(R->a.p, s, (size_t)n * sizeof(oaz_state), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_current_state((const oaz_state*)R->a.p, n, (uint8_t*)R->d.p, st));
    HIP_TRY(hipMemcpyAsync(results, R->d.p, (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

extern "C" int oaz_encode(const oaz_state* s, int n, float* planes) {
    if (!s || !planes || n < 0) return oaz_set_err(OAZ_ERR_ARG, "encode: bad arguments");
    if (n == 0) return 0;
    RulesCtx* R = nullptr;
    std::unique_lock<std::mutex> lk;
    if (int rc = rules_begin(&R, lk)) return rc;
    hipStream_t st = R->stream;
    if (int rc = R->a.ensure((size_t)n * sizeof(oaz_state))) return rc;
    if (int rc = R->b.ensure((size_t)n * 525 * 4)) return rc;
    HIP_TRY(hipMemcpyAsync(R->a.p, s, (size_t)n * sizeof(oaz_state), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_encode((const oaz_state*)R->a.p, n, (float*)R->b.p, st));
    HIP_TRY(hipMemcpyAsync(planes, R->b.p, (size_t)n * 525 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

// ---- engine ------------------------------------------------------------------------------------
constexpr int kMaxParts = 4;  // run_sims: game parts, each on its own stream (oaz_config.parts)

struct TimedLaunch {
    int kind;  // 0 select, 1 nn, 2 expand, 3 finalize, 4 root noise (second stream), 5 leaf compaction,
               // 6 expand/backup + next select (fused)
    hipEvent_t a, b;
    uint32_t samples;
};

struct oaz_engine {
    oaz_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;       // root-noise producer, overlaps the NN kernel
    int cus = 256;                       // compute units of the device (leaf-compaction threshold)
    hipStream_t stream3[kMaxParts - 1] = {nullptr, nullptr, nullptr};  // the streams of game parts 1.. (oaz_config.parts)
    hipEvent_t ev_join = nullptr, ev_part[kMaxParts] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_ready[2] = {nullptr, nullptr};
    hipEvent_t ev_consumed[2][kMaxParts] = {};  // noise ring slot done with, per game part
    noise_t* noise = nullptr;            // [2][noise_chunk][G][kNoiseStride] (f64 draws; f32 in an OAZ_NOISE_F32 build)
    uint32_t noise_chunk = 16;           // simulations per noise ring slot (noise_chunk_for)
    uint32_t G = 0, cap = 0, pathcap = 0, hcap = 0, out_cap = 0;
    int32_t sims_cap = 0;                // cfg.sims at creation: trees and paths are sized for it
    // trees
    oaz_node* nodes = nullptr;
    uint32_t *n_nodes = nullptr, *path = nullptr, *depth = nullptr, *leaf = nullptr;
    oaz_state* leaf_state = nullptr;
    uint64_t* stats = nullptr;
    uint64_t* stats_sum = nullptr;
    double* sqrt_tab = nullptr;
    float *policy = nullptr, *value = nullptr;  // evaluations by compacted row (TreeView::slot)
    uint8_t* need = nullptr;                    // leaf compaction (oaz_kernels.h TreeView)
    uint32_t *slot = nullptr, *bcnt = nullptr;
    oaz_state* cstate = nullptr;
    float* weights = nullptr;
    bool have_weights = false;
    unsigned long long* nn_fallback = nullptr;  // OAZ_FP32_SPLIT16: tiles recomputed by k_nn_x6 (fp16 range)
    // search mode
    oaz_state* s_roots = nullptr;
    oaz_move* s_move = nullptr;
    float* s_pi = nullptr;
    float* s_rootv = nullptr;
    float* s_rootp = nullptr;
    uint32_t search_calls = 0;
    uint32_t last_sims = 0;  // simulations per game of the last run_sims (Q7 budget: may be < cfg.sims)
    // Q7 on the device (the one-launch searches): the deadline on the device clock, each game's simulation
    // count (last_sims_dev: the last run_sims wrote them for its last_G games; last_sims is then their maximum)
    uint64_t* deadline = nullptr;
    uint32_t* sims_run = nullptr;
    int wall_khz = 0;  // hipDeviceAttributeWallClockRate (kHz)
    bool last_sims_dev = false;
    bool deadline_armed = false;  // begin_budget launched k_deadline_start for the current search / ply
    double t_search0 = 0.0;       // host clock at the start of the current search / ply (0: no budget)
    uint32_t last_G = 0;
    std::vector<uint32_t> sims_host;  // per-game counts of the last device-budgeted run (empty: all last_sims)
    uint32_t* s_ply = nullptr;
    // self-play
    oaz_state* root = nullptr;
    uint32_t *ply = nullptr, *seq = nullptr;
    uint64_t* game_id = nullptr;
    uint8_t* active = nullptr;
    oaz_sample* hist = nullptr;
    oaz_sample* out = nullptr;
    unsigned long long* out_count = nullptr;
    uint32_t* fin = nullptr;      // SlotView::fin / fin_pos (records of the games that ended in a ply)
    uint64_t* fin_pos = nullptr;
    unsigned long long out_read = 0;  // samples already handed out
    bool selfplay_ready = false;
    uint64_t quota = 0;
    // timing
    bool timing = false;
    int timing_every = 1;     // time the kernels of every N-th simulation step (events cost ~2 % each)
    bool timing_skip = false; // run_sims: this simulation step is not sampled
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> pool;
    oaz_kernel_times times{};
};

template <class T>
static int dalloc(T** p, size_t count) {
    HIP_TRY(hipMalloc((void**)p, count * sizeof(T) > 0 ? count * sizeof(T) : 16));
    return 0;
}

static void dfree(void* p) {
    if (p) (void)hipFree(p);
}

static TreeView tree_view(oaz_engine* e, uint32_t G) {
    TreeView t;
    t.nodes = e->nodes;
    t.n_nodes = e->n_nodes;
    t.path = e->path;
    t.depth = e->depth;
    t.leaf = e->leaf;
    t.leaf_state = e->leaf_state;
    t.stats = e->stats;
    t.sqrt_tab = e->sqrt_tab;
    t.need = e->need;
    t.slot = e->slot;
    t.cstate = e->cstate;
    t.bcnt = e->bcnt;
    t.cap = e->cap;
    t.pathcap = e->pathcap;
    t.G = G;
    return t;
}

static SlotView slot_view(oaz_engine* e) {
    SlotView s;
    s.root = e->root;
    s.ply = e->ply;
    s.seq = e->seq;
    s.game_id = e->game_id;
    s.active = e->active;
    s.hist = e->hist;
    s.out = e->out;
    s.out_count = e->out_count;
    s.fin = e->fin;
    s.fin_pos = e->fin_pos;
    s.hcap = e->hcap;
    s.out_cap = e->out_cap;
    s.max_plies = e->cfg.max_plies;
    s.fixed_deck = e->cfg.fixed_deck;
    memcpy(s.deck, e->cfg.deck, 5);
    s.seed = e->cfg.seed;
    s.G = e->G;
    s.world = (uint32_t)(e->cfg.world > 0 ? e->cfg.world : 1);
    s.rank = (uint32_t)e->cfg.rank;
    s.quota = e->quota;
    s.stagger = e->quota ? 0u : (uint32_t)(e->cfg.stagger > 0 ? e->cfg.stagger : 0);
    return s;
}

static SearchParams search_params(const oaz_engine* e) {
    SearchParams p;
    p.c_puct = e->cfg.c_puct;
    p.alpha = e->cfg.dirichlet_alpha;
    p.eps = e->cfg.dirichlet_eps;
    p.seed = e->cfg.seed;
    p.train_noise = e->cfg.train_noise;
    return p;
}

static hipEvent_t ev_get(oaz_engine* e) {
    if (!e->pool.empty()) {
        hipEvent_t ev = e->pool.back();
        e->pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    (void)hipEventCreate(&ev);
    return ev;
}

// Run a launch, bracketed by events on the engine stream when timing is on.
#ifndef OAZ_NOISE_CHUNK  // 16: C3 +0.3 % over 8 in a 4-round same-box A/B (50: +0.4 %, 3x the ring); DESIGN.md perf log
#define OAZ_NOISE_CHUNK 16
#endif
static constexpr uint32_t kNoiseChunk = OAZ_NOISE_CHUNK;  // simulations of root noise produced per launch
static uint32_t noise_chunk_for(const oaz_engine* e);  // after grp_search

static void accumulate(oaz_engine* e, const TimedLaunch& p, float ms) {
    double* acc[7] = {&e->times.select_ms, &e->times.nn_ms, &e->times.expand_ms, &e->times.finalize_ms,
                      &e->times.noise_ms, &e->times.compact_ms, &e->times.backup_select_ms};
    uint64_t* cnt[7] = {&e->times.select_n, &e->times.nn_n, &e->times.expand_n, &e->times.finalize_n,
                        &e->times.noise_n, &e->times.compact_n, &e->times.backup_select_n};
    *acc[p.kind] += ms;
    *cnt[p.kind] += 1;
    if (p.kind == 1) e->times.nn_samples += p.samples;
}

// Resolve the recorded event pairs: per-kind sums, and the NN's busy time = the length of the union
// of its launches' intervals (with game parts on several streams the NN launches of a simulation
// step overlap each other; the union is the time during which any of them ran).
static int resolve_pending(oaz_engine* e) {
    std::vector<std::pair<float, float>> nn;
    hipEvent_t ref = e->pending.empty() ? nullptr : e->pending.front().a;
    for (auto& p : e->pending) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
        accumulate(e, p, ms);
        if (p.kind == 1) {
            float t0 = 0.f;
            HIP_TRY(hipEventElapsedTime(&t0, ref, p.a));
            nn.emplace_back(t0, t0 + ms);
        }
    }
    std::sort(nn.begin(), nn.end());
    for (size_t i = 0; i < nn.size();) {
        float lo = nn[i].first, hi = nn[i].second;
        size_t j = i + 1;
        for (; j < nn.size() && nn[j].first <= hi; ++j) hi = std::max(hi, nn[j].second);
        e->times.nn_busy_ms += hi - lo;
        e->times.nn_busy_n += 1;
        i = j;
    }
    for (auto& p : e->pending) {
        e->pool.push_back(p.a);
        e->pool.push_back(p.b);
    }
    e->pending.clear();
    return 0;
}

template <class F>
static int timed(oaz_engine* e, int kind, uint32_t samples, F&& launch, hipStream_t st = nullptr) {
    if (!st) st = e->stream;
    if (!e->timing || e->timing_skip) {
        HIP_TRY(launch());
        return 0;
    }
    TimedLaunch t;
    t.kind = kind;
    t.samples = samples;
    t.a = ev_get(e);
    t.b = ev_get(e);
    HIP_TRY(hipEventRecord(t.a, st));
    HIP_TRY(launch());
    HIP_TRY(hipEventRecord(t.b, st));
    e->pending.push_back(t);
    if (e->pending.size() > 4096) {  // resolve periodically to bound the pool
        HIP_TRY(hipStreamSynchronize(e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream2));
        for (auto s3 : e->stream3) HIP_TRY(hipStreamSynchronize(s3));
        return resolve_pending(e);
    }
    return 0;
}

extern "C" oaz_engine* oaz_create(const oaz_config* cfg, int device) {
    if (!cfg) {
        oaz_set_err(OAZ_ERR_ARG, "create: null config");
        return nullptr;
    }
    if (cfg->channels != 64 || cfg->in_planes != 21) {
        oaz_set_err(OAZ_ERR_ARG, "create: only channels=64, in_planes=21 are supported");
        return nullptr;
    }
    if (cfg->blocks < 0 || cfg->blocks > 64 || cfg->sims < 1 || cfg->sims > 65535 || cfg->games < 1 ||
        cfg->max_plies < 0 || cfg->max_plies > 100000 || cfg->compact < 0 || cfg->compact > 2 || cfg->search_time_ns < 0 ||
        cfg->step_kernels < 0 || cfg->step_kernels > 1 || cfg->world < 0 || cfg->rank < 0 ||
        cfg->rank >= (cfg->world > 0 ? cfg->world : 1) ||
        (uint64_t)cfg->games * ((uint64_t)cfg->sims + 1) >= (1ull << 32) ||  // 32-bit path offsets (k_select_seg)
        (uint64_t)cfg->games * kNoiseStride * sizeof(noise_t) >= (1ull << 31) ||  // 32-bit noise offsets (root_noise_pairs)
        (cfg->parts != 0 && cfg->parts != 1 && cfg->parts != 2 && cfg->parts != 4)) {
        oaz_set_err(OAZ_ERR_ARG, "create: config out of range");
        return nullptr;
    }
    if (cfg->precision != OAZ_FP32 && cfg->precision != OAZ_BF16 && cfg->precision != OAZ_FP32_SPLIT &&
        cfg->precision != OAZ_FP32_SPLIT16) {
        oaz_set_err(OAZ_ERR_ARG, "create: precision must be OAZ_FP32, OAZ_BF16, OAZ_FP32_SPLIT or OAZ_FP32_SPLIT16");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        oaz_set_err(OAZ_ERR_NO_DEVICE, "create: no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        oaz_set_err(OAZ_ERR_ARG, "create: device %d out of range (%d visible)", device, ndev);
        return nullptr;
    }
    oaz_engine* e = new oaz_engine();
    e->cfg = *cfg;
    e->device = device;
    e->G = (uint32_t)cfg->games;
    e->sims_cap = cfg->sims;
    e->cap = 1u + (uint32_t)cfg->sims * OAZ_MAX_MOVES;  // each playout expands <= 1 node of <= 40 children
    e->pathcap = (uint32_t)cfg->sims + 1;               // depth grows by <= 1 per playout
    e->hcap = (uint32_t)cfg->max_plies + 2;             // train.rs:74-79 cut after max_plies+2 plies
    e->out_cap = cfg->sample_capacity > 0 ? (uint32_t)cfg->sample_capacity : e->G * 64u;
    auto fail = [&](void) -> oaz_engine* {
        std::string msg = g_err;
        oaz_destroy(e);
        g_err = msg;
        return nullptr;
    };
    DeviceScope dev_scope_(device);  // the caller's current device is restored on return
    if (dev_scope_.rc != hipSuccess) {
        oaz_set_err(OAZ_ERR_HIP, "hipSetDevice(%d) failed", device);
        return fail();
    }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess) {
        oaz_set_err(OAZ_ERR_HIP, "stream create failed");
        return fail();
    }
    for (int i = 0; i < kMaxParts - 1; ++i)
        if (hipStreamCreateWithFlags(&e->stream3[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_part[i + 1], hipEventDisableTiming) != hipSuccess) {
            oaz_set_err(OAZ_ERR_HIP, "stream create failed");
            return fail();
        }
    for (int i = 0; i < 2; ++i)
        if (hipEventCreateWithFlags(&e->ev_ready[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_consumed[i][0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_consumed[i][1], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_consumed[i][2], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_consumed[i][3], hipEventDisableTiming) != hipSuccess) {
            oaz_set_err(OAZ_ERR_HIP, "event create failed");
            return fail();
        }
    if (hipDeviceGetAttribute(&e->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || e->cus < 1)
        e->cus = 256;
    if (hipDeviceGetAttribute(&e->wall_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) e->wall_khz = 0;
    const size_t G = e->G;
    e->noise_chunk = noise_chunk_for(e);
    if (dalloc(&e->nodes, G * e->cap) || dalloc(&e->n_nodes, G) || dalloc(&e->path, G * e->pathcap) ||
        dalloc(&e->depth, G) || dalloc(&e->leaf, G) || dalloc(&e->leaf_state, G) ||
        dalloc(&e->stats, G * GS_COUNT) || dalloc(&e->stats_sum, (size_t)GS_COUNT) ||
        dalloc(&e->sqrt_tab, (size_t)cfg->sims + 2) || dalloc(&e->policy, G * 50) ||
        dalloc(&e->value, G) || dalloc(&e->need, G) || dalloc(&e->slot, G) || dalloc(&e->cstate, G + 16) ||
        dalloc(&e->bcnt, (size_t)buckets_of((uint32_t)G) + kMaxParts) || dalloc(&e->weights, weights_floats(cfg->blocks, cfg->precision)) ||
        dalloc(&e->s_roots, G) || dalloc(&e->s_move, G) || dalloc(&e->s_pi, G * 50) ||
        dalloc(&e->s_rootv, G) || dalloc(&e->s_rootp, G * 50) || dalloc(&e->s_ply, G) ||
        dalloc(&e->root, G) || dalloc(&e->ply, G) || dalloc(&e->seq, G) ||
        dalloc(&e->game_id, G) || dalloc(&e->active, G) || dalloc(&e->hist, G * e->hcap) ||
        dalloc(&e->out, (size_t)e->out_cap) || dalloc(&e->out_count, (size_t)1) || dalloc(&e->nn_fallback, (size_t)1) ||
        dalloc(&e->deadline, (size_t)1) || dalloc(&e->sims_run, G) || dalloc(&e->fin, G) || dalloc(&e->fin_pos, G) ||
        (cfg->train_noise && dalloc(&e->noise, 2 * (size_t)e->noise_chunk * G * kNoiseStride)))
        return fail();
    // sqrt((double)n) from the host libm (IEEE correctly rounded), so device PUCT = oracle PUCT
    std::vector<double> tab((size_t)cfg->sims + 2);
    for (size_t i = 0; i < tab.size(); ++i) tab[i] = sqrt((double)i);
    // on the engine's own stream, waited for: its streams do not synchronise with the null stream, a null-stream
    // hipMemset returns before it ran and a pageable hipMemcpy before its DMA landed, so the first kernels could
    // otherwise read these buffers early (seen with several engines created concurrently on one GPU)
    hipStream_t s0 = e->stream;
    if (hipMemcpyAsync(e->sqrt_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice, s0) != hipSuccess ||
        hipMemsetAsync(e->stats, 0, G * GS_COUNT * sizeof(uint64_t), s0) != hipSuccess ||
        hipMemsetAsync(e->out_count, 0, sizeof(unsigned long long), s0) != hipSuccess ||
        hipMemsetAsync(e->nn_fallback, 0, sizeof(unsigned long long), s0) != hipSuccess ||
        hipMemsetAsync(e->active, 0, G, s0) != hipSuccess || hipMemsetAsync(e->need, 0, G, s0) != hipSuccess ||
        hipMemsetAsync(e->slot, 0, G * sizeof(uint32_t), s0) != hipSuccess ||
        hipMemsetAsync(e->cstate, 0, (G + 16) * sizeof(oaz_state), s0) != hipSuccess ||
        hipStreamSynchronize(s0) != hipSuccess) {
        oaz_set_err(OAZ_ERR_HIP, "create: init copies failed");
        return fail();
    }
    if (cfg->evaluator == OAZ_EVAL_NN) {  // random-init weights until oaz_load_weights
        std::vector<float> w(oaz_weight_count(cfg->blocks, 64, 21));
        if (oaz_random_weights(0, cfg->blocks, w.data(), w.size()) || oaz_load_weights(e, w.data(), w.size()))
            return fail();
    }
    return e;
}

extern "C" void oaz_destroy(oaz_engine* e) {
    if (!e) return;
    DeviceScope dev_scope_(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->stream2) (void)hipStreamSynchronize(e->stream2);
    for (auto s3 : e->stream3)
        if (s3) (void)hipStreamSynchronize(s3);
    for (auto ev : e->ev_part)
        if (ev) (void)hipEventDestroy(ev);
    for (int i = 0; i < 2; ++i) {
        if (e->ev_ready[i]) (void)hipEventDestroy(e->ev_ready[i]);
        for (auto ev : e->ev_consumed[i])
            if (ev) (void)hipEventDestroy(ev);
    }
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    for (auto& p : e->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto ev : e->pool) (void)hipEventDestroy(ev);
    void* ptrs[] = {e->nodes, e->n_nodes, e->path, e->depth, e->leaf, e->leaf_state, e->stats,
                    e->stats_sum, e->sqrt_tab, e->policy, e->value, e->weights, e->s_roots,
                    e->s_move, e->s_pi, e->s_rootv, e->s_rootp, e->s_ply, e->root, e->ply,
                    e->seq, e->game_id, e->active, e->hist, e->out, e->out_count, e->noise, e->nn_fallback,
                    e->need, e->slot, e->cstate, e->bcnt, e->deadline, e->sims_run, e->fin, e->fin_pos};
    for (void* p : ptrs) dfree(p);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    for (auto s3 : e->stream3)
        if (s3) (void)hipStreamDestroy(s3);
    delete e;
}

extern "C" int oaz_set_search_params(oaz_engine* e, int sims, double c_puct, int train_noise) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "set_search_params: null");
    if (sims < 1 || sims > e->sims_cap)
        return oaz_set_err(OAZ_ERR_ARG, "set_search_params: sims %d outside [1, %d] (the creation budget)", sims,
                           e->sims_cap);
    if (!(c_puct >= 0.0) || !std::isfinite(c_puct)) return oaz_set_err(OAZ_ERR_ARG, "set_search_params: bad c_puct");
    if (train_noise && !e->noise) {  // the engine was made without root noise: its ring comes now
        OAZ_ON_DEVICE(e->device);
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (dalloc(&e->noise, 2 * (size_t)e->noise_chunk * e->G * kNoiseStride)) return OAZ_ERR_HIP;
    }
    e->cfg.sims = sims;
    e->cfg.c_puct = c_puct;
    e->cfg.train_noise = train_noise ? 1 : 0;
    return 0;
}

extern "C" int oaz_set_search_time(oaz_engine* e, int64_t search_time_ns) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "set_search_time: null");
    if (search_time_ns < 0) return oaz_set_err(OAZ_ERR_ARG, "set_search_time: negative budget");
    e->cfg.search_time_ns = search_time_ns;
    return 0;
}

// The device-budgeted searches leave each game's count on the device; read them once.
static int fetch_sims_run(oaz_engine* e) {
    if (!e->last_sims_dev) return 0;
    OAZ_ON_DEVICE(e->device);
    std::vector<uint32_t> n(e->last_G);
    if (e->last_G) {
        HIP_TRY(hipMemcpyAsync(n.data(), e->sims_run, (size_t)e->last_G * 4, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    uint32_t m = 0;
    for (uint32_t v : n) m = v > m ? v : m;
    e->last_sims = m;
    e->last_sims_dev = false;
    e->sims_host = std::move(n);
    return 0;
}

extern "C" int oaz_last_sims(oaz_engine* e, int* sims) {
    if (!e || !sims) return oaz_set_err(OAZ_ERR_ARG, "last_sims: null");
    if (int rc = fetch_sims_run(e)) return rc;
    *sims = (int)e->last_sims;
    return 0;
}

extern "C" int oaz_search_playouts(oaz_engine* e, int* out, int G) {
    if (!e || (!out && G > 0) || G < 0) return oaz_set_err(OAZ_ERR_ARG, "search_playouts: bad arguments");
    if ((uint32_t)G > e->last_G)
        return oaz_set_err(OAZ_ERR_ARG, "search_playouts: G=%d > %u games in the last search", G, e->last_G);
    if (int rc = fetch_sims_run(e)) return rc;
    for (int g = 0; g < G; ++g) out[g] = e->sims_host.empty() ? (int)e->last_sims : (int)e->sims_host[(size_t)g];
    return 0;
}

extern "C" int oaz_get_config(const oaz_engine* e, oaz_config* out) {
    if (!e || !out) return oaz_set_err(OAZ_ERR_ARG, "get_config: null");
    *out = e->cfg;
    return 0;
}

extern "C" int oaz_load_weights(oaz_engine* e, const float* blob, size_t n) {
    if (!e || !blob) return oaz_set_err(OAZ_ERR_ARG, "load_weights: null");
    const size_t need = oaz_weight_count(e->cfg.blocks, 64, 21);
    if (n != need)  // the reference silently keeps random weights on a bad file (Q13); we refuse
        return oaz_set_err(OAZ_ERR_WEIGHTS, "load_weights: got %zu floats, need %zu for %d blocks", n, need,
                       e->cfg.blocks);
    std::vector<float> packed;
    if (int rc = pack_weights(blob, e->cfg.blocks, e->cfg.precision, packed)) return rc;
    OAZ_ON_DEVICE(e->device);
    HIP_TRY(hipMemcpyAsync(e->weights, packed.data(), packed.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->have_weights = true;
    return 0;
}

extern "C" int oaz_sync(oaz_engine* e) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "sync: null");
    OAZ_ON_DEVICE(e->device);
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream2));
    for (auto s3 : e->stream3) HIP_TRY(hipStreamSynchronize(s3));
    return 0;
}

extern "C" int oaz_set_timing(oaz_engine* e, int enable) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "set_timing: null");
    if (enable < 0) return oaz_set_err(OAZ_ERR_ARG, "set_timing: enable=%d < 0", enable);
    e->timing = enable != 0;
    e->timing_every = enable > 1 ? enable : 1;
    return 0;
}

static int resolve_timing(oaz_engine* e) {
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream2));
    for (auto s3 : e->stream3) HIP_TRY(hipStreamSynchronize(s3));
    return resolve_pending(e);
}

extern "C" int oaz_kernel_times_get(oaz_engine* e, oaz_kernel_times* out) {
    if (!e || !out) return oaz_set_err(OAZ_ERR_ARG, "kernel_times: null");
    if (int rc = resolve_timing(e)) return rc;
    *out = e->times;
    return 0;
}

extern "C" int oaz_kernel_times_reset(oaz_engine* e) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "kernel_times_reset: null");
    if (int rc = resolve_timing(e)) return rc;
    memset(&e->times, 0, sizeof(e->times));
    return 0;
}

static NNView nn_view(const oaz_engine* e, const TileMap* tm) {
    NNView w;
    w.blob = e->weights;
    w.blocks = e->cfg.blocks;
    w.precision = e->cfg.precision;
    w.x6_variant = 0;
#if OAZ_AB  // A/B build only: the diagnostic builds of k_nn_h3 by environment variable
    if (const char* xv = getenv("OAZ_NN_X6_V")) w.x6_variant = atoi(xv);
#endif
    w.blob_x6 = e->cfg.precision == OAZ_FP32_SPLIT16 ? e->weights + nn_packed_floats(e->cfg.blocks, OAZ_FP32_SPLIT16)
                                                     : nullptr;
    w.fallback = e->nn_fallback;
    w.tm = tm ? *tm : TileMap{nullptr, 0, 0};
    // k_nn_h3s (one position per workgroup) while the launch fits one round of workgroups on the CUs;
    // k_nn_h3 (16 per workgroup) above. The two give bit-identical outputs.
    w.small_max = e->cus;
#if OAZ_AB  // A/B build only: OAZ_NN_SMALL_MAX=n overrides
    if (const char* v = getenv("OAZ_NN_SMALL_MAX")) w.small_max = atoi(v);
#endif
    return w;
}

// B positions d_states[0, B) -> rows [0, B); with tm (compacted leaves, run_sims) the rows of the
// bucket tiles (the HASH evaluator simply evaluates every row below B).
static int evaluate(oaz_engine* e, const oaz_state* d_states, uint32_t B, float* d_pol, float* d_val,
                    hipStream_t st = nullptr, const TileMap* tm = nullptr) {
    if (!st) st = e->stream;
    const uint32_t counted = tm ? 0u : B;  // compacted: the count is on the device (GS_EVALS)
    if (e->cfg.evaluator == OAZ_EVAL_HASH)
        return timed(e, 1, counted, [&] { return launch_hash_eval(d_states, (int)B, d_pol, d_val, st); }, st);
    const NNView w = nn_view(e, tm);
    return timed(e, 1, counted, [&] { return launch_nn_forward(w, d_states, (int)B, d_pol, d_val, st); }, st);
}

extern "C" int oaz_nn_fallbacks(oaz_engine* e, uint64_t* tiles) {
    if (!e || !tiles) return oaz_set_err(OAZ_ERR_ARG, "nn_fallbacks: null");
    OAZ_ON_DEVICE(e->device);
    unsigned long long n = 0;
    HIP_TRY(hipMemcpyAsync(&n, e->nn_fallback, sizeof(n), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    *tiles = (uint64_t)n;
    return 0;
}

extern "C" int oaz_nn_forward(oaz_engine* e, const oaz_state* s, int B, float* policy, float* value) {
    if (!e || !s || B < 0) return oaz_set_err(OAZ_ERR_ARG, "nn_forward: bad arguments");
    if ((uint32_t)B > e->G) return oaz_set_err(OAZ_ERR_CAPACITY, "nn_forward: B=%d > games=%u", B, e->G);
    if (B == 0) return 0;
    OAZ_ON_DEVICE(e->device);
    HIP_TRY(hipMemcpyAsync(e->s_roots, s, (size_t)B * sizeof(oaz_state), hipMemcpyHostToDevice, e->stream));
    if (int rc = evaluate(e, e->s_roots, (uint32_t)B, e->s_rootp, e->s_rootv)) return rc;
    if (policy) HIP_TRY(hipMemcpyAsync(policy, e->s_rootp, (size_t)B * 50 * 4, hipMemcpyDeviceToHost, e->stream));
    if (value) HIP_TRY(hipMemcpyAsync(value, e->s_rootv, (size_t)B * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return 0;
}

// Leaf compaction (oaz_config.compact; off by default: every playout evaluates its leaf, Q2) pays
// when it can remove whole rounds of NN workgroups (one 16-position tile per
// CU at a time): at C3 the ~8.7 % won leaves are 1.4 of 16 rounds. Below 12 rounds (G < 12 * 16 *
// CUs, e.g. C2's 4096 games = one round) it would only add its own launch, so the leaves are then
// evaluated in place.
static bool compact_leaves(const oaz_engine* e, uint32_t G) {
    return e->cfg.compact == 1 || (e->cfg.compact == 2 && G >= 12u * 16u * (uint32_t)e->cus);
}

// A search of G games runs as k_search_grp launches (16 games per workgroup, up to one round of workgroups,
// one launch per root-noise chunk) instead of the per-simulation-step launches. Everything it depends on is
// fixed at creation except G (any G below a qualifying engine's qualifies as well).
static bool grp_search(const oaz_engine* e, uint32_t G) {
    const bool hash = e->cfg.evaluator == OAZ_EVAL_HASH;
    return e->cfg.step_kernels == 0 && !compact_leaves(e, G) && (G + 15) / 16 <= (uint32_t)e->cus &&
           (hash || e->cfg.precision == OAZ_FP32_SPLIT16) && tree_seg_kernels();
}

// Simulations per root-noise ring slot. An engine whose searches run as k_search_grp: every chunk is one
// launch, and the noise launch of the next chunk cannot overlap it (the search holds every CU), so a chunk of
// up to 512 simulations (a C2 ply in one launch and one noise launch: 46.6-47.1 -> 49.5-50.0 M sims/s;
// DESIGN.md section 8) at a 16-simulation minimum. kNoiseChunk (16) for the per-step launches, where the
// noise overlaps the network and the first select waits for only 16 simulations' draws. Ring: 2 x chunk x
// G x 80 floats (<= 1.3 GB at 4 096 games).
static uint32_t noise_chunk_for(const oaz_engine* e) {
    if (!grp_search(e, e->G)) return kNoiseChunk;
    const uint32_t c = e->sims_cap < 512 ? (uint32_t)e->sims_cap : 512u;
    return c > kNoiseChunk ? c : kNoiseChunk;
}

// All cfg.sims simulations of one move for every game, in lock step: select -> leaf compaction ->
// evaluate -> expand/backup, where simulation s's expand/backup and simulation s+1's select run as
// one kernel (k_backup_select_seg; a game's next walk needs only its own backup). Select marks the games whose playout uses its leaf evaluation (all
// but those ending on a won, terminal-flagged node, whose evaluation the reference discards:
// mcts_arena.rs:156-176) and the compaction kernel packs their leaves per 4096-game bucket, so the
// network evaluates only those. With root noise, k_root_noise fills chunk c+1 of the
// double-buffered noise ring on stream2 while stream 1 runs chunk c (events order the ring slots).
static TreeView slice_view(const TreeView& t, uint32_t g0, uint32_t n, int b0);

// Game parts of run_sims (oaz_config.parts; 0 = auto: two from kAutoParts games; the overlap of
// one part's tree kernels and NN tail with the other's launches measured +3-4 % on C2, C3, C5).
constexpr uint32_t kAutoParts = 2048;
static int game_parts(const oaz_engine* e, uint32_t G) {
    int p = e->cfg.parts ? e->cfg.parts : (G >= kAutoParts ? 2 : 1);
#if OAZ_AB  // A/B build only: OAZ_SPLIT_HALVES=n overrides
    if (const char* v = getenv("OAZ_SPLIT_HALVES")) p = atoi(v);
#endif
    if (p != 2 && p != 4) p = 1;
    // every part non-empty: part h starts at h * ceil(G / p), so the last one needs (p - 1) * ceil(G / p) < G
    // (G = 5, p = 4 would give parts of 2, 2, 1 and an empty fourth)
    while (p > 1 && (uint32_t)(p - 1) * ((G + (uint32_t)p - 1) / (uint32_t)p) >= G) p /= 2;
    return p;
}

// Game range [g0, g0 + n) of part h of nh over G games (clamped: no part extends past G).
static void part_range(uint32_t G, int nh, int h, uint32_t* g0, uint32_t* n) {
    const uint32_t Gh = (G + (uint32_t)nh - 1) / (uint32_t)nh;
    const uint32_t s = std::min((uint32_t)h * Gh, G);
    *g0 = s;
    *n = std::min(Gh, G - s);
}

static int run_sims_body(oaz_engine* e, const TreeView& t, const oaz_state* roots, const uint8_t* active,
                         const uint64_t* gids, const uint32_t* plies);

// run_sims_body, and on an error the game parts' streams are joined into the engine stream anyway
// (its early returns skip the join), so oaz_sync and buffer reuse after an error wait for them.
static int run_sims(oaz_engine* e, const TreeView& t, const oaz_state* roots, const uint8_t* active,
                    const uint64_t* gids, const uint32_t* plies) {
    const int rc = run_sims_body(e, t, roots, active, gids, plies);
    if (rc) {
        const std::string msg = g_err;
        for (int h = 1; h < kMaxParts; ++h)
            if (hipEventRecord(e->ev_part[h], e->stream3[h - 1]) == hipSuccess)
                (void)hipStreamWaitEvent(e->stream, e->ev_part[h], 0);
        e->timing_skip = false;
        g_err = msg;
    }
    return rc;
}


// Q7: the device deadline = the device clock when k_deadline_start runs on the engine stream + the budget.
static int arm_deadline(oaz_engine* e) {
    if (e->wall_khz <= 0) return oaz_set_err(OAZ_ERR_HIP, "search_time: the device reports no wall clock rate");
    const double ticks = (double)e->cfg.search_time_ns * (double)e->wall_khz * 1e-6;
    HIP_TRY(launch_deadline_start(e->deadline, ticks < 1.8e19 ? (uint64_t)ticks : (uint64_t)1.8e19, e->stream));
    e->deadline_armed = true;
    return 0;
}

// Q7: a search's budget runs from the start of the search call, as the reference's Instant is taken at the
// top of search() (mcts_arena.rs:75-78): the host clock now (the per-step loop's reads) and, on the device,
// the deadline armed before this search's first upload or reset on the engine stream (the one-launch
// searches' reads), so the roots upload and the tree reset count against the budget on both paths. Work
// queued on the stream by earlier calls (asynchronous self-play plies) is not part of this search.
static int begin_budget(oaz_engine* e) {
    e->deadline_armed = false;
    e->t_search0 = 0.0;
    if (e->cfg.search_time_ns <= 0) return 0;
    e->t_search0 = now_ns();
    return e->wall_khz > 0 ? arm_deadline(e) : 0;
}

static int run_sims_body(oaz_engine* e, const TreeView& t, const oaz_state* roots, const uint8_t* active,
                         const uint64_t* gids, const uint32_t* plies) {
    const SearchParams prm = search_params(e);
    const uint32_t sims = (uint32_t)e->cfg.sims;
    // Q7 (opt-in, oaz_config.search_time_ns): the reference's loop runs playouts while
    // `playouts < max_playouts && elapsed < search_time` (mcts_arena.rs:78). The one-launch searches
    // (k_search_lat, k_search_grp: the Agent / arena sizes) read the device clock before every simulation
    // and each workgroup stops on its own (oaz_search_playouts: each game's count, >= 1). The per-step loop
    // (larger batches) advances all games together, so there the clock is read between simulation steps
    // (after the streams drained) and the search stops after the first step that ends at or past the
    // budget: every game then has run the same number of playouts (>= 1). pi / the move come from the
    // visits that ran.
    const double budget_ns = (double)e->cfg.search_time_ns;
    const double t_start = budget_ns > 0 ? (e->t_search0 > 0 ? e->t_search0 : now_ns()) : 0.0;
    e->last_sims = 0;
    e->last_sims_dev = false;
    e->sims_host.clear();
    e->last_G = t.G;
    // the one-launch searches check the budget on the device (oaz_search_lat.hip): the deadline is the
    // device clock when k_deadline_start runs + the budget in clock ticks
    auto device_budget = [&]() -> int {
        if (budget_ns <= 0) return 0;
        if (!e->deadline_armed)
            if (int rc = arm_deadline(e)) return rc;
        HIP_TRY(hipMemsetAsync(e->sims_run, 0, (size_t)t.G * 4, e->stream));
        e->last_sims_dev = true;
        return 0;
    };
    uint64_t* const dl = budget_ns > 0 ? e->deadline : nullptr;
    uint32_t* const sr = budget_ns > 0 ? e->sims_run : nullptr;
    const bool noise = e->cfg.train_noise && e->noise;
    // the one-launch search (oaz_search_lat.hip): a workgroup per game runs all its simulations, when the
    // per-step loop would launch one NN workgroup per game anyway and nothing needs the host or a second
    // stream between simulation steps
    const bool hash = e->cfg.evaluator == OAZ_EVAL_HASH;
    if (e->cfg.step_kernels == 0 && !noise && !compact_leaves(e, t.G) && t.G <= (uint32_t)e->cus &&
        (hash || e->cfg.precision == OAZ_FP32_SPLIT16) && tree_seg_kernels()) {
        const NNView w = nn_view(e, nullptr);
        TreeView tl = t;  // rows = game ids (no compaction arrays)
        tl.need = nullptr;
        tl.slot = nullptr;
        e->times.parts = 1;
        e->timing_skip = false;
        if (int rc = device_budget()) return rc;
        if (int rc = timed(e, 6, t.G, [&] {
                return launch_search_lat(tl, roots, active, prm, (int)sims, hash ? nullptr : &w, e->policy, e->value,
                                         dl, sr, e->stream);
            }))
            return rc;
        e->last_sims = sims;  // (with a budget: replaced by the games' largest count when it is asked for)
        return 0;
    }
    const uint32_t chunk = e->noise_chunk;
    const size_t slot_elems = (size_t)chunk * t.G * kNoiseStride;
    const uint32_t nchunks = (sims + chunk - 1) / chunk;
    // up to one round of 16-game workgroups (k_search_grp): one launch per noise chunk of simulations,
    // each workgroup walking, evaluating and backing up its 16 games without a grid-wide step
    const bool grp = grp_search(e, t.G);
    // The games in nh parts, each on its own stream: one part's tree kernels, leaf compaction and NN
    // tail run in the gaps of the others' launches (the NN holds a whole CU per workgroup, so the
    // tree kernels cannot share a CU with it, only fill the CUs it leaves idle). The parts meet only
    // through the root-noise ring: chunk c + 2 overwrites chunk c's slot once every part is done with it.
    const int nh = grp ? 1 : game_parts(e, t.G);
    if (grp)
        if (int rc = device_budget()) return rc;
    auto produce = [&](uint32_t c) -> int {
        if (c >= 2)
            for (int h = 0; h < nh; ++h) HIP_TRY(hipStreamWaitEvent(e->stream2, e->ev_consumed[c & 1][h], 0));
        e->timing_skip = false;  // every noise launch is timed (once per chunk)
        const uint32_t s0 = c * chunk, n = sims - s0 < chunk ? sims - s0 : chunk;
        noise_t* buf = e->noise + (c & 1) * slot_elems;
        if (int rc = timed(e, 4, t.G * n, [&] {
                return launch_root_noise(roots, active, gids, plies, prm, t.G, s0, n, buf, e->stream2);
            }, e->stream2))
            return rc;
        HIP_TRY(hipEventRecord(e->ev_ready[c & 1], e->stream2));
        return 0;
    };
    if (noise) {
        HIP_TRY(hipEventRecord(e->ev_consumed[0][0], e->stream));  // stream2 starts after prior work
        HIP_TRY(hipStreamWaitEvent(e->stream2, e->ev_consumed[0][0], 0));
        if (int rc = produce(0)) return rc;
    }
    TreeView tc = t;  // the compaction arrays, or none (rows = game ids)
    if (!compact_leaves(e, t.G)) {
        tc.need = nullptr;
        tc.slot = nullptr;
    }
#if OAZ_AB  // A/B build only: OAZ_TREE_FUSE=0 runs expand/backup and the next select as two launches
    static const bool fuse = !(getenv("OAZ_TREE_FUSE") && getenv("OAZ_TREE_FUSE")[0] == '0');
#else
    constexpr bool fuse = true;
#endif
    const bool split = nh > 1;
    e->times.parts = (uint64_t)nh;
    TreeView tv[kMaxParts];
    uint32_t gstart[kMaxParts] = {0, 0, 0, 0};
    hipStream_t sh[kMaxParts] = {e->stream, e->stream3[0], e->stream3[1], e->stream3[2]};
    int b0 = 0;  // a part's compaction bucket counters follow the previous parts'
    for (int h = 0; h < nh; ++h) {
        uint32_t n = t.G;
        part_range(t.G, nh, h, &gstart[h], &n);
        tv[h] = split ? slice_view(tc, gstart[h], n, b0) : tc;
        b0 += buckets_of(n);
    }
    if (split) {
        HIP_TRY(hipEventRecord(e->ev_join, e->stream));  // the other streams start after prior work
        for (int h = 1; h < nh; ++h) HIP_TRY(hipStreamWaitEvent(sh[h], e->ev_join, 0));
    }
    auto join = [&]() -> int {  // stream waits for the other parts' streams
        for (int h = 1; h < nh; ++h) {
            HIP_TRY(hipEventRecord(e->ev_part[h], sh[h]));
            HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_part[h], 0));
        }
        return 0;
    };
    bool out_of_time = false;
    for (uint32_t c = 0; c < nchunks && !out_of_time; ++c) {
        if (noise) {
            if (c + 1 < nchunks)
                if (int rc = produce(c + 1)) return rc;
            for (int h = 0; h < nh; ++h) HIP_TRY(hipStreamWaitEvent(sh[h], e->ev_ready[c & 1], 0));
        }
        const uint32_t s0 = c * chunk, s1 = s0 + chunk < sims ? s0 + chunk : sims;
        if (grp) {  // the chunk's simulations in one launch
            const NNView w = nn_view(e, nullptr);
            e->timing_skip = false;
            const noise_t* nz = noise ? e->noise + (c & 1) * slot_elems : nullptr;
            if (int rc = timed(e, 6, t.G * (s1 - s0), [&] {
                    return launch_search_grp(tv[0], roots, active, prm, (int)s0, (int)s1, nz, hash ? nullptr : &w,
                                             e->policy, e->value, dl, sr, sh[0]);
                }, sh[0]))
                return rc;
            e->last_sims = s1;
        }
        for (uint32_t s = grp ? s1 : s0; s < s1; ++s) {
            // Q7: is the budget spent after simulation s - 1? This waits for every part's stream before
            // each simulation step, so a budgeted search gives up the parts' overlap (and the root-noise
            // producer runs ahead at most to the step being waited on) and is not the one-launch search:
            // its throughput is not comparable with an unbudgeted run's (the reference's own cutoff is a
            // clock read per playout, mcts_arena.rs:78). Parity runs and the benches leave it off.
            if (budget_ns > 0 && s > 0) {
                for (int h = 0; h < nh; ++h) HIP_TRY(hipStreamSynchronize(sh[h]));
                if (now_ns() - t_start >= budget_ns) {
                    out_of_time = true;
                    break;
                }
            }
            e->last_sims = s + 1;
            // sampled steps sit mid-chunk: a chunk's first select also waits for its noise
            e->timing_skip = e->timing_every > 1 && s % (uint32_t)e->timing_every != (uint32_t)e->timing_every / 2;
            for (int h = 0; h < nh; ++h) {
                const TreeView& th = tv[h];
                const size_t go = gstart[h];
                if (th.G == 0) continue;
                const hipStream_t st = sh[h];
                const oaz_state* rh = roots + go;
                const uint8_t* ah = active ? active + go : nullptr;  // null in search mode
                float* pol = e->policy + go * 50;
                float* val = e->value + go;
                const noise_t* nz = noise ? e->noise + (c & 1) * slot_elems + ((size_t)(s - s0) * t.G + go) * kNoiseStride
                                        : nullptr;
                if (s == 0) {
                    if (int rc = timed(e, 0, th.G, [&] { return launch_select(th, rh, ah, nz, prm, st); }, st))
                        return rc;
                } else if (!fuse) {
                    if (int rc = timed(e, 2, th.G, [&] { return launch_expand_backup(th, rh, ah, pol, val, st); }, st))
                        return rc;
                    if (int rc = timed(e, 0, th.G, [&] { return launch_select(th, rh, ah, nz, prm, st); }, st))
                        return rc;
                } else if (int rc = timed(e, 6, th.G, [&] {
                               return launch_backup_select(th, rh, ah, pol, val, nz, prm, st);
                           }, st)) {
                    return rc;
                }
                if (th.need) {
                    // row loads clamped to the part's own rows (the next part's compaction writes its
                    // rows on another stream)
                    const TileMap tm{th.bcnt, buckets_of(th.G), (int32_t)th.G};
                    if (int rc = timed(e, 5, th.G, [&] { return launch_eval_compact(th, st); }, st)) return rc;
                    if (int rc = evaluate(e, th.cstate, th.G, pol, val, st, &tm)) return rc;
                } else if (int rc = evaluate(e, th.leaf_state, th.G, pol, val, st)) {
                    return rc;
                }
            }
        }
        if (noise)  // this part is done with the noise slot (no join: a part may run a chunk ahead)
            for (int h = 0; h < nh; ++h) HIP_TRY(hipEventRecord(e->ev_consumed[c & 1][h], sh[h]));
    }
    e->timing_skip = false;
    for (int h = 0; h < nh; ++h) {
        const size_t go = gstart[h];
        if (tv[h].G == 0) continue;
        if (int rc = timed(e, 2, tv[h].G, [&] {
                return launch_expand_backup(tv[h], roots + go, active ? active + go : nullptr, e->policy + go * 50,
                                            e->value + go, sh[h]);
            }, sh[h]))
            return rc;
    }
    if (split)
        if (int rc = join()) return rc;
    return 0;
}

// The trees of games [g0, g0 + n) as a view of their own: every per-game array offset by g0, the
// part's compaction buckets from bucket counter b0 (its compacted rows start at g0; the NN's row loads
// are clamped to the part's own n rows by the TileMap cap, run_sims).
static TreeView slice_view(const TreeView& t, uint32_t g0, uint32_t n, int b0) {
    TreeView v = t;
    v.nodes = t.nodes + (size_t)g0 * t.cap;
    v.n_nodes = t.n_nodes + g0;
    v.path = t.path + (size_t)g0 * t.pathcap;
    v.depth = t.depth + g0;
    v.leaf = t.leaf + g0;
    v.leaf_state = t.leaf_state + g0;
    v.stats = t.stats + (size_t)g0 * GS_COUNT;
    if (t.need) v.need = t.need + g0;
    if (t.slot) v.slot = t.slot + g0;
    v.cstate = t.cstate + g0;
    v.bcnt = t.bcnt + b0;
    v.G = n;
    return v;
}

static int reduce_stats(oaz_engine* e, uint32_t G, uint64_t out[GS_COUNT]) {
    HIP_TRY(launch_stats_reduce(e->stats, G, e->stats_sum, e->stream));
    HIP_TRY(hipMemcpyAsync(out, e->stats_sum, GS_COUNT * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return 0;
}

static void fill_search_stats(const uint64_t* s, oaz_search_stats* o) {
    o->sims = s[GS_SIMS];
    o->expansions = s[GS_EXPANSIONS];
    o->children = s[GS_CHILDREN];
    o->terminal_leaves = s[GS_TERMINAL];
    o->depth_sum = s[GS_DEPTH];
    o->stuck_leaves = s[GS_STUCK];
    o->max_nodes = s[GS_MAXNODES];
    o->nn_evals = s[GS_EVALS];
}

extern "C" int oaz_search(oaz_engine* e, const oaz_state* roots, int G, oaz_move* out_move, float* out_pi,
                          float* out_root_value, oaz_search_stats* stats) {
    if (!e || !roots || G < 0) return oaz_set_err(OAZ_ERR_ARG, "search: bad arguments");
    if ((uint32_t)G > e->G) return oaz_set_err(OAZ_ERR_CAPACITY, "search: G=%d > games=%u", G, e->G);
    if (G == 0) return 0;
    for (int i = 0; i < G; ++i)
        if (roots[i].to_move > 1) return oaz_set_err(OAZ_ERR_ARG, "search: root %d has to_move=%d", i, roots[i].to_move);
    OAZ_ON_DEVICE(e->device);
    if (int rc = begin_budget(e)) return rc;
    const TreeView t = tree_view(e, (uint32_t)G);
    HIP_TRY(hipMemcpyAsync(e->s_roots, roots, (size_t)G * sizeof(oaz_state), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemsetAsync(e->stats, 0, (size_t)G * GS_COUNT * sizeof(uint64_t), e->stream));
    std::vector<uint32_t> plies((size_t)G, e->search_calls);
    HIP_TRY(hipMemcpyAsync(e->s_ply, plies.data(), (size_t)G * 4, hipMemcpyHostToDevice, e->stream));
    e->search_calls++;
    HIP_TRY(launch_tree_reset(t, e->stream));
    if (int rc = run_sims(e, t, e->s_roots, nullptr, nullptr, e->s_ply)) {
        (void)hipStreamSynchronize(e->stream);  // the plies upload reads this frame's vector
        return rc;
    }
    if (int rc = timed(e, 3, (uint32_t)G, [&] { return launch_search_finalize(t, e->s_roots, e->s_move, e->s_pi, e->stream); }))
        return rc;
    if (out_root_value) {  // extra root evaluation (alphazero_mcts/mod.rs:137-141)
        if (int rc = evaluate(e, e->s_roots, (uint32_t)G, e->s_rootp, e->s_rootv)) return rc;
        HIP_TRY(hipMemcpyAsync(out_root_value, e->s_rootv, (size_t)G * 4, hipMemcpyDeviceToHost, e->stream));
    }
    if (out_move) HIP_TRY(hipMemcpyAsync(out_move, e->s_move, (size_t)G * sizeof(oaz_move), hipMemcpyDeviceToHost, e->stream));
    if (out_pi) HIP_TRY(hipMemcpyAsync(out_pi, e->s_pi, (size_t)G * 50 * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (stats) {
        uint64_t s[GS_COUNT];
        if (int rc = reduce_stats(e, (uint32_t)G, s)) return rc;
        memset(stats, 0, sizeof(*stats));
        fill_search_stats(s, stats);
    }
    return 0;
}

extern "C" int oaz_tree_dump(oaz_engine* e, int game, oaz_node* out, int cap, int* n_nodes) {
    if (!e || game < 0 || (uint32_t)game >= e->G) return oaz_set_err(OAZ_ERR_ARG, "tree_dump: bad game");
    OAZ_ON_DEVICE(e->device);
    uint32_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, e->n_nodes + game, 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (n_nodes) *n_nodes = (int)n;
    if (out && cap > 0) {
        const size_t m = n < (uint32_t)cap ? n : (uint32_t)cap;
        HIP_TRY(hipMemcpyAsync(out, e->nodes + (size_t)game * e->cap, m * sizeof(oaz_node), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    return 0;
}

// ---- self-play ----------------------------------------------------------------------------------
extern "C" int oaz_selfplay_reset(oaz_engine* e) {
    if (!e) return oaz_set_err(OAZ_ERR_ARG, "selfplay_reset: null");
    OAZ_ON_DEVICE(e->device);
    const TreeView t = tree_view(e, e->G);
    HIP_TRY(hipMemsetAsync(e->stats, 0, (size_t)e->G * GS_COUNT * sizeof(uint64_t), e->stream));
    HIP_TRY(hipMemsetAsync(e->out_count, 0, sizeof(unsigned long long), e->stream));
    e->out_read = 0;
    HIP_TRY(launch_selfplay_reset(t, slot_view(e), e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->selfplay_ready = true;
    return 0;
}

extern "C" int oaz_selfplay_step(oaz_engine* e, int moves) {
    if (!e || moves < 0) return oaz_set_err(OAZ_ERR_ARG, "selfplay_step: bad arguments");
    if (!e->selfplay_ready)
        if (int rc = oaz_selfplay_reset(e)) return rc;
    OAZ_ON_DEVICE(e->device);
    const TreeView t = tree_view(e, e->G);
    const SlotView sv = slot_view(e);
    for (int m = 0; m < moves; ++m) {
        if (int rc = begin_budget(e)) return rc;
        HIP_TRY(launch_tree_reset(t, e->stream));  // a fresh tree per move (the last ply's stays dumpable)
        if (int rc = run_sims(e, t, e->root, e->active, e->game_id, e->ply)) return rc;
        if (int rc = timed(e, 3, e->G, [&] { return launch_selfplay_move(t, sv, e->stream); })) return rc;
    }
    return 0;
}

extern "C" int oaz_selfplay_stats_get(oaz_engine* e, oaz_selfplay_stats* o) {
    if (!e || !o) return oaz_set_err(OAZ_ERR_ARG, "selfplay_stats: null");
    OAZ_ON_DEVICE(e->device);
    uint64_t s[GS_COUNT];
    if (int rc = reduce_stats(e, e->G, s)) return rc;
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, e->out_count, sizeof(cnt), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    memset(o, 0, sizeof(*o));
    o->moves = s[GS_MOVES];
    o->games_finished = s[GS_FINISHED];
    o->games_cut = s[GS_CUT];
    o->red_wins = s[GS_RED];
    o->blue_wins = s[GS_BLUE];
    o->passes = s[GS_PASSES];
    o->samples_dropped = s[GS_DROPPED];
    const unsigned long long avail = cnt < e->out_cap ? cnt : e->out_cap;
    o->samples_ready = avail > e->out_read ? avail - e->out_read : 0;
    fill_search_stats(s, &o->search);
    return 0;
}

static int samples_copy(oaz_engine* e, void* dst, size_t cap, size_t* n_out, hipMemcpyKind kind) {
    OAZ_ON_DEVICE(e->device);
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, e->out_count, sizeof(cnt), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const unsigned long long avail = (cnt < e->out_cap ? cnt : e->out_cap);
    const size_t ready = avail > e->out_read ? (size_t)(avail - e->out_read) : 0;
    const size_t n = ready < cap ? ready : cap;
    if (n) HIP_TRY(hipMemcpyAsync(dst, e->out + e->out_read, n * sizeof(oaz_sample), kind, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->out_read += n;
    if (e->out_read == avail && cnt >= e->out_read) {  // buffer drained: rewind
        HIP_TRY(hipMemsetAsync(e->out_count, 0, sizeof(unsigned long long), e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        e->out_read = 0;
    }
    if (n_out) *n_out = n;
    return 0;
}

// Internal (oaz_host.h), for oaz_allgather_samples: the engine's buffered samples as one contiguous
// device range [*dev, *dev + *n), after the engine's work so far is complete.
int oaz_engine_samples_peek(oaz_engine* e, const oaz_sample** dev, size_t* n, int* device) {
    OAZ_ON_DEVICE(e->device);
    HIP_TRY(hipStreamSynchronize(e->stream2));
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, e->out_count, sizeof(cnt), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const unsigned long long avail = (cnt < e->out_cap ? cnt : e->out_cap);
    *n = avail > e->out_read ? (size_t)(avail - e->out_read) : 0;
    *dev = e->out + e->out_read;
    *device = e->device;
    return 0;
}

// Drops the first n peeked samples (the caller's copies of them are complete).
int oaz_engine_samples_consume(oaz_engine* e, size_t n) {
    OAZ_ON_DEVICE(e->device);
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, e->out_count, sizeof(cnt), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const unsigned long long avail = (cnt < e->out_cap ? cnt : e->out_cap);
    e->out_read += n;
    if (e->out_read == avail && cnt >= e->out_read) {  // buffer drained: rewind
        HIP_TRY(hipMemsetAsync(e->out_count, 0, sizeof(unsigned long long), e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        e->out_read = 0;
    }
    return 0;
}

extern "C" int oaz_samples_fetch(oaz_engine* e, oaz_sample* out, size_t cap, size_t* n_out) {
    if (!e || (!out && cap)) return oaz_set_err(OAZ_ERR_ARG, "samples_fetch: bad arguments");
    return samples_copy(e, out, cap, n_out, hipMemcpyDeviceToHost);
}

extern "C" int oaz_samples_export_device(oaz_engine* e, void* dev_dst, size_t cap_bytes, size_t* n_out) {
    if (!e || (!dev_dst && cap_bytes)) return oaz_set_err(OAZ_ERR_ARG, "samples_export: bad arguments");
    return samples_copy(e, dev_dst, cap_bytes / sizeof(oaz_sample), n_out, hipMemcpyDeviceToDevice);
}

// Games of the first `quota` global ids that this rank plays: rank r owns the ids
// seq * world * G + r * G + g (g < G, seq >= 0; SlotView, k_selfplay_move).
static uint64_t rank_share(const oaz_engine* e, uint64_t quota) {
    const uint64_t G = e->G, W = (uint64_t)(e->cfg.world > 0 ? e->cfg.world : 1), r = (uint64_t)e->cfg.rank;
    const uint64_t full = quota / (W * G), rem = quota % (W * G);
    const uint64_t lo = r * G;
    return full * G + (rem > lo ? (rem - lo < G ? rem - lo : G) : 0);
}

extern "C" int oaz_selfplay_run(oaz_engine* e, int n_games, oaz_sample* out, size_t cap, size_t* n_out,
                                oaz_selfplay_stats* stats) {
    if (!e || n_games < 0) return oaz_set_err(OAZ_ERR_ARG, "selfplay_run: bad arguments");
    e->quota = (uint64_t)n_games;  // slots stop dealing at global game index >= n_games
    const uint64_t mine = rank_share(e, e->quota);  // this rank's share of the n_games (global) games
    int rc = oaz_selfplay_reset(e);
    if (rc) {
        e->quota = 0;
        return rc;
    }
    size_t got = 0;
    for (;;) {
        oaz_selfplay_stats st;
        if ((rc = oaz_selfplay_stats_get(e, &st))) break;
        if (st.games_finished >= mine) {
            if (stats) *stats = st;
            break;
        }
        if ((rc = oaz_selfplay_step(e, 8))) break;
        size_t n = 0;
        if (out && got < cap) {
            if ((rc = oaz_samples_fetch(e, out + got, cap - got, &n))) break;
            got += n;
        }
    }
    if (!rc && out && got < cap) {
        size_t n = 0;
        rc = oaz_samples_fetch(e, out + got, cap - got, &n);
        got += n;
    }
    e->quota = 0;
    e->selfplay_ready = false;
    if (n_out) *n_out = got;
    return rc;
}
