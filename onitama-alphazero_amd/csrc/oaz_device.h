// oaz_device.h — rules, RNG and evaluator primitives shared by the HIP kernels and the host
// engine (all __host__ __device__). Semantics follow the reference exactly (citations per
// function); the formulation is the GPU's own (branch-free bit ops, one lane per square).
#pragma once

#include <stdint.h>

#include "../../include/onitama_az.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define OAZ_HD __host__ __device__ __forceinline__
#else
#define OAZ_HD inline
#endif

namespace oaz {

// ---- cards: onitama-game/src/game/card.rs:17-468 -------------------------------------
// Card patterns are 25-bit masks (bit 31-i = square i) centred on square 12; `mirror` is
// the pattern Blue uses (card.rs:531-533).
constexpr uint32_t kCardPos[16] = {0x20004000u, 0x0440A000u, 0x02202000u, 0x00828000u,
                                   0x01220000u, 0x02940000u, 0x02142000u, 0x00948000u,
                                   0x0280A000u, 0x02804000u, 0x0100A000u, 0x01104000u,
                                   0x01044000u, 0x01140000u, 0x02048000u, 0x00902000u};
constexpr uint32_t kCardMir[16] = {0x01000200u, 0x02811000u, 0x02022000u, 0x00A08000u,
                                   0x00224000u, 0x0014A000u, 0x02142000u, 0x00948000u,
                                   0x0280A000u, 0x0100A000u, 0x02804000u, 0x01044000u,
                                   0x01104000u, 0x00144000u, 0x00902000u, 0x02048000u};
// Card.player_color (0 Red, 1 Blue): the first mover is the neutral card's colour.
constexpr uint8_t kCardColor[16] = {1, 0, 0, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0};

constexpr uint32_t kRedKingStart = 0x00000200u;   // state.rs:24
constexpr uint32_t kBlueKingStart = 0x20000000u;  // state.rs:31
constexpr uint32_t kBluePawnsStart = 0xD8000000u; // state.rs:38
constexpr uint32_t kRedPawnsStart = 0x00000D80u;  // state.rs:45
constexpr int kBlueTemple = 2;                    // state.rs:48
constexpr int kRedTemple = 22;                    // state.rs:49

OAZ_HD constexpr uint32_t sq_bit(int sq) { return 0x80000000u >> sq; }

// ATTACK_MAPS[color][card][from] (card.rs:476-604). The reference builds it by shifting the
// centred pattern by the square delta and masking wrapped files by (delta % 5). Here every
// pattern square is turned into a (dr, dc) offset from the centre and applied to `from`
// when it stays on the board — the same set (the file masks remove exactly the column
// wrap-arounds; tests/test_rules_host.py checks the tables against the oracle).
struct AttackTable {
    uint32_t m[2][16][25];
};

constexpr AttackTable make_attack_table() {
    AttackTable t{};
    for (int color = 0; color < 2; ++color)
        for (int card = 0; card < 16; ++card) {
            const uint32_t pat = color ? kCardMir[card] : kCardPos[card];
            for (int from = 0; from < 25; ++from) {
                uint32_t m = 0;
                for (int j = 0; j < 25; ++j) {
                    if (!(pat & sq_bit(j))) continue;
                    const int dr = j / 5 - 2, dc = j % 5 - 2;
                    const int r = from / 5 + dr, c = from % 5 + dc;
                    if (r >= 0 && r < 5 && c >= 0 && c < 5) m |= sq_bit(r * 5 + c);
                }
                t.m[color][card][from] = m;
            }
        }
    return t;
}

constexpr AttackTable kAttackHost = make_attack_table();

// ---- state helpers ----------------------------------------------------------------------
OAZ_HD bool is_win(int r) { return r == OAZ_RED_WIN || r == OAZ_BLUE_WIN; }

// State::make_move (state.rs:145-202) + Deck::rotate (deck.rs:87-90); colour = mover.
OAZ_HD int make_move(oaz_state& s, int from, int to, int piece, int slot, int color) {
    const uint32_t fb = sq_bit(from), tb = sq_bit(to);
    const int enemy = color ^ 1;
    if (piece == OAZ_PAWN) s.pawns[color] &= ~fb;
    else s.kings[color] &= ~fb;
    int res = OAZ_IN_PROGRESS;
    if (s.pawns[enemy] & tb) {
        s.pawns[enemy] &= ~tb;
        res = OAZ_CAPTURE;
    } else if (s.kings[enemy] & tb) {
        s.kings[enemy] &= ~tb;
        res = color == OAZ_RED ? OAZ_RED_WIN : OAZ_BLUE_WIN;
    }
    if (piece == OAZ_PAWN) s.pawns[color] |= tb;
    else s.kings[color] |= tb;
    if (piece == OAZ_KING && to == (color == OAZ_RED ? kBlueTemple : kRedTemple))
        res = color == OAZ_RED ? OAZ_RED_WIN : OAZ_BLUE_WIN;
    if (slot < 4) {
        const uint8_t t = s.cards[slot];
        s.cards[slot] = s.cards[4];
        s.cards[4] = t;
    }
    return res;
}

// Register-only forms of the colour- and slot-indexed accesses, for code that holds the state in registers
// across a loop (the one-launch search's walk): a runtime index into the struct (s.pawns[color],
// s.cards[slot]) can make the compiler keep the whole state in scratch memory, a memory round trip per
// access. cards[0..3] are one little-endian word.
OAZ_HD int state_card(const oaz_state& s, int i) {
    uint32_t w;
    __builtin_memcpy(&w, s.cards, 4);
    return i < 4 ? (int)((w >> (8 * i)) & 0xFFu) : (int)s.cards[4];
}
OAZ_HD void state_rotate(oaz_state& s, int slot) {  // Deck::rotate (deck.rs:87-90): cards[slot] <-> cards[4]
    uint32_t w;
    __builtin_memcpy(&w, s.cards, 4);
    const uint32_t sh = 8u * (uint32_t)slot;
    const uint8_t t = (uint8_t)(w >> sh);
    w = (w & ~(0xFFu << sh)) | ((uint32_t)s.cards[4] << sh);
    __builtin_memcpy(s.cards, &w, 4);
    s.cards[4] = t;
}
// make_move with the same result and state, through selects
OAZ_HD int make_move_regs(oaz_state& s, int from, int to, int piece, int slot, int color) {
    const uint32_t fb = sq_bit(from), tb = sq_bit(to);
    const bool blue = color != OAZ_RED;
    uint32_t mp = blue ? s.pawns[1] : s.pawns[0], mk = blue ? s.kings[1] : s.kings[0];
    uint32_t ep = blue ? s.pawns[0] : s.pawns[1], ek = blue ? s.kings[0] : s.kings[1];
    if (piece == OAZ_PAWN) mp &= ~fb;
    else mk &= ~fb;
    int res = OAZ_IN_PROGRESS;
    if (ep & tb) {
        ep &= ~tb;
        res = OAZ_CAPTURE;
    } else if (ek & tb) {
        ek &= ~tb;
        res = color == OAZ_RED ? OAZ_RED_WIN : OAZ_BLUE_WIN;
    }
    if (piece == OAZ_PAWN) mp |= tb;
    else mk |= tb;
    if (piece == OAZ_KING && to == (color == OAZ_RED ? kBlueTemple : kRedTemple))
        res = color == OAZ_RED ? OAZ_RED_WIN : OAZ_BLUE_WIN;
    s.pawns[0] = blue ? ep : mp;
    s.pawns[1] = blue ? mp : ep;
    s.kings[0] = blue ? ek : mk;
    s.kings[1] = blue ? mk : ek;
    if (slot < 4) state_rotate(s, slot);
    return res;
}

// State::current_state (state.rs:120-134)
OAZ_HD int current_state(const oaz_state& s) {
    if (s.kings[0] == 0 || s.kings[1] == kRedKingStart) return OAZ_BLUE_WIN;
    if (s.kings[1] == 0 || s.kings[0] == kBlueKingStart) return OAZ_RED_WIN;
    return OAZ_IN_PROGRESS;
}

// reward (alphazero_mcts/mod.rs:45-53)
OAZ_HD double reward(int result, int color) {
    if (!is_win(result)) return 0.0;
    return ((result == OAZ_RED_WIN) == (color == OAZ_RED)) ? 1.0 : -1.0;
}

// State::with_deck (state.rs:66-72); first mover = neutral card colour (game_state.rs:37-45)
OAZ_HD void initial_state(const uint8_t deck[5], oaz_state& s) {
    s.kings[0] = kRedKingStart;
    s.kings[1] = kBlueKingStart;
    s.pawns[0] = kRedPawnsStart;
    s.pawns[1] = kBluePawnsStart;
    for (int i = 0; i < 5; ++i) s.cards[i] = deck[i];
    s.to_move = kCardColor[deck[4] & 15];
    s.pad[0] = s.pad[1] = 0;
}

// Packed move (oaz_node.mv): from | to<<5 | slot<<10 | piece<<12
OAZ_HD uint16_t pack_move(int from, int to, int slot, int piece) {
    return (uint16_t)(from | (to << 5) | (slot << 10) | (piece << 12));
}
OAZ_HD int mv_from(uint32_t m) { return m & 31; }
OAZ_HD int mv_to(uint32_t m) { return (m >> 5) & 31; }
OAZ_HD int mv_slot(uint32_t m) { return (m >> 10) & 3; }
OAZ_HD int mv_piece(uint32_t m) { return (m >> 12) & 1; }

// ---- counter-based RNG (DESIGN.md "RNG"): Philox4x32-10 ---------------------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

OAZ_HD u32x4 philox(uint64_t key, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

// uniform in (0,1) with 53 random bits
OAZ_HD double u01(uint32_t a, uint32_t b) {
    const uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return ((double)m + 0.5) * (1.0 / 9007199254740992.0);
}

// ---- Dirichlet root noise (mcts_arena.rs:186-203) ------------------------------------------
// The reference draws a fresh Dirichlet(alpha; K) vector (f64, rand_distr 0.4.3: gamma variates,
// Marsaglia-Tsang with the u^(1/shape) boost for shape < 1, normalised) for every PUCT evaluation at
// the root and uses component child.idx-1: marginally Beta(alpha, (K-1) alpha) = X / (X + Y) with
// X ~ Gamma(alpha), Y ~ Gamma((K-1) alpha). The noise parity with the reference is distributional (its
// thread_rng is unseedable); the draw here is the same Beta marginal in f64, by Johnk's method in the log
// domain (U^(1/0.03) underflows even in f64 for U < 1e-9). log and exp are the polynomials below: only
// IEEE +, -, *, / and explicit fused multiply-adds (correctly rounded on the host, x86 vfmadd / libm fma,
// and on the device, v_fma_f64) with no compiler contraction, so the device, the host (oaz_root_noise)
// and the C oracle compute bit-identical draws.
//
// OAZ_NOISE_F32 (the A/B build only, a measured option): the previous f32 draw (one 32-bit word per
// uniform, polynomials in f32), which resolves the law's ends only to f32.
#ifndef OAZ_NOISE_F32
#define OAZ_NOISE_F32 0
#endif
#if OAZ_NOISE_F32
typedef float noise_t;
#else
typedef double noise_t;
#endif

OAZ_HD float nz_u(uint32_t x) {  // uniform in (0,1): (2k + 1) 2^-24, k = x >> 9 (exact in f32)
    return (float)(((x >> 9) << 1) | 1u) * (1.0f / 16777216.0f);
}
OAZ_HD float nz_log(float x) {  // natural log for normal x > 0 (|rel err| < 2e-7)
    uint32_t b = __builtin_bit_cast(uint32_t, x);
    int e = (int)((b >> 23) & 0xFF) - 127;
    b = (b & 0x007FFFFFu) | 0x3F800000u;  // mantissa m in [1, 2)
    float m = __builtin_bit_cast(float, b);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e += 1;
    }
    const float t = (m - 1.0f) / (m + 1.0f), t2 = t * t;
    const float p = t * (2.0f + t2 * (0.666666667f + t2 * (0.4f + t2 * (0.285714286f + t2 * 0.222222222f))));
    return (float)e * 0.693147182f + p;
}
OAZ_HD float nz_exp(float x) {  // e^x (|rel err| < 3e-7); 0 below -87, +inf above 88
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) return __builtin_bit_cast(float, 0x7F800000u);
    const float k = (float)(int)(x * 1.44269504f + (x >= 0.0f ? 0.5f : -0.5f));
    const float r = (x - k * 0.693145752f) - k * 1.42860677e-6f;  // ln2 split hi + lo
    const float q = 1.0f + r * (1.0f + r * (0.5f + r * (0.166666667f + r * (0.0416666667f + r * (0.00833333333f +
                                                                                        r * 0.00138888889f)))));
    return q * __builtin_bit_cast(float, (uint32_t)((int)k + 127) << 23);
}
// f32 draw (OAZ_NOISE_F32): idx (2j + {0: running best, 1: child j}) of comparison j; c2 = ply << 16 | sim.
// Attempt t takes Philox block (game lo, game hi, c2, idx << 12 | t), words 0, 1 and then 2, 3.
OAZ_HD float root_noise_f32(uint64_t seed, uint64_t game, uint32_t c2, uint32_t idx, float alpha, int K) {
    const float ia = 1.0f / alpha, ib = 1.0f / (alpha * (float)(K - 1));
    for (uint32_t t = 0; t < 1024u; ++t) {
        const u32x4 r = philox(seed, (uint32_t)game, (uint32_t)(game >> 32), c2, (idx << 12) | t);
        const float lx = nz_log(nz_u(r.x)) * ia, ly = nz_log(nz_u(r.y)) * ib;
        if (nz_exp(lx) + nz_exp(ly) <= 1.0f) return 1.0f / (1.0f + nz_exp(ly - lx));
        const float lx2 = nz_log(nz_u(r.z)) * ia, ly2 = nz_log(nz_u(r.w)) * ib;
        if (nz_exp(lx2) + nz_exp(ly2) <= 1.0f) return 1.0f / (1.0f + nz_exp(ly2 - lx2));
    }
    return 1.0f / (float)K;  // (never reached: 2048 rejections in a row)
}

// ln 2 split: kLn2Hi has 21 trailing zero bits (k * kLn2Hi is exact for |k| < 2^21), kLn2Lo the rest.
constexpr double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;
OAZ_HD double nz_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
// natural log for normal x > 0: x = 2^e m, m in [sqrt(1/2), sqrt(2)), t = (m - 1) / (m + 1), log m =
// 2 atanh(t) = 2 (t + t^3 / 3 + ... + t^21 / 21) (|t| <= 0.1716: the next term is < 1e-18 relative).
OAZ_HD double nz_log64(double x) {
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    int e = (int)((b >> 52) & 0x7FF) - 1023;
    double m = __builtin_bit_cast(double, (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double t = (m - 1.0) / (m + 1.0), t2 = t * t;
    double p = 2.0 / 21.0;
    p = nz_fma(p, t2, 2.0 / 19.0);
    p = nz_fma(p, t2, 2.0 / 17.0);
    p = nz_fma(p, t2, 2.0 / 15.0);
    p = nz_fma(p, t2, 2.0 / 13.0);
    p = nz_fma(p, t2, 2.0 / 11.0);
    p = nz_fma(p, t2, 2.0 / 9.0);
    p = nz_fma(p, t2, 2.0 / 7.0);
    p = nz_fma(p, t2, 2.0 / 5.0);
    p = nz_fma(p, t2, 2.0 / 3.0);
    p = nz_fma(p * t2, t, 2.0 * t);  // t (2 + t2 p)
    const double de = (double)e;
    return nz_fma(de, kLn2Hi, nz_fma(de, kLn2Lo, p));
}
// e^x: x = k ln2 + r, |r| <= ln2 / 2, Taylor to r^13 (the remainder is < 5e-18 relative); 0 below -708
// (the normal range), +inf above 709.
OAZ_HD double nz_exp64(double x) {
    if (x < -708.0) return 0.0;
    if (x > 709.0) return __builtin_bit_cast(double, 0x7FF0000000000000ull);
    const double k = (double)(int)(x * 1.4426950408889634 + (x >= 0.0 ? 0.5 : -0.5));
    const double r = (x - k * kLn2Hi) - k * kLn2Lo;
    double q = 1.0 / 6227020800.0;  // 1 / 13!
    q = nz_fma(q, r, 1.0 / 479001600.0);
    q = nz_fma(q, r, 1.0 / 39916800.0);
    q = nz_fma(q, r, 1.0 / 3628800.0);
    q = nz_fma(q, r, 1.0 / 362880.0);
    q = nz_fma(q, r, 1.0 / 40320.0);
    q = nz_fma(q, r, 1.0 / 5040.0);
    q = nz_fma(q, r, 1.0 / 720.0);
    q = nz_fma(q, r, 1.0 / 120.0);
    q = nz_fma(q, r, 1.0 / 24.0);
    q = nz_fma(q, r, 1.0 / 6.0);
    q = nz_fma(q, r, 0.5);
    q = nz_fma(q, r, 1.0);
    q = nz_fma(q, r, 1.0);
    return q * __builtin_bit_cast(double, (uint64_t)((int64_t)k + 1023) << 52);
}
// Draw idx (2j + {0: running best, 1: child j}) of comparison j; c2 = ply << 16 | sim.
// Beta(a, b), a = alpha, b = (K - 1) alpha, by Johnk's method: with U, V uniform, X = U^(1/a),
// Y = V^(1/b), the pairs with X + Y <= 1 give X / (X + Y) ~ Beta(a, b) exactly (acceptance
// Gamma(a+1) Gamma(b+1) / Gamma(a+b+1): 0.99 at K = 12, 0.96 at K = 40). In the log domain:
// lx = log(U) / a, ly = log(V) / b (as products with the rounded reciprocals), X = exp(lx), Y = exp(ly),
// accept when X + Y <= 1, eta = X / (X + Y) when both are normal, else (one of them below e^-708) in the
// log domain, eta = 1 / (1 + exp(ly - lx)). Attempt t takes Philox block (game lo, game hi, c2,
// idx << 12 | t): U from words 0, 1 and V from words 2, 3 (53-bit uniforms, u01).
// Resolution: eta is 1.0 exactly when Y / X < 2^-53, as the reference's X / (X + Y) in f64 is.
OAZ_HD double root_noise_f64(uint64_t seed, uint64_t game, uint32_t c2, uint32_t idx, double alpha, int K) {
    const double ia = 1.0 / alpha, ib = 1.0 / (alpha * (double)(K - 1));
    for (uint32_t t = 0; t < 2048u; ++t) {
        const u32x4 r = philox(seed, (uint32_t)game, (uint32_t)(game >> 32), c2, (idx << 12) | t);
        const double lx = nz_log64(u01(r.x, r.y)) * ia, ly = nz_log64(u01(r.z, r.w)) * ib;
        const double x = nz_exp64(lx), y = nz_exp64(ly), sum = x + y;
        if (sum <= 1.0) return (x > 0.0 && y > 0.0) ? x / sum : 1.0 / (1.0 + nz_exp64(ly - lx));
    }
    return 1.0 / (double)K;  // (never reached: 2048 rejections in a row)
}
// The engine's draw (k_root_noise, oaz_root_noise): f64, or f32 in an OAZ_NOISE_F32 build.
OAZ_HD noise_t root_noise(uint64_t seed, uint64_t game, uint32_t c2, uint32_t idx, double alpha, int K) {
#if OAZ_NOISE_F32
    return root_noise_f32(seed, game, c2, idx, (float)alpha, K);
#else
    return root_noise_f64(seed, game, c2, idx, alpha, K);
#endif
}

// Deck::default (deck.rs:139-151): random 5 of the 16 cards; Fisher-Yates driven by
// Philox(seed; game_id, 0xDEA1, q).
OAZ_HD void deal_deck(uint64_t seed, uint64_t game_id, uint8_t out[5]) {
    uint8_t cards[16];
    for (int i = 0; i < 16; ++i) cards[i] = (uint8_t)i;
    uint32_t w[16];
    for (uint32_t q = 0; q < 4; ++q) {
        const u32x4 r = philox(seed, (uint32_t)game_id, (uint32_t)(game_id >> 32), 0xDEA1u, q);
        w[4 * q] = r.x;
        w[4 * q + 1] = r.y;
        w[4 * q + 2] = r.z;
        w[4 * q + 3] = r.w;
    }
    for (int i = 15, k = 0; i >= 1; --i, ++k) {
        const uint32_t j = (uint32_t)(((uint64_t)w[k] * (uint64_t)(i + 1)) >> 32);
        const uint8_t t = cards[i];
        cards[i] = cards[j];
        cards[j] = t;
    }
    for (int i = 0; i < 5; ++i) out[i] = cards[i];
}

// Global game id of self-play slot g of rank r (of `world` ranks, G slots each) in the slot's seq-th
// game: (seq * world + r) * G + g. The id keys the deal and the root noise, so
// ranks play disjoint games and together every id below (seq + 1) * world * G once per sequence;
// k_selfplay_move's start_game and the host's oaz_slot_game_ids both call this.
OAZ_HD uint64_t slot_game_id(uint64_t seq, uint32_t world, uint32_t rank, uint32_t G, uint32_t g) {
    return (seq * (uint64_t)world + (uint64_t)rank) * (uint64_t)G + (uint64_t)g;
}

OAZ_HD uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// HASH test evaluator: a deterministic stand-in for the NN whose outputs are exact in fp32
// on every device, so MCTS trees can be compared bit for bit ("Hard parts").
OAZ_HD uint64_t hash_state(const oaz_state& s) {
    uint64_t h = splitmix64((uint64_t)s.kings[0] | ((uint64_t)s.kings[1] << 32));
    h = splitmix64(h ^ ((uint64_t)s.pawns[0] | ((uint64_t)s.pawns[1] << 32)));
    const uint64_t c = (uint64_t)(s.cards[0] & 15) | ((uint64_t)(s.cards[1] & 15) << 4) |
                       ((uint64_t)(s.cards[2] & 15) << 8) | ((uint64_t)(s.cards[3] & 15) << 12) |
                       ((uint64_t)(s.cards[4] & 15) << 16) | ((uint64_t)(s.to_move & 1) << 20);
    return splitmix64(h ^ c);
}
OAZ_HD float hash_policy(uint64_t h, int i) {
    return (float)((splitmix64(h + (uint64_t)i) >> 40) + 1) * (1.0f / 16777216.0f);
}
OAZ_HD float hash_value(uint64_t h) {
    const int32_t v = (int32_t)(splitmix64(h ^ 0x5DEECE66Dull) >> 40) - 8388608;
    return (float)v * (1.0f / 8388608.0f);
}

// f64::total_cmp key (argmax ties and signed zeros as Rust orders them)
OAZ_HD int64_t total_key(double x) {
    int64_t i = (int64_t)__builtin_bit_cast(uint64_t, x);
    i ^= (int64_t)(((uint64_t)(i >> 63)) >> 1);
    return i;
}

}  // namespace oaz
