/*
 * oaz_oracle.c — TEST INFRASTRUCTURE ONLY (see oaz_oracle.h).
 *
 * Plain-C restatement of the reference hot path, used as the checker for the HIP engine.
 * Every function cites the reference file:line it follows (paths relative to the
 * reference root). Built with -ffp-contract=off so the f64 MCTS arithmetic is the plain
 * IEEE sequence the Rust code performs.
 */
#include "oaz_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------------------
 * Cards — onitama-game/src/game/card.rs:17-468 (positions, mirror, player_color, index)
 * ---------------------------------------------------------------------------------- */
static const uint32_t CARD_POS[16] = {
    0x20004000u, /* TIGER    card.rs:17-42   */
    0x0440A000u, /* DRAGON   card.rs:44-69   */
    0x02202000u, /* FROG     card.rs:71-96   */
    0x00828000u, /* RABBIT   card.rs:98-123  */
    0x01220000u, /* CRAB     card.rs:125-154 */
    0x02940000u, /* ELEPHANT card.rs:156-185 */
    0x02142000u, /* GOOSE    card.rs:187-216 */
    0x00948000u, /* ROOSTER  card.rs:218-247 */
    0x0280A000u, /* MONKEY   card.rs:249-278 */
    0x02804000u, /* MANTIS   card.rs:280-309 */
    0x0100A000u, /* CRANE    = MANTIS.mirror   card.rs:311-340 */
    0x01104000u, /* HORSE    card.rs:342-371 */
    0x01044000u, /* OX       = HORSE.mirror    card.rs:373-402 */
    0x01140000u, /* BOAR     card.rs:404-433 */
    0x02048000u, /* EEL      card.rs:435-464 (sic: ends 463) */
    0x00902000u, /* COBRA    = EEL.mirror */
};
static const uint32_t CARD_MIR[16] = {
    0x01000200u, 0x02811000u, 0x02022000u, 0x00A08000u, 0x00224000u, 0x0014A000u,
    0x02142000u, 0x00948000u, 0x0280A000u, 0x0100A000u, 0x02804000u, 0x01044000u,
    0x01104000u, 0x00144000u, 0x00902000u, 0x02048000u,
};
/* player_color field of each card: 0 Red, 1 Blue */
static const uint8_t CARD_COL[16] = {1, 0, 0, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0};

uint32_t orc_card_positions(int card) { return CARD_POS[card & 15]; }
uint32_t orc_card_mirror(int card) { return CARD_MIR[card & 15]; }
int orc_card_color(int card) { return CARD_COL[card & 15]; }

/* card.rs:478-517 file masks */
#define FILE_A 0x84210800u
#define FILE_E 0x08421080u
#define FILE_AB 0xC6318C00u
#define FILE_DE 0x18C63180u

/* card.rs:553-604 generate_attack_maps_for_card */
static void attack_maps_for_card(uint32_t card, uint32_t out[25]) {
    memset(out, 0, 25 * sizeof(uint32_t));
    out[12] = card;
    for (int n = 1; n < 13; n++) {
        uint32_t left = (uint32_t)(card << n) & 0xFFFFFF80u;
        uint32_t right = (card >> n) & 0xFFFFFF80u;
        switch (n % 5) {
            case 1: left &= ~FILE_E; right &= ~FILE_A; break;
            case 2: left &= ~FILE_DE; right &= ~FILE_AB; break;
            case 3: left &= ~FILE_AB; right &= ~FILE_DE; break;
            case 4: left &= ~FILE_A; right &= ~FILE_E; break;
            default: break;
        }
        out[12 - n] = left;
        out[12 + n] = right;
    }
}

static uint32_t g_attack[2][16][25];
static pthread_once_t g_attack_once = PTHREAD_ONCE_INIT;

/* card.rs:520-541 generate_attack_maps: Blue uses the mirror */
static void attack_init(void) {
    for (int p = 0; p < 2; p++)
        for (int c = 0; c < 16; c++)
            attack_maps_for_card(p == 1 ? CARD_MIR[c] : CARD_POS[c], g_attack[p][c]);
}

void orc_attack_maps(uint32_t out[2 * 16 * 25]) {
    pthread_once(&g_attack_once, attack_init);
    memcpy(out, g_attack, sizeof(g_attack));
}

/* ------------------------------------------------------------------------------------
 * Bits — onitama-game/src/common/mod.rs:2-4 get_bit, 29-43 set/clear
 * ---------------------------------------------------------------------------------- */
static inline uint32_t get_bit(uint32_t x, int n) { return (x >> (31 - n)) & 1u; }
static inline void set_bit(uint32_t* v, int pos) { *v |= 1u << (31 - pos); }
static inline void clear_bit(uint32_t* v, int pos) { *v &= ~(1u << (31 - pos)); }

/* state.rs:24-45 start squares, 47-49 temples */
#define RED_KING_SP 0x00000200u
#define BLUE_KING_SP 0x20000000u
#define BLUE_PAWNS_SP 0xD8000000u
#define RED_PAWNS_SP 0x00000D80u
#define BLUE_TEMPLE 2
#define RED_TEMPLE 22

/* state.rs:66-72 with_deck; game_state.rs:37-45 first mover = neutral card colour */
void orc_initial_state(const uint8_t deck[5], oaz_state* out) {
    memset(out, 0, sizeof(*out));
    out->kings[0] = RED_KING_SP;
    out->kings[1] = BLUE_KING_SP;
    out->pawns[0] = RED_PAWNS_SP;
    out->pawns[1] = BLUE_PAWNS_SP;
    memcpy(out->cards, deck, 5);
    out->to_move = (uint8_t)CARD_COL[deck[4] & 15];
}

/* state.rs:323-378 generate_legal_moves for one card; appends in (from, to) order */
static int legal_moves_card(const oaz_state* s, int color, int slot, oaz_move* out, int n,
                            uint32_t* masks_row) {
    pthread_once(&g_attack_once, attack_init);
    const int card = s->cards[slot] & 15; /* deck.rs:66-69 get_card */
    const uint32_t pawns = s->pawns[color];
    const uint32_t king = s->kings[color];
    for (int sq = 0; sq < 25; sq++) {
        uint32_t pawn_bit = get_bit(pawns, sq);
        uint32_t king_bit = get_bit(king, sq);
        if (masks_row) masks_row[sq] = 0;
        if (pawn_bit == 0 && king_bit == 0) continue;
        uint32_t am = g_attack[color][card][sq];
        uint32_t map;
        int piece;
        if (pawn_bit == 1) {
            map = ((am | pawns) & ~pawns) & ~king; /* state.rs:351 */
            piece = OAZ_PAWN;
        } else {
            map = ((am | king) & ~king) & ~pawns; /* state.rs:357 */
            piece = OAZ_KING;
        }
        if (masks_row) masks_row[sq] = map;
        for (int i = 0; i < 25; i++) {
            if (get_bit(map, i) == 0) continue;
            if (out) {
                out[n].from = (uint8_t)sq;
                out[n].to = (uint8_t)i;
                out[n].piece = (uint8_t)piece;
                out[n].slot = (uint8_t)slot;
            }
            n++;
        }
    }
    return n;
}

/* state.rs:301-310 generate_all_legal_moves; deck.rs:48-53 get_player_cards_idx */
int orc_movegen(const oaz_state* s, int color, oaz_move* out) {
    int n = 0;
    const int s0 = color == OAZ_RED ? 0 : 2;
    for (int k = 0; k < 2; k++) n = legal_moves_card(s, color, s0 + k, out, n, NULL);
    return n;
}

void orc_movegen_masks(const oaz_state* s, int color, uint32_t masks[2 * 25]) {
    const int s0 = color == OAZ_RED ? 0 : 2;
    for (int k = 0; k < 2; k++) legal_moves_card(s, color, s0 + k, NULL, 0, masks + 25 * k);
}

/* state.rs:145-202 make_move; deck.rs:87-90 rotate */
int orc_make_move(oaz_state* s, const oaz_move* mv, int color) {
    const int from = mv->from, to = mv->to;
    int res = OAZ_IN_PROGRESS;
    if (mv->piece == OAZ_PAWN) clear_bit(&s->pawns[color], from);
    else clear_bit(&s->kings[color], from);
    const int enemy = color ^ 1;
    uint32_t enemy_pawn = get_bit(s->pawns[enemy], to);
    uint32_t enemy_king = get_bit(s->kings[enemy], to);
    if (enemy_pawn == 1) {
        clear_bit(&s->pawns[enemy], to);
        res = OAZ_CAPTURE;
    } else if (enemy_king == 1) {
        clear_bit(&s->kings[enemy], to);
        res = color == OAZ_RED ? OAZ_RED_WIN : OAZ_BLUE_WIN;
    }
    if (mv->piece == OAZ_PAWN) set_bit(&s->pawns[color], to);
    else set_bit(&s->kings[color], to);
    if (mv->piece == OAZ_KING) {
        if (color == OAZ_RED && to == BLUE_TEMPLE) res = OAZ_RED_WIN;
        if (color == OAZ_BLUE && to == RED_TEMPLE) res = OAZ_BLUE_WIN;
    }
    /* deck.rs:87-90: assert!(idx < 4); swap(idx, NEUTRAL) */
    if (mv->slot < 4) {
        uint8_t t = s->cards[mv->slot];
        s->cards[mv->slot] = s->cards[4];
        s->cards[4] = t;
    }
    return res;
}

/* state.rs:120-134 current_state */
int orc_current_state(const oaz_state* s) {
    if (s->kings[0] == 0 || s->kings[1] == RED_KING_SP) return OAZ_BLUE_WIN;
    if (s->kings[1] == 0 || s->kings[0] == BLUE_KING_SP) return OAZ_RED_WIN;
    return OAZ_IN_PROGRESS;
}

/* state.rs:111-117 is_terminal */
int orc_is_terminal(const oaz_state* s) {
    return s->kings[0] == 0 || s->kings[1] == 0 || s->kings[0] == BLUE_KING_SP ||
           s->kings[1] == RED_KING_SP;
}

static inline int is_win(int r) { return r == OAZ_RED_WIN || r == OAZ_BLUE_WIN; }

/* alphazero-training/src/common.rs:26-80 create_tensor_from_state */
void orc_encode(const oaz_state* s, int color, float planes[21 * 25]) {
    memset(planes, 0, 21 * 25 * sizeof(float));
    if (color == OAZ_BLUE)
        for (int i = 0; i < 25; i++) planes[20 * 25 + i] = 1.0f;
    const uint32_t src[4] = {s->pawns[0], s->kings[0], s->pawns[1], s->kings[1]};
    for (int p = 0; p < 4; p++) /* common/mod.rs:69-75 get_bit_array */
        for (int i = 0; i < 25; i++) planes[p * 25 + i] = (float)((src[p] >> (31 - i)) & 1u);
    const int s0 = color == OAZ_RED ? 0 : 2; /* deck.rs:40-46 get_player_cards */
    for (int k = 0; k < 2; k++) {
        const int c = s->cards[s0 + k] & 15;
        for (int i = 0; i < 25; i++) planes[(c + 4) * 25 + i] = 1.0f;
    }
}

/* ------------------------------------------------------------------------------------
 * RNG spec (not in the reference, which uses unseeded thread_rng: deck.rs:139-151,
 * mcts_arena.rs:188). Philox4x32-10, key = seed.
 * ---------------------------------------------------------------------------------- */
void orc_philox(uint64_t key, const uint32_t ctr[4], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline double u01_open(uint32_t a, uint32_t b) {
    uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return ((double)m + 0.5) * (1.0 / 9007199254740992.0);
}

/* deck.rs:139-151 Deck::default — shuffle the 16 cards, take 5 (here Fisher-Yates on
 * Philox keyed by (seed, game_id)). */
void orc_deal_deck(uint64_t seed, uint64_t game_id, uint8_t out[5]) {
    uint8_t cards[16];
    for (int i = 0; i < 16; i++) cards[i] = (uint8_t)i;
    uint32_t words[16];
    for (uint32_t q = 0; q < 4; q++) {
        uint32_t ctr[4] = {(uint32_t)game_id, (uint32_t)(game_id >> 32), 0xDEA1u, q};
        orc_philox(seed, ctr, words + 4 * q);
    }
    for (int i = 15, k = 0; i >= 1; i--, k++) {
        uint32_t j = (uint32_t)(((uint64_t)words[k] * (uint64_t)(i + 1)) >> 32);
        uint8_t t = cards[i];
        cards[i] = cards[j];
        cards[j] = t;
    }
    memcpy(out, cards, 5);
}

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* HASH test evaluator: integer-only, exact in fp32, identical on host and device. */
void orc_hash_eval(const oaz_state* s, float policy[50], float* value) {
    uint64_t h = splitmix64((uint64_t)s->kings[0] | ((uint64_t)s->kings[1] << 32));
    h = splitmix64(h ^ ((uint64_t)s->pawns[0] | ((uint64_t)s->pawns[1] << 32)));
    uint64_t c = (uint64_t)(s->cards[0] & 15) | ((uint64_t)(s->cards[1] & 15) << 4) |
                 ((uint64_t)(s->cards[2] & 15) << 8) | ((uint64_t)(s->cards[3] & 15) << 12) |
                 ((uint64_t)(s->cards[4] & 15) << 16) | ((uint64_t)(s->to_move & 1) << 20);
    h = splitmix64(h ^ c);
    for (int i = 0; i < 50; i++)
        policy[i] = (float)((splitmix64(h + (uint64_t)i) >> 40) + 1) * (1.0f / 16777216.0f);
    int32_t v = (int32_t)(splitmix64(h ^ 0x5DEECE66Dull) >> 40) - 8388608;
    *value = (float)v * (1.0f / 8388608.0f);
}

/* ------------------------------------------------------------------------------------
 * NN — alphazero-training/src/net.rs:9-232, eval mode, fp32.
 * Canonical weight order = tch VarStore construction order (DESIGN.md "Weights").
 * ---------------------------------------------------------------------------------- */
#define CH 64
#define INP 21
size_t orc_weight_count(int blocks) {
    size_t n = (size_t)CH * INP * 9 + CH + 4 * CH;             /* conv_init_1 + bn1 */
    n += (size_t)blocks * 2 * ((size_t)CH * CH * 9 + CH + 4 * CH); /* resnet_i */
    n += CH + 1 + 4 + (size_t)CH * 25 + CH + CH + 1;           /* value head */
    n += 2 * CH + 2 + 8 + 50 * 50 + 50;                         /* policy head */
    return n;
}

typedef struct {
    const float *w, *b, *g, *beta, *mean, *var;
} conv_bn;

static const float* take(const float** p, size_t n) {
    const float* r = *p;
    *p += n;
    return r;
}

static conv_bn take_conv_bn(const float** p, size_t w_n, int cout) {
    conv_bn c;
    c.w = take(p, w_n);
    c.b = take(p, (size_t)cout);
    c.g = take(p, (size_t)cout);
    c.beta = take(p, (size_t)cout);
    c.mean = take(p, (size_t)cout);
    c.var = take(p, (size_t)cout);
    return c;
}

/* conv3x3 stride 1 pad 1 + bias (net.rs:16-26 / 120-130), then BN eval (tch default eps 1e-5).
 * x: [cin][25], y: [CH][25]. */
static __thread float g_wT[9 * CH * CH]; /* [tap][ci][co] so the co loop vectorises */

static void conv3x3_bn(const conv_bn* c, int cin, const float* x, float* y) {
    float acc[25][CH];
    for (int co = 0; co < CH; co++)
        for (int ci = 0; ci < cin; ci++)
            for (int t = 0; t < 9; t++) g_wT[(t * cin + ci) * CH + co] = c->w[((size_t)co * cin + ci) * 9 + t];
    for (int p = 0; p < 25; p++) {
        const int r = p / 5, q = p % 5;
        float* a = acc[p];
        for (int co = 0; co < CH; co++) a[co] = 0.0f;
        for (int t = 0; t < 9; t++) {
            const int rr = r + t / 3 - 1, qq = q + t % 3 - 1;
            if (rr < 0 || rr > 4 || qq < 0 || qq > 4) continue; /* zero padding */
            const int src = rr * 5 + qq;
            for (int ci = 0; ci < cin; ci++) {
                const float xv = x[ci * 25 + src];
                const float* w = &g_wT[(t * cin + ci) * CH];
                for (int co = 0; co < CH; co++) a[co] += xv * w[co];
            }
        }
        for (int co = 0; co < CH; co++) a[co] += c->b[co];
    }
    for (int co = 0; co < CH; co++) {
        const float inv = 1.0f / sqrtf(c->var[co] + 1e-5f);
        for (int p = 0; p < 25; p++)
            y[co * 25 + p] = (acc[p][co] - c->mean[co]) * inv * c->g[co] + c->beta[co];
    }
}

static inline float reluf(float x) { return x > 0.0f ? x : 0.0f; }

static void nn_forward_one(const float* weights, int blocks, const oaz_state* s, float* policy,
                           float* value) {
    const float* p = weights;
    conv_bn init = take_conv_bn(&p, (size_t)CH * INP * 9, CH);
    float x[INP * 25], a[CH * 25], t[CH * 25], y[CH * 25];
    orc_encode(s, s->to_move, x);
    conv3x3_bn(&init, INP, x, a); /* net.rs:119-136 initial block */
    for (int i = 0; i < CH * 25; i++) a[i] = reluf(a[i]);
    for (int b = 0; b < blocks; b++) { /* net.rs:56-65 ResNetBlock::forward_t */
        conv_bn c1 = take_conv_bn(&p, (size_t)CH * CH * 9, CH);
        conv_bn c2 = take_conv_bn(&p, (size_t)CH * CH * 9, CH);
        conv3x3_bn(&c1, CH, a, t);
        for (int i = 0; i < CH * 25; i++) t[i] = reluf(t[i]);
        conv3x3_bn(&c2, CH, t, y);
        for (int i = 0; i < CH * 25; i++) a[i] = reluf(y[i] + a[i]);
    }
    /* value head net.rs:152-181 */
    const float* vw = take(&p, CH);
    const float* vb = take(&p, 1);
    const float *vg = take(&p, 1), *vbeta = take(&p, 1), *vmean = take(&p, 1), *vvar = take(&p, 1);
    const float* l1w = take(&p, (size_t)CH * 25);
    const float* l1b = take(&p, CH);
    const float* l2w = take(&p, CH);
    const float* l2b = take(&p, 1);
    float v1[25], h[CH];
    for (int q = 0; q < 25; q++) {
        float s1 = vb[0];
        for (int c = 0; c < CH; c++) s1 += vw[c] * a[c * 25 + q];
        s1 = (s1 - vmean[0]) * (1.0f / sqrtf(vvar[0] + 1e-5f)) * vg[0] + vbeta[0];
        v1[q] = reluf(s1);
    }
    for (int j = 0; j < CH; j++) {
        float s1 = l1b[j];
        for (int q = 0; q < 25; q++) s1 += l1w[j * 25 + q] * v1[q];
        h[j] = reluf(s1);
    }
    float vv = l2b[0];
    for (int j = 0; j < CH; j++) vv += l2w[j] * h[j];
    *value = tanhf(vv);
    /* policy head net.rs:183-213 */
    const float* pw = take(&p, 2 * CH);
    const float* pb = take(&p, 2);
    const float *pg = take(&p, 2), *pbeta = take(&p, 2), *pmean = take(&p, 2), *pvar = take(&p, 2);
    const float* plw = take(&p, 50 * 50);
    const float* plb = take(&p, 50);
    float f[50], lg[50];
    for (int o = 0; o < 2; o++)
        for (int q = 0; q < 25; q++) {
            float s1 = pb[o];
            for (int c = 0; c < CH; c++) s1 += pw[o * CH + c] * a[c * 25 + q];
            s1 = (s1 - pmean[o]) * (1.0f / sqrtf(pvar[o] + 1e-5f)) * pg[o] + pbeta[o];
            f[o * 25 + q] = reluf(s1); /* flatten(1,-1): index o*25+q */
        }
    float mx = -INFINITY;
    for (int m = 0; m < 50; m++) {
        float s1 = plb[m];
        for (int k = 0; k < 50; k++) s1 += plw[m * 50 + k] * f[k];
        lg[m] = s1;
        if (s1 > mx) mx = s1;
    }
    float sum = 0.0f;
    for (int m = 0; m < 50; m++) {
        lg[m] = expf(lg[m] - mx);
        sum += lg[m];
    }
    for (int m = 0; m < 50; m++) policy[m] = lg[m] / sum; /* reshape [-1,2,25], net.rs:226 */
}

int orc_nn_forward(const float* weights, int blocks, const oaz_state* s, int B, float* policy,
                   float* value) {
    if (!weights || !s || B < 0 || blocks < 0) return OAZ_ERR_ARG;
    for (int i = 0; i < B; i++)
        nn_forward_one(weights, blocks, &s[i], policy + 50 * (size_t)i, value + i);
    return 0;
}

/* ------------------------------------------------------------------------------------
 * AlphaZero MCTS — alphazero-training/src/alphazero_mcts/mcts_arena.rs
 * ---------------------------------------------------------------------------------- */
typedef struct {
    double W, P;
    uint32_t N, first;
    uint16_t nch;
    uint8_t expanded, terminal, color;
    int32_t parent;
    oaz_move mv;
} onode; /* MctsNode mcts_arena.rs:355-373 (children contiguous by construction) */

typedef struct {
    onode* a;
    int n, cap;
} arena_t;

static int arena_push(arena_t* ar, int parent, const oaz_move* mv, int color, double prob) {
    if (ar->n == ar->cap) {
        int nc = ar->cap ? ar->cap * 2 : 1024;
        onode* na = (onode*)realloc(ar->a, (size_t)nc * sizeof(onode));
        if (!na) return -1;
        ar->a = na;
        ar->cap = nc;
    }
    onode* x = &ar->a[ar->n]; /* MctsNode::new mcts_arena.rs:376-396 */
    memset(x, 0, sizeof(*x));
    x->parent = parent;
    if (mv) x->mv = *mv;
    x->color = (uint8_t)color;
    x->P = prob;
    return ar->n++;
}

/* reward — alphazero_mcts/mod.rs:45-53 */
static double reward_fn(int result, int color) {
    if (color == OAZ_RED && result == OAZ_RED_WIN) return 1.0;
    if (color == OAZ_RED && result == OAZ_BLUE_WIN) return -1.0;
    if (color == OAZ_BLUE && result == OAZ_RED_WIN) return -1.0;
    if (color == OAZ_BLUE && result == OAZ_BLUE_WIN) return 1.0;
    return 0.0;
}

/* f64::total_cmp key (Rust core::f64::total_cmp) */
static inline int64_t tkey(double x) {
    int64_t i;
    memcpy(&i, &x, 8);
    i ^= (int64_t)(((uint64_t)(i >> 63)) >> 1);
    return i;
}

/* --- Dirichlet root noise (mcts_arena.rs:186-203). Each PUCT evaluation at the root draws
 * a fresh Dirichlet(alpha; K) vector (f64) and uses component child.idx-1, i.e. a
 * Beta(alpha, (K-1)alpha) variate X/(X+Y) from two gamma variates (rand_distr 0.4.3 Gamma:
 * Marsaglia-Tsang, small-shape boost u^(1/shape)). The reference's thread_rng is unseedable, so
 * noise parity is distributional; this restates the engine's f64 log-domain formulation
 * (oaz_device.h root_noise_f64) op for op so that the engine's draws can be checked bit for bit:
 * the same Beta marginal by Johnk's method, with polynomial log/exp (+, -, *, /, explicit fma and
 * bit operations only; built with -ffp-contract=off). */
typedef struct {
    uint64_t seed, game;
    uint32_t c2;
} noise_key;

static double d_from_u(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static uint64_t u_from_d(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

/* 53-bit uniform in (0, 1) from two Philox words (oaz_device.h u01) */
static double nz_u01(uint32_t a, uint32_t b) {
    const uint64_t m = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return ((double)m + 0.5) * (1.0 / 9007199254740992.0);
}

static const double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;

/* log x for normal x > 0: x = 2^e m, m in [sqrt(1/2), sqrt(2)), 2 atanh((m-1)/(m+1)) to t^21 */
static double nz_log64(double x) {
    const uint64_t b = u_from_d(x);
    int e = (int)((b >> 52) & 0x7FF) - 1023;
    double m = d_from_u((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double t = (m - 1.0) / (m + 1.0), t2 = t * t;
    double p = 2.0 / 21.0;
    p = fma(p, t2, 2.0 / 19.0);
    p = fma(p, t2, 2.0 / 17.0);
    p = fma(p, t2, 2.0 / 15.0);
    p = fma(p, t2, 2.0 / 13.0);
    p = fma(p, t2, 2.0 / 11.0);
    p = fma(p, t2, 2.0 / 9.0);
    p = fma(p, t2, 2.0 / 7.0);
    p = fma(p, t2, 2.0 / 5.0);
    p = fma(p, t2, 2.0 / 3.0);
    p = fma(p * t2, t, 2.0 * t);
    const double de = (double)e;
    return fma(de, kLn2Hi, fma(de, kLn2Lo, p));
}

/* e^x: x = k ln2 + r, Taylor to r^13; 0 below -708, +inf above 709 */
static double nz_exp64(double x) {
    if (x < -708.0) return 0.0;
    if (x > 709.0) return d_from_u(0x7FF0000000000000ull);
    const double k = (double)(int)(x * 1.4426950408889634 + (x >= 0.0 ? 0.5 : -0.5));
    const double r = (x - k * kLn2Hi) - k * kLn2Lo;
    double q = 1.0 / 6227020800.0;
    q = fma(q, r, 1.0 / 479001600.0);
    q = fma(q, r, 1.0 / 39916800.0);
    q = fma(q, r, 1.0 / 3628800.0);
    q = fma(q, r, 1.0 / 362880.0);
    q = fma(q, r, 1.0 / 40320.0);
    q = fma(q, r, 1.0 / 5040.0);
    q = fma(q, r, 1.0 / 720.0);
    q = fma(q, r, 1.0 / 120.0);
    q = fma(q, r, 1.0 / 24.0);
    q = fma(q, r, 1.0 / 6.0);
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = fma(q, r, 1.0);
    return q * d_from_u((uint64_t)((int64_t)k + 1023) << 52);
}

/* Beta(a, b), a = alpha, b = (K-1) alpha, by Johnk's method (exact): X = U^(1/a), Y = V^(1/b),
 * accept X + Y <= 1, eta = X / (X + Y) (when X or Y is below e^-708: 1 / (1 + exp(ly - lx))); in the
 * log domain with products by the rounded reciprocals; attempt t uses Philox block (game lo, game hi, c2,
 * idx << 12 | t): U from words 0, 1, V from words 2, 3 (oaz_device.h root_noise_f64, op for op). */
static double beta_noise(const noise_key* k, uint32_t idx, double alpha, int nchild) {
    const double ia = 1.0 / alpha, ib = 1.0 / (alpha * (double)(nchild - 1));
    for (uint32_t t = 0; t < 2048u; t++) {
        uint32_t r[4];
        const uint32_t ctr[4] = {(uint32_t)k->game, (uint32_t)(k->game >> 32), k->c2, (idx << 12) | t};
        orc_philox(k->seed, ctr, r);
        const double lx = nz_log64(nz_u01(r[0], r[1])) * ia, ly = nz_log64(nz_u01(r[2], r[3])) * ib;
        const double x = nz_exp64(lx), y = nz_exp64(ly), sum = x + y;
        if (sum <= 1.0) return (x > 0.0 && y > 0.0) ? x / sum : 1.0 / (1.0 + nz_exp64(ly - lx));
    }
    return 1.0 / (double)nchild;
}

double orc_root_noise(uint64_t seed, uint64_t game_id, uint32_t c2, uint32_t draw, double alpha, int nchild) {
    const noise_key k = {seed, game_id, c2};
    return beta_noise(&k, draw, alpha, nchild);
}

typedef struct {
    const orc_search_cfg* cfg;
    arena_t ar;
    oaz_state root;
    int root_color;
    uint32_t sim;
    oaz_search_stats* st;
} search_t;

/* uct closure — mcts_arena.rs:190-209 */
static double uct(const search_t* S, const onode* parent, const onode* ch, int is_root_noise,
                  double noise) {
    const double q = ch->N ? ch->W / (double)ch->N : 0.0; /* winrate = reward / visits */
    const double c = S->cfg->c_puct;
    const double sq = sqrt((double)parent->N) / (double)(ch->N + 1);
    if (is_root_noise) {
        const double eps = S->cfg->eps;
        return q + c * (ch->P * (1.0 - eps) + noise * eps) * sq;
    }
    return q + c * ch->P * sq;
}

/* select — mcts_arena.rs:183-223. Iterator::max_by keeps the LAST maximum; the closure is
 * re-evaluated for both operands of every comparison (fresh noise each time at the root). */
static int select_child(search_t* S, int pidx) {
    const onode* parent = &S->ar.a[pidx];
    const int K = parent->nch;
    const int noise = (parent->parent < 0) && S->cfg->train_noise;
    noise_key nk = {S->cfg->seed, S->cfg->game_id,
                    ((S->cfg->ply & 0xFFFFu) << 16) | (S->sim & 0xFFFFu)};
    int acc = (int)parent->first;
    for (int j = 1; j < K; j++) {
        const int b = (int)parent->first + j;
        double na = 0.0, nb = 0.0;
        if (noise) {
            na = beta_noise(&nk, (uint32_t)(2 * j), S->cfg->alpha, K);
            nb = beta_noise(&nk, (uint32_t)(2 * j + 1), S->cfg->alpha, K);
        }
        const double ua = uct(S, parent, &S->ar.a[acc], noise, na);
        const double ub = uct(S, parent, &S->ar.a[b], noise, nb);
        /* cmp::max_by: Greater keeps a, Less/Equal takes b */
        if (!(tkey(ua) > tkey(ub))) acc = b;
    }
    return acc;
}

typedef struct {
    oaz_move moves[OAZ_MAX_MOVES];
    int nmoves;
    double value;
    double priors[2][25];
} eval_result;

/* evaluate — mcts_arena.rs:267-310 */
static void evaluate(search_t* S, const oaz_state* gs, eval_result* er) {
    float policy[50], value = 0.0f;
    const orc_search_cfg* cfg = S->cfg;
    if (cfg->evaluator == OAZ_EVAL_NN) nn_forward_one(cfg->weights, cfg->blocks, gs, policy, &value);
    else if (cfg->evaluator == OAZ_EVAL_HASH) orc_hash_eval(gs, policy, &value);
    else cfg->fn(cfg->ctx, gs, policy, &value);
    er->nmoves = orc_movegen(gs, gs->to_move, er->moves);
    memset(er->priors, 0, sizeof(er->priors));
    for (int i = 0; i < er->nmoves; i++) {
        const int row = er->moves[i].slot % 2, to = er->moves[i].to;
        er->priors[row][to] = (double)policy[row * 25 + to];
    }
    for (int row = 0; row < 2; row++) {
        double sum = 0.0;
        for (int i = 0; i < 25; i++) sum += er->priors[row][i];
        if (sum > 0.0)
            for (int i = 0; i < 25; i++) er->priors[row][i] /= sum;
    }
    er->value = (double)value;
}

/* expand — mcts_arena.rs:231-260 */
static int expand(search_t* S, int pidx, const eval_result* er) {
    const int color = S->ar.a[pidx].color;
    const int first = S->ar.n;
    for (int i = 0; i < er->nmoves; i++) {
        const oaz_move* mv = &er->moves[i];
        const double prob = er->priors[mv->slot % 2][mv->to];
        if (arena_push(&S->ar, pidx, mv, color ^ 1, prob) < 0) return -1;
    }
    S->ar.a[pidx].first = (uint32_t)first;
    S->ar.a[pidx].nch = (uint16_t)er->nmoves;
    S->ar.a[pidx].expanded = 1;
    S->st->expansions++;
    S->st->children += (uint64_t)er->nmoves;
    return 0;
}

/* back_propagate — mcts_arena.rs:312-323; MctsNode::update 398-402 */
static void back_propagate(search_t* S, int idx, double r) {
    for (;;) {
        onode* x = &S->ar.a[idx];
        x->N += 1;
        x->W += r;
        if (x->parent < 0) break;
        idx = x->parent;
        r = -r;
    }
}

/* playout — mcts_arena.rs:127-177 */
static int playout(search_t* S) {
    oaz_state gs = S->root;
    int node = 0;
    uint32_t depth = 0;
    while (S->ar.a[node].expanded && !S->ar.a[node].terminal) {
        if (S->ar.a[node].nch == 0) { /* reference panics in select (Q6): treat as a leaf */
            S->st->stuck_leaves++;
            break;
        }
        node = select_child(S, node);
        const onode* x = &S->ar.a[node];
        const int mover = S->ar.a[x->parent].color;
        const int res = orc_make_move(&gs, &x->mv, mover);
        gs.to_move ^= 1; /* game_state.player_color.switch() */
        if (is_win(res)) S->ar.a[node].terminal = 1;
        depth++;
    }
    eval_result er;
    evaluate(S, &gs, &er);
    const int expands = !S->ar.a[node].expanded && !S->ar.a[node].terminal;
    if (expands)
        if (expand(S, node, &er) < 0) return -1;
    const int parent = S->ar.a[node].parent >= 0 ? S->ar.a[node].parent : 0;
    const int reward_color = S->ar.a[parent].color;
    const int mr = orc_current_state(&gs);
    S->st->sims++;
    S->st->nn_evals += (uint64_t)(expands || !is_win(mr)); /* the evaluation is used (priors or value) */
    S->st->depth_sum += depth;
    if (is_win(mr)) {
        S->st->terminal_leaves++;
        back_propagate(S, node, reward_fn(mr, reward_color));
    } else {
        back_propagate(S, node, er.value);
    }
    return 0;
}

/* search — mcts_arena.rs:75-102; calculate_priors 104-124 */
int orc_search(const orc_search_cfg* cfg, const oaz_state* root, oaz_move* out_move,
               float out_pi[50], oaz_node* out_nodes, int cap, int* n_nodes,
               oaz_search_stats* stats) {
    if (!cfg || !root) return OAZ_ERR_ARG;
    oaz_search_stats local;
    memset(&local, 0, sizeof(local));
    search_t S;
    memset(&S, 0, sizeof(S));
    S.cfg = cfg;
    S.root = *root;
    S.root_color = root->to_move;
    S.st = stats ? stats : &local;
    if (arena_push(&S.ar, -1, NULL, root->to_move, 1.0) < 0) return OAZ_ERR_CAPACITY;
    for (S.sim = 0; S.sim < (uint32_t)cfg->sims; S.sim++)
        if (playout(&S) < 0) {
            free(S.ar.a);
            return OAZ_ERR_CAPACITY;
        }
    const onode* r = &S.ar.a[0];
    float pi[50];
    memset(pi, 0, sizeof(pi));
    float sum = 0.0f;
    for (uint32_t i = 0; i < r->nch; i++) {
        const onode* ch = &S.ar.a[r->first + i];
        pi[(ch->mv.slot % 2) * 25 + ch->mv.to] += (float)ch->N;
    }
    for (int i = 0; i < 50; i++) sum += pi[i];
    if (sum > 0.0f)
        for (int i = 0; i < 50; i++) pi[i] /= sum;
    if (out_pi) memcpy(out_pi, pi, sizeof(pi));
    oaz_move best;
    memset(&best, 0, sizeof(best));
    if (r->nch == 0) { /* no legal move (Q6): pass with the mover's first card */
        best.from = 25;
        best.to = 25;
        best.piece = 0;
        best.slot = (uint8_t)(root->to_move == OAZ_RED ? 0 : 2);
    } else {
        int bi = (int)r->first;
        double bv = (double)S.ar.a[bi].N / (double)r->N;
        for (uint32_t i = 1; i < r->nch; i++) {
            const int ci = (int)r->first + (int)i;
            const double v = (double)S.ar.a[ci].N / (double)r->N;
            if (!(tkey(bv) > tkey(v))) {
                bi = ci;
                bv = v;
            }
        }
        best = S.ar.a[bi].mv;
    }
    if (out_move) *out_move = best;
    if ((uint64_t)S.ar.n > S.st->max_nodes) S.st->max_nodes = (uint64_t)S.ar.n;
    if (n_nodes) *n_nodes = S.ar.n;
    if (out_nodes) {
        const int n = S.ar.n < cap ? S.ar.n : cap;
        for (int i = 0; i < n; i++) {
            const onode* x = &S.ar.a[i];
            oaz_node* o = &out_nodes[i];
            memset(o, 0, sizeof(*o));
            o->W = x->W;
            o->P = x->P;
            o->N = x->N;
            o->first = x->expanded ? x->first : 0;
            o->mv = (uint16_t)(x->mv.from | (x->mv.to << 5) | (x->mv.slot << 10) | (x->mv.piece << 12));
            o->nch = (uint8_t)x->nch;
            o->flags = (uint8_t)((x->expanded ? 1 : 0) | (x->terminal ? 2 : 0));
        }
    }
    free(S.ar.a);
    return 0;
}

/* ------------------------------------------------------------------------------------
 * self_play — alphazero-training/src/train.rs:35-98 (one game)
 * ---------------------------------------------------------------------------------- */
int orc_selfplay_game(const orc_selfplay_cfg* cfg, uint64_t game_id, oaz_sample* out, int cap,
                      int* result, int* plies, oaz_search_stats* stats) {
    uint8_t deck[5];
    if (cfg->fixed_deck) memcpy(deck, cfg->deck, 5);
    else orc_deal_deck(cfg->search.seed, game_id, deck);
    oaz_state st;
    orc_initial_state(deck, &st); /* colour = neutral card colour (train.rs:49) */
    int progress = OAZ_IN_PROGRESS;
    int max_plies = cfg->max_plies;
    int n = 0;
    orc_search_cfg sc = cfg->search;
    sc.game_id = game_id;
    uint32_t ply = 0;
    while (!is_win(progress)) {
        sc.ply = ply;
        oaz_move mv;
        float pi[50];
        int rc = orc_search(&sc, &st, &mv, pi, NULL, 0, NULL, stats);
        if (rc) return rc;
        if (n < cap) {
            out[n].state = st;
            memcpy(out[n].pi, pi, sizeof(pi));
            out[n].z = 0.0f;
        }
        n++;
        if (mv.from >= 25) { /* pass: rotate the card (state.rs:139-142), Q6 */
            uint8_t t = st.cards[mv.slot];
            st.cards[mv.slot] = st.cards[4];
            st.cards[4] = t;
            progress = OAZ_IN_PROGRESS;
        } else {
            progress = orc_make_move(&st, &mv, st.to_move);
        }
        st.to_move ^= 1;
        ply++;
        if (max_plies < 0) break; /* train.rs:74-79 */
        max_plies -= 1;
    }
    const int m = n < cap ? n : cap;
    for (int i = 0; i < m; i++) out[i].z = (float)reward_fn(progress, out[i].state.to_move);
    if (result) *result = progress;
    if (plies) *plies = (int)ply;
    return m;
}

/* ------------------------------------------------------------------------------------
 * CPU baseline: thread-per-worker self-play (train.rs:218-245), batch-1 NN per simulation.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    const orc_selfplay_cfg* cfg;
    int tid, threads;
    double deadline;
    int64_t sims, games, plies;
} bench_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* bench_worker(void* p) {
    bench_arg* a = (bench_arg*)p;
    orc_search_cfg sc = a->cfg->search;
    uint64_t game = (uint64_t)a->tid;
    while (now_s() < a->deadline) {
        uint8_t deck[5];
        if (a->cfg->fixed_deck) memcpy(deck, a->cfg->deck, 5);
        else orc_deal_deck(sc.seed, game, deck);
        oaz_state st;
        orc_initial_state(deck, &st);
        int progress = OAZ_IN_PROGRESS, max_plies = a->cfg->max_plies;
        uint32_t ply = 0;
        sc.game_id = game;
        while (!is_win(progress) && now_s() < a->deadline) {
            oaz_search_stats ss;
            memset(&ss, 0, sizeof(ss));
            oaz_move mv;
            sc.ply = ply;
            if (orc_search(&sc, &st, &mv, NULL, NULL, 0, NULL, &ss)) return NULL;
            a->sims += (int64_t)ss.sims;
            a->plies++;
            if (mv.from >= 25) {
                uint8_t t = st.cards[mv.slot];
                st.cards[mv.slot] = st.cards[4];
                st.cards[4] = t;
                progress = OAZ_IN_PROGRESS;
            } else {
                progress = orc_make_move(&st, &mv, st.to_move);
            }
            st.to_move ^= 1;
            ply++;
            if (max_plies < 0) break;
            max_plies--;
        }
        if (is_win(progress) || max_plies < 0) a->games++;
        game += (uint64_t)a->threads;
    }
    return NULL;
}

int64_t orc_selfplay_bench(const orc_selfplay_cfg* cfg, int threads, double seconds,
                           int64_t* games_done, int64_t* plies_done) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    bench_arg* args = (bench_arg*)calloc((size_t)threads, sizeof(bench_arg));
    const double deadline = now_s() + seconds;
    for (int i = 0; i < threads; i++) {
        args[i].cfg = cfg;
        args[i].tid = i;
        args[i].threads = threads;
        args[i].deadline = deadline;
        pthread_create(&th[i], NULL, bench_worker, &args[i]);
    }
    int64_t sims = 0, games = 0, plies = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        sims += args[i].sims;
        games += args[i].games;
        plies += args[i].plies;
    }
    free(th);
    free(args);
    if (games_done) *games_done = games;
    if (plies_done) *plies_done = plies;
    return sims;
}


/* Batch of independent searches on host threads (the checker for bench-size GPU searches): root i
 * runs orc_search with game_id = game_ids[i] (or cfg->game_id + i); workers take roots from a
 * shared counter. */
typedef struct {
    const orc_search_cfg* cfg;
    const oaz_state* roots;
    const uint64_t* game_ids;
    int n;
    oaz_move* out_move;
    float* out_pi;
    int* next;
    pthread_mutex_t* mu;
    oaz_search_stats st;
    int rc;
} batch_arg;

static void* batch_worker(void* p) {
    batch_arg* a = (batch_arg*)p;
    orc_search_cfg c = *a->cfg;
    for (;;) {
        pthread_mutex_lock(a->mu);
        const int i = (*a->next)++;
        pthread_mutex_unlock(a->mu);
        if (i >= a->n) break;
        c.game_id = a->game_ids ? a->game_ids[i] : a->cfg->game_id + (uint64_t)i;
        oaz_search_stats st;
        memset(&st, 0, sizeof(st));
        const int rc = orc_search(&c, &a->roots[i], &a->out_move[i], a->out_pi + (size_t)i * 50, NULL, 0, NULL, &st);
        if (rc < 0) a->rc = rc;
        a->st.sims += st.sims;
        a->st.expansions += st.expansions;
        a->st.children += st.children;
        a->st.terminal_leaves += st.terminal_leaves;
        a->st.nn_evals += st.nn_evals;
        a->st.depth_sum += st.depth_sum;
        a->st.stuck_leaves += st.stuck_leaves;
        if (st.max_nodes > a->st.max_nodes) a->st.max_nodes = st.max_nodes;
    }
    return NULL;
}

int orc_search_batch(const orc_search_cfg* cfg, const oaz_state* roots, const uint64_t* game_ids, int n, int threads,
                     oaz_move* out_move, float* out_pi, oaz_search_stats* stats) {
    if (!cfg || !roots || n < 0 || !out_move || !out_pi) return OAZ_ERR_ARG;
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    batch_arg* args = (batch_arg*)calloc((size_t)threads, sizeof(batch_arg));
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    int next = 0;
    for (int i = 0; i < threads; i++) {
        args[i].cfg = cfg;
        args[i].roots = roots;
        args[i].game_ids = game_ids;
        args[i].n = n;
        args[i].out_move = out_move;
        args[i].out_pi = out_pi;
        args[i].next = &next;
        args[i].mu = &mu;
        pthread_create(&th[i], NULL, batch_worker, &args[i]);
    }
    int rc = 0;
    oaz_search_stats sum;
    memset(&sum, 0, sizeof(sum));
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        if (args[i].rc < 0) rc = args[i].rc;
        sum.sims += args[i].st.sims;
        sum.expansions += args[i].st.expansions;
        sum.children += args[i].st.children;
        sum.terminal_leaves += args[i].st.terminal_leaves;
        sum.nn_evals += args[i].st.nn_evals;
        sum.depth_sum += args[i].st.depth_sum;
        sum.stuck_leaves += args[i].st.stuck_leaves;
        if (args[i].st.max_nodes > sum.max_nodes) sum.max_nodes = args[i].st.max_nodes;
    }
    free(th);
    free(args);
    if (stats) *stats = sum;
    return rc;
}

/* ---- pure MCTS (onitama-game/src/ai/mcts/mcts_arena.rs) ---------------------------------- */
typedef struct {
    uint64_t seed;
    uint32_t game, playout, d, buf[4];
} pm_rng;

static uint32_t pm_next(pm_rng* r) {
    if ((r->d & 3) == 0) {
        const uint32_t ctr[4] = {r->game, r->playout, 0x9C7A0000u, r->d >> 2};
        orc_philox(r->seed, ctr, r->buf);
    }
    return r->buf[r->d++ & 3];
}

static uint32_t pm_below(pm_rng* r, uint32_t n) { return (uint32_t)(((uint64_t)pm_next(r) * n) >> 32); }

/* mcts_arena.rs:233-241 */
static float pm_reward(int result, int color) {
    if (result == OAZ_RED_WIN) return color == OAZ_RED ? 1.0f : -1.0f;
    if (result == OAZ_BLUE_WIN) return color == OAZ_BLUE ? 1.0f : -1.0f;
    return 0.0f;
}

static uint16_t pm_pack(const oaz_move* m) {
    return (uint16_t)(m->from | (m->to << 5) | (m->slot << 10) | (m->piece << 12));
}

static void pm_unpack(uint16_t v, oaz_move* m) {
    m->from = v & 31;
    m->to = (v >> 5) & 31;
    m->slot = (v >> 10) & 3;
    m->piece = (v >> 12) & 1;
}

/* f32::total_cmp(a, b) > 0 */
static int pm_total_ge(float a, float b) {
    int32_t ia, ib;
    memcpy(&ia, &a, 4);
    memcpy(&ib, &b, 4);
    ia ^= (int32_t)((uint32_t)(ia >> 31) >> 1);
    ib ^= (int32_t)((uint32_t)(ib >> 31) >> 1);
    return ia >= ib;
}

int orc_pure_mcts(const oaz_pure_mcts_config* cfg, uint64_t game_id, const oaz_state* root, oaz_move* out_move,
                  float* out_value, oaz_pure_node* T, int cap, oaz_pure_mcts_stats* stats) {
    if (cap < 1) return -1;
    const int root_color = root->to_move & 1;
    memset(&T[0], 0, sizeof(T[0]));
    T[0].parent = 0xFFFFFFFFu;
    int n_nodes = 1;
    oaz_move moves[40];
    for (int po = 0; po < cfg->max_playouts; ++po) {  /* search, mcts_arena.rs:56-62 */
        oaz_state s = *root;
        uint32_t idx = 0;
        /* playout step 1 (:100-116): select while expanded and not terminal */
        while ((T[idx].flags & 1) && !(T[idx].flags & 2) && T[idx].nch) {
            const float lnN = logf((float)T[idx].visits);
            uint32_t best = T[idx].first;
            float bu = 0.0f;
            for (uint32_t c = T[idx].first; c < T[idx].first + T[idx].nch; ++c) {
                const float u = T[c].winrate + cfg->exploration_c * sqrtf(lnN / (float)T[c].visits); /* :141-143 */
                if (c == T[idx].first || pm_total_ge(u, bu)) { /* max_by keeps the last maximum */
                    bu = u;
                    best = c;
                }
            }
            oaz_move m;
            pm_unpack(T[best].mv, &m);
            const int res = orc_make_move(&s, &m, s.to_move & 1);
            s.to_move ^= 1;
            if (res == OAZ_RED_WIN || res == OAZ_BLUE_WIN) T[best].flags |= 2;
            idx = best;
        }
        /* step 2 (:118-124): expand (:166-185) */
        if (!(T[idx].flags & 3) && T[idx].visits > (uint32_t)cfg->min_node_visits) {
            const int n = orc_movegen(&s, s.to_move & 1, moves);
            if (n_nodes + n <= cap) {
                T[idx].first = (uint32_t)n_nodes;
                T[idx].nch = (uint8_t)n;
                for (int k = 0; k < n; ++k) {
                    oaz_pure_node* ch = &T[n_nodes + k];
                    memset(ch, 0, sizeof(*ch));
                    ch->parent = idx;
                    ch->mv = pm_pack(&moves[k]);
                }
                n_nodes += n;
                T[idx].flags |= 1;
                if (stats) stats->expansions++;
            } else if (stats) {
                stats->tree_full++;
            }
        }
        /* step 3 (:126-130, simulate :188-231): reward colour = the parent's colour */
        const int reward_color = idx == 0 ? root_color : ((s.to_move & 1) ^ 1);
        pm_rng rng = {cfg->seed, (uint32_t)game_id, (uint32_t)po, 0, {0, 0, 0, 0}};
        int mr = orc_current_state(&s);
        float r;
        if (mr == OAZ_RED_WIN || mr == OAZ_BLUE_WIN) {
            r = pm_reward(mr, reward_color);
        } else {
            int color = s.to_move & 1, plies = 0, capped = 0;
            while (mr != OAZ_RED_WIN && mr != OAZ_BLUE_WIN) {
                if (plies >= cfg->rollout_cap) {
                    capped = 1;
                    break;
                }
                const int n = orc_movegen(&s, color, moves);
                if (n == 0) { /* pass with a random own card */
                    const int slot = (color == OAZ_RED ? 0 : 2) + (int)pm_below(&rng, 2);
                    const uint8_t t = s.cards[slot];
                    s.cards[slot] = s.cards[4];
                    s.cards[4] = t;
                    color ^= 1;
                    plies++;
                    if (stats) stats->rollout_passes++;
                    continue;
                }
                const oaz_move m = moves[pm_below(&rng, (uint32_t)n)];
                mr = orc_make_move(&s, &m, color);
                color ^= 1;
                plies++;
            }
            if (stats) stats->rollout_plies += (uint64_t)plies;
            if (capped) {
                r = 0.0f;
                if (stats) stats->rollouts_capped++;
            } else {
                r = pm_reward(mr, reward_color);
            }
        }
        /* step 4 (:243-254) */
        for (uint32_t v = idx;;) {
            T[v].visits += 1;
            T[v].reward += r;
            T[v].winrate = T[v].reward / (float)T[v].visits;
            if (v == 0) break;
            v = T[v].parent;
            r = -r;
        }
        if (stats) stats->playouts++;
    }
    if (stats && (uint64_t)n_nodes > stats->max_nodes) stats->max_nodes = (uint64_t)n_nodes;
    if (T[0].nch == 0) {
        out_move->from = 25;
        out_move->to = 25;
        out_move->piece = 0;
        out_move->slot = (uint8_t)(root_color ? 2 : 0);
        *out_value = 0.0f;
    } else {
        uint32_t best = T[0].first, bv = 0;
        for (uint32_t c = T[0].first; c < T[0].first + T[0].nch; ++c)
            if (T[c].visits >= bv) { /* max_by_key: last maximum */
                bv = T[c].visits;
                best = c;
            }
        pm_unpack(T[best].mv, out_move);
        *out_value = T[best].winrate;
    }
    return n_nodes;
}

typedef struct {
    const oaz_pure_mcts_config* cfg;
    double seconds;
    int tid;
    int64_t playouts, searches;
} pm_bench_arg;

static void* pm_bench_worker(void* p) {
    pm_bench_arg* a = (pm_bench_arg*)p;
    const int cap = (int)(1 + 40 * (a->cfg->max_playouts / (a->cfg->min_node_visits + 1) + 1));
    oaz_pure_node* T = (oaz_pure_node*)malloc(sizeof(oaz_pure_node) * (size_t)cap);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t g = (uint64_t)a->tid << 32;; ++g) {
        uint8_t deck[5];
        orc_deal_deck(a->cfg->seed, g, deck);
        oaz_state root;
        orc_initial_state(deck, &root);
        oaz_move mv;
        float v;
        oaz_pure_mcts_stats st;
        memset(&st, 0, sizeof(st));
        orc_pure_mcts(a->cfg, g, &root, &mv, &v, T, cap, &st);
        a->playouts += (int64_t)st.playouts;
        a->searches++;
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if ((double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec) >= a->seconds) break;
    }
    free(T);
    return NULL;
}

int64_t orc_pure_mcts_bench(const oaz_pure_mcts_config* cfg, int threads, double seconds, int64_t* searches) {
    pthread_t th[256];
    pm_bench_arg args[256];
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (int i = 0; i < threads; ++i) {
        args[i].cfg = cfg;
        args[i].seconds = seconds;
        args[i].tid = i;
        args[i].playouts = args[i].searches = 0;
        pthread_create(&th[i], NULL, pm_bench_worker, &args[i]);
    }
    int64_t total = 0, ns = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        total += args[i].playouts;
        ns += args[i].searches;
    }
    if (searches) *searches = ns;
    return total;
}
