// oaz_kernels.hip — gfx950 kernels for the rules and the AlphaZero search.
//
// Execution model: ONE WAVEFRONT (64 lanes) PER GAME for everything tree-shaped.
//   * move generation: lane = (card k, from square) for k in {0,1}, from in 0..24 (50 lanes);
//     each lane produces one 25-bit destination mask, a wave prefix sum over popcounts gives
//     the reference order (slot, from, to) (state.rs:301-378) with no sort;
//   * PUCT select: lane = child (K <= 40 < 64); a child's 32-byte node is one coalesced
//     load per lane, the argmax (last maximum wins, mcts_arena.rs:213-220) is a butterfly
//     over the wave; one dependent memory round trip per tree level;
//   * backup: lane = depth along the recorded path, all levels updated in parallel.
// The f64 PUCT arithmetic is the reference's expression order, compiled with
// -ffp-contract=off; sqrt(N) comes from a host-built table so every bit matches the oracle.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <utility>

#include "oaz_device.h"
#include "oaz_kernels.h"

namespace oaz {

__constant__ AttackTable c_attack = make_attack_table();

constexpr int kWave = 64;
#ifndef OAZ_TREE_WPE
#define OAZ_TREE_WPE 8  // waves per SIMD the segmented tree kernels are register-budgeted for (64 VGPRs)
#endif
#ifndef OAZ_TREE_WPB
#define OAZ_TREE_WPB 8
#endif
constexpr int kWavesPerBlock = OAZ_TREE_WPB;  // waves per workgroup of the tree kernels
constexpr int kBlock = kWave * kWavesPerBlock;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint32_t wave_game() {
    return blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}
// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, off);
        if (l >= off) v += t;
    }
    return v;
}
// argmax of (key, lane) keeping the LARGEST lane among equal keys (Iterator::max_by).
// value of lane `lane` (wave-uniform index) as a wave-uniform double
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int wave_argmax_last(int64_t key) {
    int idx = lane_id();
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int64_t ok = __shfl_xor(key, off);
        const int oi = __shfl_xor(idx, off);
        if (ok > key || (ok == key && oi > idx)) {
            key = ok;
            idx = oi;
        }
    }
    return idx;
}

__device__ __forceinline__ oaz_state load_state(const oaz_state* p) {
    oaz_state s;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    uint32_t* d = reinterpret_cast<uint32_t*>(&s);
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = q[i];
    return s;
}
__device__ __forceinline__ void store_state(oaz_state* p, const oaz_state& s) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    const uint32_t* d = reinterpret_cast<const uint32_t*>(&s);
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = d[i];
}

// ---- wave-parallel move generation ------------------------------------------------------
// Lane (k, from): destination mask of the mover's piece on `from` with its k-th card.
// Pawn and king masks of the reference (state.rs:351,357) both reduce to
// attack & ~(own pawns | own king); the piece kind is the one on `from`.
struct LaneMoves {
    uint32_t mask;
    int piece;
    int slot;
    int from;
};

__device__ __forceinline__ LaneMoves lane_movegen(const oaz_state& s) {
    const int l = lane_id();
    const int color = s.to_move & 1;
    const int k = l >= 25 ? 1 : 0;
    const int from = l - 25 * k;
    const uint32_t pawns = s.pawns[color], king = s.kings[color];
    const uint32_t own = pawns | king;
    LaneMoves m;
    m.slot = (color ? 2 : 0) + k;
    m.from = from;
    m.piece = (pawns & sq_bit(from)) ? OAZ_PAWN : OAZ_KING;
    m.mask = 0;
    if (l < 50 && (own & sq_bit(from)))
        m.mask = c_attack.m[color][s.cards[m.slot] & 15][from] & ~own;
    return m;
}

__global__ void __launch_bounds__(kBlock) k_movegen(const oaz_state* __restrict__ states, int n,
                                                    uint32_t* masks, oaz_move* moves,
                                                    uint8_t* counts) {
    const uint32_t g = wave_game();
    if (g >= (uint32_t)n) return;
    const int l = lane_id();
    const oaz_state s = load_state(&states[g]);
    const LaneMoves m = lane_movegen(s);
    if (masks && l < 50) masks[(size_t)g * 50 + l] = m.mask;
    const uint32_t cnt = (uint32_t)__popc(m.mask);
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t total = (uint32_t)__shfl((int)incl, 63);
    if (moves) {
        uint32_t o = incl - cnt, mm = m.mask;
        while (mm) {
            const int to = __clz(mm);
            mm &= ~sq_bit(to);
            if (o < OAZ_MAX_MOVES) {
                oaz_move mv;
                mv.from = (uint8_t)m.from;
                mv.to = (uint8_t)to;
                mv.piece = (uint8_t)m.piece;
                mv.slot = (uint8_t)m.slot;
                moves[(size_t)g * OAZ_MAX_MOVES + o] = mv;
            }
            ++o;
        }
        // the entries past the count are zero (the whole output is defined, whatever the buffer held)
        if (l < OAZ_MAX_MOVES && (uint32_t)l >= total) moves[(size_t)g * OAZ_MAX_MOVES + l] = oaz_move{0, 0, 0, 0};
    }
    if (counts && l == 0) counts[g] = (uint8_t)total;
}

__global__ void k_step(oaz_state* states, const oaz_move* mv, int n, uint8_t* results) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    oaz_state s = states[i];
    const oaz_move m = mv[i];
    const int r = make_move(s, m.from, m.to, m.piece, m.slot, s.to_move & 1);
    s.to_move ^= 1;
    states[i] = s;
    if (results) results[i] = (uint8_t)r;
}

__global__ void k_current_state(const oaz_state* states, int n, uint8_t* results) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    results[i] = (uint8_t)current_state(states[i]);
}

// create_tensor_from_state (common.rs:26-80): one thread per (position, plane, square).
__global__ void k_encode(const oaz_state* states, int n, float* planes) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n * 525) return;
    const int b = (int)(i / 525), r = (int)(i % 525), c = r / 25, sq = r % 25;
    const oaz_state s = states[b];
    const int color = s.to_move & 1;
    float v = 0.0f;
    if (c < 4) {
        const uint32_t src = c == 0 ? s.pawns[0] : c == 1 ? s.kings[0] : c == 2 ? s.pawns[1] : s.kings[1];
        v = (src & sq_bit(sq)) ? 1.0f : 0.0f;
    } else if (c < 20) {
        const int s0 = color ? 2 : 0;
        v = ((s.cards[s0] & 15) == c - 4 || (s.cards[s0 + 1] & 15) == c - 4) ? 1.0f : 0.0f;
    } else {
        v = color == OAZ_BLUE ? 1.0f : 0.0f;
    }
    planes[i] = v;
}

__global__ void k_hash_eval(const oaz_state* states, int n, float* policy, float* value) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = hash_state(states[i]);
    for (int k = 0; k < 50; ++k) policy[(size_t)i * 50 + k] = hash_policy(h, k);
    value[i] = hash_value(h);
}

// ---- leaf compaction: the positions the NN evaluates ----------------------------------------
// One workgroup per bucket of kBucket games: the games whose playout uses its leaf evaluation
// (t.need, written by select) get consecutive rows b * kBucket + j in game order; their leaf
// positions are gathered to t.cstate, game g's row to t.slot[g], the count to t.bcnt[b]. The
// evaluator's workgroups then cover bcnt[b] rows per bucket (TileMap) and expand/backup reads
// row t.slot[g]. Thread tid owns games 4 tid .. 4 tid + 3 of the bucket.
constexpr int kCompactThreads = (int)(kBucket / 4);
__global__ void __launch_bounds__(kCompactThreads) k_eval_compact(TreeView t) {
    __shared__ uint32_t wsum[kCompactThreads / 64];
    const uint32_t base = blockIdx.x << kBucketShift;
    const int tid = threadIdx.x, w = tid >> 6;
    const uint32_t g0 = base + 4 * (uint32_t)tid;
    // the 4 leaf positions are requested with the flags (contiguous 96 B per thread), so the gather
    // below is not a second dependent round trip
    oaz_state ls[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ls[k] = load_state(&t.leaf_state[g0 + k < t.G ? g0 + k : t.G - 1]);
    uint32_t f = 0;  // need flags of the 4 games, one byte each
    if (g0 + 4 <= t.G && (reinterpret_cast<uintptr_t>(t.need + g0) & 3) == 0) {  // (a part may start unaligned)
        f = *reinterpret_cast<const uint32_t*>(t.need + g0);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (g0 + k < t.G) f |= (uint32_t)(t.need[g0 + k] != 0) << (8 * k);
    }
    f &= 0x01010101u;
    const uint32_t cnt = (uint32_t)__popc(f);
    const uint32_t incl = wave_incl_scan(cnt);
    if (lane_id() == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kCompactThreads / 64; ++i) {
        const uint32_t v = wsum[i];
        off += i < w ? v : 0u;
        tot += v;
    }
    uint32_t j = base + off + incl - cnt;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (f & (1u << (8 * k))) {
            const uint32_t g = g0 + k;
            t.slot[g] = j;
            store_state(&t.cstate[j], ls[k]);
            ++j;
        }
    }
    if (tid == 0) t.bcnt[blockIdx.x] = tot;
}

// ---- Dirichlet root noise: root_noise() in oaz_device.h ------------------------------------
// Dirichlet draws of nsims consecutive simulations for every root: out[(k*G + g)*80 + 2j + {0,1}]
// holds the noise for comparison j (operand a, operand b) of simulation sim0+k. They depend only
// on (root position, game id, ply, sim), so they are produced off the critical path (second
// stream) instead of inside the latency-bound select walk. One wave per game covers all
// nsims * 2(K-1) draws of the chunk with every lane busy.
__global__ void __launch_bounds__(kBlock) k_root_noise(const oaz_state* __restrict__ roots,
                                                       const uint8_t* __restrict__ active,
                                                       const uint64_t* __restrict__ game_ids,
                                                       const uint32_t* __restrict__ plies, SearchParams prm,
                                                       uint32_t G, uint32_t sim0, uint32_t nsims, noise_t* out) {
    const uint32_t g = wave_game();
    if (g >= G) return;
    if (active && active[g] != 1) return;
    const int l = lane_id();
    const oaz_state s = load_state(&roots[g]);
    const LaneMoves m = lane_movegen(s);
    const int K = (int)wave_sum_u32((uint32_t)__popc(m.mask));  // = root children (expand order)
    if (K < 2) return;
    const uint64_t gid = game_ids ? game_ids[g] : g;
    const uint32_t ply = plies ? plies[g] : 0u;
    const int per_sim = 2 * (K - 1);
    for (int idx = l; idx < (int)nsims * per_sim; idx += 64) {
        const int k = idx / per_sim, r = idx - k * per_sim;
        const uint32_t d = 2u + (uint32_t)r;  // draw index 2j + which, j = 1 + r/2
        const uint32_t c2 = (ply << 16) | ((sim0 + k) & 0xFFFFu);
        out[((size_t)k * G + g) * kNoiseStride + d] = root_noise(prm.seed, gid, c2, d, prm.alpha, K);
    }
}

// ---- MCTS kernels -------------------------------------------------------------------------
struct NodeRegs {  // one node held in registers (all 32 bytes)
    double W, P;
    uint32_t N, first, misc;  // misc = mv | nch<<16 | flags<<24
};

__device__ __forceinline__ NodeRegs load_node(const oaz_node* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    NodeRegs r;
    r.W = __builtin_bit_cast(double, ((uint64_t)a.y << 32) | a.x);
    r.P = __builtin_bit_cast(double, ((uint64_t)a.w << 32) | a.z);
    r.N = b.x;
    r.first = b.y;
    r.misc = b.z;
    return r;
}
__device__ __forceinline__ int node_nch(uint32_t misc) { return (misc >> 16) & 0xFF; }
__device__ __forceinline__ int node_flags(uint32_t misc) { return misc >> 24; }
__device__ __forceinline__ uint8_t* flags_ptr(oaz_node* n) { return &n->flags; }
// The playout uses the leaf's evaluation (mcts_arena.rs:156-176) to expand the leaf (neither
// expanded nor terminal-flagged) or to back up its value (the position is not won). Otherwise the
// reference evaluates the leaf and discards the result, and the leaf is left out of the NN batch.
__device__ __forceinline__ bool leaf_needs_eval(uint32_t misc, const oaz_state& s) {
    return !(node_flags(misc) & 3) || !is_win(current_state(s));
}

__device__ __forceinline__ void store_fresh_node(oaz_node* p, double P, uint32_t mv) {
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint64_t pb = __builtin_bit_cast(uint64_t, P);
    q[0] = make_uint4(0u, 0u, (uint32_t)pb, (uint32_t)(pb >> 32));
    q[1] = make_uint4(0u, 0u, mv & 0xFFFFu, 0u);
}

__global__ void __launch_bounds__(kBlock) k_tree_reset(TreeView t) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.G) return;
    store_fresh_node(&t.nodes[(size_t)g * t.cap], 1.0, 0);  // root: probability 1. (mcts_arena.rs:57)
    t.n_nodes[g] = 1;
}

// playout step 1 (mcts_arena.rs:131-153): walk from the root while the node is expanded and
// not terminal; replay each chosen move; mark children whose move wins as terminal.
__global__ void __launch_bounds__(kBlock) k_select(TreeView t, const oaz_state* __restrict__ roots,
                                                   const uint8_t* __restrict__ active,
                                                   const noise_t* __restrict__ noise,
                                                   SearchParams prm) {
    const uint32_t g = wave_game();
    if (g >= t.G) return;
    if (active && active[g] != 1) {
        if (t.need && lane_id() == 0) t.need[g] = 0;
        return;
    }
    const int l = lane_id();
    oaz_node* T = t.nodes + (size_t)g * t.cap;
    uint32_t* path = t.path + (size_t)g * t.pathcap;
    oaz_state s = load_state(&roots[g]);
    int color = s.to_move & 1;

    NodeRegs nd = load_node(&T[0]);
    uint32_t node = 0, depth = 0;
    if (l == 0) path[0] = 0;
    bool stuck = false;
    while ((node_flags(nd.misc) & 1) && !(node_flags(nd.misc) & 2)) {
        const int K = node_nch(nd.misc);
        if (K == 0) {  // reference would panic in select (Q6): stop here, treat as a leaf
            stuck = true;
            break;
        }
        NodeRegs ch;
        ch.W = 0.0;
        ch.P = 0.0;
        ch.N = 0;
        ch.first = 0;
        ch.misc = 0;
        if (l < K) ch = load_node(&T[nd.first + l]);
        // winrate (reward / visits; 0 before the first visit) and sqrt(N_parent)/(N_child+1)
        const double q = ch.N ? ch.W / (double)ch.N : 0.0;
        const double sq = t.sqrt_tab[nd.N] / (double)(ch.N + 1);
        int best;
        if (depth == 0 && prm.train_noise && noise) {
            // sequential Iterator::max_by fold; each comparison re-evaluates both operands
            // with fresh noise (draw indices 2j and 2j+1 for comparison j)
            // draws precomputed by k_root_noise (same root, game id, ply and sim)
            // Operand b of comparison j is child j with its own draw: every lane evaluates its
            // own in parallel. Only operand a (the running best, with comparison j's fresh draw)
            // is sequential; the fold runs on wave-uniform values read with v_readlane.
            double na = 0.0, nb = 0.0;
            if (l >= 1 && l < K) {
                na = (double)noise[(size_t)g * kNoiseStride + 2 * l];
                nb = (double)noise[(size_t)g * kNoiseStride + 2 * l + 1];
            }
            const double base = ch.P * (1.0 - prm.eps);
            const double ubl = q + prm.c_puct * (base + nb * prm.eps) * sq;
            int acc = 0;
            double qa = readlane_f64(q, 0), ba = readlane_f64(base, 0), sa = readlane_f64(sq, 0);
            for (int j = 1; j < K; ++j) {
                const double ua = qa + prm.c_puct * (ba + readlane_f64(na, j) * prm.eps) * sa;
                const double ub = readlane_f64(ubl, j);
                if (!(total_key(ua) > total_key(ub))) {
                    acc = j;
                    qa = readlane_f64(q, j);
                    ba = readlane_f64(base, j);
                    sa = readlane_f64(sq, j);
                }
            }
            best = acc;
        } else {
            const double u = q + prm.c_puct * ch.P * sq;  // mcts_arena.rs:204-207
            best = wave_argmax_last(l < K ? total_key(u) : INT64_MIN);
        }
        NodeRegs c;
        c.W = __shfl(ch.W, best);
        c.P = __shfl(ch.P, best);
        c.N = (uint32_t)__shfl((int)ch.N, best);
        c.first = (uint32_t)__shfl((int)ch.first, best);
        c.misc = (uint32_t)__shfl((int)ch.misc, best);
        const uint32_t cidx = nd.first + (uint32_t)best;
        const int res = make_move(s, mv_from(c.misc), mv_to(c.misc), mv_piece(c.misc),
                                  mv_slot(c.misc), color);
        color ^= 1;  // game_state.player_color.switch()
        if (is_win(res)) {
            c.misc |= 2u << 24;
            if (l == 0) *flags_ptr(&T[cidx]) = (uint8_t)(node_flags(c.misc));
        }
        ++depth;
        if (l == 0 && depth < t.pathcap) path[depth] = cidx;
        node = cidx;
        nd = c;
    }
    s.to_move = (uint8_t)color;
    if (l == 0) {
        const bool need = leaf_needs_eval(nd.misc, s);
        store_state(&t.leaf_state[g], s);
        t.leaf[g] = node;
        t.depth[g] = depth;
        if (t.need) t.need[g] = need;
        uint64_t* st = t.stats + (size_t)g * GS_COUNT;
        st[GS_SIMS] += 1;
        st[GS_DEPTH] += depth;
        st[GS_EVALS] += need;
        if (stuck) st[GS_STUCK] += 1;
    }
}

// playout steps 3-4 (mcts_arena.rs:158-176): expand the leaf if it is neither expanded nor
// terminal (evaluate() priors, mcts_arena.rs:275-301; expand, 231-260), then back up either
// the terminal reward (from the leaf parent's perspective) or the raw NN value.
__global__ void __launch_bounds__(kBlock) k_expand_backup(TreeView t, const oaz_state* __restrict__ roots,
                                                          const uint8_t* __restrict__ active,
                                                          const float* __restrict__ policy,
                                                          const float* __restrict__ value) {
    const uint32_t g = wave_game();
    if (g >= t.G) return;
    if (active && active[g] != 1) return;
    const int l = lane_id();
    oaz_node* T = t.nodes + (size_t)g * t.cap;
    const uint32_t* path = t.path + (size_t)g * t.pathcap;
    const oaz_state s = load_state(&t.leaf_state[g]);
    const uint32_t leaf = t.leaf[g], depth = t.depth[g];
    const uint32_t row = t.slot ? t.slot[g] : g;  // the leaf's evaluation (read only if it was made)
    const NodeRegs nd = load_node(&T[leaf]);
    uint64_t* st = t.stats + (size_t)g * GS_COUNT;
    const float* pol = policy + (size_t)row * 50;

    if (!(node_flags(nd.misc) & 3)) {
        const LaneMoves m = lane_movegen(s);
        const uint32_t cnt = (uint32_t)__popc(m.mask);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t K = (uint32_t)__shfl((int)incl, 63);
        const uint32_t row0 = wave_or(l < 25 ? m.mask : 0u);
        const uint32_t row1 = wave_or(l >= 25 ? m.mask : 0u);
        // per-card renormalisation; sequential f64 sums in square order (mcts_arena.rs:288-301)
        double sum0 = 0.0, sum1 = 0.0;
        for (int sq = 0; sq < 25; ++sq) {
            if (row0 & sq_bit(sq)) sum0 += (double)pol[sq];
            if (row1 & sq_bit(sq)) sum1 += (double)pol[25 + sq];
        }
        const uint32_t base = t.n_nodes[g];
        const int row = m.slot & 1;
        const double rs = row ? sum1 : sum0;
        uint32_t o = incl - cnt, mm = m.mask;
        while (mm) {
            const int to = __clz(mm);
            mm &= ~sq_bit(to);
            double p = (double)pol[row * 25 + to];
            if (rs > 0.0) p = p / rs;
            store_fresh_node(&T[base + o], p, pack_move(m.from, to, m.slot, m.piece));
            ++o;
        }
        if (l == 0) {
            t.n_nodes[g] = base + K;
            oaz_node* lp = &T[leaf];
            lp->first = base;
            lp->nch = (uint8_t)K;
            lp->flags = 1;
            st[GS_EXPANSIONS] += 1;
            st[GS_CHILDREN] += K;
            if (base + K > st[GS_MAXNODES]) st[GS_MAXNODES] = base + K;
        }
    }
    const int res = current_state(s);
    double r;
    if (is_win(res)) {
        // reward colour = colour of the leaf's parent (root if the leaf is the root)
        const int root_color = roots[g].to_move & 1;
        const int pc = depth == 0 ? root_color : (root_color ^ (int)((depth - 1) & 1));
        r = reward(res, pc);
        if (l == 0) st[GS_TERMINAL] += 1;
    } else {
        r = (double)value[row];
    }
    // back_propagate (mcts_arena.rs:312-323): node at depth k gets (-1)^(depth-k) * r
    const uint32_t plen = depth < t.pathcap ? depth : t.pathcap - 1;
    for (uint32_t k = (uint32_t)l; k <= plen; k += 64) {
        const uint32_t n = path[k];
        const double rk = ((depth - k) & 1) ? -r : r;
        T[n].N += 1;
        T[n].W += rk;
    }
}

// ---- segmented tree kernels: FOUR GAMES PER WAVE (16-lane segments) ----------------------
// The select / expand-backup walks are chains of dependent memory round trips (one per tree
// level), so their time is the number of such chains in flight per CU, not bandwidth: with one
// game per wave a CU holds 32 games, with one per 16-lane segment 128. A segment is active or
// idle as a whole (every branch condition below is uniform over its 16 lanes), and segment-wide
// reductions use DPP row operations (quad swaps, half-row and row mirrors), which never leave
// the 16-lane row. Results are bit-identical to k_select / k_expand_backup (same f64 expressions,
// same sequential fold and summation orders); tests/test_gpu.py compares whole trees to the oracle.
constexpr int kSegLanes = 16;
__device__ __forceinline__ int seg_lane() { return (int)(threadIdx.x & 15); }
__device__ __forceinline__ int seg_base() { return (int)(threadIdx.x & 63) & ~15; }
__device__ __forceinline__ uint32_t seg_game() {
    return (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 4 + ((threadIdx.x >> 4) & 3);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
// argmax of (key, idx) over the segment, the larger idx winning among equal keys (max_by)
template <int CTRL>
__device__ __forceinline__ void seg_amax_step(int64_t& key, int& idx) {
    const uint64_t kb = (uint64_t)key;
    const uint32_t lo = dpp_u32<CTRL>((uint32_t)kb), hi = dpp_u32<CTRL>((uint32_t)(kb >> 32));
    const int64_t ok = (int64_t)(((uint64_t)hi << 32) | lo);
    const int oi = (int)dpp_u32<CTRL>((uint32_t)idx);
    if (ok > key || (ok == key && oi > idx)) {
        key = ok;
        idx = oi;
    }
}
__device__ __forceinline__ int seg_argmax_last(int64_t key, int idx) {
    seg_amax_step<0xB1>(key, idx);   // quad_perm [1,0,3,2]
    seg_amax_step<0x4E>(key, idx);   // quad_perm [2,3,0,1]
    seg_amax_step<0x141>(key, idx);  // row_half_mirror
    seg_amax_step<0x140>(key, idx);  // row_mirror
    return idx;
}
__device__ __forceinline__ uint32_t seg_or(uint32_t v) {
    v |= dpp_u32<0xB1>(v);
    v |= dpp_u32<0x4E>(v);
    v |= dpp_u32<0x141>(v);
    v |= dpp_u32<0x140>(v);
    return v;
}
__device__ __forceinline__ uint32_t seg_incl_scan(uint32_t v) {  // row_shr 1, 2, 4, 8 (zero fill)
    v += dpp_u32<0x111>(v);
    v += dpp_u32<0x112>(v);
    v += dpp_u32<0x114>(v);
    v += dpp_u32<0x118>(v);
    return v;
}
template <class T>
__device__ __forceinline__ T pick3(int c, const T& a, const T& b, const T& d) {
    return c == 0 ? a : c == 1 ? b : d;
}

// Per-game statistics from the segmented tree kernels: relaxed atomics whose result is unused
// (no-return global atomics), so the update costs no load round trip at the end of a walk; each game's
// counters have one writer at a time, the atomic form only drops the read.
__device__ __forceinline__ void stat_add(uint64_t* p, uint64_t v) {
    (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stat_max(uint64_t* p, uint64_t v) {
    (void)__hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane n of every 16-lane row, to the whole row (DPP row_newbcast)
template <int N>
__device__ __forceinline__ double bcast_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    // (every lane of a row is a valid source for row_newbcast, so bound_ctrl changes nothing but lets
    // the compiler drop the zero it would otherwise write into the destination first)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x150 + N, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x150 + N, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// Root fold operands of this lane's child in one chunk: q, base = P (1 - eps), sq = sqrt(N_parent)
// / (N + 1), nae = (operand-a draw) * eps and kub = total_key(operand b) -- everything of
// comparison j that does not depend on the running best, computed in parallel per child.
struct FoldCh {
    double q, base, sq, nae, kub;
};
__device__ __forceinline__ FoldCh fold_chunk(const NodeRegs& ch, noise_t na, noise_t nb, double sqn,
                                             const SearchParams& prm) {
    FoldCh f;
    f.q = ch.N ? ch.W / (double)ch.N : 0.0;
    f.sq = sqn / (double)(ch.N + 1);
    f.base = ch.P * (1.0 - prm.eps);
    f.nae = (double)na * prm.eps;
    const double ub = f.q + prm.c_puct * (f.base + (double)nb * prm.eps) * f.sq;
    f.kub = __builtin_bit_cast(double, total_key(ub));  // the key, carried in a double
    return f;
}
// comparison j of the root fold (k_select): operand a = the running best with comparison j's
// fresh draw, operand b = child j with its own draw. A chunk's operands are built when the fold
// reaches it (j = 16, 32), so only one chunk's are live at a time.
template <int J>
__device__ __forceinline__ void fold_step(int& acc, double& qa, double& ba, double& sa, int K, FoldCh& f,
                                          const NodeRegs (&ch)[3], const noise_t (&na)[3], const noise_t (&nb)[3],
                                          double sqn, const SearchParams& prm) {
    constexpr int c = J >> 4, n = J & 15;
    if constexpr (n == 0) f = fold_chunk(ch[c], na[c], nb[c], sqn, prm);
    const double ua = qa + prm.c_puct * (ba + bcast_f64<n>(f.nae)) * sa;
    const int64_t kb = __builtin_bit_cast(int64_t, bcast_f64<n>(f.kub));
    const double qj = bcast_f64<n>(f.q), bj = bcast_f64<n>(f.base), sj = bcast_f64<n>(f.sq);
    if (J < K && !(total_key(ua) > kb)) {
        acc = J;
        qa = qj;
        ba = bj;
        sa = sj;
    }
}
template <int... I>
__device__ __forceinline__ int root_fold(int K, int Kmax, const NodeRegs (&ch)[3], const noise_t (&na)[3],
                                         const noise_t (&nb)[3], double sqn, const SearchParams& prm,
                                         std::integer_sequence<int, I...>) {
    FoldCh f = fold_chunk(ch[0], na[0], nb[0], sqn, prm);
    int acc = 0;
    double qa = bcast_f64<0>(f.q), ba = bcast_f64<0>(f.base), sa = bcast_f64<0>(f.sq);
    // j = I + 1 = 1 .. 39; stop once every segment's K is passed (wave-uniform)
    (void)((I + 1 < Kmax ? (fold_step<I + 1>(acc, qa, ba, sa, K, f, ch, na, nb, sqn, prm), true) : false) && ...);
    return acc;
}

// k_select with 16 lanes per game: lane sl holds children j = 16c + sl (c < 3, K <= 40).
// Where node i of a game's tree lives: its slot of t.nodes (the per-step kernels), or, in the one-launch
// search (oaz_search_lat.hip), LDS for the first n nodes of the workgroup's one game (the top of the tree,
// allocated first) and t.nodes beyond. Generic pointers: the same loads and stores reach either.
// The same accessor serves the walk's other per-level / per-simulation reads: sqrt(N) from the host-built
// table (one dependent load per tree level) and the game's root position.
struct NodesGlobal {
    __device__ __forceinline__ oaz_node* at(oaz_node* T, uint32_t i) const { return T + i; }
    __device__ __forceinline__ double sqrt_n(const TreeView& t, uint32_t n) const { return t.sqrt_tab[n]; }
    __device__ __forceinline__ const oaz_state* root(const oaz_state* roots, uint32_t g) const { return &roots[g]; }
    __device__ __forceinline__ void add(uint64_t* st, int f, uint64_t v) const { stat_add(&st[f], v); }
    __device__ __forceinline__ void max(uint64_t* st, int f, uint64_t v) const { stat_max(&st[f], v); }
    __device__ __forceinline__ uint32_t pawns(const oaz_state& s, int c) const { return s.pawns[c]; }
    __device__ __forceinline__ uint32_t kings(const oaz_state& s, int c) const { return s.kings[c]; }
    __device__ __forceinline__ int card(const oaz_state& s, int i) const { return s.cards[i]; }
    __device__ __forceinline__ int move(oaz_state& s, int from, int to, int piece, int slot, int color) const {
        return make_move(s, from, to, piece, slot, color);
    }
};
// The bodies called as functions (k_search_grp's walker waves): the same global nodes, the position's
// colour- and slot-indexed fields read and written register-only (make_move_regs, state_card): in a called
// function a runtime index into the state otherwise sends it through scratch memory.
struct NodesGlobalRegs : NodesGlobal {
    __device__ __forceinline__ uint32_t pawns(const oaz_state& s, int c) const { return c ? s.pawns[1] : s.pawns[0]; }
    __device__ __forceinline__ uint32_t kings(const oaz_state& s, int c) const { return c ? s.kings[1] : s.kings[0]; }
    __device__ __forceinline__ int card(const oaz_state& s, int i) const { return state_card(s, i); }
    __device__ __forceinline__ int move(oaz_state& s, int from, int to, int piece, int slot, int color) const {
        return make_move_regs(s, from, to, piece, slot, color);
    }
};
struct NodesCached {
    oaz_node* L;        // LDS: nodes [0, n)
    uint32_t n;
    const double* sq;   // LDS: sqrt_tab [0, nsq)
    uint32_t nsq;
    const oaz_state* rt;  // LDS: the workgroup's game's root position
    uint64_t* stl;        // LDS: the game's statistics, added to its global slots once at the end of the launch
    __device__ __forceinline__ oaz_node* at(oaz_node* T, uint32_t i) const { return i < n ? L + i : T + i; }
    __device__ __forceinline__ double sqrt_n(const TreeView& t, uint32_t k) const {
        return k < nsq ? sq[k] : t.sqrt_tab[k];
    }
    __device__ __forceinline__ const oaz_state* root(const oaz_state*, uint32_t) const { return rt; }
    __device__ __forceinline__ void add(uint64_t*, int f, uint64_t v) const {
        (void)__hip_atomic_fetch_add(&stl[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void max(uint64_t*, int f, uint64_t v) const {
        (void)__hip_atomic_fetch_max(&stl[f], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // the one-launch search holds the leaf position in registers across its calls: register-only reads
    // (state_card; a runtime index would put the state in scratch memory)
    __device__ __forceinline__ uint32_t pawns(const oaz_state& s, int c) const { return c ? s.pawns[1] : s.pawns[0]; }
    __device__ __forceinline__ uint32_t kings(const oaz_state& s, int c) const { return c ? s.kings[1] : s.kings[0]; }
    __device__ __forceinline__ int card(const oaz_state& s, int i) const { return state_card(s, i); }
    __device__ __forceinline__ int move(oaz_state& s, int from, int to, int piece, int slot, int color) const {
        return make_move_regs(s, from, to, piece, slot, color);
    }
};

// Per-wave statistics: the segment leads (lane 0 of each 16-lane segment) set in m contribute; the first
// of them adds the wave's sums to its own game's row, one atomic per counter, so four segments' counters
// dirty one line instead of four (the rows are only summed, and GS_MAXNODES maximised, over the games:
// oaz_search_stats). m comes from a ballot, so a lead outside the exec mask never contributes.
constexpr uint64_t kLeadLanes = 0x0001000100010001ull;
__device__ __forceinline__ uint32_t lead_sum(uint32_t v, uint64_t m) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if ((m >> (16 * k)) & 1) r += (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * k);
    return r;
}
__device__ __forceinline__ uint32_t lead_max(uint32_t v, uint64_t m) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if ((m >> (16 * k)) & 1) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * k);
            r = x > r ? x : r;
        }
    return r;
}

// The root's noise draw pairs (operand a, operand b) of this lane's children j = 16c + sl, 1 <= j < K:
// buffer loads whose lanes past K (or idle) get an offset past the resource's range, which returns 0
// without a memory access (the noise ring holds 80 draws per game and simulation, most of them past a
// root's K). Unconditional instructions, so all three chunks' loads are in flight together: one round
// trip (exec-masked loads in branches get a wait each). Byte offsets are 32-bit: G * 80 * sizeof(noise_t)
// < 2^31 (oaz_create bounds G).
// C0 .. C1 - 1: the chunks loaded (the workgroup fold loads chunk 2 only for its rare second pass).
template <int C0 = 0, int C1 = 3>
__device__ __forceinline__ void root_noise_pairs(const TreeView& t, const noise_t* noise, uint32_t g, bool go, int K,
                                                 noise_t (&na)[3], noise_t (&nb)[3]) {
    const int sl = seg_lane();
    constexpr uint32_t kB = (uint32_t)sizeof(noise_t);
    const __amdgpu_buffer_rsrc_t nr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)noise, (short)0, (int)(t.G * (uint32_t)kNoiseStride * kB), 0x00020000);
#pragma unroll
    for (int c = C0; c < C1; ++c) {
        const int j = 16 * c + sl;
        const uint32_t off =
            go && j >= 1 && j < K ? (g * (uint32_t)kNoiseStride + 2u * (uint32_t)j) * kB : 0x80000000u;
#if OAZ_NOISE_F32
        const auto d = __builtin_amdgcn_raw_buffer_load_b64(nr, (int)off, 0, 0);
        na[c] = __uint_as_float(d[0]);
        nb[c] = __uint_as_float(d[1]);
#else
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(nr, (int)off, 0, 0);
        na[c] = __builtin_bit_cast(double, ((uint64_t)d[1] << 32) | d[0]);
        nb[c] = __builtin_bit_cast(double, ((uint64_t)d[3] << 32) | d[2]);
#endif
    }
}

// The root noise folds of a workgroup's 32 games, one lane per game (k_select_seg / k_backup_select_seg).
// The fold is sequential by definition (a fresh draw per comparison against the running best,
// mcts_arena.rs:183-223), so in the per-segment form every wave issued ~27 instructions per comparison for
// its 4 games, Kmax - 1 times; here every segment stages its children's fold operands (everything that
// does not depend on the running best, computed in parallel per child as before) in LDS, and ONE wave folds
// all 32 games at once: ~1/6 of the fold's instructions per workgroup. Structure of arrays [child][game],
// so the folding lanes' reads are bank-conflict free. The arrays hold 32 children (two 16-lane chunks):
// a game with more (K <= 40, rare at a root) is folded in a second pass over children 32 .. K - 1 in the same
// rows. Row 0's kub is never a fold operand (the fold starts with child 0 as the running best), so it
// carries K in and the chosen child out. 40 KB (f64 draws): four 8-wave workgroups per CU, 8 waves per SIMD.
constexpr int kWgGames = kWavesPerBlock * 4;
constexpr int kFoldRows = 32;
struct WgFold {
    int64_t kub[kFoldRows][kWgGames];  // total_key of operand b (child j with its own draw); row 0: K, then best
    double q[kFoldRows][kWgGames];     // operand a's parts when child j is the running best
    double base[kFoldRows][kWgGames];
    double sq[kFoldRows][kWgGames];
    double nae[kFoldRows][kWgGames];   // operand a's draw of comparison j x eps
};
static_assert(sizeof(WgFold) <= 40960, "four workgroups' fold operands per CU");
// The running best of a lane's fold across its passes (registers of the folding lane).
struct FoldAcc {
    int K, acc;
    double qa, ba, sa;
};
// lane = game gi of the workgroup (threadIdx.x < kWgGames): fold_step's comparisons in the same order and
// with the same operands and expressions, so the same best child. Pass 0 starts the fold from row 0 (child 0)
// and compares children 1 .. min(K, 32) - 1; pass 1 compares children 32 .. K - 1 from rows 0 .. K - 33.
// Comparison j's operands are read one comparison ahead (the LDS latency off the sequential chain; the row
// read past the game's last comparison is never used), child j's q / base / sq at the start of comparison j,
// so a takeover is four selects, not a dependent read.
__device__ __forceinline__ void wg_fold_pass(const WgFold* wf, const SearchParams& prm, FoldAcc& f, int pass) {
    const int gi = (int)threadIdx.x;
    const int off = pass ? kFoldRows : 0;
    const int j0 = pass ? kFoldRows : 1;
    const int jend = pass ? f.K : (f.K < kFoldRows ? f.K : kFoldRows);
    double nae = wf->nae[j0 - off][gi];
    int64_t kb = wf->kub[j0 - off][gi];
    for (int j = j0; __ballot(j < jend) != 0; ++j) {  // uniform: until every game's bound is passed
        const int r = j - off, rn = r + 1 < kFoldRows ? r + 1 : kFoldRows - 1;
        const double qj = wf->q[r][gi], bj = wf->base[r][gi], sj = wf->sq[r][gi];  // used after the chain
        const double nae_n = wf->nae[rn][gi];
        const int64_t kb_n = wf->kub[rn][gi];
        const double ua = f.qa + prm.c_puct * (f.ba + nae) * f.sa;
        const bool take = j < jend && !(total_key(ua) > kb);
        f.acc = take ? j : f.acc;
        f.qa = take ? qj : f.qa;
        f.ba = take ? bj : f.ba;
        f.sa = take ? sj : f.sa;
        nae = nae_n;
        kb = kb_n;
    }
}

// g: this segment's game (>= t.G: an idle segment); leaf_lds: also store the leaf position there (LDS of
// the one-launch search, whose network reads it without a global round trip), or null.
// WGF (k_select_seg / k_backup_select_seg: every thread of the workgroup calls this body): the root's noise
// fold for the workgroup's games at once in wf (WgFold), the root level peeled off the walk so that every
// wave reaches its two barriers; otherwise each segment folds its own game (16 lanes, DPP broadcasts).
template <class NA = NodesGlobal, bool WGF = false, bool WF_ALIASED = false>
__device__ __forceinline__ void select_seg_body(const TreeView& t, const oaz_state* __restrict__ roots,
                                                const uint8_t* __restrict__ active, const noise_t* __restrict__ noise,
                                                const SearchParams& prm, uint32_t g, oaz_state* leaf_lds = nullptr,
                                                const NA& na = NA{}, WgFold* wf = nullptr) {
    const int sl = seg_lane(), sb = seg_base();
    const bool on = g < t.G && !(active && active[g] != 1);
    const bool fold_mode = prm.train_noise && noise;
    oaz_node* T = t.nodes + (size_t)(on ? g : 0) * t.cap;
    // the path by a 32-bit element offset from the (scalar) base, not a 64-bit per-lane pointer: the walk
    // keeps it live across every level, and as a VGPR pair it was the fused kernel's spill (a scratch
    // round trip per level); G * pathcap < 2^32 (oaz_create bounds both)
    const uint32_t pbase = (on ? g : 0u) * t.pathcap;
    uint32_t* const path = t.path;
    oaz_state s = load_state(na.root(roots, on ? g : 0));
    int color = s.to_move & 1;
    NodeRegs nd = load_node(na.at(T, 0));
    uint32_t node = 0, depth = 0;
    if (on && sl == 0) path[pbase] = 0;
    bool stuck = false;
    bool go = on && (node_flags(nd.misc) & 1) && !(node_flags(nd.misc) & 2);
    // one level down: the chosen child of node nd (children in ch[], this segment's best index)
    auto descend = [&](int best, const NodeRegs (&ch)[3]) {
        const int bc = best >> 4, src = sb + (best & 15);
        NodeRegs c;  // (the walk reads only N, first and misc of the node it descends to)
        c.W = 0.0;
        c.P = 0.0;
        c.N = (uint32_t)__shfl((int)pick3(bc, ch[0].N, ch[1].N, ch[2].N), src);
        c.first = (uint32_t)__shfl((int)pick3(bc, ch[0].first, ch[1].first, ch[2].first), src);
        c.misc = (uint32_t)__shfl((int)pick3(bc, ch[0].misc, ch[1].misc, ch[2].misc), src);
        if (go) {
            const uint32_t cidx = nd.first + (uint32_t)best;
            const int res = na.move(s, mv_from(c.misc), mv_to(c.misc), mv_piece(c.misc), mv_slot(c.misc), color);
            color ^= 1;  // game_state.player_color.switch()
            if (is_win(res)) {
                c.misc |= 2u << 24;
                if (sl == 0) *flags_ptr(na.at(T, cidx)) = (uint8_t)(node_flags(c.misc));
            }
            ++depth;
            if (sl == 0 && depth < t.pathcap) path[pbase + depth] = cidx;
            node = cidx;
            nd = c;
            go = (node_flags(nd.misc) & 1) && !(node_flags(nd.misc) & 2);
        }
    };
    if (WGF && fold_mode) {  // the root level, every thread of the workgroup (uniform: kernel arguments)
        const int gi = (int)(threadIdx.x >> 4);
        const int K = go ? node_nch(nd.misc) : 0;
        if (go && K == 0) {  // reference would panic in select (Q6): stop here, treat as a leaf
            stuck = true;
            go = false;
        }
        NodeRegs ch[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int j = 16 * c + sl;
            ch[c].W = 0.0;
            ch[c].P = 0.0;
            ch[c].N = 0;
            ch[c].first = 0;
            ch[c].misc = 0;
            if (go && j < K) ch[c] = load_node(na.at(T, nd.first + j));
        }
        const double sqn = go ? na.sqrt_n(t, nd.N) : 0.0;
        noise_t nza[3], nzb[3];
        root_noise_pairs<0, 2>(t, noise, g, go, K, nza, nzb);
        // wf overlays the expand/backup's policy rows (k_backup_select_seg): every wave is past its backup
        // before any writes the fold operands (the operand loads above are already in flight)
        if constexpr (WF_ALIASED) __syncthreads();
        auto stage = [&](int c, int r0) {  // chunk c's operands into rows j - r0
            const int j = 16 * c + sl;
            if (go && j < K) {
                const FoldCh f = fold_chunk(ch[c], nza[c], nzb[c], sqn, prm);
                if (j != 0) wf->kub[j - r0][gi] = __builtin_bit_cast(int64_t, f.kub);  // (child 0's row: K)
                wf->q[j - r0][gi] = f.q;
                wf->base[j - r0][gi] = f.base;
                wf->sq[j - r0][gi] = f.sq;
                wf->nae[j - r0][gi] = f.nae;
            }
        };
        stage(0, 0);
        stage(1, 0);
        if (sl == 0) wf->kub[0][gi] = go ? K : 0;
        __syncthreads();
        FoldAcc fa;
        if (threadIdx.x < (unsigned)kWgGames) {
            fa.K = (int)wf->kub[0][threadIdx.x];
            fa.acc = 0;
            fa.qa = wf->q[0][threadIdx.x];
            fa.ba = wf->base[0][threadIdx.x];
            fa.sa = wf->sq[0][threadIdx.x];
            wg_fold_pass(wf, prm, fa, 0);
            // whether any game has children 32 .. K - 1, for every wave: the last row (free after this
            // pass's reads; a second pass fills rows 0 .. 7), not __syncthreads_or, whose LDS word would
            // make the workgroup 256 B too large for four per CU
            const bool more = __ballot(fa.K > kFoldRows) != 0;
            if (threadIdx.x == 0) wf->kub[kFoldRows - 1][0] = more ? 1 : 0;
        }
        __syncthreads();
        // children 32 .. K - 1 of any game: a second pass in the same rows, after the first pass's reads
        if (wf->kub[kFoldRows - 1][0] != 0) {
            root_noise_pairs<2, 3>(t, noise, g, go, K, nza, nzb);
            stage(2, kFoldRows);
            __syncthreads();
            if (threadIdx.x < (unsigned)kWgGames) wg_fold_pass(wf, prm, fa, 1);
            __syncthreads();
        }
        if (threadIdx.x < (unsigned)kWgGames) wf->kub[0][threadIdx.x] = fa.acc;
        __syncthreads();
        descend(go ? (int)wf->kub[0][gi] : 0, ch);
    }
    while (__builtin_amdgcn_read_exec() && __ballot(go)) {  // some segment is still walking
        const int K = go ? node_nch(nd.misc) : 0;
        if (go && K == 0) {  // reference would panic in select (Q6): stop here, treat as a leaf
            stuck = true;
            go = false;
        }
        NodeRegs ch[3];
        int64_t bkey = INT64_MIN;
        int bidx = sl;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int j = 16 * c + sl;
            ch[c].W = 0.0;
            ch[c].P = 0.0;
            ch[c].N = 0;
            ch[c].first = 0;
            ch[c].misc = 0;
            if (go && j < K) ch[c] = load_node(na.at(T, nd.first + j));
        }
        const double sqn = go ? na.sqrt_n(t, nd.N) : 0.0;
        int best = 0;
        if (!WGF && depth == 0 && fold_mode) {
            // root with noise: the sequential Iterator::max_by fold of k_select, every segment's
            // fold state (acc, operand a) held uniformly across its 16 lanes; child j's operands
            // are broadcast within each 16-lane row by DPP row_newbcast (j compile-time)
            noise_t na[3], nb[3];
            root_noise_pairs(t, noise, g, go, K, na, nb);
            const int Kmax = max(max(__builtin_amdgcn_readlane(K, 0), __builtin_amdgcn_readlane(K, 16)),
                                 max(__builtin_amdgcn_readlane(K, 32), __builtin_amdgcn_readlane(K, 48)));
            best = root_fold(K, Kmax, ch, na, nb, sqn, prm, std::make_integer_sequence<int, 39>{});
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int j = 16 * c + sl;
                if (go && j < K) {
                    const double q = ch[c].N ? ch[c].W / (double)ch[c].N : 0.0;
                    const double sq = sqn / (double)(ch[c].N + 1);
                    const double u = q + prm.c_puct * ch[c].P * sq;  // mcts_arena.rs:204-207
                    const int64_t key = total_key(u);
                    if (key >= bkey) {  // ascending j: the last maximum
                        bkey = key;
                        bidx = j;
                    }
                }
            }
            best = seg_argmax_last(bkey, bidx);
        }
        // the chosen child's node from the lane that holds it (chunk best >> 4 of lane best & 15)
        descend(best, ch);
    }
    s.to_move = (uint8_t)color;
    const bool need = leaf_needs_eval(nd.misc, s);
    if (on && sl == 0) {
        store_state(&t.leaf_state[g], s);
        if (leaf_lds) *leaf_lds = s;
        t.leaf[g] = node;
        t.depth[g] = depth;
        if (t.need) t.need[g] = need;
    } else if (!on && g < t.G && sl == 0 && t.need) {
        t.need[g] = 0;  // an idle slot: nothing to evaluate
    }
    const uint64_t m = __ballot(on && sl == 0) & kLeadLanes;
    if (m) {
        const uint32_t dsum = lead_sum(depth, m), esum = lead_sum(need ? 1u : 0u, m), ssum = lead_sum(stuck ? 1u : 0u, m);
        if (lane_id() == __builtin_ctzll(m)) {
            uint64_t* st = t.stats + (size_t)g * GS_COUNT;
            na.add(st, GS_SIMS, (uint64_t)__popcll(m));
            na.add(st, GS_DEPTH, dsum);
            na.add(st, GS_EVALS, esum);
            if (ssum) na.add(st, GS_STUCK, ssum);
        }
    }
}

#ifndef OAZ_WG_FOLD
#define OAZ_WG_FOLD 1  // the workgroup's root noise folds on one wave (WgFold); 0: per segment (A/B build)
#endif
// register budget: 64 VGPRs = 8 waves/SIMD, no spill (the fold operands 40 KB: four workgroups per CU)
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OAZ_TREE_WPE)))
k_select_seg(TreeView t, const oaz_state* __restrict__ roots, const uint8_t* __restrict__ active,
             const noise_t* __restrict__ noise, SearchParams prm) {
    __shared__ WgFold wf;
    select_seg_body<NodesGlobalRegs, OAZ_WG_FOLD>(t, roots, active, noise, prm, seg_game(), nullptr, NodesGlobalRegs{},
                                                  &wf);
}

template <int N>
__device__ __forceinline__ float bcast_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + N, 0xF, 0xF, false));
}
// polm: the lane's policy entries with the squares no child moves to already zeroed (+0.0), so each
// term is one broadcast-convert and one add
template <int SQ>
__device__ __forceinline__ void policy_sum_step(const float (&polm)[4], double& sum0, double& sum1) {
    constexpr int i0 = SQ, i1 = 25 + SQ;
    sum0 += (double)bcast_f32<(i0 & 15)>(polm[i0 >> 4]);
    sum1 += (double)bcast_f32<(i1 & 15)>(polm[i1 >> 4]);
}
template <int... SQ>
__device__ __forceinline__ void policy_sums(const float (&polm)[4], double& sum0, double& sum1,
                                            std::integer_sequence<int, SQ...>) {
    (policy_sum_step<SQ>(polm, sum0, sum1), ...);
}

// k_expand_backup with 16 lanes per game: lane sl generates the moves of (card, from) combos
// 4 sl .. 4 sl + 3 (combo = card * 25 + from, the reference order), one segment scan places them.
// g: this segment's game (>= t.G: an idle segment); sp: 52 floats of LDS for the segment's policy row.
template <class NA = NodesGlobal>
__device__ __forceinline__ void expand_backup_seg_body(const TreeView& t, const oaz_state* __restrict__ roots,
                                                      const uint8_t* __restrict__ active,
                                                      const float* __restrict__ policy,
                                                      const float* __restrict__ value, uint32_t g, float* sp,
                                                      const NA& na = NA{}) {
    const int sl = seg_lane();
    if (g >= t.G) return;                  // whole segments (G is not a multiple of 4 only at the end)
    if (active && active[g] != 1) return;  // uniform over the segment
    oaz_node* T = t.nodes + (size_t)g * t.cap;
    const uint32_t* path = t.path + (size_t)g * t.pathcap;
    // Two dependent round trips: (1) the leaf record, this lane's first path entry and the node
    // count; (2) the leaf node, its policy row and value (read whether or not the playout uses them:
    // the rows are always in bounds) and N / W of this lane's path node. Everything after is stores.
    const oaz_state s = load_state(&t.leaf_state[g]);
    const uint32_t leaf = t.leaf[g], depth = t.depth[g];
    const uint32_t row = t.slot ? t.slot[g] : g;  // the leaf's evaluation row
    const uint32_t pn = (uint32_t)sl < t.pathcap ? path[sl] : 0u;
    const uint32_t nn0 = t.n_nodes[g];
    const NodeRegs nd = load_node(na.at(T, leaf));
    uint64_t* st = t.stats + (size_t)g * GS_COUNT;
    const float* pol = policy + (size_t)row * 50;
    float polr[4];  // lane sl: policy entries sl, 16+sl, 32+sl, 48+sl
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int idx = 16 * c + sl;
        polr[c] = idx < 50 ? pol[idx] : 0.0f;
    }
    const float vrow = value[row];
    const uint32_t plen = depth < t.pathcap ? depth : t.pathcap - 1;
    const bool mine = (uint32_t)sl <= plen;  // this lane backs up path node sl
    uint32_t pN = 0;
    double pW = 0.0;
    if (mine) {
        pN = na.at(T, pn)->N;
        pW = na.at(T, pn)->W;
    }
    asm volatile("" ::"v"(polr[0]), "v"(polr[1]), "v"(polr[2]), "v"(polr[3]), "v"(vrow));  // issued in trip 2
    bool expanded = false;  // this segment's statistics (summed per wave below)
    uint32_t kids = 0, nodes_end = 0;

    if (!(node_flags(nd.misc) & 3)) {
        // the policy row kept in registers for the renormalisation sums and in LDS (sp) for the
        // children's priors
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int idx = 16 * c + sl;
            if (idx < 50) sp[idx] = polr[c];
        }
        const int color = s.to_move & 1;
        const uint32_t pawns = na.pawns(s, color), king = na.kings(s, color), own = pawns | king;
        uint32_t mask[4];
        uint32_t cnt = 0, r0 = 0, r1 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int cb = 4 * sl + i, k = cb >= 25 ? 1 : 0, from = cb - 25 * k;
            uint32_t m = 0;
            if (cb < 50 && (own & sq_bit(from))) m = c_attack.m[color][na.card(s, (color ? 2 : 0) + k) & 15][from] & ~own;
            mask[i] = m;
            cnt += (uint32_t)__popc(m);
            if (k) r1 |= m; else r0 |= m;
        }
        const uint32_t incl = seg_incl_scan(cnt);
        const uint32_t K = (uint32_t)__shfl((int)incl, seg_base() + 15);
        const uint32_t row0 = seg_or(r0), row1 = seg_or(r1);
        // per-card renormalisation; sequential f64 sums in square order (mcts_arena.rs:288-301).
        // Entry idx comes from lane idx & 15 by DPP row_newbcast; an unset square adds +0.0, which
        // leaves a non-negative sum unchanged bit for bit (the old loop loaded and waited 50 times).
        double sum0 = 0.0, sum1 = 0.0;
        float polm[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int idx = 16 * c + sl, k = idx >= 25 ? 1 : 0, sq = idx - 25 * k;
            polm[c] = idx < 50 && ((k ? row1 : row0) & sq_bit(sq)) ? polr[c] : 0.0f;
        }
        policy_sums(polm, sum0, sum1, std::make_integer_sequence<int, 25>{});
        const uint32_t base = nn0;
        uint32_t o = incl - cnt;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int cb = 4 * sl + i, k = cb >= 25 ? 1 : 0, from = cb - 25 * k;
            const int slot = (color ? 2 : 0) + k;
            const int piece = (pawns & sq_bit(from)) ? OAZ_PAWN : OAZ_KING;
            const double rs = k ? sum1 : sum0;
            uint32_t mm = mask[i];
            while (mm) {
                const int to = __clz(mm);
                mm &= ~sq_bit(to);
                double p = (double)sp[k * 25 + to];
                if (rs > 0.0) p = p / rs;
                store_fresh_node(na.at(T, base + o), p, pack_move(from, to, slot, piece));
                ++o;
            }
        }
        if (sl == 0) {
            t.n_nodes[g] = base + K;
            oaz_node* lp = na.at(T, leaf);
            lp->first = base;
            lp->nch = (uint8_t)K;
            lp->flags = 1;
        }
        expanded = true;
        kids = K;
        nodes_end = base + K;
    }
    const int res = current_state(s);
    double r;
    if (is_win(res)) {
        const int root_color = na.root(roots, g)->to_move & 1;
        const int pc = depth == 0 ? root_color : (root_color ^ (int)((depth - 1) & 1));
        r = reward(res, pc);
    } else {
        r = (double)vrow;
    }
    {  // the statistics of the wave's segments that got here (the others returned above), per wave
        const uint64_t m = __ballot(sl == 0) & kLeadLanes;
        const uint32_t xs = lead_sum(expanded ? 1u : 0u, m), ks = lead_sum(kids, m), mx = lead_max(nodes_end, m);
        const uint32_t ts = lead_sum(is_win(res) ? 1u : 0u, m);
        if (m && lane_id() == __builtin_ctzll(m)) {
            if (xs) {
                na.add(st, GS_EXPANSIONS, xs);
                na.add(st, GS_CHILDREN, ks);
                na.max(st, GS_MAXNODES, mx);
            }
            if (ts) na.add(st, GS_TERMINAL, ts);
        }
    }
    if (mine) {
        const double rk = ((depth - (uint32_t)sl) & 1) ? -r : r;
        oaz_node* pp = na.at(T, pn);
        pp->N = pN + 1;
        pp->W = pW + rk;
    }
    for (uint32_t k = (uint32_t)sl + kSegLanes; k <= plen; k += kSegLanes) {  // paths deeper than 16
        const uint32_t n = path[k];
        const double rk = ((depth - k) & 1) ? -r : r;
        oaz_node* np = na.at(T, n);
        np->N += 1;
        np->W += rk;
    }
}

__global__ void __launch_bounds__(kBlock) k_expand_backup_seg(TreeView t, const oaz_state* __restrict__ roots,
                                                              const uint8_t* __restrict__ active,
                                                              const float* __restrict__ policy,
                                                              const float* __restrict__ value) {
    __shared__ float spol[kWavesPerBlock * 4][52];
    expand_backup_seg_body(t, roots, active, policy, value, seg_game(), spol[threadIdx.x >> 4]);
}

// Simulation s's expand/backup and simulation s+1's select of the same four games in one launch:
// a game's next walk needs only its own backup (the wave's own writes, ordered by a workgroup-scope
// fence), so every segment goes straight on to its next select instead of waiting for the whole
// grid; one launch and one grid ramp per simulation step fewer.
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OAZ_TREE_WPE)))
k_backup_select_seg(TreeView t, const oaz_state* __restrict__ roots, const uint8_t* __restrict__ active,
                    const float* __restrict__ policy, const float* __restrict__ value, const noise_t* __restrict__ noise,
                    SearchParams prm) {
    // the backup's policy rows and the select's fold operands share the LDS (40 KB: four 8-wave
    // workgroups per CU, 8 waves per SIMD; side by side they would be 47 KB and three)
    union BackupSelectLds {
        float spol[kWavesPerBlock * 4][52];
        WgFold wf;
    };
    __shared__ BackupSelectLds lds;
    const uint32_t g = seg_game();
    expand_backup_seg_body(t, roots, active, policy, value, g, lds.spol[threadIdx.x >> 4], NodesGlobalRegs{});
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    select_seg_body<NodesGlobalRegs, OAZ_WG_FOLD, true>(t, roots, active, noise, prm, g, nullptr, NodesGlobalRegs{},
                                                        &lds.wf);
}

// calculate_priors (mcts_arena.rs:104-124) + best child (87-94) for every root.
__device__ __forceinline__ void root_pi_best(const oaz_node* T, float* pi_out /*50, may be null*/,
                                             float& pi_lane, int& best_lane, int& K_out,
                                             uint32_t& best_mv) {
    const int l = lane_id();
    const NodeRegs root = load_node(&T[0]);
    const int K = (node_flags(root.misc) & 1) ? node_nch(root.misc) : 0;
    NodeRegs ch;
    ch.N = 0;
    ch.misc = 0;
    if (l < K) ch = load_node(&T[root.first + l]);
    const int bin = l < K ? (mv_slot(ch.misc) & 1) * 25 + mv_to(ch.misc) : -1;
    // integer visit sums per (card row, destination): f32 sums of integers are exact
    uint32_t cnt = 0;
    for (int j = 0; j < K; ++j) {
        const int bj = __shfl(bin, j);
        const uint32_t nj = (uint32_t)__shfl((int)ch.N, j);
        if (bj == l) cnt += nj;
    }
    const uint32_t total = wave_sum_u32(l < 50 ? cnt : 0u);
    pi_lane = total > 0 ? (float)cnt / (float)total : (float)cnt;
    if (pi_out && l < 50) pi_out[l] = pi_lane;
    // argmax of visits / root.visits: with N < 2^53 the quotient is monotone and injective
    // in N, so the last maximum of N is the reference's choice
    const int64_t key = l < K ? (int64_t)ch.N : INT64_MIN;
    best_lane = wave_argmax_last(key);
    best_mv = (uint32_t)__shfl((int)ch.misc, best_lane) & 0xFFFFu;
    K_out = K;
}

__global__ void __launch_bounds__(kBlock) k_search_finalize(TreeView t, const oaz_state* __restrict__ roots,
                                                            oaz_move* out_move, float* out_pi) {
    const uint32_t g = wave_game();
    if (g >= t.G) return;
    const int l = lane_id();
    const oaz_node* T = t.nodes + (size_t)g * t.cap;
    float pl;
    int best, K;
    uint32_t mv;
    root_pi_best(T, out_pi ? out_pi + (size_t)g * 50 : nullptr, pl, best, K, mv);
    if (l == 0 && out_move) {
        oaz_move m;
        if (K == 0) {  // no legal move (Q6): pass with the mover's first card
            m.from = 25;
            m.to = 25;
            m.piece = 0;
            m.slot = (uint8_t)((roots[g].to_move & 1) ? 2 : 0);
        } else {
            m.from = (uint8_t)mv_from(mv);
            m.to = (uint8_t)mv_to(mv);
            m.piece = (uint8_t)mv_piece(mv);
            m.slot = (uint8_t)mv_slot(mv);
        }
        out_move[g] = m;
    }
}

__device__ void start_game(const SlotView& sv, uint32_t g, uint32_t seq, bool lane0) {
    const uint64_t gid = slot_game_id(seq, sv.world, sv.rank, sv.G, g);
    const bool act = sv.quota == 0 || gid < sv.quota;
    uint8_t deck[5];
    if (sv.fixed_deck) {
        for (int i = 0; i < 5; ++i) deck[i] = sv.deck[i];
    } else {
        deal_deck(sv.seed, gid, deck);
    }
    oaz_state s;
    initial_state(deck, s);
    if (lane0) {
        store_state(&sv.root[g], s);
        sv.ply[g] = 0;
        sv.seq[g] = seq;
        sv.game_id[g] = gid;
        sv.active[g] = act ? 1 : 0;
    }
}

__global__ void __launch_bounds__(kBlock) k_selfplay_reset(TreeView t, SlotView sv) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.G) return;
    start_game(sv, g, 0, true);
    if (sv.stagger > 1 && sv.active[g] == 1) sv.active[g] = (uint8_t)(1 + g % (sv.stagger > 255 ? 255 : sv.stagger));
    store_fresh_node(&t.nodes[(size_t)g * t.cap], 1.0, 0);
    t.n_nodes[g] = 1;
}

// One ply of self_play (train.rs:55-80) per slot: record (state, pi, colour), play the most
// visited move (no temperature, Q9), detect the end (win, or the 152-ply cut of
// train.rs:74-79), emit z = reward(result, colour) for every sample (train.rs:83-85) and deal the
// next game. The tree is reset before the next ply's search (oaz_selfplay_step: k_tree_reset, a fresh
// tree per move, alphazero_mcts/mod.rs:68-77), so the ply's tree can be dumped in between.
__global__ void __launch_bounds__(kBlock) k_selfplay_move(TreeView t, SlotView sv) {
    const uint32_t g = wave_game();
    if (g >= t.G) return;
    const uint8_t act = sv.active[g];
    if (act != 1) {  // finished (0) or still waiting for its staggered start (> 1)
        if (lane_id() == 0) {
            if (act > 1) sv.active[g] = act - 1;
            sv.fin[g] = 0u;
        }
        return;
    }
    const int l = lane_id();
    oaz_node* T = t.nodes + (size_t)g * t.cap;
    uint64_t* st = t.stats + (size_t)g * GS_COUNT;
    oaz_state s = load_state(&sv.root[g]);
    const uint32_t ply = sv.ply[g];
    oaz_sample* hist = sv.hist + (size_t)g * sv.hcap;
    float pl;
    int best, K;
    uint32_t mv;
    const uint32_t hslot = ply < sv.hcap ? ply : sv.hcap - 1;
    root_pi_best(T, hist[hslot].pi, pl, best, K, mv);
    if (l == 0) {
        store_state(&hist[hslot].state, s);
        hist[hslot].z = 0.0f;
    }
    const int color = s.to_move & 1;
    int res;
    if (K == 0) {  // pass (state.rs:139-142) with the mover's first card (Q6)
        const int slot = color ? 2 : 0;
        const uint8_t c = s.cards[slot];
        s.cards[slot] = s.cards[4];
        s.cards[4] = c;
        res = OAZ_IN_PROGRESS;
        if (l == 0) st[GS_PASSES] += 1;
    } else {
        res = make_move(s, mv_from(mv), mv_to(mv), mv_piece(mv), mv_slot(mv), color);
    }
    s.to_move ^= 1;
    const uint32_t nply = ply + 1;
    const bool over = is_win(res) || (int)nply >= sv.max_plies + 2;
    if (l == 0) st[GS_MOVES] += 1;
    if (over) {
        // the game's records go out after the ply, in slot order (k_samples_scan, k_samples_emit): the
        // history stays until the slot's next game writes its first record in the next ply
        const uint32_t n = nply < sv.hcap ? nply : sv.hcap;
        if (l == 0) {
            sv.fin[g] = n | ((uint32_t)res << 24);
            st[GS_FINISHED] += 1;
            if (!is_win(res)) st[GS_CUT] += 1;
            if (res == OAZ_RED_WIN) st[GS_RED] += 1;
            if (res == OAZ_BLUE_WIN) st[GS_BLUE] += 1;
        }
        start_game(sv, g, sv.seq[g] + 1, l == 0);
    } else if (l == 0) {
        store_state(&sv.root[g], s);
        sv.ply[g] = nply;
        sv.fin[g] = 0u;
    }
    // the tree stays as searched (oaz_tree_dump after a ply); the next ply starts from k_tree_reset
}

// The records of the games that ended in this ply, in slot order (the reference appends a worker's
// games in the order they finish, train.rs:86-97; here a ply's finished games in slot order, so two
// engines playing the same games hold the same bytes in the same order). One workgroup: each thread
// sums a run of consecutive slots' record counts, the workgroup scans the runs in LDS, and every slot's
// first record position (the buffer's count so far + the slots before it) lands in fin_pos; the count
// grows by the ply's total.
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) k_samples_scan(SlotView sv) {
    const uint32_t per = (sv.G + kScanThreads - 1) / kScanThreads;
    const uint32_t g0 = threadIdx.x * per, g1 = g0 + per < sv.G ? g0 + per : sv.G;
    uint64_t sum = 0;
#pragma unroll 16
    for (uint32_t g = g0; g < g1; ++g) sum += sv.fin[g] & 0xFFFFFFu;  // (unrolled: the loads in flight together)
    __shared__ uint64_t run[kScanThreads];
    run[threadIdx.x] = sum;
    __syncthreads();
    for (int d = 1; d < kScanThreads; d <<= 1) {  // inclusive Hillis-Steele scan of the runs
        const uint64_t v = (int)threadIdx.x >= d ? run[threadIdx.x - d] : 0ull;
        __syncthreads();
        run[threadIdx.x] += v;
        __syncthreads();
    }
    const unsigned long long base = *sv.out_count;
    uint64_t pos = base + run[threadIdx.x] - sum;
#pragma unroll 16
    for (uint32_t g = g0; g < g1; ++g) {
        sv.fin_pos[g] = pos;
        pos += sv.fin[g] & 0xFFFFFFu;
    }
    __syncthreads();  // every thread read the count before it moves
    if (threadIdx.x == kScanThreads - 1) *sv.out_count = base + run[kScanThreads - 1];
}

// One wave per slot whose game ended in this ply: its records with z = reward(result, colour)
// (train.rs:83-85) at fin_pos; the records past the buffer's capacity are counted as dropped.
__global__ void __launch_bounds__(kBlock) k_samples_emit(TreeView t, SlotView sv) {
    const uint32_t g = wave_game();
    if (g >= sv.G) return;
    const uint32_t f = sv.fin[g], n = f & 0xFFFFFFu;
    if (n == 0) return;
    const int res = (int)(f >> 24), l = lane_id();
    const oaz_sample* hist = sv.hist + (size_t)g * sv.hcap;
    const uint64_t base = sv.fin_pos[g];
    for (uint32_t i = (uint32_t)l; i < n; i += 64) {
        oaz_sample smp = hist[i];
        smp.z = (float)reward(res, smp.state.to_move & 1);
        if (base + i < sv.out_cap) sv.out[base + i] = smp;
    }
    if (l == 0 && base + n > sv.out_cap)
        t.stats[(size_t)g * GS_COUNT + GS_DROPPED] += (base >= sv.out_cap) ? n : (uint32_t)(base + n - sv.out_cap);
}

__global__ void k_stats_reduce(const uint64_t* per_game, uint32_t G, uint64_t* out) {
    const int c = blockIdx.x;  // one block per counter
    uint64_t acc = 0;
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) {
        const uint64_t v = per_game[(size_t)g * GS_COUNT + c];
        acc = c == GS_MAXNODES ? (v > acc ? v : acc) : acc + v;
    }
    __shared__ uint64_t red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            const uint64_t o = red[threadIdx.x + s];
            red[threadIdx.x] = c == GS_MAXNODES ? (o > red[threadIdx.x] ? o : red[threadIdx.x])
                                                : red[threadIdx.x] + o;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = red[0];
}

// ---- launchers ----------------------------------------------------------------------------
static inline unsigned wave_grid(uint32_t n) { return (n + kWavesPerBlock - 1) / kWavesPerBlock; }
static inline unsigned thread_grid(long long n, int b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_movegen(const oaz_state* s, int n, uint32_t* masks, oaz_move* moves,
                          uint8_t* counts, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_movegen, dim3(wave_grid(n)), dim3(kBlock), 0, st, s, n, masks, moves, counts);
    return hipGetLastError();
}
hipError_t launch_step(oaz_state* s, const oaz_move* mv, int n, uint8_t* results, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_step, dim3(thread_grid(n, 256)), dim3(256), 0, st, s, mv, n, results);
    return hipGetLastError();
}
hipError_t launch_current_state(const oaz_state* s, int n, uint8_t* results, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_current_state, dim3(thread_grid(n, 256)), dim3(256), 0, st, s, n, results);
    return hipGetLastError();
}
hipError_t launch_encode(const oaz_state* s, int n, float* planes, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode, dim3(thread_grid((long long)n * 525, 256)), dim3(256), 0, st, s, n, planes);
    return hipGetLastError();
}
hipError_t launch_hash_eval(const oaz_state* s, int B, float* policy, float* value, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hash_eval, dim3(thread_grid(B, 256)), dim3(256), 0, st, s, B, policy, value);
    return hipGetLastError();
}
hipError_t launch_eval_compact(const TreeView& t, hipStream_t st) {
    if (t.G == 0 || !t.need) return hipSuccess;
    hipLaunchKernelGGL(k_eval_compact, dim3((unsigned)buckets_of(t.G)), dim3(kCompactThreads), 0, st, t);
    return hipGetLastError();
}
hipError_t launch_tree_reset(const TreeView& t, hipStream_t st) {
    hipLaunchKernelGGL(k_tree_reset, dim3(thread_grid(t.G, kBlock)), dim3(kBlock), 0, st, t);
    return hipGetLastError();
}
// Four games per wave (k_select_seg, k_backup_select_seg). A/B build only: OAZ_TREE_SEG=0 selects the
// one-game-per-wave kernels (the parity tests' second implementation of the same tree steps).
static bool tree_seg() {
#if OAZ_AB
    static const bool v = !(getenv("OAZ_TREE_SEG") && getenv("OAZ_TREE_SEG")[0] == '0');
    return v;
#else
    return true;
#endif
}
bool tree_seg_kernels() { return tree_seg(); }
hipError_t launch_select(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                         const noise_t* noise, SearchParams p, hipStream_t st) {
    if (tree_seg())
        hipLaunchKernelGGL(k_select_seg, dim3(wave_grid((t.G + 3) / 4)), dim3(kBlock), 0, st, t, roots, active, noise,
                           p);
    else
        hipLaunchKernelGGL(k_select, dim3(wave_grid(t.G)), dim3(kBlock), 0, st, t, roots, active, noise, p);
    return hipGetLastError();
}
hipError_t launch_root_noise(const oaz_state* roots, const uint8_t* active, const uint64_t* game_id,
                             const uint32_t* ply, SearchParams p, uint32_t G, uint32_t sim0, uint32_t nsims,
                             noise_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_root_noise, dim3(wave_grid(G)), dim3(kBlock), 0, st, roots, active, game_id, ply, p, G,
                       sim0, nsims, out);
    return hipGetLastError();
}
hipError_t launch_expand_backup(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                const float* policy, const float* value, hipStream_t st) {
    if (tree_seg())
        hipLaunchKernelGGL(k_expand_backup_seg, dim3(wave_grid((t.G + 3) / 4)), dim3(kBlock), 0, st, t, roots, active,
                           policy, value);
    else
        hipLaunchKernelGGL(k_expand_backup, dim3(wave_grid(t.G)), dim3(kBlock), 0, st, t, roots, active, policy,
                           value);
    return hipGetLastError();
}
hipError_t launch_backup_select(const TreeView& t, const oaz_state* roots, const uint8_t* active, const float* policy,
                                const float* value, const noise_t* noise, SearchParams p, hipStream_t st) {
    if (!tree_seg()) {  // the one-game-per-wave kernels, one after the other
        if (hipError_t err = launch_expand_backup(t, roots, active, policy, value, st)) return err;
        return launch_select(t, roots, active, noise, p, st);
    }
    hipLaunchKernelGGL(k_backup_select_seg, dim3(wave_grid((t.G + 3) / 4)), dim3(kBlock), 0, st, t, roots, active,
                       policy, value, noise, p);
    return hipGetLastError();
}
hipError_t launch_search_finalize(const TreeView& t, const oaz_state* roots, oaz_move* out_move,
                                  float* out_pi, hipStream_t st) {
    hipLaunchKernelGGL(k_search_finalize, dim3(wave_grid(t.G)), dim3(kBlock), 0, st, t, roots,
                       out_move, out_pi);
    return hipGetLastError();
}
hipError_t launch_selfplay_move(const TreeView& t, const SlotView& s, hipStream_t st) {
    hipLaunchKernelGGL(k_selfplay_move, dim3(wave_grid(t.G)), dim3(kBlock), 0, st, t, s);
    hipLaunchKernelGGL(k_samples_scan, dim3(1), dim3(kScanThreads), 0, st, s);
    hipLaunchKernelGGL(k_samples_emit, dim3(wave_grid(t.G)), dim3(kBlock), 0, st, t, s);
    return hipGetLastError();
}
hipError_t launch_selfplay_reset(const TreeView& t, const SlotView& s, hipStream_t st) {
    hipLaunchKernelGGL(k_selfplay_reset, dim3(thread_grid(t.G, kBlock)), dim3(kBlock), 0, st, t, s);
    return hipGetLastError();
}
hipError_t launch_stats_reduce(const uint64_t* per_game, uint32_t G, uint64_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(GS_COUNT), dim3(256), 0, st, per_game, G, out);
    return hipGetLastError();
}

// Q7 search_time on the device: the search's deadline on the device's constant-rate clock, taken when this
// kernel runs (just before the search's first kernel on the same stream; mcts_arena.rs:75-78 starts its
// Instant at the top of search()).
__global__ void k_deadline_start(uint64_t* deadline, uint64_t ticks) {
    if (threadIdx.x == 0) *deadline = (uint64_t)wall_clock64() + ticks;
}
hipError_t launch_deadline_start(uint64_t* deadline, uint64_t ticks, hipStream_t st) {
    hipLaunchKernelGGL(k_deadline_start, dim3(1), dim3(64), 0, st, deadline, ticks);
    return hipGetLastError();
}

}  // namespace oaz
