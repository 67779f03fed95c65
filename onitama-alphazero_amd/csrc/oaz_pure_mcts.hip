// oaz_pure_mcts.hip — the reference's pure-MCTS (random-rollout UCT) agent on gfx950
// (SURVEY.md 8f next #4): onitama-game/src/ai/mcts/mcts_arena.rs:56-264 + mod.rs:37-52.
//
// One thread per game runs the whole search (all playouts) in one launch: UCT selection in
// f32 with the last maximum winning ties (Iterator::max_by + f32::total_cmp, :147-156), expansion
// of a leaf once its visits exceed min_node_visits (:118-124, children in generate_all_legal_moves
// order), a uniformly random rollout to the end of the game with a random own card passed when
// no move exists (:190-230), and the +-1 reward backed up with a sign flip per level (:243-254).
// The final move is the most-visited root child (max_by_key, last maximum; :64-79) and the
// returned value its winrate.
//
// Defined where the reference is not: rollouts draw from a counter-based Philox stream keyed by
// (seed, game, playout) instead of thread_rng (draw = (u32 * n) >> 32); a rollout longer than
// rollout_cap plies scores 0 (the reference would keep playing); an expanded node without
// children (no legal move) is a leaf instead of a panic, and a root without children returns the
// pass move (from = to = 25, slot = the mover's first card) like oaz_search.
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_device.h"
#include "oaz_host.h"

using namespace oaz;

namespace pm {

__constant__ AttackTable c_att = make_attack_table();

constexpr uint8_t kExpanded = 1, kTerminal = 2;
constexpr uint32_t kTag = 0x9C7A0000u;  // Philox counter word 2 for rollout draws

struct Rng {  // draw d of (game, playout): Philox(seed; game, playout, kTag, d / 4), word d % 4
    uint64_t seed;
    uint32_t game, playout, d;
    u32x4 buf;
    __device__ uint32_t next() {
        if ((d & 3) == 0) buf = philox(seed, game, playout, kTag, d >> 2);
        const uint32_t w = d & 3;
        ++d;
        return w == 0 ? buf.x : w == 1 ? buf.y : w == 2 ? buf.z : buf.w;
    }
    __device__ uint32_t below(uint32_t n) { return (uint32_t)(((uint64_t)next() * n) >> 32); }
};

// generate_all_legal_moves order (state.rs:301-378): card slot, from square, to square.
// Returns the number of moves; with k >= 0 also the k-th move (packed).
// (The state's colour- and slot-indexed fields are read through selects (state_card, make_move_regs): a
// runtime index into the struct put the whole state in scratch memory.)
__device__ __forceinline__ int movegen_kth(const oaz_state& s, int color, const uint32_t (*att)[25], int k,
                                          uint32_t* kth) {
    const uint32_t P = color ? s.pawns[1] : s.pawns[0], K = color ? s.kings[1] : s.kings[0], occ = P | K;
    const int s0 = color ? 2 : 0;
    int n = 0;
    for (int si = 0; si < 2; ++si) {
        const int card = state_card(s, s0 + si) & 15;
        uint32_t pieces = occ;
        while (pieces) {
            const int from = __clz(pieces);
            pieces &= ~sq_bit(from);
            uint32_t map = att[card][from] & ~occ;
            const int c = __popc(map);
            if (k >= n && k < n + c) {
                for (int j = k - n; j > 0; --j) map &= ~sq_bit(__clz(map));
                const int to = __clz(map);
                *kth = pack_move(from, to, s0 + si, (P & sq_bit(from)) ? OAZ_PAWN : OAZ_KING);
            }
            n += c;
        }
    }
    return n;
}

// A rollout ply's random move (mcts_arena.rs:190-230): the same move movegen_kth(s, color, att, k) returns for
// k = rng.below(n), n = the move count, from one pass over the mover's pieces (the masks of both cards kept in
// registers, then k located by the two cards' counts), not a counting pass and a second search pass. Returns n
// (0: no legal move; no draw is taken then, as before).
__device__ __forceinline__ int rollout_pick(const oaz_state& s, int color, const uint32_t (*att)[25], Rng& rng,
                                            uint32_t* mv) {
    const uint32_t P = color ? s.pawns[1] : s.pawns[0], K = color ? s.kings[1] : s.kings[0], occ = P | K;
    const int s0 = color ? 2 : 0;
    const uint32_t (*a0)[25] = att + (state_card(s, s0) & 15), (*a1)[25] = att + (state_card(s, s0 + 1) & 15);
    uint32_t m0[5], m1[5];
    int fr[5];
    int n0 = 0, n1 = 0;
    uint32_t pieces = occ;
#pragma unroll
    for (int i = 0; i < 5; ++i) {  // at most 5 pieces, in square order (generate_all_legal_moves)
        const int from = pieces ? __clz(pieces) : 0;
        fr[i] = from;
        m0[i] = pieces ? (*a0)[from] & ~occ : 0u;
        m1[i] = pieces ? (*a1)[from] & ~occ : 0u;
        n0 += __popc(m0[i]);
        n1 += __popc(m1[i]);
        pieces &= pieces ? ~sq_bit(from) : ~0u;
    }
    const int n = n0 + n1;
    if (n == 0) return 0;
    int k = (int)rng.below((uint32_t)n);
    const bool second = k >= n0;
    k -= second ? n0 : 0;
    uint32_t map = 0;
    int from = 0;
    bool found = false;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t m = second ? m1[i] : m0[i];
        const int c = __popc(m);
        if (!found && k < c) {
            map = m;
            from = fr[i];
            found = true;
        } else if (!found) {
            k -= c;
        }
    }
    for (; k > 0; --k) map &= ~sq_bit(__clz(map));
    *mv = pack_move(from, __clz(map), s0 + (second ? 1 : 0), (P & sq_bit(from)) ? OAZ_PAWN : OAZ_KING);
    return n;
}

__device__ __forceinline__ float reward_f(int result, int color) {  // mcts_arena.rs:233-241
    if (!is_win(result)) return 0.0f;
    return ((result == OAZ_RED_WIN) == (color == OAZ_RED)) ? 1.0f : -1.0f;
}

__device__ __forceinline__ int32_t total_key(float x) {  // f32::total_cmp as a signed integer order
    int32_t i = __float_as_int(x);
    return i ^ (int32_t)((uint32_t)(i >> 31) >> 1);
}

struct Params {
    int playouts, min_visits, rollout_cap;
    float c;
    uint64_t seed, game0;
    uint32_t cap;
};

#ifndef OAZ_PM_SELB
#define OAZ_PM_SELB 4
#endif
constexpr int kSelBatch = OAZ_PM_SELB;
#ifndef OAZ_PM_WPE
#define OAZ_PM_WPE 6
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OAZ_PM_WPE))) void k_pure_mcts(const oaz_state* roots, int G, Params p, const float* ln_tab,
                                                  oaz_pure_node* nodes, oaz_move* out_move, float* out_value,
                                                  uint64_t* stats /* [G][8] */) {
    __shared__ uint32_t att_s[2][16][25];
    for (int i = threadIdx.x; i < 2 * 16 * 25; i += blockDim.x) (&att_s[0][0][0])[i] = (&c_att.m[0][0][0])[i];
    __syncthreads();
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    oaz_pure_node* T = nodes + (size_t)g * p.cap;
    const int root_color = roots[g].to_move & 1;
    T[0] = oaz_pure_node{0u, 0.0f, 0.0f, 0u, 0xFFFFFFFFu, 0, 0, 0};
    uint32_t n_nodes = 1;
    // the search's counters in LDS (the thread's own slots), out of the registers the walk and rollout need
    __shared__ uint64_t stl[5][64];
    uint64_t& st_plies = stl[0][threadIdx.x];
    uint64_t& st_pass = stl[1][threadIdx.x];
    uint64_t& st_exp = stl[2][threadIdx.x];
    uint64_t& st_capped = stl[3][threadIdx.x];
    uint64_t& st_over = stl[4][threadIdx.x];
    st_plies = st_pass = st_exp = st_capped = st_over = 0;
    for (int po = 0; po < p.playouts; ++po) {
        oaz_state s = roots[g];  // (reloaded per playout: an L2 hit, six registers fewer)
        uint32_t idx = 0;
        // 1. selection (mcts_arena.rs:100-116)
        while ((T[idx].flags & kExpanded) && !(T[idx].flags & kTerminal) && T[idx].nch) {
            const float lnN = ln_tab[T[idx].visits];
            const uint32_t first = T[idx].first, nch = T[idx].nch;
            uint32_t best = first;
            int32_t bk = INT32_MIN;
            // the children's (visits, winrate) kSelBatch at a time, all loads in flight before the fold (the
            // fold itself stays sequential in child order)
            for (uint32_t c0 = 0; c0 < nch; c0 += kSelBatch) {
                uint32_t vis[kSelBatch];
                float wr[kSelBatch];
#pragma unroll
                for (int j = 0; j < kSelBatch; ++j)
                    if (c0 + j < nch) {
                        vis[j] = T[first + c0 + j].visits;
                        wr[j] = T[first + c0 + j].winrate;
                    }
#pragma unroll
                for (int j = 0; j < kSelBatch; ++j)
                    if (c0 + j < nch) {
                        const float u = wr[j] + p.c * sqrtf(lnN / (float)vis[j]);
                        const int32_t k = total_key(u);
                        if (k >= bk) {  // max_by: the last maximum wins
                            bk = k;
                            best = first + c0 + j;
                        }
                    }
            }
            const uint32_t m = T[best].mv;
            const int color = s.to_move & 1;
            const int res = make_move_regs(s, mv_from(m), mv_to(m), mv_piece(m), mv_slot(m), color);
            s.to_move ^= 1;
            if (is_win(res)) T[best].flags |= kTerminal;
            idx = best;
        }
        // 2. expansion (mcts_arena.rs:118-124, 166-185)
        if (!(T[idx].flags & (kExpanded | kTerminal)) && T[idx].visits > (uint32_t)p.min_visits) {
            const int color = s.to_move & 1;
            const int n = movegen_kth(s, color, att_s[color], -1, nullptr);
            if (n_nodes + (uint32_t)n <= p.cap) {
                T[idx].first = n_nodes;
                T[idx].nch = (uint8_t)n;
                for (int k = 0; k < n; ++k) {
                    uint32_t m = 0;
                    movegen_kth(s, color, att_s[color], k, &m);
                    T[n_nodes + k] = oaz_pure_node{0u, 0.0f, 0.0f, 0u, idx, (uint16_t)m, 0, 0};
                }
                n_nodes += n;
                T[idx].flags |= kExpanded;
                ++st_exp;
            } else {
                ++st_over;  // capacity reached: the node stays a leaf
            }
        }
        // 3. simulation (mcts_arena.rs:188-231); reward colour = the colour that moved into idx
        const int reward_color = idx == 0 ? root_color : ((s.to_move & 1) ^ 1);
        Rng rng{p.seed, (uint32_t)(p.game0 + g), (uint32_t)po, 0u, {}};
        int mr = current_state(s);
        float r;
        if (is_win(mr)) {
            r = reward_f(mr, reward_color);
        } else {
            int color = s.to_move & 1, plies = 0;
            bool capped = false;
            while (!is_win(mr)) {
                if (plies >= p.rollout_cap) {
                    capped = true;
                    break;
                }
                uint32_t m = 0;
                const int n = rollout_pick(s, color, att_s[color], rng, &m);
                if (n == 0) {  // pass with a random own card (state.rs:139-142)
                    state_rotate(s, (color ? 2 : 0) + (int)rng.below(2));
                    color ^= 1;
                    ++st_pass;
                    ++plies;
                    continue;
                }
                mr = make_move_regs(s, mv_from(m), mv_to(m), mv_piece(m), mv_slot(m), color);
                color ^= 1;
                ++plies;
            }
            st_plies += plies;
            if (capped) {
                ++st_capped;
                r = 0.0f;
            } else {
                r = reward_f(mr, reward_color);
            }
        }
        // 4. backpropagation (mcts_arena.rs:243-254, MctsNode::update :361-365)
        for (uint32_t v = idx;;) {
            T[v].visits += 1;
            T[v].reward += r;
            T[v].winrate = T[v].reward / (float)T[v].visits;
            if (v == 0) break;
            v = T[v].parent;
            r = -r;
        }
    }
    // best root child by visits, last maximum (mcts_arena.rs:64-79)
    oaz_move mv;
    float value = 0.0f;
    if (T[0].nch == 0) {
        mv.from = 25;
        mv.to = 25;
        mv.piece = 0;
        mv.slot = (uint8_t)(root_color ? 2 : 0);
    } else {
        uint32_t best = T[0].first, bv = 0;
        for (uint32_t c = T[0].first; c < T[0].first + T[0].nch; ++c)
            if (T[c].visits >= bv) {
                bv = T[c].visits;
                best = c;
            }
        const uint32_t m = T[best].mv;
        mv.from = (uint8_t)mv_from(m);
        mv.to = (uint8_t)mv_to(m);
        mv.piece = (uint8_t)mv_piece(m);
        mv.slot = (uint8_t)mv_slot(m);
        value = T[best].winrate;
    }
    out_move[g] = mv;
    out_value[g] = value;
    uint64_t* st = stats + (size_t)g * 8;
    st[0] = (uint64_t)p.playouts;
    st[1] = st_exp;
    st[2] = st_plies;
    st[3] = st_pass;
    st[4] = st_capped;
    st[5] = n_nodes;
    st[6] = st_over;
    st[7] = 0;
}

}  // namespace pm

extern "C" void oaz_pure_mcts_config_default(oaz_pure_mcts_config* c) {  // ai/mcts/mod.rs:21-30
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->max_playouts = 5000;
    c->min_node_visits = 5;
    c->exploration_c = 1.41421354f;  // 2f32.sqrt()
    c->rollout_cap = 1000;
    c->seed = 20260101ull;
    c->game_id0 = 0;
}

extern "C" size_t oaz_pure_mcts_tree_capacity(const oaz_pure_mcts_config* c) {
    if (!c || c->max_playouts < 0) return 0;
    // every expanded node first collects min_node_visits + 1 playouts as a leaf, so a search
    // expands at most playouts / (min_node_visits + 1) nodes, each with <= 40 children
    const size_t exp = (size_t)c->max_playouts / (size_t)(c->min_node_visits + 1) + 1;
    return 1 + 40 * exp;
}

// The search's device buffers as one allocation, and the last one of each device kept for the next call: a
// 1 M-search launch's trees take 64 GB, and allocating and freeing that per call cost 0.02-1.9 s on top of a
// 0.42 s search depending on the box (bench.py --mode pure_mcts). A call finding the kept buffer in use (a
// concurrent search on the same device) allocates its own and frees it on return.
// oaz_pure_mcts_release_workspace returns a device's kept buffer.
namespace {
struct PureWorkspace {
    std::mutex mu;
    void* p = nullptr;
    size_t n = 0;
    bool busy = false;
};
constexpr int kPureMaxDevices = 64;
PureWorkspace g_pure_ws[kPureMaxDevices];

// (on the calling thread's current device, which is `dev`)
hipError_t ws_acquire(int dev, size_t bytes, void** out, bool* kept) {
    PureWorkspace& w = g_pure_ws[dev];
    {
        std::lock_guard<std::mutex> lk(w.mu);
        if (!w.busy) {
            if (w.n < bytes) {
                if (w.p) (void)hipFree(w.p);
                w.p = nullptr;
                w.n = 0;
                if (hipError_t e = hipMalloc(&w.p, bytes)) return e;
                w.n = bytes;
            }
            w.busy = true;
            *out = w.p;
            *kept = true;
            return hipSuccess;
        }
    }
    *kept = false;
    return hipMalloc(out, bytes);
}
void ws_release(int dev, void* p, bool kept) {
    if (!p) return;
    if (!kept) {
        (void)hipFree(p);
        return;
    }
    std::lock_guard<std::mutex> lk(g_pure_ws[dev].mu);
    g_pure_ws[dev].busy = false;
}
size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }
}  // namespace

extern "C" int oaz_pure_mcts_release_workspace(int device) {
    if (device < 0 || device >= kPureMaxDevices) return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: device %d", device);
    PureWorkspace& w = g_pure_ws[device];
    std::lock_guard<std::mutex> lk(w.mu);
    if (w.busy) return oaz_set_err(OAZ_ERR_STATE, "pure_mcts: the workspace of device %d is in use", device);
    if (w.p) {
        DeviceScope dev_scope_(device);
        (void)hipFree(w.p);
    }
    w.p = nullptr;
    w.n = 0;
    return 0;
}

extern "C" int oaz_pure_mcts_search(const oaz_state* roots, int G, const oaz_pure_mcts_config* cfg,
                                    oaz_move* out_move, float* out_value, oaz_pure_mcts_stats* stats,
                                    oaz_pure_node* tree_out, size_t tree_cap) {
    if (G < 0 || (G > 0 && (!roots || !out_move || !out_value)) || !cfg)
        return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: null argument");
    if (cfg->max_playouts < 0 || cfg->min_node_visits < 0 || cfg->rollout_cap < 0)
        return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: negative playouts / min_node_visits / rollout_cap");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return oaz_set_err(OAZ_ERR_NO_DEVICE, "pure_mcts: no HIP device");
    if (cfg->device < 0 || cfg->device >= ndev)
        return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: device %d of %d", cfg->device, ndev);
    for (int g = 0; g < G; ++g)
        if ((roots[g].to_move & ~1) || (roots[g].cards[0] | roots[g].cards[1] | roots[g].cards[2] | roots[g].cards[3] |
                                        roots[g].cards[4]) > 15)
            return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: root %d is not a valid state", g);
    if (stats) memset(stats, 0, sizeof(*stats));
    if (G == 0) return 0;
    const size_t cap = oaz_pure_mcts_tree_capacity(cfg);
    if (cap > 0xFFFFFFF0u) return oaz_set_err(OAZ_ERR_ARG, "pure_mcts: tree capacity too large");
    std::vector<float> ln((size_t)cfg->max_playouts + 2);
    for (size_t n = 0; n < ln.size(); ++n) ln[n] = logf((float)n);  // (parent.visits as f32).ln()
    pm::Params p{cfg->max_playouts, cfg->min_node_visits, cfg->rollout_cap, cfg->exploration_c, cfg->seed,
                 cfg->game_id0, (uint32_t)cap};
    oaz_state* d_roots = nullptr;
    float *d_ln = nullptr, *d_val = nullptr;
    oaz_pure_node* d_nodes = nullptr;
    oaz_move* d_mv = nullptr;
    uint64_t* d_st = nullptr;
    void* ws = nullptr;
    bool ws_kept = false;
    // the workspace: roots, ln table, values, moves, statistics, trees (256-byte aligned sections)
    const size_t o_ln = align256(sizeof(oaz_state) * G), o_val = o_ln + align256(sizeof(float) * ln.size());
    const size_t o_mv = o_val + align256(sizeof(float) * G), o_st = o_mv + align256(sizeof(oaz_move) * G);
    const size_t o_nodes = o_st + align256(sizeof(uint64_t) * 8 * G);
    const size_t ws_bytes = o_nodes + sizeof(oaz_pure_node) * cap * G;
    int rc = 0;
    auto fail = [&](hipError_t e, const char* what) {
        rc = oaz_set_err(OAZ_ERR_HIP, "pure_mcts: %s: %s", what, hipGetErrorString(e));
    };
    hipError_t e;
    // on cfg->device, on a stream of its own: a search on a worker thread neither lands on the thread's
    // default device nor waits for (or stalls) the engines searching on the same GPU meanwhile
    hipStream_t sm = nullptr;
    int prev_dev = -1;  // the calling thread's current device, restored on return
    if ((e = hipGetDevice(&prev_dev)) != hipSuccess) prev_dev = -1;
    if ((e = hipSetDevice(cfg->device)) != hipSuccess) fail(e, "set device");
    else if ((e = hipStreamCreateWithFlags(&sm, hipStreamNonBlocking)) != hipSuccess) fail(e, "stream");
    else if (cfg->device >= kPureMaxDevices) rc = oaz_set_err(OAZ_ERR_ARG, "pure_mcts: device %d unsupported", cfg->device);
    else if ((e = ws_acquire(cfg->device, ws_bytes, &ws, &ws_kept)) != hipSuccess) fail(e, "alloc");
    if (!rc) {
        char* b = static_cast<char*>(ws);
        d_roots = reinterpret_cast<oaz_state*>(b);
        d_ln = reinterpret_cast<float*>(b + o_ln);
        d_val = reinterpret_cast<float*>(b + o_val);
        d_mv = reinterpret_cast<oaz_move*>(b + o_mv);
        d_st = reinterpret_cast<uint64_t*>(b + o_st);
        d_nodes = reinterpret_cast<oaz_pure_node*>(b + o_nodes);
    }
    if (!rc) {
        (void)hipMemcpyAsync(d_roots, roots, sizeof(oaz_state) * G, hipMemcpyHostToDevice, sm);
        (void)hipMemcpyAsync(d_ln, ln.data(), sizeof(float) * ln.size(), hipMemcpyHostToDevice, sm);
        hipLaunchKernelGGL(pm::k_pure_mcts, dim3((G + 63) / 64), dim3(64), 0, sm, d_roots, G, p, d_ln, d_nodes, d_mv,
                           d_val, d_st);
        if ((e = hipGetLastError()) != hipSuccess || (e = hipStreamSynchronize(sm)) != hipSuccess) fail(e, "kernel");
    }
    if (!rc) {
        std::vector<uint64_t> st((size_t)G * 8);
        (void)hipMemcpyAsync(out_move, d_mv, sizeof(oaz_move) * G, hipMemcpyDeviceToHost, sm);
        (void)hipMemcpyAsync(out_value, d_val, sizeof(float) * G, hipMemcpyDeviceToHost, sm);
        (void)hipMemcpyAsync(st.data(), d_st, sizeof(uint64_t) * st.size(), hipMemcpyDeviceToHost, sm);
        if ((e = hipStreamSynchronize(sm)) != hipSuccess) fail(e, "copy");
        if (stats && !rc)
            for (int g = 0; g < G; ++g) {
                stats->playouts += st[g * 8 + 0];
                stats->expansions += st[g * 8 + 1];
                stats->rollout_plies += st[g * 8 + 2];
                stats->rollout_passes += st[g * 8 + 3];
                stats->rollouts_capped += st[g * 8 + 4];
                if (st[g * 8 + 5] > stats->max_nodes) stats->max_nodes = st[g * 8 + 5];
                stats->tree_full += st[g * 8 + 6];
            }
        if (tree_out && tree_cap && !rc) {
            for (int g = 0; g < G; ++g)
                (void)hipMemcpyAsync(tree_out + (size_t)g * tree_cap, d_nodes + (size_t)g * cap,
                                     sizeof(oaz_pure_node) * (tree_cap < cap ? tree_cap : cap), hipMemcpyDeviceToHost, sm);
            if ((e = hipStreamSynchronize(sm)) != hipSuccess) fail(e, "tree copy");
        }
    }
    if (sm) (void)hipStreamSynchronize(sm);
    if (ws) ws_release(cfg->device, ws, ws_kept);
    if (sm) (void)hipStreamDestroy(sm);
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
    return rc;
}
