// oaz_search_lat.hip — the whole search of a small batch in ONE launch: one workgroup per game runs all
// of its `sims` simulations (mcts_arena.rs:75-102: playout = select -> evaluate -> expand / back up,
// 127-177), for the Agent API's generate_move (alphazero_mcts/mod.rs:122-144: one game, 400 playouts)
// and an arena fight's last games (evaluator.rs:355-399).
//
// Why: with few games a simulation step is two dependent launches (the fused expand/backup + select,
// then the network) whose work is a few microseconds of dependent memory round trips and one small
// network evaluation; each launch adds its dispatch and ramp (~2.5 us of a ~28 us step at G = 1),
// and the network's first weights cannot be requested before its launch starts. Here the games are
// independent workgroups that never wait for each other (no grid-wide step), the tree walk of wave 4
// runs while the compute waves already hold the first conv's weights, and nothing is launched per
// simulation.
//
// Same arithmetic as the per-step launches, bit for bit: the tree work is the segmented kernels' own
// bodies (select_seg_body, expand_backup_seg_body: one 16-lane segment of wave 4 holds the game, the
// other segments idle), the network is k_nn_h3s's body (bit-identical to k_nn_h3) with its in-kernel
// fp16-range recompute, or the HASH test evaluator. Used when the per-step loop would launch one NN
// workgroup per game anyway (games <= CUs), with the fp16x3 network or HASH, no root noise (the
// Agent / arena config, train = false) and no leaf compaction (oaz_engine.cpp run_sims;
// oaz_config.step_kernels = 1 turns it off).
//
// Q7 search_time on the device (both kernels): the reference's loop runs a playout while
// `playouts < max_playouts && elapsed < search_time` (mcts_arena.rs:75-81), one clock read per playout.
// Here thread 0 of a workgroup reads the device's constant-rate clock (wall_clock64) before every
// simulation after the first and the workgroup stops there when it is at or past `*deadline` (written by
// k_deadline_start on the same stream just before the search: its start + the budget), so a budgeted
// search is still one launch (k_search_lat) or one launch per noise chunk (k_search_grp), never a host
// round trip per simulation. Each workgroup stops on its own clock read: k_search_lat's games (one per
// workgroup, as each reference agent has its own clock) and k_search_grp's 16-game groups may run different
// playout counts (>= 1); sims_run[g] records game g's.
namespace oaz {

constexpr int kLatThreads = 512;  // 8 waves: k_nn_h3s's geometry; wave 4 also walks the tree

// LDS of k_search_lat beside the network's (h3s::kBytes): the walker's per-game records (leaf position,
// leaf, depth, node count), the leaf's evaluation (the network's heads write it here), the game's statistics,
// its path, the root position and the sqrt(N) table (each walk level and each simulation would otherwise wait
// on a global round trip for them), and the top of the game's tree (its first nodes, as many as fit: the root
// and the first expansions, which every walk passes through; lat_layout).
constexpr int kLatStateOff = h3s::kBytes;          // oaz_state
constexpr int kLatVarsOff = kLatStateOff + 32;     // leaf, depth, n_nodes
constexpr int kLatPolOff = kLatVarsOff + 16;       // the leaf's evaluation: policy[50], value
constexpr int kLatStatOff = kLatPolOff + 52 * 4;   // the game's statistics (added to its global slots at the end)
constexpr int kLatPathOff = kLatStatOff + GS_COUNT * 8;
constexpr int kLatPath = 2048;                     // most path entries held in LDS (pathcap = sims + 1)
constexpr int kLatSq = 2048;                       // most sqrt(N) entries held in LDS
constexpr int kLatLds = H3Fallback<H3Cfg<0>>::kLds * 4;
// From kLatPathOff on the layout follows the launch's simulation count: the path (pathcap entries), the
// root position, sqrt(0 .. sims), then as many tree nodes as the rest of the LDS holds.
struct LatLayout {
    int root, sq, cache;
    uint32_t nsq, ncached;
};
__device__ __forceinline__ LatLayout lat_layout(uint32_t pathcap, bool path_lds, int sims, uint32_t cap) {
    LatLayout l;
    l.root = kLatPathOff + (path_lds ? (int)((pathcap * 4 + 15) & ~15u) : 0);
    l.sq = l.root + 32;
    l.nsq = (uint32_t)sims + 1 < (uint32_t)kLatSq ? (uint32_t)sims + 1 : (uint32_t)kLatSq;
    l.cache = (l.sq + (int)l.nsq * 8 + 31) & ~31;
    const uint32_t fit = (uint32_t)((kLatLds - l.cache) / (int)sizeof(oaz_node));
    l.ncached = fit < cap ? fit : cap;
    return l;
}

// The tree walk (wave 4 only) as calls of their own: the walk needs ~80 VGPRs, the network ~240 (the
// compute waves hold a conv's weights), and inlined into one loop the two allocations spill; a call
// per simulation costs a few register saves.
__device__ __noinline__ void lat_backup(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                        const float* policy, const float* value, uint32_t gs, float* sp,
                                        const NodesCached& na) {
    expand_backup_seg_body(t, roots, active, policy, value, gs, sp, na);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// The walk of the workgroup's one game on the whole walker wave: lane l holds child l (K <= 40 < 64), so a
// level evaluates each child's PUCT once instead of three children per lane of a 16-lane segment. Same
// expressions and the same last-maximum rule as select_seg_body / k_select (mcts_arena.rs:183-223): the
// arg-max runs within each 16-lane row by DPP and across the four rows on scalars, the chosen child's
// fields are read from its lane with v_readlane. No root noise here (k_search_lat's condition).
// DBG (diagnostic build): s_memtime cycles of the prologue (root position and node) into GS_MOVES and of each
// level's child loads + PUCT keys into GS_FINISHED
template <int DBG = 0>
__device__ __noinline__ void lat_select_wide(const TreeView& t, const SearchParams& prm, const NodesCached& na) {
    uint64_t d0 = DBG ? __builtin_amdgcn_s_memtime() : 0, dl = 0;
    const int l = (int)(threadIdx.x & 63);
    oaz_node* T = t.nodes;
    uint32_t* path = t.path;
    oaz_state s = load_state(na.rt);
    int color = s.to_move & 1;
    NodeRegs nd = load_node(na.at(T, 0));
    uint32_t node = 0, depth = 0;
    if (l == 0) path[0] = 0;
    bool stuck = false;
    if constexpr (DBG) {
        asm volatile("" ::"v"(nd.misc), "v"(s.pawns[0]));
        const uint64_t d1 = __builtin_amdgcn_s_memtime();
        if (l == 0) na.add(nullptr, GS_MOVES, d1 - d0);
    }
    while ((node_flags(nd.misc) & 1) && !(node_flags(nd.misc) & 2)) {
        const int K = node_nch(nd.misc);
        if (K == 0) {  // reference would panic in select (Q6): stop here, treat as a leaf
            stuck = true;
            break;
        }
        const uint64_t da = DBG ? __builtin_amdgcn_s_memtime() : 0;
        NodeRegs ch;
        ch.W = 0.0;
        ch.P = 0.0;
        ch.N = 0;
        ch.first = 0;
        ch.misc = 0;
        if (l < K) ch = load_node(na.at(T, nd.first + l));
        const double sqn = na.sqrt_n(t, nd.N);
        int64_t key = INT64_MIN;
        if (l < K) {
            const double q = ch.N ? ch.W / (double)ch.N : 0.0;
            const double sq = sqn / (double)(ch.N + 1);
            const double u = q + prm.c_puct * ch.P * sq;  // mcts_arena.rs:204-207
            key = total_key(u);
        }
        if constexpr (DBG) {
            asm volatile("" ::"v"(key));
            dl += __builtin_amdgcn_s_memtime() - da;
        }
        int idx = l;
        seg_amax_step<0xB1>(key, idx);   // within each row of 16 lanes (every lane ends with its row's best)
        seg_amax_step<0x4E>(key, idx);
        seg_amax_step<0x141>(key, idx);
        seg_amax_step<0x140>(key, idx);
        int best = __builtin_amdgcn_readlane(idx, 0);
        int64_t bkey = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)key >> 32), 0) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)key, 0));
#pragma unroll
        for (int r = 1; r < 4; ++r) {  // rows hold ascending children: a tie goes to the later row
            const int64_t rk =
                (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)key >> 32), 16 * r) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)key, 16 * r));
            const int ri = __builtin_amdgcn_readlane(idx, 16 * r);
            if (rk > bkey || (rk == bkey && ri > best)) {
                bkey = rk;
                best = ri;
            }
        }
        NodeRegs c;  // (the walk reads only N, first and misc of the node it descends to)
        c.W = 0.0;
        c.P = 0.0;
        c.N = (uint32_t)__builtin_amdgcn_readlane((int)ch.N, best);
        c.first = (uint32_t)__builtin_amdgcn_readlane((int)ch.first, best);
        c.misc = (uint32_t)__builtin_amdgcn_readlane((int)ch.misc, best);
        const uint32_t cidx = nd.first + (uint32_t)best;
        const int res = make_move_regs(s, mv_from(c.misc), mv_to(c.misc), mv_piece(c.misc), mv_slot(c.misc), color);
        color ^= 1;  // game_state.player_color.switch()
        if (is_win(res)) {
            c.misc |= 2u << 24;
            if (l == 0) *flags_ptr(na.at(T, cidx)) = (uint8_t)(node_flags(c.misc));
        }
        ++depth;
        if (l == 0 && depth < t.pathcap) path[depth] = cidx;
        node = cidx;
        nd = c;
    }
    s.to_move = (uint8_t)color;
    if (l == 0) {
        const bool need = leaf_needs_eval(nd.misc, s);
        store_state(t.leaf_state, s);
        *t.leaf = node;
        *t.depth = depth;
        na.add(nullptr, GS_SIMS, 1);
        na.add(nullptr, GS_DEPTH, depth);
        na.add(nullptr, GS_EVALS, need);
        if (stuck) na.add(nullptr, GS_STUCK, 1);
        if constexpr (DBG) na.add(nullptr, GS_FINISHED, dl);
    }
}

// DBG 2 probe: a call with the walker's arguments that only reads two of them
__device__ __noinline__ void lat_probe(const TreeView& t, const oaz_state*, const uint8_t*, const SearchParams& prm,
                                       uint32_t gs, const NodesCached& na) {
    if (gs == 0 && threadIdx.x == 1000) *t.leaf = na.n + (uint32_t)prm.seed;  // never true: keeps the reads
}

// Copies the LDS-held tree state of the game to its global slots (out = true) or back (out = false):
// before the fp16-range recompute (which uses the whole LDS) and, for the nodes and the node count, at
// the end. All threads of the workgroup; the caller places the barriers.
__device__ __forceinline__ void lat_sync_tree(const TreeView& tl, const TreeView& tg, const NodesCached& na,
                                              bool path_lds, bool out) {
    const int tid = (int)threadIdx.x;
    const uint32_t nn = out ? *tl.n_nodes : *tg.n_nodes;
    const uint32_t nc = nn < na.n ? nn : na.n;
    uint4* lq = reinterpret_cast<uint4*>(na.L);
    uint4* gq = reinterpret_cast<uint4*>(tg.nodes);
    for (uint32_t k = (uint32_t)tid; k < 2 * nc; k += blockDim.x) {
        if (out) gq[k] = lq[k];
        else lq[k] = gq[k];
    }
    if (path_lds)
        for (uint32_t k = (uint32_t)tid; k < tg.pathcap; k += blockDim.x) {
            if (out) tg.path[k] = tl.path[k];
            else tl.path[k] = tg.path[k];
        }
    if (tid == 0) {
        if (out) {
            *tg.n_nodes = *tl.n_nodes;
            *tg.leaf = *tl.leaf;
            *tg.depth = *tl.depth;
            *tg.leaf_state = *tl.leaf_state;
        } else {
            *tl.n_nodes = *tg.n_nodes;
            *tl.leaf = *tg.leaf;
            *tl.depth = *tg.depth;
            *tl.leaf_state = *tg.leaf_state;
        }
    }
}

// DBG 1 (diagnostic, A/B build only: OAZ_LAT_DBG=1; 2 adds a probe call, GS_DROPPED): the walker's s_memtime cycles in the expand / back up, the
// select, and the wait for the evaluation (barriers + network or HASH) are added to the game's statistics slots
// GS_CUT / GS_RED / GS_BLUE (and the whole loop to GS_PASSES); the search's results are unchanged.
template <int DBG = 0>
__global__ void __launch_bounds__(kLatThreads) k_search_lat(TreeView t, const oaz_state* __restrict__ roots,
                                                            const uint8_t* __restrict__ active, SearchParams prm,
                                                            int sims, int hash_eval, const float* __restrict__ blob,
                                                            int blocks, const float* __restrict__ xblob,
                                                            unsigned long long* __restrict__ fallback, float* policy,
                                                            float* value, const uint64_t* __restrict__ deadline,
                                                            uint32_t* __restrict__ sims_run) {
    using C = H3Cfg<0>;
    __shared__ __attribute__((aligned(16))) float lds[H3Fallback<C>::kLds];
    static_assert(kLatPathOff + kLatPath * 4 + 32 + kLatSq * 8 + 64 * (int)sizeof(oaz_node) <= kLatLds,
                  "k_search_lat LDS");
    const uint32_t g = blockIdx.x;
    if (g >= t.G || (active && active[g] != 1)) return;  // uniform over the workgroup
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const bool walker = wave == 4;
    char* const lb = reinterpret_cast<char*>(lds);
    // the game's slice of the tree arrays (one game: index 0), and the same with the per-game records,
    // the path and the top of the tree in LDS
    TreeView tg = t;
    tg.nodes = t.nodes + (size_t)g * t.cap;
    tg.n_nodes = t.n_nodes + g;
    tg.path = t.path + (size_t)g * t.pathcap;
    tg.depth = t.depth + g;
    tg.leaf = t.leaf + g;
    tg.leaf_state = t.leaf_state + g;
    tg.stats = t.stats + (size_t)g * GS_COUNT;
    tg.need = nullptr;
    tg.slot = nullptr;
    tg.G = 1;
    const bool path_lds = t.pathcap <= (uint32_t)kLatPath;
    TreeView tl = tg;
    tl.leaf_state = reinterpret_cast<oaz_state*>(lb + kLatStateOff);
    tl.leaf = reinterpret_cast<uint32_t*>(lb + kLatVarsOff);
    tl.depth = tl.leaf + 1;
    tl.n_nodes = tl.leaf + 2;
    if (path_lds) tl.path = reinterpret_cast<uint32_t*>(lb + kLatPathOff);
    // tl.nodes stays the game's global slot: the node accessor maps nodes [0, ncached) to the LDS copy
    const LatLayout ly = lat_layout(t.pathcap, path_lds, sims, t.cap);
    const uint32_t ncached = ly.ncached, nsq = ly.nsq;
    uint64_t* const stl = reinterpret_cast<uint64_t*>(lb + kLatStatOff);
    const NodesCached na{reinterpret_cast<oaz_node*>(lb + ly.cache), ncached,
                         reinterpret_cast<const double*>(lb + ly.sq), nsq,
                         reinterpret_cast<const oaz_state*>(lb + ly.root), stl};
    float* const pol = reinterpret_cast<float*>(lb + kLatPolOff);  // the leaf's policy row, value at [50]
    // the root position and sqrt(0 .. sims) (read-only for the launch) and zeroed statistics: at the start and
    // after an fp16-range recompute (which uses the whole LDS)
    auto fill_resident = [&] {
        double* sq = reinterpret_cast<double*>(lb + ly.sq);
        for (uint32_t k = threadIdx.x; k < nsq; k += kLatThreads) sq[k] = t.sqrt_tab[k];
        static_assert(sizeof(oaz_state) % 4 == 0 && sizeof(oaz_state) <= 32, "root copy");
        if (threadIdx.x < sizeof(oaz_state) / 4)
            reinterpret_cast<uint32_t*>(lb + ly.root)[threadIdx.x] =
                reinterpret_cast<const uint32_t*>(roots + g)[threadIdx.x];
        if (threadIdx.x < GS_COUNT) stl[threadIdx.x] = 0;
    };
    auto flush_stats = [&] {  // the statistics gathered in LDS to the game's slots (one writer: this workgroup)
        if (threadIdx.x < GS_COUNT) {
            const uint64_t v = stl[threadIdx.x];
            if (threadIdx.x == GS_MAXNODES) {
                if (v > tg.stats[threadIdx.x]) tg.stats[threadIdx.x] = v;
            } else if (v) {
                tg.stats[threadIdx.x] += v;
            }
        }
    };
    fill_resident();
    const oaz_state* rg = roots + g;
    const uint8_t* ag = active ? active + g : nullptr;
    const uint32_t gs = walker && lane < 16 ? 0u : 1u;  // the walker's segment 0 holds the game
    // the segment's policy row for expand: LDS the network rebuilds in every evaluation anyway
    float* const sp = lds + (threadIdx.x >> 4) * 52;
    lat_sync_tree(tl, tg, na, path_lds, false);  // the root (k_tree_reset) and the node count
    __syncthreads();
    bool resident = false;  // the network's head parameters are in LDS (H3sResident)
    uint64_t cyc[5] = {0, 0, 0, 0, 0}, tm0 = 0, tm = 0;  // DBG: backup, select, evaluation, loop, probe call
    auto lap = [&](int k) {
        if constexpr (DBG >= 1) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
            cyc[k] += n - tm;
            tm = n;
        }
    };
    if constexpr (DBG >= 1) tm0 = tm = __builtin_amdgcn_s_memtime();
    const uint64_t dl = deadline ? *deadline : 0;  // Q7 (null: no budget, exactly `sims` simulations)
    int ran = sims;
    for (int s = 0; s < sims; ++s) {
        if (!hash_eval && !resident) {  // at the start, and after an fp16-range recompute used the whole LDS
            const float* ph0 = blob + nn::kL1B + nn::kCh + nn::kL1Table + (size_t)blocks * 2 * (h3::kW + 2 * nn::kCh);
            float4* hd = reinterpret_cast<float4*>(lb + h3s::kHeadOff);
            for (int k = (int)threadIdx.x; k < h3s::kHeadF / 4; k += kLatThreads)
                hd[k] = reinterpret_cast<const float4*>(ph0)[k];
            __syncthreads();
            resident = true;
        }
        if (walker) {
            lap(2);
            if (s > 0) lat_backup(tl, rg, ag, pol, pol + 50, gs, sp, na);  // simulation s - 1's
            lap(0);
            lat_select_wide<DBG>(tl, prm, na);
            lap(1);
            if constexpr (DBG == 2) {  // the cost of a call alone: same arguments, no work (timed into slot 4)
                lat_probe(tl, rg, ag, prm, gs, na);
                lap(4);
            }
        }
        __syncthreads();  // the leaf position of simulation s is in LDS
        if (hash_eval) {
            if (threadIdx.x < 64) {
                const oaz_state st = *tl.leaf_state;
                const uint64_t h = hash_state(st);
                if (lane < 50) pol[lane] = hash_policy(h, lane);
                if (lane == 0) pol[50] = hash_value(h);
            }
        } else {
            int opaque;  // 0, opaque to the compiler: no lane offset of the body is hoisted out of this loop
            asm volatile("v_mov_b32 %0, 0" : "=v"(opaque));
            // row 0 of (pol, pol + 50): the heads write the evaluation to LDS, where the backup reads it
            const bool ovf = nn_h3s_body<C>(t.leaf_state, 0, blob, blocks, pol, pol + 50, lds, opaque,
                                            H3sResident{tl.leaf_state, nullptr, true});
            if (__syncthreads_or(ovf)) {  // k_nn_h3s's recompute of this position (the k_nn_x6 body), which
                                          // needs the whole LDS: the tree state goes out and comes back
                flush_stats();
                lat_sync_tree(tl, tg, na, path_lds, true);
                __syncthreads();
                using X = typename H3Fallback<C>::X;
                const TileSpan span{(int)g, (int)g + 1, (int)t.G};
                if ((threadIdx.x >> 8) == 0)
                    nn_h3_fallback<X, X::GRP0>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                else
                    nn_h3_fallback<X, X::GRP1>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                if (threadIdx.x == 0) atomicAdd(fallback, 1ull);
                __syncthreads();
                lat_sync_tree(tl, tg, na, path_lds, false);
                fill_resident();
                if (threadIdx.x < 51) pol[threadIdx.x] = threadIdx.x < 50 ? policy[(size_t)g * 50 + threadIdx.x] : value[g];
                resident = false;
            }
        }
        // policy / value row g written; the network's LDS is free for the tree again. With a budget, thread 0's
        // clock read decides for the workgroup whether simulation s + 1 runs (its backup of s follows the loop)
        if (deadline) {
            if (__syncthreads_or(threadIdx.x == 0 && (uint64_t)wall_clock64() >= dl) && s + 1 < sims) {
                ran = s + 1;
                break;
            }
        } else {
            __syncthreads();
        }
    }
    if (walker) {
        lap(2);
        lat_backup(tl, rg, ag, pol, pol + 50, gs, sp, na);  // the last simulation's
        lap(0);
        if constexpr (DBG >= 1) {
            cyc[3] = tm - tm0;
            if (lane == 0) {
                uint64_t* st = tg.stats;
                atomicAdd((unsigned long long*)&st[GS_CUT], (unsigned long long)cyc[0]);
                atomicAdd((unsigned long long*)&st[GS_RED], (unsigned long long)cyc[1]);
                atomicAdd((unsigned long long*)&st[GS_BLUE], (unsigned long long)cyc[2]);
                atomicAdd((unsigned long long*)&st[GS_PASSES], (unsigned long long)cyc[3]);
                atomicAdd((unsigned long long*)&st[GS_DROPPED], (unsigned long long)cyc[4]);
            }
        }
    }
    __syncthreads();
    lat_sync_tree(tl, tg, na, path_lds, true);  // the tree's top and the node count to global memory
    flush_stats();
    if (deadline && threadIdx.x == 0) sims_run[g] = (uint32_t)ran;
}

// ---- one launch per noise chunk for up to 16 x CU-count games (k_search_grp) ---------------------------
// The per-step loop's trouble at a few thousand games (BASELINE C2: 4 096) is that a simulation step is
// one round of 16-position NN workgroups that does not fill the CUs (two game parts on two streams
// half-fill them each), and every step waits for the slowest game's tree walk across the grid. Here a
// workgroup owns 16 games for a chunk of simulations: waves 0-3 walk the 16 trees (one 16-lane segment
// per game, the segmented kernels' bodies), then all 8 waves evaluate the 16 leaves with k_nn_h3's body
// (16-position square-major tile, its fp16-range recompute), then the backups; no grid-wide step, no
// launch per simulation. Root noise comes from the same ring k_root_noise fills per chunk of
// simulations on the second stream. Results are bit-identical to the per-step launches.
__device__ __noinline__ void grp_backup(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                        const float* policy, const float* value, uint32_t gs, float* sp) {
    expand_backup_seg_body(t, roots, active, policy, value, gs, sp, NodesGlobalRegs{});
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __noinline__ void grp_select(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                        const noise_t* noise, const SearchParams& prm, uint32_t gs) {
    select_seg_body(t, roots, active, noise, prm, gs, nullptr, NodesGlobalRegs{});
}

// DBG 1 (diagnostic, A/B build only: OAZ_GRP_DBG=1): thread 0's s_memtime cycles in the backups (wave 0's
// four games), the selects, the barrier after them (the other walker waves' walks), and the evaluation with
// its barriers, added to game b0's statistics slots GS_CUT / GS_RED / GS_MOVES / GS_BLUE (the whole loop to
// GS_PASSES); the search's results are unchanged.
template <class C, int DBG = 0>
__global__ void __launch_bounds__(kLatThreads) k_search_grp(TreeView t, const oaz_state* __restrict__ roots,
                                                            const uint8_t* __restrict__ active, SearchParams prm,
                                                            int s0, int s1, const noise_t* __restrict__ noise,
                                                            int hash_eval, const float* __restrict__ blob, int blocks,
                                                            const float* __restrict__ xblob,
                                                            unsigned long long* __restrict__ fallback, float* policy,
                                                            float* value, const uint64_t* __restrict__ deadline,
                                                            uint32_t* __restrict__ sims_run) {
    __shared__ __attribute__((aligned(16))) float lds[H3Fallback<C>::kLds];
    const int b0 = (int)blockIdx.x * nn::kSB;
    // Q7: a group that stopped in an earlier chunk stays stopped (its count is below this chunk's start; the
    // count is the same for the group's 16 games). Stopping before simulation s leaves s - 1's expand / back up
    // pending, which the caller's final launch_expand_backup runs as after an unbudgeted search.
    const uint64_t dl = deadline ? *deadline : 0;
    if (deadline && s0 > 0 && sims_run[b0] < (uint32_t)s0) return;  // uniform over the workgroup
    int s = s0;
    const int tid = (int)threadIdx.x, wave = tid >> 6;
    const bool walker = wave < 4;  // waves 0-3: four games each (segments)
    const uint32_t gs = walker ? (uint32_t)b0 + (uint32_t)(wave * 4 + ((tid >> 4) & 3)) : t.G;  // >= G: idle
    float* const sp = lds + (tid >> 4) * 52;  // the segment's policy row (the network's LDS, free meanwhile)
    const TileSpan span{b0, b0 + nn::kSB < (int)t.G ? b0 + nn::kSB : (int)t.G, (int)t.G};
    uint64_t cyc[5] = {0, 0, 0, 0, 0}, tm = 0, tm0 = 0;  // DBG: backup, select, walk barrier, evaluation, loop
    auto lap = [&](int k) {
        if constexpr (DBG >= 1) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
            cyc[k] += n - tm;
            tm = n;
        }
    };
    if constexpr (DBG >= 1) tm0 = tm = __builtin_amdgcn_s_memtime();
    for (; s < s1; ++s) {
        if (deadline && s > 0 && __syncthreads_or(tid == 0 && (uint64_t)wall_clock64() >= dl)) break;
        if (walker) {
            lap(3);
            if (s > 0) grp_backup(t, roots, active, policy, value, gs, sp);  // simulation s - 1's expand / back up
            lap(0);
            grp_select(t, roots, active, noise ? noise + (size_t)(s - s0) * t.G * kNoiseStride : nullptr, prm, gs);
            lap(1);
        }
        __syncthreads();  // the 16 leaf positions of simulation s
        lap(2);
        if (hash_eval) {
            for (int k = tid; k < nn::kSB * 50; k += kLatThreads) {
                const int gi = b0 + k / 50, e = k % 50;
                if (gi < (int)t.G) {
                    const uint64_t h = hash_state(load_state(&t.leaf_state[gi]));
                    policy[(size_t)gi * 50 + e] = hash_policy(h, e);
                    if (e == 0) value[gi] = hash_value(h);
                }
            }
        } else {
            int opaque;  // 0, opaque to the compiler: no lane offset of the body is hoisted out of this loop
            asm volatile("v_mov_b32 %0, 0" : "=v"(opaque));
            bool ovf;
            if ((tid >> 8) == 0) {
                __builtin_amdgcn_s_setprio(1);
                ovf = nn_h3_body<C, C::GRP0>(t.leaf_state, span, blob, blocks, policy, value, lds, opaque);
            } else {
                ovf = nn_h3_body<C, C::GRP1>(t.leaf_state, span, blob, blocks, policy, value, lds, opaque);
            }
            if constexpr (H3Fallback<C>::kOn) {
                using X = typename H3Fallback<C>::X;
                if (__syncthreads_or(ovf)) {
                    if ((tid >> 8) == 0)
                        nn_h3_fallback<X, X::GRP0>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                    else
                        nn_h3_fallback<X, X::GRP1>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                    if (tid == 0) atomicAdd(fallback, 1ull);
                }
            }
        }
        __syncthreads();  // policy / value rows written; the LDS is the tree's again
    }
    if constexpr (DBG >= 1) {
        lap(3);
        if (tid == 0 && b0 < (int)t.G) {
            uint64_t* st = t.stats + (size_t)b0 * GS_COUNT;
            atomicAdd((unsigned long long*)&st[GS_CUT], (unsigned long long)cyc[0]);
            atomicAdd((unsigned long long*)&st[GS_RED], (unsigned long long)cyc[1]);
            atomicAdd((unsigned long long*)&st[GS_MOVES], (unsigned long long)cyc[2]);
            atomicAdd((unsigned long long*)&st[GS_BLUE], (unsigned long long)cyc[3]);
            atomicAdd((unsigned long long*)&st[GS_PASSES], (unsigned long long)(tm - tm0));
        }
    }
    if (deadline && tid < nn::kSB && b0 + tid < (int)t.G) sims_run[b0 + tid] = (uint32_t)s;  // simulations run
}

hipError_t launch_search_grp(const TreeView& t, const oaz_state* roots, const uint8_t* active, SearchParams p, int s0,
                             int s1, const noise_t* noise, const NNView* w, float* policy, float* value,
                             const uint64_t* deadline, uint32_t* sims_run, hipStream_t st) {
    if (deadline && !sims_run) return hipErrorInvalidValue;
    if (t.G == 0 || s1 <= s0) return hipSuccess;
    if (w && (!w->fallback || !w->blob_x6 || w->precision != OAZ_FP32_SPLIT16)) return hipErrorInvalidValue;
    const unsigned grid = (t.G + nn::kSB - 1) / nn::kSB;
#if OAZ_AB
    static const int dbg = getenv("OAZ_GRP_DBG") ? atoi(getenv("OAZ_GRP_DBG")) : 0;
    if (dbg == 1) {
        hipLaunchKernelGGL((k_search_grp<H3Cfg<0>, 1>), dim3(grid), dim3(kLatThreads), 0, st, t, roots, active, p, s0, s1,
                           noise, w ? 0 : 1, w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                           w ? w->fallback : nullptr, policy, value, deadline, sims_run);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(k_search_grp<H3Cfg<0>>, dim3(grid), dim3(kLatThreads), 0, st, t, roots, active, p, s0, s1, noise,
                       w ? 0 : 1, w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                       w ? w->fallback : nullptr, policy, value, deadline, sims_run);
    return hipGetLastError();
}

hipError_t launch_search_lat(const TreeView& t, const oaz_state* roots, const uint8_t* active, SearchParams p,
                             int sims, const NNView* w, float* policy, float* value, const uint64_t* deadline,
                             uint32_t* sims_run, hipStream_t st) {
    if (deadline && !sims_run) return hipErrorInvalidValue;
    if (t.G == 0 || sims <= 0) return hipSuccess;
    if (w && (!w->fallback || !w->blob_x6 || w->precision != OAZ_FP32_SPLIT16)) return hipErrorInvalidValue;
#if OAZ_AB
    static const int dbg = getenv("OAZ_LAT_DBG") ? atoi(getenv("OAZ_LAT_DBG")) : 0;
    if (dbg == 2) {
        hipLaunchKernelGGL(k_search_lat<2>, dim3(t.G), dim3(kLatThreads), 0, st, t, roots, active, p, sims, w ? 0 : 1,
                           w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                           w ? w->fallback : nullptr, policy, value, deadline, sims_run);
        return hipGetLastError();
    }
    if (dbg == 1) {
        hipLaunchKernelGGL(k_search_lat<1>, dim3(t.G), dim3(kLatThreads), 0, st, t, roots, active, p, sims, w ? 0 : 1,
                           w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                           w ? w->fallback : nullptr, policy, value, deadline, sims_run);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(k_search_lat<0>, dim3(t.G), dim3(kLatThreads), 0, st, t, roots, active, p, sims, w ? 0 : 1,
                       w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                       w ? w->fallback : nullptr, policy, value, deadline, sims_run);
    return hipGetLastError();
}

}  // namespace oaz
