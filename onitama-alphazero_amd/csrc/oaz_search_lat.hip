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
// Agent / arena config, train = false), no search-time budget and no leaf compaction
// (oaz_engine.cpp run_sims; oaz_config.step_kernels = 1 turns it off).
namespace oaz {

constexpr int kLatThreads = 512;  // 8 waves: k_nn_h3s's geometry; wave 4 also walks the tree

// The tree walk (wave 4 only) as calls of their own: the walk needs ~80 VGPRs, the network ~240 (the
// compute waves hold a conv's weights), and inlined into one loop the two allocations spill; a call
// per simulation costs a few register saves.
__device__ __noinline__ void lat_backup(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                        const float* policy, const float* value, uint32_t gs, float* sp) {
    expand_backup_seg_body(t, roots, active, policy, value, gs, sp);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __noinline__ void lat_select(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                        const SearchParams& prm, uint32_t gs, oaz_state* leaf_lds) {
    select_seg_body(t, roots, active, nullptr, prm, gs, leaf_lds);
}

__global__ void __launch_bounds__(kLatThreads) k_search_lat(TreeView t, const oaz_state* __restrict__ roots,
                                                            const uint8_t* __restrict__ active, SearchParams prm,
                                                            int sims, int hash_eval, const float* __restrict__ blob,
                                                            int blocks, const float* __restrict__ xblob,
                                                            unsigned long long* __restrict__ fallback, float* policy,
                                                            float* value) {
    using C = H3Cfg<0>;
    __shared__ __attribute__((aligned(16))) float lds[H3Fallback<C>::kLds];
    const uint32_t g = blockIdx.x;
    if (g >= t.G || (active && active[g] != 1)) return;  // uniform over the workgroup
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const bool walker = wave == 4;
    const uint32_t gs = walker && lane < 16 ? g : t.G;  // segments 1-3 of wave 4 idle (game >= G)
    // the segment's policy row for expand: LDS the network rebuilds in every evaluation anyway
    float* const sp = lds + (threadIdx.x >> 4) * 52;
    char* const lb = reinterpret_cast<char*>(lds);
    static_assert(h3s::kResidentBytes <= H3Fallback<C>::kLds * 4, "k_search_lat LDS");
    oaz_state* const leaf_lds = reinterpret_cast<oaz_state*>(lb + h3s::kStateOff);
    bool resident = false;  // the network's resident operands are in LDS (H3sResident)
    for (int s = 0; s < sims; ++s) {
        if (!hash_eval && !resident) {  // at the start, and after an fp16-range recompute used the whole LDS
            h3s_load_resident(lb, blob, blocks);
            resident = true;
        }
        if (walker) {
            if (s > 0) lat_backup(t, roots, active, policy, value, gs, sp);  // simulation s - 1's expand / back up
            lat_select(t, roots, active, prm, gs, leaf_lds);
        }
        __syncthreads();  // the leaf position of simulation s is in t.leaf_state[g] and in LDS
        if (hash_eval) {
            if (threadIdx.x < 64) {
                const oaz_state st = load_state(&t.leaf_state[g]);
                const uint64_t h = hash_state(st);
                if (lane < 50) policy[(size_t)g * 50 + lane] = hash_policy(h, lane);
                if (lane == 0) value[g] = hash_value(h);
            }
        } else {
            int opaque;  // 0, opaque to the compiler: no lane offset of the body is hoisted out of this loop
            asm volatile("v_mov_b32 %0, 0" : "=v"(opaque));
            const bool ovf = nn_h3s_body<C>(t.leaf_state, (int)g, blob, blocks, policy, value, lds, opaque,
                                            H3sResident{leaf_lds, lb + h3s::kL1Off, true});
            if (__syncthreads_or(ovf)) {  // k_nn_h3s's recompute of this position (the k_nn_x6 body)
                resident = false;
                using X = typename H3Fallback<C>::X;
                const TileSpan span{(int)g, (int)g + 1, (int)t.G};
                if ((threadIdx.x >> 8) == 0)
                    nn_h3_fallback<X, X::GRP0>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                else
                    nn_h3_fallback<X, X::GRP1>(t.leaf_state, span, xblob, blocks, policy, value, lds);
                if (threadIdx.x == 0) atomicAdd(fallback, 1ull);
            }
        }
        __syncthreads();  // policy / value row g written; the network's LDS is free for the tree again
    }
    if (walker) lat_backup(t, roots, active, policy, value, gs, sp);  // the last simulation's
}

hipError_t launch_search_lat(const TreeView& t, const oaz_state* roots, const uint8_t* active, SearchParams p,
                             int sims, const NNView* w, float* policy, float* value, hipStream_t st) {
    if (t.G == 0 || sims <= 0) return hipSuccess;
    if (w && (!w->fallback || !w->blob_x6 || w->precision != OAZ_FP32_SPLIT16)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_search_lat, dim3(t.G), dim3(kLatThreads), 0, st, t, roots, active, p, sims, w ? 0 : 1,
                       w ? w->blob : nullptr, w ? w->blocks : 0, w ? w->blob_x6 : nullptr,
                       w ? w->fallback : nullptr, policy, value);
    return hipGetLastError();
}

}  // namespace oaz
