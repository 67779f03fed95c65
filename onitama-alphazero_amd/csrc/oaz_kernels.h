// oaz_kernels.h — launchers for the gfx950 kernels (defined in oaz_kernels.hip / oaz_nn.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/onitama_az.h"
#include "oaz_device.h"  // noise_t

namespace oaz {

// Per-game statistics slots (summed on demand): see oaz_search_stats / oaz_selfplay_stats.
enum GameStat {
    GS_SIMS = 0,
    GS_EXPANSIONS,
    GS_CHILDREN,
    GS_TERMINAL,
    GS_DEPTH,
    GS_STUCK,
    GS_MAXNODES,
    GS_MOVES,
    GS_FINISHED,
    GS_CUT,
    GS_RED,
    GS_BLUE,
    GS_PASSES,
    GS_DROPPED,
    GS_EVALS,  // leaves whose evaluation the playout uses (oaz_search_stats.nn_evals)
    GS_COUNT = 16
};

// Device view of the search trees of G games (one region of `cap` nodes per game).
struct TreeView {
    oaz_node* nodes;        // [G][cap]
    uint32_t* n_nodes;      // [G]
    uint32_t* path;         // [G][pathcap] node ids root..leaf of the current playout
    uint32_t* depth;        // [G]
    uint32_t* leaf;         // [G] leaf node id
    oaz_state* leaf_state;  // [G] position at the leaf (to_move = leaf colour)
    uint64_t* stats;        // [G][GS_COUNT]
    const double* sqrt_tab; // [sims+1] correctly rounded sqrt(n) (host libm)
    // leaf compaction (null need: none, the evaluator reads leaf_state[g] and writes row g)
    uint8_t* need;          // [G] 1 = the playout uses the leaf's evaluation (written by select)
    uint32_t* slot;         // [G] row of game g's evaluation in the compacted policy / value
    oaz_state* cstate;      // [G + 16] compacted leaf positions (bucket b's at b * kBucket ..)
    uint32_t* bcnt;         // [nb] positions per bucket
    uint32_t cap;
    uint32_t pathcap;
    uint32_t G;
};

struct SearchParams {
    double c_puct;
    double alpha;
    double eps;
    uint64_t seed;
    int32_t train_noise;
};

// Self-play slot state (continuous batching).
struct SlotView {
    oaz_state* root;      // [G] current position of the game in the slot
    uint32_t* ply;        // [G]
    uint32_t* seq;        // [G] games started in this slot
    uint64_t* game_id;    // [G] global game id (deal + noise key)
    uint8_t* active;      // [G] 1 = playing, 0 = done (quota), k > 1 = starts in k-1 plies
    oaz_sample* hist;     // [G][hcap] samples of the running game (z filled at the end)
    oaz_sample* out;      // [out_cap] finished samples
    unsigned long long* out_count;  // appended samples (may exceed out_cap: dropped)
    uint32_t* fin;        // [G] records of the game that ended in the slot this ply | result << 24 (0: none)
    uint64_t* fin_pos;    // [G] their first position in out (k_samples_scan)
    uint32_t hcap;
    uint32_t out_cap;
    int32_t max_plies;
    int32_t fixed_deck;
    uint8_t deck[5];
    uint64_t seed;
    uint32_t G;            // slots of this engine
    uint32_t world;        // ranks (oaz_config.world, >= 1)
    uint32_t rank;         // this engine's rank (slot_game_id, oaz_device.h)
    uint64_t quota;        // stop starting games at this global index (0 = unlimited)
    uint32_t stagger;      // slot g waits g % stagger plies before its first game (0: none)
};

// Evaluator tiles over the compacted leaves: bucket b (games [b * kBucket, (b + 1) * kBucket)) holds
// its bcnt[b] positions at rows b * kBucket ..; workgroup i takes tile i / nb of bucket i % nb, so the
// buckets' full tiles come first and the empty tail workgroups exit after their first loads.
constexpr int kBucketShift = 12;
constexpr uint32_t kBucket = 1u << kBucketShift;
struct TileMap {
    const uint32_t* bcnt;  // null: plain tiles over rows [0, B)
    int32_t nb;            // buckets
    int32_t cap;           // readable rows (loads are clamped to it, stores are guarded by the count)
};
inline int32_t buckets_of(uint32_t G) { return (int32_t)((G + kBucket - 1) >> kBucketShift); }

struct NNView {
    const float* blob;  // packed, BN-folded weights (DESIGN.md "NN weights layout")
    int32_t blocks;
    int32_t precision;  // OAZ_FP32 (exact fp32 MFMA), OAZ_BF16 (bf16 inputs), OAZ_FP32_SPLIT (bf16x6 split),
                        // OAZ_FP32_SPLIT16 (fp16x3 split)
    int32_t x6_variant; // A/B build only (OAZ_NN_X6_V): a diagnostic build of k_nn_h3 (timing only)
    const float* blob_x6;             // OAZ_FP32_SPLIT16: the OAZ_FP32_SPLIT blob of the same weights
    unsigned long long* fallback;     // OAZ_FP32_SPLIT16: tiles recomputed by the k_nn_x6 body (fp16 range)
    TileMap tm;                       // compacted leaves (tm.bcnt null: rows [0, B))
    int32_t small_max;                // OAZ_FP32_SPLIT16: launches of <= this many positions run k_nn_h3s
};

// rules
hipError_t launch_movegen(const oaz_state* s, int n, uint32_t* masks, oaz_move* moves,
                          uint8_t* counts, hipStream_t st);
hipError_t launch_step(oaz_state* s, const oaz_move* mv, int n, uint8_t* results, hipStream_t st);
hipError_t launch_current_state(const oaz_state* s, int n, uint8_t* results, hipStream_t st);
hipError_t launch_encode(const oaz_state* s, int n, float* planes, hipStream_t st);

// evaluators
hipError_t launch_nn_forward(const NNView& w, const oaz_state* s, int B, float* policy,
                             float* value, hipStream_t st);
hipError_t launch_hash_eval(const oaz_state* s, int B, float* policy, float* value, hipStream_t st);
// gather the leaves the playouts use (t.need) into t.cstate / t.slot / t.bcnt, bucket by bucket
hipError_t launch_eval_compact(const TreeView& t, hipStream_t st);
size_t nn_packed_floats(int blocks, int precision);

// MCTS
hipError_t launch_tree_reset(const TreeView& t, hipStream_t st);
constexpr int kNoiseStride = 2 * OAZ_MAX_MOVES;  // noise_t draws per (sim, game) in the noise ring
hipError_t launch_select(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                         const noise_t* noise /* [G][kNoiseStride] or null */, SearchParams p, hipStream_t st);
hipError_t launch_root_noise(const oaz_state* roots, const uint8_t* active, const uint64_t* game_id,
                             const uint32_t* ply, SearchParams p, uint32_t G, uint32_t sim0, uint32_t nsims,
                             noise_t* out /* [nsims][G][kNoiseStride] */, hipStream_t st);
hipError_t launch_expand_backup(const TreeView& t, const oaz_state* roots, const uint8_t* active,
                                const float* policy, const float* value, hipStream_t st);
// expand/backup of simulation s, then select of simulation s+1 (noise: its root noise), fused
hipError_t launch_backup_select(const TreeView& t, const oaz_state* roots, const uint8_t* active, const float* policy,
                                const float* value, const noise_t* noise, SearchParams p, hipStream_t st);
hipError_t launch_search_finalize(const TreeView& t, const oaz_state* roots, oaz_move* out_move,
                                  float* out_pi, hipStream_t st);
// false when OAZ_TREE_SEG=0 selected the one-game-per-wave tree kernels
bool tree_seg_kernels();
// All `sims` simulations of every game in one launch, one workgroup per game (oaz_search_lat.hip):
// w = the fp16x3 network, or null for the HASH test evaluator; no root noise; rows = game ids.
// deadline / sims_run (Q7 search_time, both null without a budget): each workgroup stops before a simulation
// s >= 1 at which the device clock is at or past *deadline; sims_run[g] = the simulations game g ran.
hipError_t launch_search_lat(const TreeView& t, const oaz_state* roots, const uint8_t* active, SearchParams p,
                             int sims, const NNView* w, float* policy, float* value, const uint64_t* deadline,
                             uint32_t* sims_run, hipStream_t st);
// Simulations [s0, s1) of every game, 16 games per workgroup, in one launch (oaz_search_lat.hip): noise =
// the ring chunk holding simulation s0's draws ([s1 - s0][G][kNoiseStride]) or null; w as above. The
// last simulation's expand / backup is the caller's (launch_expand_backup). deadline / sims_run as above, per
// 16-game group; a group that stopped in an earlier chunk exits at once (sims_run must start at 0).
hipError_t launch_search_grp(const TreeView& t, const oaz_state* roots, const uint8_t* active, SearchParams p, int s0,
                             int s1, const noise_t* noise, const NNView* w, float* policy, float* value,
                             const uint64_t* deadline, uint32_t* sims_run, hipStream_t st);
// *deadline = the device clock (wall_clock64, hipDeviceAttributeWallClockRate) when the kernel runs + ticks
hipError_t launch_deadline_start(uint64_t* deadline, uint64_t ticks, hipStream_t st);
hipError_t launch_selfplay_move(const TreeView& t, const SlotView& s, hipStream_t st);
hipError_t launch_selfplay_reset(const TreeView& t, const SlotView& s, hipStream_t st);
hipError_t launch_stats_reduce(const uint64_t* per_game, uint32_t G, uint64_t* out /* GS_COUNT */,
                               hipStream_t st);

}  // namespace oaz
