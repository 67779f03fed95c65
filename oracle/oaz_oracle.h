/*
 * oaz_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path (cyoq/onitama-alphazero), written in plain C
 * from the Rust sources, function by function (each definition in oaz_oracle.c cites the
 * reference file:line it follows). It is the checker for the HIP engine: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product library
 * (libonitama_az.so) never links or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - rules: the reference's own unit tests (onitama-game/src/game/state.rs:381-890,
 *     common/mod.rs:77-135) and the expansion-order fixtures of
 *     onitama-game/src/ai/mcts/mcts_arena.rs:403-457, committed under tests/golden/;
 *   - NN: goldens produced by torch 2.10 CPU (F.conv2d/batch_norm/linear/softmax/tanh,
 *     the op graph of net.rs) on the reference's trained 3-block weights
 *     (models/model_5e-3_3_resnet.ot) — libtorch 2.10, not the reference's tch 0.10.3 /
 *     libtorch 1.13.1, so NN parity is pinned to torch's arithmetic within 1e-4;
 *   - MCTS/self-play: no reference test pins them (alphazero-training has no tests);
 *     the restatement follows mcts_arena.rs line by line and is cross-checked against
 *     a second, independent Python restatement in tests/ (parity of the search itself is
 *     therefore "restatement-pinned", not reference-pinned).
 */
#ifndef OAZ_ORACLE_H
#define OAZ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/onitama_az.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rules */
void orc_attack_maps(uint32_t out[2 * 16 * 25]);
uint32_t orc_card_positions(int card);
uint32_t orc_card_mirror(int card);
int orc_card_color(int card);
void orc_initial_state(const uint8_t deck[5], oaz_state* out);
int orc_movegen(const oaz_state* s, int color, oaz_move* out /* >= 40 */);
void orc_movegen_masks(const oaz_state* s, int color, uint32_t masks[2 * 25]);
int orc_make_move(oaz_state* s, const oaz_move* mv, int color);
int orc_current_state(const oaz_state* s);
int orc_is_terminal(const oaz_state* s);
void orc_encode(const oaz_state* s, int color, float planes[21 * 25]);

/* counter-based RNG + deals (shared spec with the engine, DESIGN.md "RNG") */
void orc_philox(uint64_t key, const uint32_t ctr[4], uint32_t out[4]);
void orc_deal_deck(uint64_t seed, uint64_t game_id, uint8_t out[5]);
void orc_hash_eval(const oaz_state* s, float policy[50], float* value);
/* root-noise draw (see oaz_oracle.c beta_noise): c2 = ply << 16 | sim */
double orc_root_noise(uint64_t seed, uint64_t game_id, uint32_t c2, uint32_t draw, double alpha, int nchild);

/* NN: raw (un-folded) weights in canonical order, fp32 */
size_t orc_weight_count(int blocks);
int orc_nn_forward(const float* weights, int blocks, const oaz_state* s, int B, float* policy,
                   float* value);

/* MCTS */
typedef void (*orc_eval_fn)(void* ctx, const oaz_state* s, float policy[50], float* value);

typedef struct orc_search_cfg {
    int sims;
    double c_puct;
    int train_noise;
    double alpha, eps;
    uint64_t seed;     /* noise RNG key */
    uint64_t game_id;  /* noise RNG counter words */
    uint32_t ply;
    int evaluator;     /* OAZ_EVAL_NN, OAZ_EVAL_HASH, or 2 = callback */
    const float* weights;
    int blocks;
    orc_eval_fn fn;
    void* ctx;
} orc_search_cfg;

/* Runs one search from `root` (colour root->to_move). Returns 0 / <0. out_nodes (optional)
 * receives the tree in arena order (cap nodes). */
int orc_search(const orc_search_cfg* cfg, const oaz_state* root, oaz_move* out_move,
               float out_pi[50], oaz_node* out_nodes, int cap, int* n_nodes,
               oaz_search_stats* stats);

/* n independent searches on `threads` host threads; root i uses game_id = game_ids[i], or
 * cfg->game_id + i when game_ids is NULL (the GPU's search mode keys root i's noise by batch index
 * i). out_move[n], out_pi[n*50]; stats summed (max_nodes: maximum). The evaluator must be
 * thread-safe (HASH or NN; not a Python callback). */
int orc_search_batch(const orc_search_cfg* cfg, const oaz_state* roots, const uint64_t* game_ids, int n, int threads,
                     oaz_move* out_move, float* out_pi, oaz_search_stats* stats);

typedef struct orc_selfplay_cfg {
    orc_search_cfg search;
    int max_plies;
    int fixed_deck;
    uint8_t deck[5];
} orc_selfplay_cfg;

/* One self_play game (train.rs:35-98) for global game id `game_id`. Returns #samples
 * written (<= cap) or <0. *result = final MoveResult, *plies = plies played. */
int orc_selfplay_game(const orc_selfplay_cfg* cfg, uint64_t game_id, oaz_sample* out, int cap,
                      int* result, int* plies, oaz_search_stats* stats);

/* CPU baseline: `threads` workers, each playing self-play games (one game per worker at a
 * time, like train.rs:218-245) until `seconds` elapse; returns simulations done. */
int64_t orc_selfplay_bench(const orc_selfplay_cfg* cfg, int threads, double seconds,
                           int64_t* games_done, int64_t* plies_done);

/* Pure MCTS agent (onitama-game/src/ai/mcts/mcts_arena.rs): one search from `root`.
 * Tree nodes use the ABI's oaz_pure_node layout so tests can compare them byte for byte.
 * Rollout draws: Philox(seed; game_id, playout, 0x9C7A0000, d/4) word d%4, uniform int
 * (u32 * n) >> 32 — the stream the GPU uses. Returns the node count or <0. */
int orc_pure_mcts(const oaz_pure_mcts_config* cfg, uint64_t game_id, const oaz_state* root, oaz_move* out_move,
                  float* out_value, oaz_pure_node* nodes, int cap, oaz_pure_mcts_stats* stats);
int64_t orc_pure_mcts_bench(const oaz_pure_mcts_config* cfg, int threads, double seconds, int64_t* searches);

#ifdef __cplusplus
}
#endif
#endif
