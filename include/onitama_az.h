/*
 * onitama_az.h — C ABI of the MI355X-native Onitama AlphaZero self-play engine.
 *
 * This is the drop-in boundary for the reference's hot path (cyoq/onitama-alphazero):
 * batched 5x5-bitboard move generation / state stepping (onitama-game) plus
 * leaf-evaluated AlphaZero MCTS (select/expand/backup) and the ResNet policy-value
 * evaluation (alphazero-training). The reference is Rust calling libtorch through
 * tch-rs; a Rust host binds this header with one `extern "C"` block
 * and tch is no longer needed on the path.
 *
 * Conventions
 *   - Plain C, POD structs, caller-owned buffers, no torch types.
 *   - Every function returning int: 0 = OK, < 0 = error; the message is then in
 *     oaz_last_error() (thread-local). Nothing throws or aborts across the ABI:
 *     the reference's panics (e.g. "Must find the best child",
 *     alphazero-training/src/alphazero_mcts/mcts_arena.rs:94,220) become defined
 *     behaviour or an error code.
 *   - An engine is owned by one host thread and bound to one GPU (one process per
 *     GPU, one engine per process in the self-play bench). Distinct engines are
 *     independent, also when several threads create and drive engines on one GPU at
 *     once (creation zeroes and uploads on the engine's own stream and waits for it).
 *   - Engine, trainer and communicator calls run on their object's device and restore
 *     the calling thread's current HIP device before returning (so do the pure-MCTS
 *     search on cfg->device); the stateless rules entry points (oaz_movegen, oaz_step,
 *     oaz_current_state, oaz_encode) run on the thread's current device.
 *   - Compute entry points need a gfx950 GPU. Without one oaz_create() returns
 *     NULL and the rules entry points return OAZ_ERR_NO_DEVICE; there is no CPU
 *     fallback in this library.
 *
 * Reference interfaces replaced (file:line under the reference root):
 *   oaz_movegen        <- State::generate_all_legal_moves   onitama-game/src/game/state.rs:301-378
 *   oaz_step           <- State::make_move + Deck::rotate    onitama-game/src/game/state.rs:145-202, deck.rs:87-90
 *   oaz_current_state  <- State::current_state               onitama-game/src/game/state.rs:120-134
 *   oaz_encode         <- create_tensor_from_state           alphazero-training/src/common.rs:26-80
 *   oaz_nn_forward     <- ConvResNet::forward(train=false)   alphazero-training/src/net.rs:215-232
 *   oaz_search         <- MctsArena::new + search            alphazero-training/src/alphazero_mcts/mcts_arena.rs:48-124
 *                         (TrainingAlphaZeroMcts::generate_move_tensor, alphazero_mcts/mod.rs:63-78,
 *                          and Agent::generate_move for AlphaZeroMcts, alphazero_mcts/mod.rs:122-144)
 *   oaz_selfplay_*     <- self_play                           alphazero-training/src/train.rs:35-98
 *   oaz_load_weights   <- AlphaZeroMcts::from_model_file      alphazero-training/src/alphazero_mcts/mod.rs:89-105
 *   oaz_pure_mcts_*    <- Mcts agent (random-rollout UCT)     onitama-game/src/ai/mcts/mcts_arena.rs:56-264, mod.rs:37-52
 *   oaz_trainer_*      <- the training loop body               alphazero-training/src/train.rs:264-313
 *                         (ConvResNet::forward(train=true) net.rs:215-232, alphaloss net.rs:234-243,
 *                          nn::Sgd{momentum 0.9} + set_weight_decay train.rs:181-186, opt.backward_step)
 */
#ifndef ONITAMA_AZ_H
#define ONITAMA_AZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OAZ_ABI_VERSION 5

/* ---- enums mirroring the reference --------------------------------------- */
enum { OAZ_RED = 0, OAZ_BLUE = 1 };                 /* PlayerColor, player_color.rs:7-10 */
enum { OAZ_PAWN = 0, OAZ_KING = 1 };                /* PieceKind, piece.rs:5-9 */
enum {                                              /* MoveResult, move_result.rs:4-9 */
    OAZ_CAPTURE = 0,
    OAZ_RED_WIN = 1,
    OAZ_BLUE_WIN = 2,
    OAZ_IN_PROGRESS = 3
};
/* Card ids are indices into ORIGINAL_CARDS (card.rs:465-468):
 * 0 Tiger 1 Dragon 2 Frog 3 Rabbit 4 Crab 5 Elephant 6 Goose 7 Rooster
 * 8 Monkey 9 Mantis 10 Crane 11 Horse 12 Ox 13 Boar 14 Eel 15 Cobra. */
enum { OAZ_NUM_CARDS = 16, OAZ_MAX_MOVES = 40 };    /* 2 cards x 5 pieces x 4 squares */

enum {
    OAZ_OK = 0,
    OAZ_ERR_ARG = -1,
    OAZ_ERR_NO_DEVICE = -2,
    OAZ_ERR_HIP = -3,
    OAZ_ERR_CAPACITY = -4,
    OAZ_ERR_STATE = -5,
    OAZ_ERR_WEIGHTS = -6,
    OAZ_ERR_RANGE = -7,     /* ABI 1 only: ABI 2 recomputes fp16-range tiles instead (oaz_nn_fallbacks) */
    OAZ_ERR_COMM = -8       /* RCCL communicator error (oaz_comm_*, oaz_allgather_samples) */
};

enum { OAZ_EVAL_NN = 0, OAZ_EVAL_HASH = 1 };        /* leaf evaluator (HASH: test evaluator, below) */
/* NN arithmetic. OAZ_FP32: exact fp32 MFMA products (v_mfma_f32_16x16x4_f32). OAZ_BF16: bf16 MFMA
 * inputs, fp32 accumulate (BASELINE C5). OAZ_FP32_SPLIT: fp32 operands split exactly into three
 * bf16 terms (hi + mid + lo), the six products above 2^-24 relative on bf16 MFMA, fp32
 * accumulate: fp32-level error (DESIGN.md "fp32 split") at bf16 MFMA rates. OAZ_FP32_SPLIT16: fp32
 * operands split into two fp16 terms (hi = fp16(x), lo = fp16(x - hi): 22 significant bits), the
 * three products hi*hi, hi*lo, lo*hi on fp16 MFMA, fp32 accumulate; conv weights are pre-scaled per
 * output channel by a power of two (exact). Errors vs a float64 forward are at the fp32 level
 * (DESIGN.md "fp16 split") at half the MFMA work of OAZ_FP32_SPLIT. fp16 terms cover |x| < 65504:
 * a workgroup whose 16 positions split an activation beyond that recomputes them in the same launch
 * with the OAZ_FP32_SPLIT arithmetic (fp32 range), so no result is ever silently wrong and no run
 * fails; oaz_nn_fallbacks() counts the recomputed 16-position tiles. */
enum { OAZ_FP32 = 0, OAZ_BF16 = 1, OAZ_FP32_SPLIT = 2, OAZ_FP32_SPLIT16 = 3 };

/* ---- PODs ----------------------------------------------------------------- */

/* State (state.rs:51-56) plus the side to move (MctsState.player_color, mcts_arena.rs:24-28).
 * Bitboards: square i = row*5+col, (0,0) = a5 top-left, bit for square i is 1u<<(31-i)
 * (common/mod.rs:2-16). cards[] are deck slots R0,R1,B2,B3,N4 (deck.rs:14-18). */
typedef struct oaz_state {
    uint32_t kings[2];
    uint32_t pawns[2];
    uint8_t cards[5];
    uint8_t to_move;
    uint8_t pad[2];
} oaz_state; /* 24 bytes */

/* DoneMove (done_move.rs:3-7): Move{from,to,piece} (move.rs:20-25) + used_card_idx (deck slot). */
typedef struct oaz_move {
    uint8_t from;
    uint8_t to;
    uint8_t piece;
    uint8_t slot;
} oaz_move;

/* One MCTS node as stored on the GPU (MctsNode, mcts_arena.rs:355-373). Children of a node
 * are contiguous: [first, first+nch). Node indices are the reference arena indices
 * (allocation order), so a dump compares index-for-index with the reference tree. */
typedef struct oaz_node {
    double W;        /* reward sum ("reward") */
    double P;        /* prior ("probability") */
    uint32_t N;      /* visits */
    uint32_t first;  /* first child (valid when expanded) */
    uint16_t mv;     /* packed move: from | to<<5 | slot<<10 | piece<<12 */
    uint8_t nch;     /* number of children */
    uint8_t flags;   /* bit0 expanded, bit1 terminal */
    uint32_t pad;
} oaz_node; /* 32 bytes */

/* Self-play training sample (SelfPlayData, train.rs:27-33): encoded compactly; the 21x5x5
 * planes are recoverable with oaz_encode(state). */
typedef struct oaz_sample {
    oaz_state state;  /* position before the move; state.to_move = player_color */
    float pi[50];     /* visit distribution [2][25] (calculate_priors, mcts_arena.rs:104-124) */
    float z;          /* reward(final result, player_color) (train.rs:83-85) */
} oaz_sample; /* 228 bytes */

typedef struct oaz_config {
    int32_t blocks;          /* ConvResNetConfig.resnet_block_amnt (net.rs:74-89) */
    int32_t channels;        /* hidden_channels: 64 (only value supported) */
    int32_t in_planes;       /* input_channels: 21 (only value supported) */
    int32_t sims;            /* AlphaZeroMctsConfig.max_playouts; search_time is not used */
    double c_puct;           /* exploration_c */
    int32_t train_noise;     /* AlphaZeroMctsConfig.train: Dirichlet noise at the root */
    int32_t max_plies;       /* TrainConfig.max_plies (train.rs:52,74-79): 150 => 152 plies */
    double dirichlet_alpha;  /* 0.03 (mcts_arena.rs:187) */
    double dirichlet_eps;    /* 0.25 (mcts_arena.rs:186) */
    int32_t games;           /* parallel game slots G (also the max batch of oaz_search) */
    int32_t evaluator;       /* OAZ_EVAL_NN or OAZ_EVAL_HASH */
    int32_t precision;       /* OAZ_FP32, OAZ_BF16, OAZ_FP32_SPLIT or OAZ_FP32_SPLIT16 (default) */
    int32_t fixed_deck;      /* 1: every game uses deck[]; 0: random 5 of 16 per game (deck.rs:139-151) */
    uint8_t deck[5];
    uint8_t pad0[3];
    uint64_t seed;           /* counter-based RNG key for deals and Dirichlet noise */
    int32_t rank;            /* global game id = (k * world + rank) * games + slot */
    int32_t world;
    int32_t sample_capacity; /* max samples buffered on the device (0: auto) */
    int32_t stagger;         /* self-play: slot g starts playing after g % stagger plies (steady-state
                                game ages for throughput measurement); 0 = all slots start at once */
    int32_t compact;         /* leaf compaction: only the leaves whose evaluation the playout uses go to
                                the evaluator (a won, terminal-flagged leaf's is computed and discarded by
                                the reference, Q2). 0 = off: every playout evaluates its leaf, as the
                                reference (default); 1 = always; 2 = when it saves NN workgroup rounds
                                (games >= 12 * 16 * CUs). Trees, pi and samples are identical either way */
    int32_t parts;           /* the simulation loop runs the games in this many parts (1, 2 or 4), each
                                on its own stream so one part's tree kernels fill the others' NN gaps;
                                0 = auto (2 from 2048 games); results are identical either way */
    int64_t search_time_ns;  /* Q7, AlphaZeroMctsConfig.search_time (mcts_arena.rs:78: playouts run while
                                `playouts < max_playouts && elapsed < search_time`). 0 = off (default, the
                                parity mode: exactly `sims` playouts). > 0: a search (or self-play ply) stops
                                after the first simulation step that ends at or past this wall-clock budget
                                from its start, and pi / the move come from the visits that ran. A search
                                of the one-launch sizes (step_kernels 0: <= CU-count games without root
                                noise, or <= 16 x CU-count games) reads the device clock before every
                                simulation, each game (k_search_grp: each 16-game group) on its own, so the
                                games of a batch may run different counts (>= 1, <= sims;
                                oaz_search_playouts); larger batches stop together after a simulation step */
    int32_t step_kernels;    /* 0 = auto: a search of at most CU-count games with the fp16x3 network (or
                                HASH), no root noise and no leaf compaction runs as ONE
                                launch, a workgroup per game doing all its simulations (the Agent API's
                                one-position latency path); 1 = always the per-simulation-step launches.
                                Trees, pi and samples are identical either way */
    int32_t reserved;
} oaz_config;

typedef struct oaz_search_stats {
    uint64_t sims;            /* simulations run (= NN leaf evaluations, Q2) */
    uint64_t expansions;      /* leaves actually expanded (non-terminal, first visit) */
    uint64_t children;        /* children created */
    uint64_t terminal_leaves; /* playouts that ended on a won position */
    uint64_t depth_sum;       /* sum of select path depths */
    uint64_t stuck_leaves;    /* expanded nodes with no legal move (reference panics, Q6) */
    uint64_t max_nodes;       /* largest tree seen */
    uint64_t nn_evals;        /* leaf evaluations whose policy or value the playout uses: every
                               * playout except those ending on a won, already terminal-flagged
                               * node, whose evaluation the reference computes and then discards
                               * (mcts_arena.rs:156-176); only these are sent to the network */
} oaz_search_stats;

typedef struct oaz_selfplay_stats {
    uint64_t moves;           /* plies played over all slots */
    uint64_t games_finished;
    uint64_t games_cut;       /* finished by the ply cap (z = 0) */
    uint64_t red_wins, blue_wins;
    uint64_t samples_ready;   /* samples buffered on the device */
    uint64_t samples_dropped; /* overflowed the device buffer */
    uint64_t passes;          /* root positions with no legal move: pass (Q6) */
    oaz_search_stats search;
} oaz_selfplay_stats;

typedef struct oaz_kernel_times {
    /* accumulated HIP-event time (ms) and launches per kernel class; enabled with
     * oaz_set_timing(eng, 1) */
    double select_ms, nn_ms, expand_ms, finalize_ms;
    uint64_t select_n, nn_n, expand_n, finalize_n;
    uint64_t nn_samples;  /* positions of the timed nn launches outside the simulation loop (oaz_nn_forward,
                           * root values); in the loop the count is on the device: oaz_search_stats.nn_evals */
    double noise_ms;      /* Dirichlet root-noise producer (second stream, overlaps the NN) */
    uint64_t noise_n;
    double compact_ms;    /* leaf compaction (the positions the NN evaluates, per 4096-game bucket) */
    uint64_t compact_n;
    double backup_select_ms; /* expand/backup of simulation s fused with the select of s + 1 (every
                              * simulation step but the first select and the last expand/backup) */
    uint64_t backup_select_n;
    double nn_busy_ms;    /* length of the union of the timed nn launches' intervals (the game parts'
                           * launches of one simulation step overlap; oaz_config.parts) */
    uint64_t nn_busy_n;   /* disjoint intervals in that union */
    uint64_t parts;       /* game parts (streams) of the last simulation loop: nn launches per step */
} oaz_kernel_times;

typedef struct oaz_engine oaz_engine;

/* ---- library ---------------------------------------------------------------- */
int oaz_abi_version(void);
const char* oaz_last_error(void);
void oaz_config_default(oaz_config* cfg);   /* canonical self-play config (bin/train.rs:50-78) */
int oaz_device_count(int* n);               /* number of visible HIP devices */

/* ---- host-side helpers (no GPU needed) ---------------------------------------- */
/* ATTACK_MAPS[color][card][from] (card.rs:476-604), as compiled into the kernels. */
void oaz_attack_maps(uint32_t out[2 * 16 * 25]);
/* Number of fp32 values in the canonical weight blob (tch VarStore order). */
size_t oaz_weight_count(int blocks, int channels, int in_planes);
/* Bytes of the packed, BN-folded weight image the network kernels read for `precision` (OAZ_FP32 ...
 * OAZ_FP32_SPLIT16): every launch streams it into each XCD's L2 once (the L2s are written back and
 * invalidated at kernel boundaries), which is the per-launch weight traffic bench.py's roofline counts. */
size_t oaz_nn_device_bytes(int blocks, int precision);
/* Random-init weights in canonical order: conv/linear U(-1/sqrt(fan_in), +1/sqrt(fan_in)),
 * BN gamma 1, beta 0, mean 0, var 1. */
int oaz_random_weights(uint64_t seed, int blocks, float* out, size_t n);
/* Deck of global game `game_id` under `seed` (random 5 of 16, Fisher-Yates on Philox). */
void oaz_deal_deck(uint64_t seed, uint64_t game_id, uint8_t out[5]);
/* Global game ids of the `games` self-play slots of rank `rank` of `world` in their seq-th game:
 * out[g] = (seq * world + rank) * games + g, the rule the self-play kernel keys deals and root noise with
 * (replaces the reference's per-worker games, train.rs:218-238: ranks play disjoint game ids). */
int oaz_slot_game_ids(int rank, int world, int games, uint64_t seq, uint64_t* out);
/* Start position with `deck`; to_move = colour of the neutral card (game_state.rs:19-24). */
void oaz_initial_state(const uint8_t deck[5], oaz_state* out);
/* The HASH test evaluator (identical on host and device; documented in DESIGN.md). */
void oaz_hash_eval(const oaz_state* s, float policy[50], float* value);
/* One root-noise draw (replaces the per-comparison Dirichlet(alpha; K) sample of
 * mcts_arena.rs:186-203, marginally Beta(alpha, (K-1) alpha), f64 as the reference's): draw `draw`
 * (2j + 0 for the running best, 2j + 1 for child j of comparison j) of simulation `sim` at ply `ply`
 * of global game `game_id`. Host computation of the exact value the GPU's root-noise kernel stores. */
double oaz_root_noise(uint64_t seed, uint64_t game_id, uint32_t ply, uint32_t sim, uint32_t draw, double alpha,
                      int nchild);

/* ---- rules on the GPU (bit-exact with the reference) ---------------------------- */
/* Legal moves of s[i].to_move. masks[i][k][from] = destination mask of own piece on
 * `from` with the mover's k-th card (slot 0/1 for Red, 2/3 for Blue), 0 if no own piece.
 * moves[i][*] in reference order (slot, from, to ascending), the entries past counts[i] zero;
 * counts[i] = #moves.
 * Any output pointer may be NULL. Host pointers. */
int oaz_movegen(const oaz_state* s, int n, uint32_t* masks /* n*2*25 */,
                oaz_move* moves /* n*40 */, uint8_t* counts /* n */);
/* make_move(mv[i], s[i].to_move, mv[i].slot) in place, then switch to_move;
 * results[i] = MoveResult. Host pointers. */
int oaz_step(oaz_state* s, const oaz_move* mv, int n, uint8_t* results);
/* current_state() of each position. */
int oaz_current_state(const oaz_state* s, int n, uint8_t* results);
/* 21x5x5 planes of s[i] for colour s[i].to_move (fp32, n*525). */
int oaz_encode(const oaz_state* s, int n, float* planes);

/* ---- engine --------------------------------------------------------------------- */
oaz_engine* oaz_create(const oaz_config* cfg, int device);
void oaz_destroy(oaz_engine* eng);
int oaz_get_config(const oaz_engine* eng, oaz_config* out);
/* Per-agent search parameters for the following searches / self-play plies (AlphaZeroMctsConfig,
 * alphazero_mcts/mod.rs:26-43: max_playouts <= the creation cfg.sims, exploration_c, train), so
 * agents with different configs can share one engine as the reference's agents share one
 * Arc<Mutex<ConvResNet>> (mod.rs:84,124). */
int oaz_set_search_params(oaz_engine* eng, int sims, double c_puct, int train_noise);
/* Q7 wall-clock budget per search (AlphaZeroMctsConfig.search_time, alphazero_mcts/mod.rs:26-43;
 * the reference's default agent: 400 ms / 5000 playouts, its tournament: 1 s / 5000,
 * bin/tournament.rs:121-129) for the following searches / plies: oaz_config.search_time_ns. 0 = off. */
int oaz_set_search_time(oaz_engine* eng, int64_t search_time_ns);
/* Simulations per game run by the last search / self-play ply (= sims unless a search_time_ns budget
 * stopped it earlier; with per-game counts, their maximum). */
int oaz_last_sims(oaz_engine* eng, int* sims);
/* Playouts each of the first G games of the last search / ply ran (the reference's
 * MctsArena.playouts after search(), mcts_arena.rs:75-81); G <= the last call's games. */
int oaz_search_playouts(oaz_engine* eng, int* out, int G);
/* Weights in canonical order (n == oaz_weight_count). BN is folded on the host. */
int oaz_load_weights(oaz_engine* eng, const float* blob, size_t n);

/* ---- model loading by name (AlphaZeroMcts::from_model_file: `vs.load(model_path)` on the
 * ConvResNet of net.rs:101-213, alphazero_mcts/mod.rs:89-105) ----------------------------------
 * The canonical tensor table = the VarStore variables net.rs creates, in creation order (the blob
 * layout of oaz_load_weights): names joined with '|' as in the .ot files ('.' — tch's in-memory
 * separator — is accepted everywhere a name is taken). Host-only helpers (no GPU). */
size_t oaz_weight_tensor_count(int blocks);
int oaz_weight_tensor_info(int blocks, size_t i, char* name, size_t name_cap, size_t* numel);
/* n named fp32 tensors (any order, e.g. tch's `vs.variables()` HashMap: name, data pointer, numel)
 * -> the canonical blob (out_n >= oaz_weight_count). A missing, duplicate, unknown or wrongly sized
 * tensor is OAZ_ERR_WEIGHTS naming it (the reference silently keeps random weights, Q13). */
int oaz_weights_from_named(int blocks, const char* const* names, const float* const* data, const size_t* sizes,
                           size_t n, float* out, size_t out_n);
/* The same, straight into an engine (blocks = the engine's). */
int oaz_load_weights_named(oaz_engine* eng, const char* const* names, const float* const* data,
                           const size_t* sizes, size_t n);
/* A VarStore::save .ot archive (train.rs:414-430; TorchScript zip with stored members) -> canonical
 * blob; *blocks_out = residual blocks found in it. data.pkl is read by a restricted pickle machine
 * that builds plain values only (nothing is imported or executed). out may be NULL to size. */
int oaz_ot_read(const char* path, float* out, size_t cap, size_t* n_out, int* blocks_out);
/* oaz_ot_read + oaz_load_weights; the file must hold a network of the engine's block count. */
int oaz_load_ot(oaz_engine* eng, const char* path);
/* ---- checkpoints (save_vs, alphazero-training/src/train.rs:414-430: `vs.save(&path)`) ---------
 * A canonical blob (n == oaz_weight_count(blocks, 64, 21)) -> a VarStore .ot archive at `path`: the
 * TorchScript zip layout VarStore::load, oaz_ot_read and torch.jit.load read (stored members under
 * "<file stem>/", '|' names, 64-byte aligned fp32 storages). Written to "<path>.tmp" and renamed
 * over `path`. Host only. */
int oaz_ot_write(const char* path, const float* blob, size_t n, int blocks);
/* save_vs naming: "<folder>/[best_]model_<iteration>_<stamp>.ot", stamp NULL = the local time as
 * "%Y%m%d_%H%M%S" (chrono Local::now()). OAZ_ERR_CAPACITY if out[cap] is too small. */
int oaz_checkpoint_path(const char* folder, int64_t iteration, int is_best, const char* stamp, char* out,
                        size_t cap);
int oaz_sync(oaz_engine* eng);
/* enable: 0 off, 1 HIP events around every launch, N > 1 around the kernels of every N-th
 * simulation step only (the events cost ~2 % of a C3 step when every launch is timed). */
int oaz_set_timing(oaz_engine* eng, int enable);
int oaz_kernel_times_get(oaz_engine* eng, oaz_kernel_times* out);
int oaz_kernel_times_reset(oaz_engine* eng);

/* policy [B][2][25] (softmax over all 50), value [B]. Host pointers. B <= cfg.games. */
int oaz_nn_forward(oaz_engine* eng, const oaz_state* s, int B, float* policy, float* value);
/* OAZ_FP32_SPLIT16: 16-position tiles recomputed with the OAZ_FP32_SPLIT arithmetic because an
 * activation left the fp16 range, since the engine was created (0 for other precisions). */
int oaz_nn_fallbacks(oaz_engine* eng, uint64_t* tiles);

/* One search per root (root colour = roots[i].to_move), cfg.sims simulations each, all
 * G searches advanced together. out_pi [G][50] f32, out_root_value [G] = an extra NN
 * evaluation of the root (Agent::generate_move, mod.rs:137-141). Any output may be NULL. */
int oaz_search(oaz_engine* eng, const oaz_state* roots, int G, oaz_move* out_move,
               float* out_pi, float* out_root_value, oaz_search_stats* stats);
/* Tree of `game` left by the last oaz_search, or of slot `game` by the last self-play ply (the tree that
 * ply's move and pi came from): nodes [0, *n_nodes) in reference arena order. */
int oaz_tree_dump(oaz_engine* eng, int game, oaz_node* out, int cap, int* n_nodes);

/* ---- self-play (continuous batching over cfg.games slots, device resident) ------ */
int oaz_selfplay_reset(oaz_engine* eng);                 /* deal a fresh game in every slot */
int oaz_selfplay_step(oaz_engine* eng, int moves);       /* play `moves` plies in every slot */
int oaz_selfplay_stats_get(oaz_engine* eng, oaz_selfplay_stats* out);
/* Copy up to cap buffered samples to host memory and drop them from the device buffer. */
int oaz_samples_fetch(oaz_engine* eng, oaz_sample* out, size_t cap, size_t* n_out);
/* Device-to-device copy of up to cap_bytes/sizeof(oaz_sample) buffered samples into a
 * device buffer on the engine's GPU (e.g. a tensor that is then all-gathered over RCCL). */
int oaz_samples_export_device(oaz_engine* eng, void* dev_dst, size_t cap_bytes, size_t* n_out);
/* self_play(): play exactly n_games games and return their samples. n_games counts global game
 * ids over all ranks (cfg.world): this rank plays the ids below n_games that it owns
 * ((k * world + rank) * games + slot) and returns when those are finished. */
int oaz_selfplay_run(oaz_engine* eng, int n_games, oaz_sample* out, size_t cap,
                     size_t* n_out, oaz_selfplay_stats* stats);

/* ---- multi-GPU: RCCL over xGMI ------------------------------
 * One process (or host thread) per GPU, one engine per GPU, games sharded by global game id with
 * no exchange inside the simulation loop. The one data exchange of the path replaces the
 * reference's join of its self-play workers' buffers (alphazero-training/src/train.rs:241-244:
 * `for handle in handles { data_buffer.extend(handle.join()) }`): every rank ends with every
 * rank's (s, pi, z) records. The communicator wraps an RCCL communicator (librccl.so.1, loaded on
 * first use); rank 0 makes the id and the host sends it to the other ranks out of band (a file,
 * a socket, torch.distributed, MPI). All oaz_comm_* calls with a `comm` are collective. */
typedef struct oaz_comm oaz_comm;
typedef struct oaz_comm_id { char internal[128]; } oaz_comm_id;  /* = ncclUniqueId */

int oaz_comm_unique_id(oaz_comm_id* out);
/* Joins `world` ranks on GPU `device`; blocks until all ranks joined. NULL on error. */
oaz_comm* oaz_comm_init(const oaz_comm_id* id, int rank, int world, int device);
void oaz_comm_destroy(oaz_comm* comm);
/* All-gather of the engines' buffered samples: every rank's samples_ready records land in
 * dev_out (device memory on the engine's GPU, cap records) in rank order, and are dropped from each
 * engine's buffer (as oaz_samples_fetch does). counts_out[world] (host, optional) = records per
 * rank; *n_total = their sum. Counts are all-gathered first, then each rank's block is one
 * broadcast into its offset, all in one RCCL group: an all-gatherv with no padding and no scratch.
 * OAZ_ERR_CAPACITY (on every rank alike) when the total exceeds cap; nothing is consumed then. */
int oaz_allgather_samples(oaz_engine* eng, oaz_comm* comm, oaz_sample* dev_out, size_t cap, size_t* n_total,
                          uint64_t* counts_out);
/* In-place sum all-reduce of n floats in device memory (data-parallel gradients), on `stream`
 * (a hipStream_t; NULL = the communicator's own stream); returns when enqueued. */
int oaz_comm_allreduce_sum_f32(oaz_comm* comm, float* dev, size_t n, void* stream);
/* In-place broadcast of `bytes` bytes of device memory from `root` (new best weights),
 * on `stream` (NULL = the communicator's stream); returns when enqueued. */
int oaz_comm_broadcast(oaz_comm* comm, void* dev, size_t bytes, int root, void* stream);
/* Waits for the communicator's own stream. */
int oaz_comm_sync(oaz_comm* comm);
/* What RCCL itself reports for the communicator, and the last oaz_allgather_samples timed by HIP events
 * on the communicator's stream (host copies and any caller-side post-processing excluded). */
typedef struct oaz_comm_stats {
    int32_t ranks;              /* ncclCommCount(): ranks in the RCCL communicator */
    int32_t rank;
    uint64_t allgather_calls;
    double counts_ms;           /* last all-gather: the uint64 counts all-gather (+ its 8-byte host copies) */
    double allgather_ms;        /* last all-gather: the grouped per-rank broadcasts of the 228-byte records */
    uint64_t allgather_records; /* records every rank received in the last all-gather (sum of the counts) */
    uint64_t allgather_bytes;   /* = allgather_records * sizeof(oaz_sample) */
    uint64_t own_records;       /* this rank's contribution to the last all-gather */
} oaz_comm_stats;
int oaz_comm_stats_get(oaz_comm* comm, oaz_comm_stats* out);

/* ---- training step ---------------------------------
 * One trainer = one GPU. Parameters live on the device in the canonical blob
 * layout (the VarStore order, see oaz_weight_count); BN running statistics are
 * part of the blob and are updated by the train-mode forward (momentum 0.1,
 * unbiased variance), as tch's batch_norm2d does. A step is
 *   gather batch -> forward(train=true) -> alphaloss -> backward -> SGD
 * with the reference's optimiser: d = g + wd*p; buf = momentum*buf + d; p -= lr*buf
 * over the trainable variables (weights, biases, BN gamma/beta). */
typedef struct oaz_train_config {
    int32_t blocks;               /* residual blocks (ConvResNetConfig::resnet_block_amnt) */
    int32_t max_batch;            /* largest batch (multiple of 16); train_batch_size 512 (train.rs:142) */
    double learning_rate;         /* 5e-3 (bin/train.rs:69) */
    double momentum;              /* 0.9 (train.rs:182) */
    double weight_decay;          /* l2_const 1e-4 (train.rs:139,186) */
    double bn_momentum;           /* 0.1 (tch BatchNormConfig default) */
    double bn_eps;                /* 1e-5 */
    int32_t value_loss_broadcast; /* 1 = reference (Q16: z[B] - v[B,1] broadcasts to [B,B]), 0 = elementwise */
    int32_t reserved[7];
} oaz_train_config;

typedef struct oaz_trainer oaz_trainer;

void oaz_train_config_default(oaz_train_config* cfg);
oaz_trainer* oaz_trainer_create(const oaz_train_config* cfg, int device);  /* NULL on error */
void oaz_trainer_destroy(oaz_trainer* t);
/* Run the trainer's kernels on `stream` (a hipStream_t; NULL = the trainer's own stream). */
int oaz_trainer_set_stream(oaz_trainer* t, void* stream);
/* Parameters + running stats, canonical blob (n = oaz_weight_count(blocks, 64, 21)).
 * set_weights also clears the momentum buffers (a fresh nn::Sgd). */
int oaz_trainer_set_weights(oaz_trainer* t, const float* blob, size_t n);
int oaz_trainer_get_weights(oaz_trainer* t, float* blob, size_t n);
/* The trainer's parameters (and BN running statistics) as a .ot checkpoint (oaz_ot_write): the
 * reference's save_vs on the training VarStore (train.rs:383-403, 414-430). */
int oaz_trainer_save_ot(oaz_trainer* t, const char* path);
/* The replay buffer: copy n host samples to the device (owned), or bind n samples already
 * resident on this GPU (e.g. oaz_samples_export_device; not owned, must outlive use). */
int oaz_trainer_load_samples(oaz_trainer* t, const oaz_sample* samples, size_t n);
int oaz_trainer_bind_device_samples(oaz_trainer* t, const oaz_sample* dev_samples, size_t n);
/* Upload batch indices (n_batches x batch int32 into the replay buffer), e.g. one epoch of
 * choose_multiple draws (train.rs:272-276). */
int oaz_trainer_set_batches(oaz_trainer* t, const int32_t* idx, int n_batches, int batch);
/* Forward + loss + backward for batch `b` of the uploaded indices: gradients land in the
 * device gradient buffer (oaz_trainer_grads); no parameter changes except BN running stats. */
int oaz_trainer_backward(oaz_trainer* t, int b);
/* Device gradient buffer (canonical blob layout; running-stat slots unused) for an external
 * all-reduce between backward and apply (data-parallel training). */
int oaz_trainer_grads(oaz_trainer* t, float** dev_grads, size_t* n);
int oaz_trainer_get_grads(oaz_trainer* t, float* host, size_t n);
/* SGD step on the gradient buffer (scaled by grad_scale, e.g. 1/world after a sum all-reduce). */
int oaz_trainer_apply(oaz_trainer* t, float grad_scale);
/* BN running statistics (running_mean + running_var of every BN layer, canonical order) as one
 * contiguous device range of oaz_trainer_bn_stats_count(blocks) floats, so a data-parallel host can
 * average them over ranks (pack, oaz_comm_allreduce_sum_f32, unpack with scale = 1/world) and every
 * rank keeps identical inference weights (ranks' batch statistics differ; DDP without SyncBN). Both
 * run on the trainer's stream. */
size_t oaz_trainer_bn_stats_count(int blocks);
int oaz_trainer_bn_stats_pack(oaz_trainer* t, float* dev_out);
int oaz_trainer_bn_stats_unpack(oaz_trainer* t, const float* dev_in, float scale);
/* backward(b) + apply(1) for batches [first, first+count). */
int oaz_trainer_train(oaz_trainer* t, int first, int count);
/* Loss sums since the last call: out[0] value loss, out[1] policy loss, out[2] steps. */
int oaz_trainer_losses(oaz_trainer* t, double out[3]);
int oaz_trainer_sync(oaz_trainer* t);

/* ---- pure MCTS agent --------------------------------
 * The reference's `Mcts` agent: UCT (f32, winrate + c*sqrt(ln N / n)) over a tree expanded once a
 * leaf has more than min_node_visits visits, random rollouts to the end of the game, +-1 backed up
 * with a sign flip. One GPU thread runs one game's whole search. Rollout draws come from Philox
 * (seed; game_id0 + g, playout, 0x9C7A0000, d/4); a rollout longer than rollout_cap plies scores 0. */
typedef struct oaz_pure_mcts_config {
    int32_t max_playouts;     /* 5000 (ai/mcts/mod.rs:25); the arena's opponent uses 400 (evaluator.rs:340-345) */
    int32_t min_node_visits;  /* 5 */
    float exploration_c;      /* sqrt(2) as f32 (the arena's opponent: 1.41) */
    int32_t rollout_cap;      /* plies per rollout before it is scored as a draw (reference: none) */
    uint64_t seed;
    uint64_t game_id0;        /* RNG stream of root g = game_id0 + g */
    int32_t device;           /* HIP device the search runs on (its own stream; other work on it is not waited for) */
    int32_t reserved[3];
} oaz_pure_mcts_config;

typedef struct oaz_pure_node { /* MctsNode (mcts_arena.rs:330-352) */
    uint32_t visits;
    float reward;
    float winrate;
    uint32_t first;   /* first child (children are contiguous) */
    uint32_t parent;  /* 0xFFFFFFFF for the root */
    uint16_t mv;      /* from | to<<5 | slot<<10 | piece<<12 */
    uint8_t nch;
    uint8_t flags;    /* 1 expanded, 2 terminal */
} oaz_pure_node;  /* 24 bytes */

typedef struct oaz_pure_mcts_stats {
    uint64_t playouts, expansions, rollout_plies, rollout_passes, rollouts_capped, max_nodes, tree_full;
} oaz_pure_mcts_stats;

void oaz_pure_mcts_config_default(oaz_pure_mcts_config* cfg);
/* Nodes one search may allocate (the per-game capacity of tree_out). */
size_t oaz_pure_mcts_tree_capacity(const oaz_pure_mcts_config* cfg);
/* One search per root (colour = root.to_move). out_value = winrate of the chosen child. A root with
 * no legal move returns the pass move (from = to = 25). tree_out (optional, G x tree_cap nodes)
 * receives each game's tree. Runs on cfg->device on a stream of its own; the calling thread's current
 * HIP device is restored before the call returns. */
int oaz_pure_mcts_search(const oaz_state* roots, int G, const oaz_pure_mcts_config* cfg, oaz_move* out_move,
                         float* out_value, oaz_pure_mcts_stats* stats, oaz_pure_node* tree_out, size_t tree_cap);
/* A search's device buffers are one allocation (G x oaz_pure_mcts_tree_capacity nodes + ~100 B per root), and the
 * last one of each device is kept for the next search (a 1 M-search launch's trees are 64 GB); this frees a
 * device's kept buffer (OAZ_ERR_STATE while a search uses it). */
int oaz_pure_mcts_release_workspace(int device);

#ifdef __cplusplus
}
#endif
#endif /* ONITAMA_AZ_H */
