/* abi_smoke.c — the C ABI used from plain C, as a Rust/C host would bind it.
 * Built by tests/test_c_abi.py with gcc against include/onitama_az.h and libonitama_az.so.
 * Without a GPU it checks the host-side entry points and the loud no-device errors; with one it
 * runs a batched search, a self-play game batch and the pure-MCTS agent. Prints "OK ..." lines.
 *   abi_smoke [model.ot golden.bin]: also loads the model the way AlphaZeroMcts::from_model_file
 *   does (alphazero_mcts/mod.rs:89-105) — by path (oaz_load_ot) and by name (oaz_load_weights_named,
 *   the tensors in shuffled order with tch's '.' separator, as `vs.variables()` hands them over) —
 *   and compares oaz_nn_forward with the golden policy/value (golden.bin: n, then n states, n x 50
 *   policy and n values).
 *   abi_smoke model.ot golden.bin out_dir: also writes the model back as a checkpoint the way save_vs
 *   does (train.rs:414-430: oaz_checkpoint_path + oaz_ot_write, <out_dir>/best_model_7_<stamp>.ot),
 *   reads it back bit-equal, and (with a GPU) saves the trainer's weights with oaz_trainer_save_ot. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "onitama_az.h"

/* A host allocates the device buffer the all-gather writes into with HIP itself (the Rust host
 * links libamdhip64 too); plain-C prototypes of the three calls used (extern "C" in HIP). */
int hipMalloc(void** ptr, size_t size);
int hipFree(void* ptr);
int hipMemcpy(void* dst, const void* src, size_t bytes, int kind); /* kind 2 = device to host */

#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, oaz_last_error()); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

/* The model file by path and by name (host side: no GPU). Fills *blob (canonical order). */
static int model_host(const char* ot, const char* out_dir, float** blob, size_t* nblob) {
    size_t n = 0;
    int blocks = -1;
    CHECK(oaz_ot_read(ot, NULL, 0, &n, &blocks) == 0 && blocks == 3 && n == oaz_weight_count(3, 64, 21));
    float* w = (float*)malloc(n * sizeof(float));
    CHECK(oaz_ot_read(ot, w, n, &n, &blocks) == 0);
    /* by name: the canonical table, tensors handed over in a shuffled order with '.' separators */
    const size_t nt = oaz_weight_tensor_count(3);
    CHECK(nt == 60);
    char(*names)[96] = malloc(nt * sizeof(*names));
    const char** np = malloc(nt * sizeof(char*));
    const float** dp = malloc(nt * sizeof(float*));
    size_t* sz = malloc(nt * sizeof(size_t));
    size_t off = 0;
    for (size_t i = 0; i < nt; ++i) {
        const size_t j = (i * 37) % nt; /* 37 is coprime with 60: a permutation */
        size_t numel = 0;
        CHECK(oaz_weight_tensor_info(3, i, names[j], sizeof(names[j]), &numel) == 0);
        for (char* c = names[j]; *c; ++c)
            if (*c == '|') *c = '.';
        np[j] = names[j];
        dp[j] = w + off;
        sz[j] = numel;
        off += numel;
    }
    CHECK(off == n);
    float* w2 = (float*)malloc(n * sizeof(float));
    CHECK(oaz_weights_from_named(3, np, dp, sz, nt, w2, n) == 0 && memcmp(w, w2, n * sizeof(float)) == 0);
    sz[5] += 1; /* a wrongly sized tensor is refused, naming it */
    CHECK(oaz_weights_from_named(3, np, dp, sz, nt, w2, n) == OAZ_ERR_WEIGHTS && strstr(oaz_last_error(), "elements"));
    sz[5] -= 1;
    CHECK(oaz_weights_from_named(3, np, dp, sz, nt - 1, w2, n) == OAZ_ERR_WEIGHTS && strstr(oaz_last_error(), "missing"));
    CHECK(oaz_weights_from_named(2, np, dp, sz, nt, w2, n) == OAZ_ERR_WEIGHTS); /* resnet_2 is not in 2 blocks */
    free(w2);
    if (out_dir) { /* save_vs: the checkpoint path and the archive, read back bit-equal */
        char path[1024];
        CHECK(oaz_checkpoint_path(out_dir, 7, 1, "20260101_120000", path, 8) == OAZ_ERR_CAPACITY);
        CHECK(oaz_checkpoint_path(out_dir, 7, 1, "20260101_120000", path, sizeof path) == 0);
        CHECK(strstr(path, "/best_model_7_20260101_120000.ot") != NULL);
        CHECK(oaz_ot_write(path, w, n - 1, 3) == OAZ_ERR_ARG); /* wrong size for 3 blocks */
        CHECK(oaz_ot_write(path, w, n, 3) == 0);
        float* w3 = (float*)malloc(n * sizeof(float));
        size_t n3 = 0;
        int b3 = -1;
        CHECK(oaz_ot_read(path, w3, n, &n3, &b3) == 0 && n3 == n && b3 == 3 && memcmp(w, w3, n * sizeof(float)) == 0);
        free(w3);
        printf("OK ot-write %s\n", path);
    }
    free(names);
    free(np);
    free(dp);
    free(sz);
    *blob = w;
    *nblob = n;
    return 0;
}

/* On the GPU: load by path and by name, forward the golden positions, compare. */
static int model_gpu(const char* ot, const char* golden, const float* w, size_t nw) {
    FILE* f = fopen(golden, "rb");
    CHECK(f != NULL);
    int32_t n = 0;
    CHECK(fread(&n, 4, 1, f) == 1 && n > 0 && n <= 4096);
    oaz_state* st = malloc(n * sizeof(oaz_state));
    float *gp = malloc(n * 50 * sizeof(float)), *gv = malloc(n * sizeof(float));
    float *p = malloc(n * 50 * sizeof(float)), *v = malloc(n * sizeof(float));
    float *p2 = malloc(n * 50 * sizeof(float)), *v2 = malloc(n * sizeof(float));
    CHECK(fread(st, sizeof(oaz_state), n, f) == (size_t)n && fread(gp, 4, n * 50, f) == (size_t)n * 50 &&
          fread(gv, 4, n, f) == (size_t)n);
    fclose(f);
    oaz_config cfg;
    oaz_config_default(&cfg);
    cfg.blocks = 3;
    cfg.sims = 1;
    cfg.games = n;
    cfg.precision = OAZ_FP32_SPLIT16;
    oaz_engine* e = oaz_create(&cfg, 0);
    CHECK(e != NULL);
    CHECK(oaz_load_ot(e, ot) == 0 && oaz_nn_forward(e, st, n, p, v) == 0);
    double err = 0;
    for (int i = 0; i < n * 50; ++i) err = fabs(p[i] - gp[i]) > err ? fabs(p[i] - gp[i]) : err;
    for (int i = 0; i < n; ++i) err = fabs(v[i] - gv[i]) > err ? fabs(v[i] - gv[i]) : err;
    CHECK(err < 1e-5);
    /* by name: the same tensors from host memory, bit-identical forward */
    const size_t nt = oaz_weight_tensor_count(3);
    char(*names)[96] = malloc(nt * sizeof(*names));
    const char** np = malloc(nt * sizeof(char*));
    const float** dp = malloc(nt * sizeof(float*));
    size_t* sz = malloc(nt * sizeof(size_t));
    size_t off = 0;
    for (size_t i = 0; i < nt; ++i) {
        CHECK(oaz_weight_tensor_info(3, i, names[i], sizeof(names[i]), &sz[i]) == 0);
        np[i] = names[i];
        dp[i] = w + off;
        off += sz[i];
    }
    CHECK(off == nw);
    CHECK(oaz_load_weights_named(e, np, dp, sz, nt) == 0 && oaz_nn_forward(e, st, n, p2, v2) == 0);
    CHECK(memcmp(p, p2, n * 50 * sizeof(float)) == 0 && memcmp(v, v2, n * sizeof(float)) == 0);
    CHECK(oaz_load_weights_named(e, np, dp, sz, nt - 2) == OAZ_ERR_WEIGHTS);
    oaz_destroy(e);
    printf("OK model %d positions max err %.2e\n", n, err);
    free(names);
    free(np);
    free(dp);
    free(sz);
    free(st);
    free(gp);
    free(gv);
    free(p);
    free(v);
    free(p2);
    free(v2);
    return 0;
}

int main(int argc, char** argv) {
    CHECK(oaz_abi_version() == OAZ_ABI_VERSION);
    oaz_config cfg;
    oaz_config_default(&cfg);
    CHECK(cfg.blocks == 5 && cfg.sims == 400 && cfg.max_plies == 150);
    CHECK(oaz_weight_count(3, 64, 21) == 240006);
    uint32_t maps[2 * 16 * 25];
    oaz_attack_maps(maps);
    uint8_t deck[5] = {0, 1, 2, 3, 4};
    oaz_state s;
    oaz_initial_state(deck, &s);
    CHECK(s.kings[0] == 0x200u && s.kings[1] == 0x20000000u && s.to_move == 1); /* Crab neutral: Blue starts */
    printf("OK host\n");
    float* model = NULL;
    size_t nmodel = 0;
    if (argc >= 3) {
        if (model_host(argv[1], argc >= 4 ? argv[3] : NULL, &model, &nmodel)) return 1;
        printf("OK model-host\n");
    }
    int ndev = 0;
    oaz_device_count(&ndev);
    if (ndev == 0) {
        CHECK(oaz_create(&cfg, 0) == NULL && strstr(oaz_last_error(), "device") != NULL);
        CHECK(oaz_movegen(&s, 1, NULL, NULL, NULL) == OAZ_ERR_NO_DEVICE);
        printf("OK no-device\n");
        return 0;
    }
    if (model && model_gpu(argv[1], argv[2], model, nmodel)) return 1;
    /* rules */
    oaz_move moves[40];
    uint8_t count = 0;
    CHECK(oaz_movegen(&s, 1, NULL, moves, &count) == 0 && count == 8); /* Frog + Rabbit from the start (oracle) */
    /* one batched search per root (mirrors generate_move_tensor) */
    cfg.blocks = 3;
    cfg.sims = 64;
    cfg.games = 4;
    cfg.train_noise = 0;
    oaz_engine* e = oaz_create(&cfg, 0);
    CHECK(e != NULL);
    size_t nw = oaz_weight_count(3, 64, 21);
    float* w = (float*)malloc(nw * sizeof(float));
    CHECK(oaz_random_weights(0, 3, w, nw) == 0 && oaz_load_weights(e, w, nw) == 0);
    oaz_state roots[4];
    for (int g = 0; g < 4; ++g) {
        uint8_t d[5];
        oaz_deal_deck(20260101ull, (uint64_t)g, d);
        oaz_initial_state(d, &roots[g]);
    }
    oaz_move out[4];
    float pi[4 * 50], rv[4];
    oaz_search_stats st;
    CHECK(oaz_search(e, roots, 4, out, pi, rv, &st) == 0 && st.sims == 4 * 64);
    for (int g = 0; g < 4; ++g) {
        float sum = 0;
        for (int k = 0; k < 50; ++k) sum += pi[g * 50 + k];
        CHECK(sum > 0.999f && sum < 1.001f && out[g].from < 25);
    }
    printf("OK search\n");
    /* self-play */
    oaz_sample* buf = (oaz_sample*)malloc(sizeof(oaz_sample) * 4 * 152);
    size_t n = 0;
    oaz_selfplay_stats sp;
    CHECK(oaz_selfplay_run(e, 4, buf, 4 * 152, &n, &sp) == 0 && sp.games_finished + sp.games_cut == 4 && n > 0);
    printf("OK selfplay %zu samples\n", n);
    /* RCCL communicator at world 1: all-gather the buffered samples device to device */
    CHECK(oaz_selfplay_reset(e) == 0 && oaz_selfplay_step(e, 40) == 0 && oaz_selfplay_stats_get(e, &sp) == 0);
    const size_t ready = sp.samples_ready;
    CHECK(ready > 0);
    oaz_comm_id cid;
    CHECK(oaz_comm_unique_id(&cid) == 0);
    oaz_comm* comm = oaz_comm_init(&cid, 0, 1, 0);
    CHECK(comm != NULL);
    void* dev = NULL;
    CHECK(hipMalloc(&dev, ready * sizeof(oaz_sample)) == 0);
    size_t total = 0;
    uint64_t counts[1] = {0};
    CHECK(oaz_allgather_samples(e, comm, (oaz_sample*)dev, ready - 1, &total, counts) == OAZ_ERR_CAPACITY &&
          total == ready);
    CHECK(oaz_allgather_samples(e, comm, (oaz_sample*)dev, ready, &total, counts) == 0 && total == ready &&
          counts[0] == ready);
    oaz_sample* hs = (oaz_sample*)malloc(ready * sizeof(oaz_sample));
    CHECK(hipMemcpy(hs, dev, ready * sizeof(oaz_sample), 2) == 0);
    for (size_t i = 0; i < ready; ++i) {
        float sum = 0;
        for (int k = 0; k < 50; ++k) sum += hs[i].pi[k];
        CHECK(sum > 0.999f && sum < 1.001f && (hs[i].z == 0.0f || hs[i].z == 1.0f || hs[i].z == -1.0f));
    }
    CHECK(oaz_selfplay_stats_get(e, &sp) == 0 && sp.samples_ready == 0); /* consumed */
    oaz_comm_stats cs;
    CHECK(oaz_comm_stats_get(comm, &cs) == 0 && cs.ranks == 1 && cs.rank == 0 && cs.allgather_calls == 1 &&
          cs.allgather_records == ready && cs.allgather_bytes == ready * sizeof(oaz_sample) && cs.allgather_ms >= 0.0);
    CHECK(oaz_comm_allreduce_sum_f32(comm, (float*)dev, 16, NULL) == 0 && oaz_comm_sync(comm) == 0);
    CHECK(oaz_comm_broadcast(comm, dev, 64, 0, NULL) == 0 && oaz_comm_sync(comm) == 0);
    oaz_comm_destroy(comm);
    hipFree(dev);
    free(hs);
    printf("OK comm %zu samples\n", ready);
    /* pure MCTS agent */
    oaz_pure_mcts_config pc;
    oaz_pure_mcts_config_default(&pc);
    pc.max_playouts = 200;
    oaz_move pm[4];
    float pv[4];
    oaz_pure_mcts_stats ps;
    CHECK(oaz_pure_mcts_search(roots, 4, &pc, pm, pv, &ps, NULL, 0) == 0 && ps.playouts == 800);
    printf("OK pure_mcts\n");
    /* training step */
    oaz_train_config tc;
    oaz_train_config_default(&tc);
    tc.blocks = 3;
    tc.max_batch = 32;
    oaz_trainer* t = oaz_trainer_create(&tc, 0);
    CHECK(t != NULL && oaz_trainer_set_weights(t, w, nw) == 0 && oaz_trainer_load_samples(t, buf, n) == 0);
    int32_t idx[32];
    for (int i = 0; i < 32; ++i) idx[i] = (int32_t)(i % n);
    double losses[3];
    CHECK(oaz_trainer_set_batches(t, idx, 1, 32) == 0 && oaz_trainer_train(t, 0, 1) == 0);
    CHECK(oaz_trainer_losses(t, losses) == 0 && losses[2] == 1.0 && losses[0] >= 0.0 && losses[1] > 0.0);
    printf("OK train loss %.4f %.4f\n", losses[0], losses[1]);
    if (argc >= 4) { /* the trained weights as a checkpoint (save_vs on the training VarStore) */
        char path[1024];
        CHECK(oaz_checkpoint_path(argv[3], 1, 0, NULL, path, sizeof path) == 0);
        CHECK(oaz_trainer_save_ot(t, path) == 0);
        float *tw = (float*)malloc(nw * sizeof(float)), *rw = (float*)malloc(nw * sizeof(float));
        size_t nr = 0;
        int br = -1;
        CHECK(oaz_trainer_get_weights(t, tw, nw) == 0 && oaz_ot_read(path, rw, nw, &nr, &br) == 0 && nr == nw && br == 3);
        CHECK(memcmp(tw, rw, nw * sizeof(float)) == 0 && memcmp(tw, w, nw * sizeof(float)) != 0);
        free(tw);
        free(rw);
        printf("OK trainer-save %s\n", path);
    }
    oaz_trainer_destroy(t);
    oaz_destroy(e);
    free(buf);
    free(w);
    free(model);
    return 0;
}
