/* comm_multirank.c — the product multi-GPU exchange (csrc/oaz_comm.cpp) at world > 1, from plain C.
 * Each rank is a host thread with its own engine and communicator on GPU 0; librccl.so.1 is the
 * test double tests/c/rccl_stub.c (put first on LD_LIBRARY_PATH by tests/test_c_abi.py), so the
 * grouped-broadcast all-gatherv, the counts all-gather, the failure sentinel, the broadcast and the
 * all-reduce run with several ranks on a one-GPU box. Reference: the join of the self-play workers'
 * buffers, alphazero-training/src/train.rs:241-244 (`data_buffer.extend(handle.join())` in worker
 * order = rank order here).
 *
 *   comm_multirank W        (2 <= W <= 8; 8 = the C4 node's rank count)
 *   comm_multirank 8 c4     (the C4 volume: 65,536 slots per rank, > 2^31 bytes gathered into every rank)
 *
 * Per rank r: engine A (the exchange) and engine B (the expectation) get the same config (G_r game
 * slots, rank r of W, HASH evaluator, root noise on) and play the same number of plies P_r, ragged
 * over the ranks and 0 for rank 1 (a rank with no samples). B's samples are fetched to the host;
 * self-play is deterministic, records included (a ply's finished games append their records in slot
 * order), so they are byte for byte what A holds. Then, on every rank:
 *   1. oaz_allgather_samples with cap = total - 1: OAZ_ERR_CAPACITY, *n_total = total, nothing consumed;
 *   2. the last rank passes a NULL engine: it gets OAZ_ERR_ARG, every other rank OAZ_ERR_COMM naming
 *      that rank (the kLocalFailure sentinel through the counts all-gather), nothing consumed;
 *   3. cap = total: counts_out = every rank's count; every rank's device output byte-equal to every
 *      other rank's and to the rank-order concatenation of the B engines' fetches; own buffer drained;
 *      stats (ranks, records, own records);
 *   4. again with every buffer empty: total 0, success;
 *   5. oaz_comm_broadcast from each root in turn (in place, NULL and explicit streams);
 *   6. oaz_comm_allreduce_sum_f32 (exact small sums) on the communicator's and on a caller stream.
 * The stub is asynchronous as RCCL is (a collective is enqueued on the caller's stream and the call
 * returns before it ran), so these results also check the product's stream ordering: the counts copy
 * and the records behind the collectives on the communicator's stream, the read cursor advanced only
 * after the exchange completed, the all-reduce ordered on a caller's stream.
 * Prints "OK rank r ..." per rank and "OK multirank W" at the end; exit 0 only if every rank passed. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "onitama_az.h"

typedef void* hipStream_t;
int hipMalloc(void** ptr, size_t size);
int hipFree(void* ptr);
int hipMemcpy(void* dst, const void* src, size_t bytes, int kind); /* 1 = H2D, 2 = D2H */
int hipStreamCreateWithFlags(hipStream_t* s, unsigned flags); /* 1 = hipStreamNonBlocking */
int hipStreamDestroy(hipStream_t s);
int hipStreamSynchronize(hipStream_t s);
uint64_t rccl_stub_ops(void); /* from the stub: proves it served the calls */
uint64_t rccl_stub_pending_at_return(void); /* ... and that they returned before their operations ran */

#define MAXW 8
static int W;
static oaz_comm_id g_id;
static oaz_sample* g_expect[MAXW]; /* rank r's samples, sorted (bytewise) */
static oaz_sample* g_out[MAXW];    /* rank r's whole all-gather output, as received */
static size_t g_count[MAXW];
/* host barrier between the rank threads, with a timeout so a rank that fails early ends the run
 * instead of leaving the others waiting */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;
static int g_arrived;
static unsigned g_gen;
static int bar_wait(void) {
    pthread_mutex_lock(&g_mu);
    const unsigned gen = g_gen;
    if (++g_arrived == W) {
        g_arrived = 0;
        g_gen++;
        pthread_cond_broadcast(&g_cv);
        pthread_mutex_unlock(&g_mu);
        return 1;
    }
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    ts.tv_sec += 150;
    while (g_gen == gen)
        if (pthread_cond_timedwait(&g_cv, &g_mu, &ts) != 0) break;
    const int ok = g_gen != gen;
    pthread_mutex_unlock(&g_mu);
    return ok;
}
static int g_fail[MAXW];

static const int kGames[MAXW] = {24, 16, 32, 8, 8, 24, 16, 32};
static const int kPlies[MAXW] = {45, 0, 70, 30, 45, 30, 70, 45};
/* c4 mode: BASELINE C4's 65,536 slots per rank, 2 simulations, games cut after 20 plies (max_plies 18),
 * 30 plies on every rank (the zero-count rank is the small mode's): ~1.4 M records = ~0.3 GB per rank, > 2^31
 * bytes gathered into each of the 8 ranks */
static int g_c4;
static const int kC4Games = 65536, kC4Plies = 30;
static int games_of(int rank) { return g_c4 ? kC4Games : kGames[rank]; }
static int plies_of(int rank) { return g_c4 ? kC4Plies : kPlies[rank]; }

#define CHECK(c)                                                                                          \
    do {                                                                                                  \
        if (!(c)) {                                                                                       \
            fprintf(stderr, "FAIL rank %d %s:%d %s (%s)\n", rank, __FILE__, __LINE__, #c, oaz_last_error()); \
            g_fail[rank] = 1;                                                                             \
            goto done;                                                                                    \
        }                                                                                                 \
    } while (0)

static oaz_engine* make_engine(int rank) {
    oaz_config cfg;
    oaz_config_default(&cfg);
    cfg.blocks = 0;
    cfg.evaluator = OAZ_EVAL_HASH;
    cfg.sims = g_c4 ? 2 : 12;
    cfg.games = games_of(rank);
    cfg.train_noise = 1;
    cfg.max_plies = g_c4 ? 18 : 150;
    if (g_c4) cfg.sample_capacity = kC4Games * 32;
    cfg.seed = 20260101ull;
    cfg.rank = rank;
    cfg.world = W;
    return oaz_create(&cfg, 0);
}

static void* rank_main(void* arg) {
    const int rank = (int)(intptr_t)arg;
    oaz_engine *a = NULL, *b = NULL;
    oaz_comm* comm = NULL;
    void *dev = NULL, *buf = NULL;
    oaz_sample* host = NULL;
    float* fh = NULL;
    hipStream_t s = NULL;
    int synced = 0;
    /* expectation: engine B plays the same plies and hands its samples to the host */
    a = make_engine(rank);
    b = make_engine(rank);
    CHECK(a && b);
    CHECK(oaz_selfplay_reset(a) == 0 && oaz_selfplay_reset(b) == 0);
    CHECK(oaz_selfplay_step(a, plies_of(rank)) == 0 && oaz_selfplay_step(b, plies_of(rank)) == 0);
    oaz_selfplay_stats sa, sb;
    CHECK(oaz_selfplay_stats_get(a, &sa) == 0 && oaz_selfplay_stats_get(b, &sb) == 0);
    if (!(sa.samples_ready == sb.samples_ready && sa.samples_dropped == 0))
        fprintf(stderr, "rank %d: engine A %llu samples (%llu dropped), engine B %llu (%llu dropped)\n", rank,
                (unsigned long long)sa.samples_ready, (unsigned long long)sa.samples_dropped,
                (unsigned long long)sb.samples_ready, (unsigned long long)sb.samples_dropped);
    CHECK(sa.samples_ready == sb.samples_ready && sa.samples_dropped == 0);
    g_count[rank] = sb.samples_ready;
    g_expect[rank] = (oaz_sample*)malloc((g_count[rank] + 1) * sizeof(oaz_sample));
    size_t got = 0;
    CHECK(oaz_samples_fetch(b, g_expect[rank], g_count[rank], &got) == 0 && got == g_count[rank]);
    oaz_destroy(b); /* (its memory back before the exchange's outputs) */
    b = NULL;
    CHECK(g_c4 ? g_count[rank] > 0 : (rank == 1) == (g_count[rank] == 0)); /* rank 1 played no ply: the zero-count rank */
    comm = oaz_comm_init(&g_id, rank, W, 0);
    CHECK(comm != NULL);
    synced = 1;
    CHECK(bar_wait()); /* every g_count / g_expect is written */
    size_t total = 0;
    for (int r = 0; r < W; ++r) total += g_count[r];
    CHECK(total > 0);
    CHECK(hipMalloc(&dev, (total + 1) * sizeof(oaz_sample)) == 0);
    host = (oaz_sample*)malloc((total + 1) * sizeof(oaz_sample));
    uint64_t counts[MAXW];
    size_t n_total = 0;
    /* 1. capacity error on every rank alike, nothing consumed */
    CHECK(oaz_allgather_samples(a, comm, (oaz_sample*)dev, total - 1, &n_total, counts) == OAZ_ERR_CAPACITY);
    CHECK(n_total == total && strstr(oaz_last_error(), "cap") != NULL);
    CHECK(oaz_selfplay_stats_get(a, &sa) == 0 && sa.samples_ready == g_count[rank]);
    /* 2. a local failure on the last rank reaches every rank through the counts all-gather */
    const int bad = W - 1;
    const int rc2 = oaz_allgather_samples(rank == bad ? NULL : a, comm, (oaz_sample*)dev, total, &n_total, counts);
    if (rank == bad) {
        CHECK(rc2 == OAZ_ERR_ARG);
    } else {
        char want[64];
        snprintf(want, sizeof want, "rank %d failed", bad);
        CHECK(rc2 == OAZ_ERR_COMM && strstr(oaz_last_error(), want) != NULL);
    }
    CHECK(oaz_selfplay_stats_get(a, &sa) == 0 && sa.samples_ready == g_count[rank]);
    /* 3. the exchange: every rank's records, in rank order */
    memset(counts, 0xff, sizeof counts);
    CHECK(oaz_allgather_samples(a, comm, (oaz_sample*)dev, total, &n_total, counts) == 0 && n_total == total);
    for (int r = 0; r < W; ++r) CHECK(counts[r] == g_count[r]);
    CHECK(hipMemcpy(host, dev, total * sizeof(oaz_sample), 2) == 0);
    size_t off = 0;
    for (int r = 0; r < W; ++r) { /* train.rs:241-244: the workers' buffers joined in worker order */
        CHECK(g_count[r] == 0 || memcmp(host + off, g_expect[r], g_count[r] * sizeof(oaz_sample)) == 0);
        off += g_count[r];
    }
    g_out[rank] = host;
    CHECK(bar_wait());
    int same = 1;
    for (int r = 0; r < W; ++r) same &= memcmp(g_out[r], host, total * sizeof(oaz_sample)) == 0;
    CHECK(bar_wait()); /* every rank compared before any frees its copy */
    CHECK(same);
    CHECK(oaz_selfplay_stats_get(a, &sa) == 0 && sa.samples_ready == 0);
    oaz_comm_stats cs;
    CHECK(oaz_comm_stats_get(comm, &cs) == 0 && cs.ranks == W && cs.rank == rank && cs.allgather_calls == 1 &&
          cs.allgather_records == total && cs.own_records == g_count[rank] &&
          cs.allgather_bytes == total * sizeof(oaz_sample));
    /* 4. every buffer empty: a zero-total exchange succeeds */
    CHECK(oaz_allgather_samples(a, comm, (oaz_sample*)dev, total, &n_total, counts) == 0 && n_total == 0);
    for (int r = 0; r < W; ++r) CHECK(counts[r] == 0);
    /* 5. broadcast from every root, in place */
    const size_t nb = 4096 + 36; /* not a multiple of anything convenient */
    CHECK(hipMalloc(&buf, nb) == 0);
    unsigned char* hb = (unsigned char*)malloc(nb);
    for (int root = 0; root < W; ++root) {
        for (size_t i = 0; i < nb; ++i) hb[i] = (unsigned char)(rank * 37 + i * 7 + 1);
        CHECK(hipMemcpy(buf, hb, nb, 1) == 0);
        CHECK(oaz_comm_broadcast(comm, buf, nb, root, NULL) == 0 && oaz_comm_sync(comm) == 0);
        CHECK(hipMemcpy(hb, buf, nb, 2) == 0);
        for (size_t i = 0; i < nb; ++i) CHECK(hb[i] == (unsigned char)(root * 37 + i * 7 + 1));
    }
    CHECK(oaz_comm_broadcast(comm, buf, nb, W, NULL) == OAZ_ERR_ARG); /* root out of range: local, no collective */
    free(hb);
    /* 6. all-reduce (sum), exact: x_i = (rank + 1) * i + 0.5 -> sum = i * W(W+1)/2 + W/2 */
    const size_t nf = 1000;
    fh = (float*)malloc(nf * sizeof(float));
    /* non-blocking, as a multi-GPU host's streams are: the ranks here share one process, whose legacy
     * default stream (the hipMemcpy calls) would otherwise wait on this stream's pending collective while
     * its peers have not yet issued theirs */
    CHECK(hipStreamCreateWithFlags(&s, 1) == 0);
    for (int pass = 0; pass < 2; ++pass) {
        for (size_t i = 0; i < nf; ++i) fh[i] = (float)((rank + 1) * (int)i) + 0.5f;
        CHECK(hipMemcpy(dev, fh, nf * sizeof(float), 1) == 0);
        if (pass == 0) {
            CHECK(oaz_comm_allreduce_sum_f32(comm, (float*)dev, nf, NULL) == 0 && oaz_comm_sync(comm) == 0);
        } else {
            CHECK(oaz_comm_allreduce_sum_f32(comm, (float*)dev, nf, s) == 0 && hipStreamSynchronize(s) == 0);
        }
        CHECK(hipMemcpy(fh, dev, nf * sizeof(float), 2) == 0);
        for (size_t i = 0; i < nf; ++i) CHECK(fh[i] == (float)((int)i * W * (W + 1) / 2) + 0.5f * (float)W);
    }
    if (g_c4) CHECK(total * sizeof(oaz_sample) > ((size_t)1 << 31)); /* the C4 volume: > 2^31 bytes per rank */
    printf("OK rank %d: %zu own of %zu records (%.3f GB) gathered byte-equal; capacity, failure sentinel, empty, "
           "broadcast x%d, allreduce x2\n", rank, g_count[rank], total, (double)total * sizeof(oaz_sample) * 1e-9, W);
done:
    if (!synced) bar_wait(); /* never leave the others waiting at the first barrier */
    if (s) hipStreamDestroy(s);
    if (comm) oaz_comm_destroy(comm);
    if (buf) hipFree(buf);
    if (dev) hipFree(dev);
    free(host);
    free(fh);
    if (a) oaz_destroy(a);
    if (b) oaz_destroy(b);
    return NULL;
}

int main(int argc, char** argv) {
    W = argc > 1 ? atoi(argv[1]) : 2;
    g_c4 = argc > 2 && strcmp(argv[2], "c4") == 0;
    if (W < 2 || W > MAXW || (argc > 2 && !g_c4)) {
        fprintf(stderr, "usage: comm_multirank W [c4]   (2 <= W <= %d)\n", MAXW);
        return 2;
    }
    int ndev = 0;
    if (oaz_device_count(&ndev) != 0 || ndev == 0) {
        fprintf(stderr, "no GPU\n");
        return 2;
    }
    if (oaz_comm_unique_id(&g_id) != 0) {
        fprintf(stderr, "FAIL unique id: %s\n", oaz_last_error());
        return 1;
    }
    pthread_t th[MAXW];
    for (int r = 0; r < W; ++r) pthread_create(&th[r], NULL, rank_main, (void*)(intptr_t)r);
    for (int r = 0; r < W; ++r) pthread_join(th[r], NULL);
    int fails = 0;
    for (int r = 0; r < W; ++r) fails += g_fail[r];
    for (int r = 0; r < W; ++r) free(g_expect[r]);
    if (fails) return 1;
    printf("OK multirank %d%s (%llu stub collectives, %llu calls returned before their collective ran)\n", W, g_c4 ? " c4" : "",
           (unsigned long long)rccl_stub_ops(), (unsigned long long)rccl_stub_pending_at_return());
    return 0;
}
