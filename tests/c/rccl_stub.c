/* rccl_stub.c — test double for librccl.so.1: the 10 RCCL entry points csrc/oaz_comm.cpp resolves
 * (oaz_comm.cpp:55-60), implemented for ranks that are HOST THREADS OF ONE PROCESS sharing GPU 0.
 *
 * Purpose: run the product exchange (oaz_allgather_samples, oaz_comm_broadcast,
 * oaz_comm_allreduce_sum_f32 — the replacement of the reference's buffer join,
 * alphazero-training/src/train.rs:241-244) at world > 1 on a one-GPU box, where real RCCL cannot
 * form a multi-rank communicator. Test infrastructure only: built by tests/test_c_abi.py (gcc, like
 * abi_smoke.c) into a temporary directory as `librccl.so.1` and put first on LD_LIBRARY_PATH of a
 * plain C process (tests/c/comm_multirank.c) that never loads torch's RCCL. libonitama_az.so has a
 * RUNPATH, not an RPATH, so LD_LIBRARY_PATH wins its dlopen("librccl.so.1").
 *
 * Stream semantics are RCCL's: a collective is ENQUEUED on the caller's stream and the call returns
 * without waiting for the GPU (no stream or device synchronisation anywhere in a collective call). Its
 * copies read the send buffers when the streams reach them (after the work each rank enqueued before its
 * call) and every rank's later stream work runs after them. Mechanism: the ranks' calls meet on the host
 * (a barrier, so each learns the others' buffers and events; real RCCL meets on the GPU instead); each
 * rank's stream waits for the peers' "ready" events (recorded at their calls), runs the copies
 * (device-to-device, same GPU; the all-reduce stages the peers' buffers in pinned memory and sums them in
 * a host function on the stream, in rank order and fp64 so the sums are exact for the tests), records a
 * "done" event, and waits for the peers' "done" events (no rank's later work may overwrite a buffer a
 * peer still reads). Every GPU-side wait is on an event recorded before it was enqueued, so ranks whose
 * streams share a hardware queue cannot deadlock (a wait on a FUTURE host release — a flag a proxy would
 * write later — can: the HIP runtime multiplexes a process's streams onto 4 hardware queues).
 * rccl_stub_pending_at_return() counts the calls that returned while their copies were still pending on
 * the GPU: the proof that the callers' stream ordering, not a synchronous double, made their results right.
 * RCCL_STUB_DELAY_US=n puts an n-microsecond host function (a sleep) on the stream before each operation's
 * copies, so that every call returns long before its data moves: a caller that reads a result without
 * ordering itself after the collective on the stream then reads stale data.
 *
 * Semantics kept from NCCL: every call of a communicator is collective and must be issued by every
 * rank in the same order with the same sizes / root; inside ncclGroupStart/End the operations are
 * queued and issued at the outermost ncclGroupEnd; ncclBroadcast ignores a non-root's send buffer;
 * in-place forms are allowed. Differences (harmless for the callers under test): a call returns once
 * every rank has issued it (the host rendezvous); a rank whose peers issue a different operation gets
 * ncclInvalidUsage on every rank instead of a hang; a rendezvous that does not complete in STUB_TIMEOUT_S
 * seconds fails with ncclSystemError instead of blocking forever.
 *
 * Protocol of one operation, rank r: record ready_r -> post (kind, buffers, bytes, root, ready_r) ->
 * barrier -> check that all posts agree -> wait ready_p of the peers read -> copies [all-reduce: copies
 * to pinned staging, record read_r, barrier, wait read_p of every peer, host sum, copy back] -> record
 * done_r -> barrier -> wait done_p of every peer -> barrier (events released). */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

/* HIP calls used (extern "C" in libamdhip64); kind 4 = hipMemcpyDefault (unified addressing). */
typedef void* hipStream_t;
typedef void* hipEvent_t;
typedef void (*hipHostFn_t)(void* user);
int hipMemcpyAsync(void* dst, const void* src, size_t bytes, int kind, hipStream_t stream);
int hipEventCreateWithFlags(hipEvent_t* ev, unsigned flags);
int hipEventRecord(hipEvent_t ev, hipStream_t stream);
int hipEventQuery(hipEvent_t ev);
int hipEventSynchronize(hipEvent_t ev);
int hipEventDestroy(hipEvent_t ev);
int hipStreamWaitEvent(hipStream_t stream, hipEvent_t ev, unsigned flags);
int hipLaunchHostFunc(hipStream_t stream, hipHostFn_t fn, void* user);
int hipHostMalloc(void** p, size_t bytes, unsigned flags);
int hipHostFree(void* p);
#define HIP_EVENT_DISABLE_TIMING 0x2

typedef int ncclResult_t; /* rccl.h values */
enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
       ncclInvalidArgument = 4, ncclInvalidUsage = 5 };
enum { ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5, ncclFloat32 = 7,
       ncclFloat64 = 8 };
enum { ncclSum = 0 };
typedef struct { char internal[128]; } ncclUniqueId;

#define STUB_MAX_RANKS 16
#define STUB_MAX_WORLDS 16
#define STUB_MAX_GROUP 256
#define STUB_TIMEOUT_S 60

enum { OP_ALLGATHER = 1, OP_BROADCAST = 2, OP_ALLREDUCE = 3 };
typedef struct {
    int kind, dtype, root;
    const void* send;
    void* recv;
    size_t count;
    hipStream_t stream;
} stub_op;

/* what a rank posts for one operation */
typedef struct {
    stub_op op;
    hipEvent_t ready, read, done;
} stub_post;

typedef struct {
    int used, nranks, joined, refs;
    uint64_t key;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int arrived;
    uint64_t gen;
    int failed; /* sticky: a rendezvous timed out */
    stub_post post[STUB_MAX_RANKS];
} stub_world;

/* all-reduce host sum, run as a host function on the caller's stream (no HIP calls inside) */
typedef struct stub_sum {
    int n, f32;
    size_t count;
    void* staging; /* pinned: n rank buffers, rank order */
    void* out;     /* pinned */
    hipEvent_t fin;
    struct stub_sum* next;
} stub_sum;

typedef struct stub_comm {
    stub_world* w;
    int rank;
    stub_sum* sums; /* pinned buffers of the all-reduces, freed at destroy once their streams passed */
} * ncclComm_t;

static stub_world g_worlds[STUB_MAX_WORLDS];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_next_key = 1;
static uint64_t g_ops;     /* operations run by this process */
static uint64_t g_pending; /* operations whose copies were still pending on the GPU when the call returned */

static __thread int t_group_depth;
static __thread int t_group_n;
static __thread ncclComm_t t_group_comm[STUB_MAX_GROUP];
static __thread stub_op t_group_ops[STUB_MAX_GROUP];

static const uint64_t kMagic = 0x4255545343434152ull; /* "RCCLSTUB" */

/* Barrier with a timeout; returns 0 or ncclSystemError (and marks the world failed). */
static int wbarrier(stub_world* w) {
    pthread_mutex_lock(&w->mu);
    if (w->failed) {
        pthread_mutex_unlock(&w->mu);
        return ncclSystemError;
    }
    const uint64_t gen = w->gen;
    if (++w->arrived == w->nranks) {
        w->arrived = 0;
        w->gen++;
        pthread_cond_broadcast(&w->cv);
        pthread_mutex_unlock(&w->mu);
        return 0;
    }
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    ts.tv_sec += STUB_TIMEOUT_S;
    while (w->gen == gen && !w->failed) {
        if (pthread_cond_timedwait(&w->cv, &w->mu, &ts) != 0 && w->gen == gen) {
            w->failed = 1;
            pthread_cond_broadcast(&w->cv);
            fprintf(stderr, "rccl_stub: rendezvous timed out after %d s\n", STUB_TIMEOUT_S);
        }
    }
    const int rc = (w->gen == gen) ? ncclSystemError : 0;
    pthread_mutex_unlock(&w->mu);
    return rc;
}

static size_t dtype_size(int t) {
    switch (t) {
        case ncclUint8: return 1;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

static void host_sleep(void* user) { usleep((useconds_t)(uintptr_t)user); }
static unsigned delay_us(void) {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("RCCL_STUB_DELAY_US");
        v = e ? atoi(e) : 0;
        if (v < 0 || v > 1000000) v = 0;
    }
    return (unsigned)v;
}

static void host_sum(void* user) {
    const stub_sum* s = (const stub_sum*)user;
    for (size_t i = 0; i < s->count; ++i) {
        double acc = 0.0;
        for (int r = 0; r < s->n; ++r)
            acc += s->f32 ? (double)((const float*)s->staging)[(size_t)r * s->count + i]
                          : ((const double*)s->staging)[(size_t)r * s->count + i];
        if (s->f32)
            ((float*)s->out)[i] = (float)acc;
        else
            ((double*)s->out)[i] = acc;
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof(*id));
    pthread_mutex_lock(&g_mu);
    const uint64_t key = g_next_key++;
    pthread_mutex_unlock(&g_mu);
    memcpy(id->internal, &kMagic, 8);
    memcpy(id->internal + 8, &key, 8);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    uint64_t magic = 0, key = 0;
    memcpy(&magic, id.internal, 8);
    memcpy(&key, id.internal + 8, 8);
    if (!comm || magic != kMagic || nranks < 1 || nranks > STUB_MAX_RANKS || rank < 0 || rank >= nranks)
        return ncclInvalidArgument;
    pthread_mutex_lock(&g_mu);
    stub_world* w = NULL;
    for (int i = 0; i < STUB_MAX_WORLDS && !w; ++i)
        if (g_worlds[i].used && g_worlds[i].key == key) w = &g_worlds[i];
    for (int i = 0; i < STUB_MAX_WORLDS && !w; ++i)
        if (!g_worlds[i].used) {
            w = &g_worlds[i];
            memset(w, 0, sizeof(*w));
            w->used = 1;
            w->key = key;
            w->nranks = nranks;
            pthread_mutex_init(&w->mu, NULL);
            pthread_cond_init(&w->cv, NULL);
        }
    if (!w || w->nranks != nranks || (w->joined >> rank) & 1) {
        pthread_mutex_unlock(&g_mu);
        return ncclInvalidUsage;
    }
    w->joined |= 1 << rank;
    w->refs++;
    pthread_mutex_unlock(&g_mu);
    ncclComm_t c = (ncclComm_t)calloc(1, sizeof(*c));
    c->w = w;
    c->rank = rank;
    const int rc = wbarrier(w); /* blocks until every rank joined, as ncclCommInitRank does */
    if (rc) {
        free(c);
        return rc;
    }
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    for (stub_sum* s = c->sums; s;) {
        stub_sum* nx = s->next;
        (void)hipEventSynchronize(s->fin); /* the stream has passed the host sum and the copy back */
        (void)hipEventDestroy(s->fin);
        (void)hipHostFree(s->staging);
        (void)hipHostFree(s->out);
        free(s);
        s = nx;
    }
    pthread_mutex_lock(&g_mu);
    if (--c->w->refs == 0) c->w->used = 0;
    pthread_mutex_unlock(&g_mu);
    free(c);
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t c, int* count) {
    if (!c || !count) return ncclInvalidArgument;
    *count = c->w->nranks;
    return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (rccl_stub)";
        case ncclUnhandledCudaError: return "unhandled HIP error (rccl_stub)";
        case ncclSystemError: return "rendezvous timed out (rccl_stub)";
        case ncclInvalidArgument: return "invalid argument (rccl_stub)";
        case ncclInvalidUsage: return "ranks issued different operations (rccl_stub)";
        default: return "internal error (rccl_stub)";
    }
}

static hipEvent_t mkevent(int* err) {
    hipEvent_t e = NULL;
    if (hipEventCreateWithFlags(&e, HIP_EVENT_DISABLE_TIMING)) *err = 1;
    return e;
}

/* One collective operation, enqueued by every rank of c's world on its own stream (see the header). */
static ncclResult_t run_op(ncclComm_t c, const stub_op* op) {
    stub_world* w = c->w;
    const int me = c->rank, n = w->nranks;
    const size_t es = dtype_size(op->dtype);
    if (!es) return ncclInvalidArgument;
    hipStream_t st = op->stream;
    int he = 0;
    stub_post mine = {*op, mkevent(&he), NULL, NULL};
    if (!he) he |= hipEventRecord(mine.ready, st);
    w->post[me] = mine;
    int rc = wbarrier(w);
    if (rc) goto out;
    for (int r = 0; r < n; ++r) { /* every rank checks every post: all agree on the verdict */
        const stub_op* p = &w->post[r].op;
        if (p->kind != op->kind || p->dtype != op->dtype || p->count != op->count || p->root != op->root) {
            rc = ncclInvalidUsage;
            break;
        }
    }
    const size_t bytes = op->count * es;
    if (!rc && bytes && delay_us()) he |= hipLaunchHostFunc(st, host_sleep, (void*)(uintptr_t)delay_us());
    if (!rc && bytes) {
        if (op->kind == OP_ALLGATHER) {
            for (int r = 0; r < n; ++r) {
                char* dst = (char*)op->recv + (size_t)r * bytes;
                if ((const void*)dst == w->post[r].op.send) continue;
                if (r != me) he |= hipStreamWaitEvent(st, w->post[r].ready, 0);
                he |= hipMemcpyAsync(dst, w->post[r].op.send, bytes, 4, st);
            }
        } else if (op->kind == OP_BROADCAST) {
            const int rt = op->root;
            if (op->recv != w->post[rt].op.send) {
                if (rt != me) he |= hipStreamWaitEvent(st, w->post[rt].ready, 0);
                he |= hipMemcpyAsync(op->recv, w->post[rt].op.send, bytes, 4, st);
            }
        } else { /* all-reduce (sum): every rank's buffer to pinned staging, then (after every rank read ours) the sum */
            stub_sum* s = (stub_sum*)calloc(1, sizeof(*s));
            s->n = n;
            s->f32 = op->dtype == ncclFloat32;
            s->count = op->count;
            he |= hipHostMalloc(&s->staging, bytes * (size_t)n, 0);
            he |= hipHostMalloc(&s->out, bytes, 0);
            s->fin = mkevent(&he);
            s->next = c->sums;
            c->sums = s;
            for (int r = 0; r < n && !he; ++r) {
                if (r != me) he |= hipStreamWaitEvent(st, w->post[r].ready, 0);
                he |= hipMemcpyAsync((char*)s->staging + (size_t)r * bytes, w->post[r].op.send, bytes, 4, st);
            }
            w->post[me].read = mkevent(&he);
            if (!he) he |= hipEventRecord(w->post[me].read, st);
            rc = wbarrier(w);
            if (rc) goto out;
            for (int r = 0; r < n && !he; ++r)
                if (r != me) he |= hipStreamWaitEvent(st, w->post[r].read, 0);
            if (!he) he |= hipLaunchHostFunc(st, host_sum, s);
            if (!he) he |= hipMemcpyAsync(op->recv, s->out, bytes, 4, st);
            if (!he) he |= hipEventRecord(s->fin, st);
        }
    }
    w->post[me].done = mkevent(&he);
    if (!he) he |= hipEventRecord(w->post[me].done, st);
    {
        const int rc2 = wbarrier(w); /* every rank's copies are enqueued */
        if (!rc) rc = rc2;
    }
    if (!rc)
        for (int r = 0; r < n; ++r) /* peers done reading our buffers before our later work */
            if (r != me && w->post[r].done) he |= hipStreamWaitEvent(st, w->post[r].done, 0);
    if (!rc && !he && bytes && hipEventQuery(w->post[me].done) != 0) __atomic_add_fetch(&g_pending, 1, __ATOMIC_RELAXED);
    {
        const int rc3 = wbarrier(w); /* nobody refers to another rank's events any more */
        if (!rc) rc = rc3;
    }
    __atomic_add_fetch(&g_ops, 1, __ATOMIC_RELAXED);
out:
    if (w->post[me].ready) (void)hipEventDestroy(w->post[me].ready);
    if (w->post[me].read) (void)hipEventDestroy(w->post[me].read);
    if (w->post[me].done) (void)hipEventDestroy(w->post[me].done);
    memset(&w->post[me], 0, sizeof(w->post[me]));
    if (rc) return rc;
    return he ? ncclUnhandledCudaError : ncclSuccess;
}

static ncclResult_t submit(ncclComm_t c, const stub_op* op) {
    if (!c) return ncclInvalidArgument;
    if (t_group_depth > 0) {
        if (t_group_n >= STUB_MAX_GROUP) return ncclInvalidUsage;
        t_group_comm[t_group_n] = c;
        t_group_ops[t_group_n++] = *op;
        return ncclSuccess;
    }
    return run_op(c, op);
}

ncclResult_t ncclGroupStart(void) {
    t_group_depth++;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void) {
    if (t_group_depth <= 0) return ncclInvalidUsage;
    if (--t_group_depth > 0) return ncclSuccess;
    ncclResult_t rc = ncclSuccess;
    const int n = t_group_n;
    t_group_n = 0;
    for (int i = 0; i < n; ++i) {
        const ncclResult_t r = run_op(t_group_comm[i], &t_group_ops[i]);
        if (r && !rc) rc = r;
    }
    return rc;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, int dtype, ncclComm_t c, hipStream_t s) {
    if ((!send || !recv) && count) return ncclInvalidArgument;
    stub_op op = {OP_ALLGATHER, dtype, 0, send, recv, count, s};
    return submit(c, &op);
}

ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, int dtype, int root, ncclComm_t c,
                           hipStream_t s) {
    if (!c || root < 0 || root >= c->w->nranks || (!recv && count) || (c->rank == root && !send && count))
        return ncclInvalidArgument;
    stub_op op = {OP_BROADCAST, dtype, root, send, recv, count, s};
    return submit(c, &op);
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int redop, ncclComm_t c,
                           hipStream_t s) {
    if ((!send || !recv) && count) return ncclInvalidArgument;
    if (redop != ncclSum || (dtype != ncclFloat32 && dtype != ncclFloat64)) return ncclInvalidArgument;
    stub_op op = {OP_ALLREDUCE, dtype, 0, send, recv, count, s};
    return submit(c, &op);
}

/* Not RCCL symbols: let the test confirm that this library, not a real RCCL, served the calls, and that
 * the calls returned before their copies had run. */
uint64_t rccl_stub_ops(void) { return __atomic_load_n(&g_ops, __ATOMIC_RELAXED); }
uint64_t rccl_stub_pending_at_return(void) { return __atomic_load_n(&g_pending, __ATOMIC_RELAXED); }
