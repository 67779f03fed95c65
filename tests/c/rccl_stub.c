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
 * Semantics kept from NCCL: every call of a communicator is collective and must be issued by every
 * rank in the same order with the same sizes / root; inside ncclGroupStart/End the operations are
 * queued and issued at the outermost ncclGroupEnd; ncclBroadcast ignores a non-root's send buffer;
 * in-place forms are allowed. Differences (documented, harmless for the callers under test): each
 * operation completes before the call returns (the caller's stream is synchronised first, so the
 * send data its earlier work produced is ready, and the copies are enqueued on that stream and
 * waited for); a rank whose peers issue a different operation gets ncclInvalidUsage on every rank
 * instead of a hang; a rendezvous that does not complete in STUB_TIMEOUT_S seconds fails with
 * ncclSystemError (every rank waiting alike) instead of blocking forever.
 *
 * Protocol of one operation: sync the stream -> post (kind, buffers, bytes, root) -> barrier ->
 * check that all posts agree -> copy from the peers' buffers (device-to-device, same GPU) [for the
 * all-reduce: read all to host, barrier, write] -> sync -> barrier (no rank may reuse a buffer a
 * peer still reads). */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* HIP calls used (extern "C" in libamdhip64); kind 4 = hipMemcpyDefault (unified addressing). */
typedef void* hipStream_t;
int hipMemcpyAsync(void* dst, const void* src, size_t bytes, int kind, hipStream_t stream);
int hipStreamSynchronize(hipStream_t stream);

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
#define STUB_TIMEOUT_S 120

enum { OP_ALLGATHER = 1, OP_BROADCAST = 2, OP_ALLREDUCE = 3 };
typedef struct {
    int kind, dtype, root;
    const void* send;
    void* recv;
    size_t count;
    hipStream_t stream;
} stub_op;

typedef struct {
    int used, nranks, joined, refs;
    uint64_t key;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int arrived;
    uint64_t gen;
    int failed; /* sticky: a rendezvous timed out */
    stub_op post[STUB_MAX_RANKS];
    double* red[STUB_MAX_RANKS]; /* all-reduce host staging (fp64 so the sum order is exact for tests) */
} stub_world;

typedef struct stub_comm {
    stub_world* w;
    int rank;
} * ncclComm_t;

static stub_world g_worlds[STUB_MAX_WORLDS];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_next_key = 1;
static uint64_t g_ops; /* operations run by this process (reported on stderr at the end) */

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
    pthread_mutex_lock(&g_mu);
    if (--c->w->refs == 0) {
        for (int r = 0; r < STUB_MAX_RANKS; ++r) free(c->w->red[r]);
        c->w->used = 0;
    }
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

/* One collective operation, run by every rank of c's world. */
static ncclResult_t run_op(ncclComm_t c, const stub_op* op) {
    stub_world* w = c->w;
    const int me = c->rank, n = w->nranks;
    const size_t es = dtype_size(op->dtype);
    if (!es) return ncclInvalidArgument;
    if (hipStreamSynchronize(op->stream)) return ncclUnhandledCudaError;
    w->post[me] = *op;
    int rc = wbarrier(w);
    if (rc) return rc;
    for (int r = 0; r < n; ++r) { /* every rank checks every post: all agree on the verdict */
        const stub_op* p = &w->post[r];
        if (p->kind != op->kind || p->dtype != op->dtype || p->count != op->count || p->root != op->root) {
            rc = ncclInvalidUsage;
            break;
        }
    }
    const size_t bytes = op->count * es;
    int hip_err = 0;
    if (!rc && bytes) {
        if (op->kind == OP_ALLGATHER) {
            for (int r = 0; r < n; ++r) {
                char* dst = (char*)op->recv + (size_t)r * bytes;
                if ((const void*)dst != w->post[r].send)
                    hip_err |= hipMemcpyAsync(dst, w->post[r].send, bytes, 4, op->stream);
            }
        } else if (op->kind == OP_BROADCAST) {
            if (op->recv != w->post[op->root].send)
                hip_err |= hipMemcpyAsync(op->recv, w->post[op->root].send, bytes, 4, op->stream);
        } else { /* all-reduce (sum): read every rank's buffer, then (after all reads) write our own */
            double* acc = (double*)calloc(op->count, sizeof(double));
            void* tmp = malloc(bytes);
            for (int r = 0; r < n && !hip_err; ++r) {
                hip_err |= hipMemcpyAsync(tmp, w->post[r].send, bytes, 4, op->stream);
                hip_err |= hipStreamSynchronize(op->stream);
                for (size_t i = 0; i < op->count; ++i)
                    acc[i] += op->dtype == ncclFloat32 ? (double)((const float*)tmp)[i] : ((const double*)tmp)[i];
            }
            rc = wbarrier(w);
            if (!rc && !hip_err) {
                for (size_t i = 0; i < op->count; ++i) {
                    if (op->dtype == ncclFloat32)
                        ((float*)tmp)[i] = (float)acc[i];
                    else
                        ((double*)tmp)[i] = acc[i];
                }
                hip_err |= hipMemcpyAsync(op->recv, tmp, bytes, 4, op->stream);
                hip_err |= hipStreamSynchronize(op->stream);
            }
            free(acc);
            free(tmp);
        }
        hip_err |= hipStreamSynchronize(op->stream);
    }
    const int rc2 = wbarrier(w); /* peers are done reading our buffers */
    __atomic_add_fetch(&g_ops, 1, __ATOMIC_RELAXED);
    if (rc) return rc;
    if (rc2) return rc2;
    return hip_err ? ncclUnhandledCudaError : ncclSuccess;
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

/* Not an RCCL symbol: lets the test confirm that this library, not a real RCCL, served the calls. */
uint64_t rccl_stub_ops(void) { return __atomic_load_n(&g_ops, __ATOMIC_RELAXED); }
