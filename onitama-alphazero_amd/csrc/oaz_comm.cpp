// oaz_comm.cpp — the multi-GPU exchange of the self-play path over RCCL (xGMI within a node):
// communicator lifecycle, the (s, pi, z) sample all-gather (replaces the buffer join of
// alphazero-training/src/train.rs:241-244), and the in-place all-reduce / broadcast the
// data-parallel trainer and the weight distribution need.
//
// RCCL is loaded on first use with dlopen("librccl.so.1"): a process that already loaded an RCCL
// (e.g. PyTorch's bundled copy, same soname) shares that one, a plain C/Rust host gets the ROCm
// one; engines that never make a communicator never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/onitama_az.h"
#include "oaz_host.h"

static_assert(sizeof(oaz_comm_id) == sizeof(ncclUniqueId), "oaz_comm_id must hold an ncclUniqueId");

namespace {
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*group_start)(void);
    ncclResult_t (*group_end)(void);
    ncclResult_t (*comm_count)(const ncclComm_t, int*);
    const char* (*error_string)(ncclResult_t);
};
Rccl g_rccl;
std::mutex g_rccl_mu;

template <class F>
bool sym(void* h, const char* name, F& f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

int rccl_load() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.tried) return g_rccl.ok ? 0 : oaz_set_err(OAZ_ERR_COMM, "RCCL unavailable (librccl.so.1 did not load)");
    g_rccl.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return oaz_set_err(OAZ_ERR_COMM, "dlopen(librccl.so.1): %s", dlerror());
    Rccl& r = g_rccl;
    r.ok = sym(h, "ncclGetUniqueId", r.get_unique_id) && sym(h, "ncclCommInitRank", r.comm_init_rank) &&
           sym(h, "ncclCommDestroy", r.comm_destroy) && sym(h, "ncclAllGather", r.all_gather) &&
           sym(h, "ncclBroadcast", r.broadcast) && sym(h, "ncclAllReduce", r.all_reduce) &&
           sym(h, "ncclGroupStart", r.group_start) && sym(h, "ncclGroupEnd", r.group_end) &&
           sym(h, "ncclCommCount", r.comm_count) &&
           sym(h, "ncclGetErrorString", r.error_string);
    if (!r.ok) return oaz_set_err(OAZ_ERR_COMM, "librccl.so.1 lacks an expected symbol");
    return 0;
}
}  // namespace

#define NCCL_TRY(expr)                                                                                   \
    do {                                                                                                 \
        ncclResult_t r_ = (expr);                                                                        \
        if (r_ != ncclSuccess)                                                                           \
            return oaz_set_err(OAZ_ERR_COMM, "%s failed: %s (%s:%d)", #expr, g_rccl.error_string(r_),    \
                               __FILE__, __LINE__);                                                      \
    } while (0)

struct oaz_comm {
    ncclComm_t nc = nullptr;
    int rank = 0, world = 1, device = 0;
    hipStream_t stream = nullptr;
    uint64_t* d_counts = nullptr;  // [world] all-gathered sample counts
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // last all-gather: start, counts done, records done
    oaz_comm_stats st{};
};

extern "C" int oaz_comm_unique_id(oaz_comm_id* out) {
    if (!out) return oaz_set_err(OAZ_ERR_ARG, "comm_unique_id: null");
    if (int rc = rccl_load()) return rc;
    ncclUniqueId id;
    NCCL_TRY(g_rccl.get_unique_id(&id));
    memcpy(out->internal, id.internal, sizeof(id.internal));
    return 0;
}

extern "C" void oaz_comm_destroy(oaz_comm* c) {
    if (!c) return;
    DeviceScope dev_scope_(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->nc) (void)g_rccl.comm_destroy(c->nc);
    if (c->d_counts) (void)hipFree(c->d_counts);
    for (auto ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int comm_init(const oaz_comm_id* id, int rank, int world, int device, oaz_comm** out) {
    if (!id || world < 1 || rank < 0 || rank >= world) return oaz_set_err(OAZ_ERR_ARG, "comm_init: rank %d of %d", rank, world);
    if (int rc = rccl_load()) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return oaz_set_err(OAZ_ERR_NO_DEVICE, "comm_init: no HIP device");
    if (device < 0 || device >= ndev) return oaz_set_err(OAZ_ERR_ARG, "comm_init: device %d of %d", device, ndev);
    oaz_comm* c = new oaz_comm();
    *out = c;
    c->rank = rank;
    c->world = world;
    c->device = device;
    OAZ_ON_DEVICE(device);
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(hipMalloc((void**)&c->d_counts, (size_t)world * sizeof(uint64_t)));
    for (auto& ev : c->ev) HIP_TRY(hipEventCreate(&ev));
    ncclUniqueId uid;
    memcpy(uid.internal, id->internal, sizeof(uid.internal));
    NCCL_TRY(g_rccl.comm_init_rank(&c->nc, world, uid, rank));
    int n = 0;
    NCCL_TRY(g_rccl.comm_count(c->nc, &n));
    if (n != world) return oaz_set_err(OAZ_ERR_COMM, "comm_init: RCCL communicator holds %d ranks, expected %d", n, world);
    c->st.ranks = n;
    c->st.rank = rank;
    return 0;
}

extern "C" oaz_comm* oaz_comm_init(const oaz_comm_id* id, int rank, int world, int device) {
    oaz_comm* c = nullptr;
    if (int rc = comm_init(id, rank, world, device, &c)) {
        (void)rc;
        oaz_comm_destroy(c);
        return nullptr;
    }
    return c;
}

extern "C" int oaz_comm_sync(oaz_comm* c) {
    if (!c) return oaz_set_err(OAZ_ERR_ARG, "comm_sync: null");
    OAZ_ON_DEVICE(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int oaz_comm_stats_get(oaz_comm* c, oaz_comm_stats* out) {
    if (!c || !out) return oaz_set_err(OAZ_ERR_ARG, "comm_stats: null");
    int n = 0;
    NCCL_TRY(g_rccl.comm_count(c->nc, &n));
    c->st.ranks = n;
    *out = c->st;
    return 0;
}

// A rank whose own part fails before the exchange (bad engine / device, the sample peek) still joins
// the counts all-gather with this count, so every rank sees the failure and returns an error instead
// of the others blocking in the collective.
static constexpr uint64_t kLocalFailure = UINT64_MAX;

extern "C" int oaz_allgather_samples(oaz_engine* eng, oaz_comm* c, oaz_sample* dev_out, size_t cap, size_t* n_total,
                                     uint64_t* counts_out) {
    if (!c) return oaz_set_err(OAZ_ERR_ARG, "allgather_samples: null communicator");
    const oaz_sample* src = nullptr;
    size_t n = 0;
    int dev = c->device, rc_local = 0;
    std::string why;
    if (!eng || (!dev_out && cap)) {
        rc_local = oaz_set_err(OAZ_ERR_ARG, "allgather_samples: bad arguments");
    } else if ((rc_local = oaz_engine_samples_peek(eng, &src, &n, &dev)) == 0 && dev != c->device) {
        rc_local = oaz_set_err(OAZ_ERR_ARG, "allgather_samples: engine on GPU %d, comm on GPU %d", dev, c->device);
    }
    if (rc_local) why = oaz_last_error();
    OAZ_ON_DEVICE(c->device);
    // 1. counts (every rank joins, also after a local failure)
    const uint64_t mine = rc_local ? kLocalFailure : (uint64_t)n;
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_counts + c->rank, &mine, sizeof(mine), hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(g_rccl.all_gather(c->d_counts + c->rank, c->d_counts, 1, ncclUint64, c->nc, c->stream));
    std::vector<uint64_t> counts((size_t)c->world);
    HIP_TRY(hipMemcpyAsync(counts.data(), c->d_counts, counts.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (rc_local) return oaz_set_err(rc_local, "%s", why.c_str());
    uint64_t total = 0;
    for (int r = 0; r < c->world; ++r) {
        if (counts[r] == kLocalFailure)  // every rank sees the same counts: all fail alike, nothing consumed
            return oaz_set_err(OAZ_ERR_COMM, "allgather_samples: rank %d failed before the exchange", r);
        total += counts[r];
    }
    if (counts[c->rank] != mine) return oaz_set_err(OAZ_ERR_COMM, "allgather_samples: own count not gathered");
    if (counts_out) memcpy(counts_out, counts.data(), counts.size() * sizeof(uint64_t));
    if (n_total) *n_total = (size_t)total;
    if (total > cap)  // every rank sees the same counts: all fail alike, nothing consumed
        return oaz_set_err(OAZ_ERR_CAPACITY, "allgather_samples: %llu samples over all ranks > cap %zu",
                           (unsigned long long)total, cap);
    // 2. one broadcast per rank into its offset (grouped: an all-gatherv without padding)
    NCCL_TRY(g_rccl.group_start());
    uint64_t off = 0;
    for (int r = 0; r < c->world; ++r) {
        if (counts[r]) {
            const void* send = r == c->rank ? (const void*)src : (const void*)(dev_out + off);
            ncclResult_t res = g_rccl.broadcast(send, dev_out + off, counts[r] * sizeof(oaz_sample), ncclUint8, r,
                                                c->nc, c->stream);
            if (res != ncclSuccess) {
                (void)g_rccl.group_end();
                return oaz_set_err(OAZ_ERR_COMM, "ncclBroadcast(root %d): %s", r, g_rccl.error_string(res));
            }
        }
        off += counts[r];
    }
    NCCL_TRY(g_rccl.group_end());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    float ms_counts = 0.f, ms_data = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms_counts, c->ev[0], c->ev[1]));
    HIP_TRY(hipEventElapsedTime(&ms_data, c->ev[1], c->ev[2]));
    c->st.allgather_calls += 1;
    c->st.counts_ms = ms_counts;
    c->st.allgather_ms = ms_data;
    c->st.allgather_records = total;
    c->st.allgather_bytes = total * sizeof(oaz_sample);
    c->st.own_records = mine;
    return oaz_engine_samples_consume(eng, n);
}

extern "C" int oaz_comm_allreduce_sum_f32(oaz_comm* c, float* dev, size_t n, void* stream) {
    if (!c || (!dev && n)) return oaz_set_err(OAZ_ERR_ARG, "allreduce: bad arguments");
    OAZ_ON_DEVICE(c->device);
    NCCL_TRY(g_rccl.all_reduce(dev, dev, n, ncclFloat32, ncclSum, c->nc, stream ? (hipStream_t)stream : c->stream));
    return 0;
}

extern "C" int oaz_comm_broadcast(oaz_comm* c, void* dev, size_t bytes, int root, void* stream) {
    if (!c || (!dev && bytes) || root < 0 || root >= c->world) return oaz_set_err(OAZ_ERR_ARG, "broadcast: bad arguments");
    OAZ_ON_DEVICE(c->device);
    NCCL_TRY(g_rccl.broadcast(dev, dev, bytes, ncclUint8, root, c->nc, stream ? (hipStream_t)stream : c->stream));
    return 0;
}
