// sharded.hip -- one data part sharded by row range over the GPUs of a node:
// mqvs_comm_* (an RCCL communicator, one rank per GPU) and mqvs_sharded_search.
//
// The reference runs one scan per data part and merges the parts' top-k on
// the host (MergeTreeBaseSearchManager.cpp:207-297; across servers, the
// Distributed engine's per-shard LIMIT + initiator merge, StorageDistributed.cpp).
// Here a part too big or too hot for one GPU is split into granule-aligned row
// ranges, one per rank, each a resident segment with row_offset = its first
// row (ids stay part-global).  A search is:
//   1. cosine only: every rank counts the granule chunks of its range that the
//      reference searches; one all-gather of those counts (8 B per rank) gives
//      each rank its chunk-ordinal base (the query is re-normalised once per
//      searched chunk, VIWithDataPart.h:358, so the ordinal picks the variant);
//   2. the local top-k on every rank (mqvs_search_ex with that base);
//   3. ONE all-gather over xGMI of the per-rank (id, distance) lists,
//      nq*k*12 bytes per rank, grouped as two RCCL calls;
//   4. the device merge by (distance, rank, position) = the unsharded order.
// Every rank ends with the merged result, bit-identical to a single-GPU
// search of the whole part.
//
// RCCL is loaded at first use (dlopen librccl.so.1): PyTorch-ROCm processes
// already hold one, and a process that never shards does not need it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mqvs_internal.h"

namespace mqvs {

struct Rccl {
    void *handle = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char *(*errorString)(ncclResult_t) = nullptr;
};

static Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.handle = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r.handle) break;
        }
        if (!r.handle) return;
        r.getUniqueId = (decltype(r.getUniqueId))dlsym(r.handle, "ncclGetUniqueId");
        r.commInitRank = (decltype(r.commInitRank))dlsym(r.handle, "ncclCommInitRank");
        r.commDestroy = (decltype(r.commDestroy))dlsym(r.handle, "ncclCommDestroy");
        r.allGather = (decltype(r.allGather))dlsym(r.handle, "ncclAllGather");
        r.groupStart = (decltype(r.groupStart))dlsym(r.handle, "ncclGroupStart");
        r.groupEnd = (decltype(r.groupEnd))dlsym(r.handle, "ncclGroupEnd");
        r.errorString = (decltype(r.errorString))dlsym(r.handle, "ncclGetErrorString");
    });
    if (!r.getUniqueId || !r.commInitRank || !r.commDestroy || !r.allGather || !r.groupStart || !r.groupEnd)
        fail(MQVS_ERR_DEVICE, "RCCL (librccl.so.1) not available: the sharded path needs it");
    return r;
}

#define MQVS_RCCL(call)                                                                                     \
    do {                                                                                                    \
        const ncclResult_t rc_ = (call);                                                                    \
        if (rc_ != ncclSuccess)                                                                             \
            fail(MQVS_ERR_DEVICE, std::string(#call) + ": " +                                               \
                                      (rccl().errorString ? rccl().errorString(rc_) : std::to_string(rc_))); \
    } while (0)

// Loopback transport: N virtual ranks of one process on one device (a thread
// per rank), the all-gathers done as device copies through a shared buffer
// between host barriers.  It runs exactly the code of mqvs_sharded_search that
// an RCCL communicator runs, so the multi-rank path is tested on one GPU.
struct LoopGroup {
    int nranks = 0;
    int device = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    void *buf = nullptr;  // shared device buffer, nranks * bytes of the current gather
    size_t cap = 0;
    int refs = 0;
    // every rank of the group waits here; the last arriver runs `last` first
    template <class F>
    void barrier(F &&last) {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            last();
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

}  // namespace mqvs

struct mqvs_comm {
    ncclComm_t comm = nullptr;
    mqvs::LoopGroup *loop = nullptr;  // loopback transport (mqvs_comm_init_loopback)
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;
    mqvs::DevBuf queries, filter, exists, local_ids, local_dist, all_ids, all_dist, out_ids, out_dist, flags, counts,
        scratch, hdr;
    std::mutex mu;  // one search at a time per communicator (RCCL comms are not re-entrant)
};

using namespace mqvs;

namespace {

// all-gather of `bytes` per rank (rank-major into recv), on stream s
void comm_all_gather(mqvs_comm *c, const void *send, void *recv, size_t bytes, hipStream_t s) {
    if (!c->loop) {
        MQVS_RCCL(rccl().allGather(send, recv, bytes, ncclUint8, c->comm, s));
        return;
    }
    LoopGroup &g = *c->loop;
    const size_t need = bytes * (size_t)g.nranks;
    g.barrier([&] {
        if (g.cap < need) {
            if (g.buf) (void)hipFree(g.buf);
            g.buf = nullptr;
            g.cap = 0;
            MQVS_HIP(hipMalloc(&g.buf, need));
            g.cap = need;
        }
    });
    if (bytes) MQVS_HIP(hipMemcpyAsync((char *)g.buf + bytes * c->rank, send, bytes, hipMemcpyDeviceToDevice, s));
    MQVS_HIP(hipStreamSynchronize(s));
    g.barrier([] {});
    if (bytes) MQVS_HIP(hipMemcpyAsync(recv, g.buf, need, hipMemcpyDeviceToDevice, s));
    MQVS_HIP(hipStreamSynchronize(s));
    g.barrier([] {});
}

void comm_group_start(mqvs_comm *c) {
    if (!c->loop) MQVS_RCCL(rccl().groupStart());
}
void comm_group_end(mqvs_comm *c) {
    if (!c->loop) MQVS_RCCL(rccl().groupEnd());
}

// per-rank header of a sharded search, exchanged before any search work:
// the shard's place in the part and this rank's view of the call
enum { kHdrOffset, kHdrRows, kHdrGranule, kHdrDim, kHdrCall, kHdrOk, kHdrChunks, kHdrWords = 8 };

}  // namespace

extern "C" {

int mqvs_comm_unique_id(uint8_t *id) {
    return guarded([&] {
        if (!id) fail(MQVS_ERR_BAD_ARGUMENTS, "null id buffer");
        static_assert(sizeof(ncclUniqueId) == MQVS_COMM_ID_BYTES, "RCCL unique id size");
        ncclUniqueId u;
        MQVS_RCCL(rccl().getUniqueId(&u));
        std::memcpy(id, &u, sizeof(u));
    });
}

int mqvs_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, mqvs_comm_t *out) {
    return guarded([&] {
        if (!out || !id) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        *out = nullptr;
        if (nranks < 1 || rank < 0 || rank >= nranks) fail(MQVS_ERR_BAD_ARGUMENTS, "bad rank / nranks");
        auto *c = new mqvs_comm();
        c->nranks = nranks;
        c->rank = rank;
        try {
            MQVS_HIP(hipGetDevice(&c->device));
            MQVS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            ncclUniqueId u;
            std::memcpy(&u, id, sizeof(u));
            MQVS_RCCL(rccl().commInitRank(&c->comm, nranks, u, rank));
        } catch (...) {
            if (c->stream) (void)hipStreamDestroy(c->stream);
            delete c;
            throw;
        }
        *out = c;
    });
}

int mqvs_comm_init_loopback(int32_t nranks, mqvs_comm_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        if (nranks < 1 || nranks > 64) fail(MQVS_ERR_BAD_ARGUMENTS, "loopback nranks must be in [1, 64]");
        for (int r = 0; r < nranks; ++r) out[r] = nullptr;
        auto *g = new LoopGroup();
        g->nranks = nranks;
        MQVS_HIP(hipGetDevice(&g->device));
        g->refs = nranks;
        for (int r = 0; r < nranks; ++r) {
            auto *c = new mqvs_comm();
            c->nranks = nranks;
            c->rank = r;
            c->device = g->device;
            c->loop = g;
            MQVS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            out[r] = c;
        }
    });
}

int mqvs_comm_free(mqvs_comm_t c) {
    return guarded([&] {
        if (!c) return;
        DeviceGuard guard(c->device);
        if (c->comm) (void)rccl().commDestroy(c->comm);
        DevBuf *all[] = {&c->queries,  &c->filter,  &c->exists,   &c->local_ids, &c->local_dist,
                         &c->all_ids,  &c->all_dist, &c->out_ids, &c->out_dist,  &c->flags,
                         &c->counts,   &c->scratch, &c->hdr};
        for (auto *b : all) b->release();
        if (c->stream) (void)hipStreamDestroy(c->stream);
        if (c->loop) {
            LoopGroup *g = c->loop;
            bool last = false;
            {
                std::lock_guard<std::mutex> lk(g->mu);
                last = --g->refs == 0;
            }
            if (last) {
                if (g->buf) (void)hipFree(g->buf);
                delete g;
            }
        }
        delete c;
    });
}

int mqvs_sharded_search(mqvs_comm_t c, mqvs_segment_t shard, const float *queries, int32_t nq, int32_t k,
                        int32_t metric, const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids,
                        float *out_dist, uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        // (a call that cannot take part in the exchange fails alone)
        if (!c || !shard) fail(MQVS_ERR_BAD_ARGUMENTS, "null communicator or shard");
        if (shard->device != c->device) fail(MQVS_ERR_BAD_ARGUMENTS, "shard and communicator on different devices");
        std::lock_guard<std::mutex> lock(c->mu);
        DeviceGuard guard(c->device);
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        const bool dev = flags & MQVS_F_DEVICE_PTRS;
        const int64_t n = shard->n, bm = (n + 7) / 8;
        const size_t nk = (size_t)std::max(nq, 0) * (size_t)std::max(k, 0);
        // Argument errors of this rank are exchanged in the header, so that
        // every rank fails together instead of the others waiting in a
        // collective this rank never joins.
        std::string local_err;
        int local_code = MQVS_OK;
        const float *dq = queries;
        const uint8_t *dfilter = filter, *dexists = row_exists;
        try {
            if (shard->binary) fail(MQVS_ERR_LOGICAL, "binary segments are not sharded");
            if (nq < 0 || k < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "nq and k must be non-negative");
            if (k > kMaxK) fail(MQVS_ERR_BAD_ARGUMENTS, "k above " + std::to_string(kMaxK) + " not supported");
            if (nq > 0 && k > 0 && (!queries || !out_ids || !out_dist))
                fail(MQVS_ERR_BAD_ARGUMENTS, "null query or output pointer");
            if (!dev) {
                if (nk) {
                    auto *q = (float *)c->queries.get(sizeof(float) * (size_t)nq * shard->d);
                    MQVS_HIP(hipMemcpyAsync(q, queries, sizeof(float) * (size_t)nq * shard->d, hipMemcpyHostToDevice,
                                            s));
                    dq = q;
                }
                if (filter) {
                    auto *f = (uint8_t *)c->filter.get(bm);
                    MQVS_HIP(hipMemcpyAsync(f, filter, bm, hipMemcpyHostToDevice, s));
                    dfilter = f;
                }
                if (row_exists) {
                    auto *f = (uint8_t *)c->exists.get(bm);
                    MQVS_HIP(hipMemcpyAsync(f, row_exists, bm, hipMemcpyHostToDevice, s));
                    dexists = f;
                }
            }
        } catch (const Error &e) {
            local_err = e.msg;
            local_code = e.code;
        }
        // 1. header exchange: shard placement, the call, this rank's state and,
        // for cosine, how many granule chunks of its range the reference
        // searches (the chunk-ordinal base of the ranks above it)
        auto *hd = (int64_t *)c->hdr.get(sizeof(int64_t) * kHdrWords * (size_t)(c->nranks + 1));
        int64_t *mine = hd + (size_t)kHdrWords * c->nranks;
        const int64_t nch = (n + shard->granule - 1) / shard->granule;
        const bool cos_counts = metric == MQVS_METRIC_COSINE && c->nranks > 1 && local_code == MQVS_OK;
        if (cos_counts) {
            launch_count_active_chunks(dfilter, shard->nonempty_bits, dexists, n, shard->granule,
                                       (int *)c->flags.get(sizeof(int) * (size_t)std::max<int64_t>(nch, 1)),
                                       mine + kHdrChunks, s);
            MQVS_HIP(hipGetLastError());
        }
        int64_t h_mine[kHdrWords] = {shard->row_offset, n, shard->granule, shard->d,
                                     ((int64_t)nq << 40) ^ ((int64_t)k << 8) ^ (int64_t)(metric & 0xFF),
                                     local_code == MQVS_OK ? 1 : 0, 0, 0};
        // (the chunk count, when computed, is already in place on the device)
        MQVS_HIP(hipMemcpyAsync(mine, h_mine, sizeof(int64_t) * kHdrChunks, hipMemcpyHostToDevice, s));
        if (!cos_counts) MQVS_HIP(hipMemsetAsync(mine + kHdrChunks, 0, sizeof(int64_t) * 2, s));
        comm_all_gather(c, mine, hd, sizeof(int64_t) * kHdrWords, s);
        std::vector<int64_t> h((size_t)kHdrWords * c->nranks);
        MQVS_HIP(hipMemcpyAsync(h.data(), hd, sizeof(int64_t) * h.size(), hipMemcpyDeviceToHost, s));
        MQVS_HIP(hipStreamSynchronize(s));
        // every rank checks the same table and so decides the same way
        for (int r = 0; r < c->nranks; ++r) {
            const int64_t *x = &h[(size_t)kHdrWords * r];
            if (!x[kHdrOk])
                fail(r == c->rank ? local_code : MQVS_ERR_BAD_ARGUMENTS,
                     r == c->rank ? local_err : "sharded search failed on rank " + std::to_string(r));
        }
        for (int r = 1; r < c->nranks; ++r) {
            const int64_t *a = &h[(size_t)kHdrWords * (r - 1)], *b = &h[(size_t)kHdrWords * r];
            if (b[kHdrOffset] != a[kHdrOffset] + a[kHdrRows])
                fail(MQVS_ERR_BAD_ARGUMENTS, "shards out of row order: rank " + std::to_string(r) + " starts at row " +
                                                 std::to_string(b[kHdrOffset]) + ", rank " + std::to_string(r - 1) +
                                                 " ends at " + std::to_string(a[kHdrOffset] + a[kHdrRows]));
            if (b[kHdrGranule] != a[kHdrGranule] || b[kHdrDim] != a[kHdrDim] || b[kHdrCall] != a[kHdrCall])
                fail(MQVS_ERR_BAD_ARGUMENTS, "ranks disagree on granule, dimension, nq, k or metric");
        }
        if (c->nranks > 1 && h[kHdrGranule] > 0)
            for (int r = 0; r + 1 < c->nranks; ++r)
                if (h[(size_t)kHdrWords * (r + 1) + kHdrOffset] % h[kHdrGranule])
                    fail(MQVS_ERR_BAD_ARGUMENTS, "shard boundaries must be granule aligned");
        int64_t ord_base = -1;
        if (metric == MQVS_METRIC_COSINE && c->nranks > 1) {
            ord_base = 0;
            for (int r = 0; r < c->rank; ++r) ord_base += h[(size_t)kHdrWords * r + kHdrChunks];
        }
        if (nk == 0) return;
        // 2. local top-k (ids part-global: the shard's row_offset applied); a
        // failure still joins the exchange, with its status
        auto *li = (int64_t *)c->local_ids.get(sizeof(int64_t) * nk);
        auto *ld = (float *)c->local_dist.get(sizeof(float) * nk);
        int64_t st_mine = 1;
        try {
            search_segment(shard, dq, nq, k, metric, dfilter, dexists, li, ld,
                           flags & ~(MQVS_F_ASYNC | MQVS_F_DEVICE_PTRS), s, ord_base);
        } catch (const Error &e) {
            local_err = e.msg;
            local_code = e.code;
            st_mine = 0;
        }
        // 3. one exchange: (ids, distances) of every rank, rank-major, and
        // each rank's status
        auto *ai = (int64_t *)c->all_ids.get(sizeof(int64_t) * nk * c->nranks);
        auto *ad = (float *)c->all_dist.get(sizeof(float) * nk * c->nranks);
        int64_t *stv = hd;  // (the header table is no longer needed)
        MQVS_HIP(hipMemcpyAsync(mine, &st_mine, sizeof(int64_t), hipMemcpyHostToDevice, s));
        comm_group_start(c);
        comm_all_gather(c, li, ai, sizeof(int64_t) * nk, s);
        comm_all_gather(c, ld, ad, sizeof(float) * nk, s);
        comm_all_gather(c, mine, stv, sizeof(int64_t), s);
        comm_group_end(c);
        std::vector<int64_t> sts(c->nranks);
        MQVS_HIP(hipMemcpyAsync(sts.data(), stv, sizeof(int64_t) * c->nranks, hipMemcpyDeviceToHost, s));
        MQVS_HIP(hipStreamSynchronize(s));
        for (int r = 0; r < c->nranks; ++r)
            if (!sts[r])
                fail(r == c->rank ? local_code : MQVS_ERR_DEVICE,
                     r == c->rank ? local_err : "sharded search failed on rank " + std::to_string(r));
        // 4. merge by (distance, rank, position): the unsharded order
        int64_t *oi = out_ids;
        float *od = out_dist;
        if (!dev) {
            oi = (int64_t *)c->out_ids.get(sizeof(int64_t) * nk);
            od = (float *)c->out_dist.get(sizeof(float) * nk);
        }
        uint4 *scratch = (int64_t)c->nranks * k > kSortCap
                             ? (uint4 *)c->scratch.get(sizeof(uint4) * 2 * (size_t)c->nranks * k * nq)
                             : nullptr;
        launch_merge_shards(c->nranks, nq, k, metric, ai, ad, oi, od, false, scratch, s);
        MQVS_HIP(hipGetLastError());
        if (!dev) {
            MQVS_HIP(hipMemcpyAsync(out_ids, oi, sizeof(int64_t) * nk, hipMemcpyDeviceToHost, s));
            MQVS_HIP(hipMemcpyAsync(out_dist, od, sizeof(float) * nk, hipMemcpyDeviceToHost, s));
        }
        if (!(dev && (flags & MQVS_F_ASYNC))) MQVS_HIP(hipStreamSynchronize(s));
    });
}

}  // extern "C"
