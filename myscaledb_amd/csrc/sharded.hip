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
//      reference searches (the query is re-normalised once per searched
//      chunk, VIWithDataPart.h:358, so the ranks below fix a shard's
//      chunk-ordinal base, i.e. its query variant);
//   2. the local top-k on every rank (mqvs_search_ex with that base);
//   3. the exchange over xGMI: a 128-B header per rank (shard placement, the
//      call, outcome, fallback flags, chunk count), then the per-rank
//      (id, distance) lists, nq*k*12 bytes per rank, as one RCCL group (the
//      same two collectives on every path, so ranks on different paths
//      still pair their operations);
//   4. the device merge by (distance, rank, position) = the unsharded order.
// Every rank ends with the merged result, bit-identical to a single-GPU
// search of the whole part.
//
// Host round trips.  A call equal to the last call all ranks validated
// together (same shard, nq, k, metric, bitmaps present) takes the FAST path:
// 1-4 are enqueued back to back (the local search without its own sync, the
// cosine base taken from the last validated call) and the host synchronises
// ONCE, to read the exchanged table -- every rank reads the same table and so
// decides alike: done; or fail everywhere (a rank's error); or, when a local
// search needed a host-driven fallback or a cosine base was wrong (PREWHERE
// filters that empty whole chunks), re-run on the validated path together.
// The VALIDATED path (first call, changed call, re-run) allocates everything
// first, exchanges the header and synchronises (shard order, agreement on the
// call, statuses, exact cosine bases), runs the local search with its
// fallbacks, exchanges lists + statuses and synchronises again.  A rank that
// fails at any step still joins every exchange, so no rank is left waiting
// in a collective.
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
// per rank), the all-gathers done as device copies through a shared buffer.
// It runs exactly the code of mqvs_sharded_search that an RCCL communicator
// runs, so the multi-rank path is tested on one GPU.  Like an RCCL
// collective, a gather is only ENQUEUED: the ranks meet at host barriers to
// publish their events, but no rank synchronises its stream -- each stream
// waits on device for the other ranks' copy-in events before its copy-out
// (and, before overwriting the buffer, for their copy-outs of the last
// gather).  A caller that read a result before its stream got there would
// see it here as it would on RCCL.
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
    std::vector<hipEvent_t> in_ev, out_ev;  // per rank: its copy into buf done; its copy out of buf done
    int err_code = MQVS_OK;  // failure of the `last` step of generation err_gen
    std::string err_msg;
    uint64_t err_gen = ~(uint64_t)0;
    // every rank of the group waits here; the last arriver runs `last` first.
    // A failing `last` still releases the group, and every rank then fails
    // with its error (none is left waiting for a generation that never ends).
    template <class F>
    void barrier(F &&last) {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            try {
                last();
            } catch (const Error &e) {
                err_code = e.code;
                err_msg = e.msg;
                err_gen = gen;
            } catch (...) {
                err_code = MQVS_ERR_DEVICE;
                err_msg = "loopback exchange failed";
                err_gen = gen;
            }
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
        if (err_gen == gen) fail(err_code, err_msg);
    }
};

}  // namespace mqvs

// The last call every rank validated together (the fast path's key): set and
// cleared only from exchanged tables, which every rank reads alike, so all
// ranks hold the same validation state.
struct ShardCall {
    bool valid = false;
    const void *shard = nullptr;
    int64_t row_offset = 0, rows = 0, nq = 0, k = 0, metric = 0, d = 0;
    bool filter = false, exists = false, dev = false;
    int64_t ord_base = -1;  // cosine, no PREWHERE filter: the verified chunk-ordinal base
    bool same(const ShardCall &o) const {
        return valid && o.shard == shard && o.row_offset == row_offset && o.rows == rows && o.nq == nq &&
               o.k == k && o.metric == metric && o.d == d && o.filter == filter && o.exists == exists &&
               o.dev == dev;
    }
};

struct mqvs_comm {
    ncclComm_t comm = nullptr;
    mqvs::LoopGroup *loop = nullptr;  // loopback transport (mqvs_comm_init_loopback)
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;
    mqvs::DevBuf queries, filter, exists, local_ids, local_dist, all_ids, all_dist, out_ids, out_dist, flags, counts,
        scratch, hdr;
    int64_t *h_hdr = nullptr;  // pinned: this rank's header [kHdrWords], then the table [nranks][kHdrWords]
    ShardCall last;
    int64_t fast_calls = 0, redo_calls = 0;  // mqvs_comm_stats
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
            // (a larger buffer: the last gather's copies out of the old one
            // finish first -- the only host wait of the transport)
            for (hipEvent_t e : g.out_ev) MQVS_HIP(hipEventSynchronize(e));
            if (g.buf) (void)hipFree(g.buf);
            g.buf = nullptr;
            g.cap = 0;
            MQVS_HIP(hipMalloc(&g.buf, need));
            g.cap = need;
        }
    });
    // every rank has recorded its copy-out of the last gather (before this
    // barrier): the buffer is free once the streams pass those events
    for (int r = 0; r < g.nranks; ++r)
        if (r != c->rank) MQVS_HIP(hipStreamWaitEvent(s, g.out_ev[r], 0));
    if (bytes) MQVS_HIP(hipMemcpyAsync((char *)g.buf + bytes * c->rank, send, bytes, hipMemcpyDeviceToDevice, s));
    MQVS_HIP(hipEventRecord(g.in_ev[c->rank], s));
    g.barrier([] {});
    for (int r = 0; r < g.nranks; ++r)
        if (r != c->rank) MQVS_HIP(hipStreamWaitEvent(s, g.in_ev[r], 0));
    if (bytes) MQVS_HIP(hipMemcpyAsync(recv, g.buf, need, hipMemcpyDeviceToDevice, s));
    MQVS_HIP(hipEventRecord(g.out_ev[c->rank], s));
}

void comm_group_start(mqvs_comm *c) {
    if (!c->loop) MQVS_RCCL(rccl().groupStart());
}
void comm_group_end(mqvs_comm *c) {
    if (!c->loop) MQVS_RCCL(rccl().groupEnd());
}

// per-rank header of a sharded search: the shard's place in the part, this
// rank's view of the call and its outcome.  kHdrFast: the rank took the fast
// path; kHdrOrd: the cosine chunk-ordinal base it searched with; kHdrFlags:
// its local search's fallback flags (an int in the low half); kHdrNk: nq * k;
// kHdrCode: the status code of a failed rank.
enum {
    kHdrOffset,
    kHdrRows,
    kHdrGranule,
    kHdrDim,
    kHdrCall,
    kHdrOk,
    kHdrChunks,
    kHdrFast,
    kHdrOrd,
    kHdrFlags,
    kHdrNk,
    kHdrCode,
    kHdrWords = 16
};

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
            MQVS_HIP(hipHostMalloc((void **)&c->h_hdr, sizeof(int64_t) * kHdrWords * (size_t)(nranks + 1),
                                   hipHostMallocDefault));
            c->hdr.get(sizeof(int64_t) * kHdrWords * (size_t)(nranks + 1));
            ncclUniqueId u;
            std::memcpy(&u, id, sizeof(u));
            MQVS_RCCL(rccl().commInitRank(&c->comm, nranks, u, rank));
        } catch (...) {
            if (c->stream) (void)hipStreamDestroy(c->stream);
            if (c->h_hdr) (void)hipHostFree(c->h_hdr);
            c->hdr.release();
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
        g->in_ev.assign(nranks, nullptr);
        g->out_ev.assign(nranks, nullptr);
        for (int r = 0; r < nranks; ++r) {
            MQVS_HIP(hipEventCreateWithFlags(&g->in_ev[r], hipEventDisableTiming));
            MQVS_HIP(hipEventCreateWithFlags(&g->out_ev[r], hipEventDisableTiming));
        }
        for (int r = 0; r < nranks; ++r) {
            auto *c = new mqvs_comm();
            c->nranks = nranks;
            c->rank = r;
            c->device = g->device;
            c->loop = g;
            out[r] = c;
            MQVS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            MQVS_HIP(hipHostMalloc((void **)&c->h_hdr, sizeof(int64_t) * kHdrWords * (size_t)(nranks + 1),
                                   hipHostMallocDefault));
            c->hdr.get(sizeof(int64_t) * kHdrWords * (size_t)(nranks + 1));
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
        if (c->h_hdr) (void)hipHostFree(c->h_hdr);
        if (c->loop) {
            LoopGroup *g = c->loop;
            bool last = false;
            {
                std::lock_guard<std::mutex> lk(g->mu);
                last = --g->refs == 0;
            }
            if (last) {
                for (hipEvent_t e : g->out_ev)
                    if (e) (void)hipEventSynchronize(e);
                if (g->buf) (void)hipFree(g->buf);
                for (auto *v : {&g->in_ev, &g->out_ev})
                    for (hipEvent_t e : *v)
                        if (e) (void)hipEventDestroy(e);
                delete g;
            }
        }
        delete c;
    });
}

}  // extern "C"

namespace {

// this rank's header words (the outcome fields ok / code / flags as given)
void fill_header(int64_t *h, const mqvs_segment *shard, int nq, int k, int metric, bool fast, int64_t ord,
                 int64_t nk, int code) {
    for (int i = 0; i < kHdrWords; ++i) h[i] = 0;
    h[kHdrOffset] = shard->row_offset;
    h[kHdrRows] = shard->n;
    h[kHdrGranule] = shard->granule;
    h[kHdrDim] = shard->d;
    h[kHdrCall] = ((int64_t)nq << 40) ^ ((int64_t)k << 8) ^ (int64_t)(metric & 0xFF);
    h[kHdrOk] = code == MQVS_OK ? 1 : 0;
    h[kHdrCode] = code;
    h[kHdrFast] = fast ? 1 : 0;
    h[kHdrOrd] = ord;
    h[kHdrNk] = nk;
}

const int64_t *row(const int64_t *table, int r) { return table + (size_t)kHdrWords * r; }

// The checks every rank makes on the same exchanged table (so every rank
// decides the same way): a failed rank fails the call everywhere with its
// code; shards must follow each other in row order on granule boundaries and
// the ranks must agree on granule, dimension, nq, k and metric.
void check_table(const mqvs_comm *c, const int64_t *t, int local_code, const std::string &local_err) {
    for (int r = 0; r < c->nranks; ++r)
        if (!row(t, r)[kHdrOk])
            fail(r == c->rank ? local_code : (int)row(t, r)[kHdrCode],
                 r == c->rank ? local_err : "sharded search failed on rank " + std::to_string(r));
    for (int r = 1; r < c->nranks; ++r) {
        const int64_t *a = row(t, r - 1), *b = row(t, r);
        if (b[kHdrOffset] != a[kHdrOffset] + a[kHdrRows])
            fail(MQVS_ERR_BAD_ARGUMENTS, "shards out of row order: rank " + std::to_string(r) + " starts at row " +
                                             std::to_string(b[kHdrOffset]) + ", rank " + std::to_string(r - 1) +
                                             " ends at " + std::to_string(a[kHdrOffset] + a[kHdrRows]));
        if (b[kHdrGranule] != a[kHdrGranule] || b[kHdrDim] != a[kHdrDim] || b[kHdrCall] != a[kHdrCall])
            fail(MQVS_ERR_BAD_ARGUMENTS, "ranks disagree on granule, dimension, nq, k or metric");
    }
    if (c->nranks > 1 && t[kHdrGranule] > 0)
        for (int r = 0; r + 1 < c->nranks; ++r)
            if (row(t, r + 1)[kHdrOffset] % t[kHdrGranule])
                fail(MQVS_ERR_BAD_ARGUMENTS, "shard boundaries must be granule aligned");
}

struct CallArgs {
    mqvs_segment *shard;
    const float *queries;
    int nq, k, metric;
    const uint8_t *filter, *exists;
    int64_t *out_ids;
    float *out_dist;
    uint32_t search_flags;  // per-call path flags for the local search
    bool dev;
    hipStream_t s;
    size_t nk;
    bool cos;  // cosine over more than one rank: chunk-ordinal bases exchanged
};

// Inputs on the device (host pointers: copied into the communicator's
// buffers) and the argument checks of mqvs_search.
void stage_inputs(mqvs_comm *c, const CallArgs &a, const float *&dq, const uint8_t *&dfilter,
                  const uint8_t *&dexists) {
    mqvs_segment *shard = a.shard;
    if (shard->binary) fail(MQVS_ERR_LOGICAL, "binary segments are not sharded");
    if (a.nq < 0 || a.k < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "nq and k must be non-negative");
    if (a.k > kMaxK) fail(MQVS_ERR_BAD_ARGUMENTS, "k above " + std::to_string(kMaxK) + " not supported");
    if (a.nk && (!a.queries || !a.out_ids || !a.out_dist))
        fail(MQVS_ERR_BAD_ARGUMENTS, "null query or output pointer");
    dq = a.queries;
    dfilter = a.filter;
    dexists = a.exists;
    if (a.dev) return;
    const int64_t bm = (shard->n + 7) / 8;
    if (a.nk) {
        auto *q = (float *)c->queries.get(sizeof(float) * (size_t)a.nq * shard->d);
        MQVS_HIP(hipMemcpyAsync(q, a.queries, sizeof(float) * (size_t)a.nq * shard->d, hipMemcpyHostToDevice, a.s));
        dq = q;
    }
    if (a.filter) {
        auto *f = (uint8_t *)c->filter.get(bm);
        MQVS_HIP(hipMemcpyAsync(f, a.filter, bm, hipMemcpyHostToDevice, a.s));
        dfilter = f;
    }
    if (a.exists) {
        auto *f = (uint8_t *)c->exists.get(bm);
        MQVS_HIP(hipMemcpyAsync(f, a.exists, bm, hipMemcpyHostToDevice, a.s));
        dexists = f;
    }
}

// The exchange buffers of a call of nk results per rank (local lists, the
// gathered lists, host-pointer outputs, the merge's sort scratch) and the
// chunk-flag scratch of the cosine count.
struct Bufs {
    int64_t *li = nullptr, *ai = nullptr, *oi = nullptr;
    float *ld = nullptr, *ad = nullptr, *od = nullptr;
    uint4 *scratch = nullptr;
    int *chunk_flags = nullptr;
};
Bufs get_bufs(mqvs_comm *c, const CallArgs &a, size_t nk) {
    Bufs b;
    const int64_t nch = (a.shard->n + a.shard->granule - 1) / a.shard->granule;
    b.chunk_flags = (int *)c->flags.get(sizeof(int) * (size_t)std::max<int64_t>(nch, 1));
    if (!nk) return b;
    b.li = (int64_t *)c->local_ids.get(sizeof(int64_t) * nk);
    b.ld = (float *)c->local_dist.get(sizeof(float) * nk);
    b.ai = (int64_t *)c->all_ids.get(sizeof(int64_t) * nk * c->nranks);
    b.ad = (float *)c->all_dist.get(sizeof(float) * nk * c->nranks);
    b.oi = a.out_ids;
    b.od = a.out_dist;
    if (!a.dev) {
        b.oi = (int64_t *)c->out_ids.get(sizeof(int64_t) * nk);
        b.od = (float *)c->out_dist.get(sizeof(float) * nk);
    }
    if ((int64_t)c->nranks * a.k > kSortCap)
        b.scratch = (uint4 *)c->scratch.get(sizeof(uint4) * 2 * (size_t)c->nranks * a.k * a.nq);
    return b;
}

// merge by (distance, rank, position) = the unsharded order, then the
// results to the caller's host buffers
void merge_out(mqvs_comm *c, const CallArgs &a, const Bufs &b) {
    if (!a.nk) return;
    launch_merge_shards(c->nranks, a.nq, a.k, a.metric, b.ai, b.ad, b.oi, b.od, false, b.scratch, a.s);
    MQVS_HIP(hipGetLastError());
    if (!a.dev) {
        MQVS_HIP(hipMemcpyAsync(a.out_ids, b.oi, sizeof(int64_t) * a.nk, hipMemcpyDeviceToHost, a.s));
        MQVS_HIP(hipMemcpyAsync(a.out_dist, b.od, sizeof(float) * a.nk, hipMemcpyDeviceToHost, a.s));
    }
}

enum class Fast { kDone, kRedo };

// The fast path: this rank's call equals the call every rank validated last
// (so its buffers are in place and nothing is allocated).  Header, local
// search, exchange and merge are all enqueued; ONE host sync reads the
// exchanged table.  The table holds every rank's outcome, its local search's
// fallback flags and, for cosine, the chunk-ordinal base it assumed next to
// its chunk count: a failure fails every rank, a fallback or a wrong base
// (PREWHERE filters that empty whole chunks) makes every rank re-run the
// validated path.
Fast fast_search(mqvs_comm *c, const CallArgs &a) {
    mqvs_segment *shard = a.shard;
    auto *hd = (int64_t *)c->hdr.p;  // [nranks][kHdrWords] table, then this rank's header
    int64_t *mine = hd + (size_t)kHdrWords * c->nranks;
    int64_t *hm = c->h_hdr, *ht = c->h_hdr + kHdrWords;
    const int64_t ord = !a.cos ? -1
                        : (!a.filter && c->last.ord_base >= 0) ? c->last.ord_base
                                                              : shard->row_offset / shard->granule;
    std::string local_err;
    int local_code = MQVS_OK;
    fill_header(hm, shard, a.nq, a.k, a.metric, true, ord, (int64_t)a.nk, MQVS_OK);
    MQVS_HIP(hipMemcpyAsync(mine, hm, sizeof(int64_t) * kHdrWords, hipMemcpyHostToDevice, a.s));
    Bufs b;
    try {
        const float *dq;
        const uint8_t *dfilter, *dexists;
        stage_inputs(c, a, dq, dfilter, dexists);
        b = get_bufs(c, a, a.nk);
        if (a.cos)
            launch_count_active_chunks(dfilter, shard->nonempty_bits, dexists, shard->n, shard->granule,
                                       b.chunk_flags, mine + kHdrChunks, a.s);
        if (a.nk)
            search_segment_async(shard, dq, a.nq, a.k, a.metric, dfilter, dexists, b.li, b.ld, a.search_flags, a.s,
                                 ord, (int *)(mine + kHdrFlags));
    } catch (const Error &e) {
        local_err = e.msg;
        local_code = e.code;
        // (this rank still joins the exchange, with its failure in the header;
        // the staging buffer is rewritten whole, so the copy above is harmless)
        fill_header(hm, shard, a.nq, a.k, a.metric, true, ord, (int64_t)a.nk, e.code);
        MQVS_HIP(hipMemcpyAsync(mine, hm, sizeof(int64_t) * kHdrWords, hipMemcpyHostToDevice, a.s));
    }
    const bool have = local_code == MQVS_OK;
    // The collective sequence is the one every path issues: the header
    // all-gather ON ITS OWN, then the two list gathers as one group.  A rank
    // on the validated path (slow_search) cannot know that this rank took the
    // fast path until its header gather returns; it then joins the list group
    // with the same two operations.  (One group of all three here would pair
    // a grouped launch with an ungrouped one, and RCCL splits grouped
    // collectives over channels by the group's contents.)
    comm_all_gather(c, mine, hd, sizeof(int64_t) * kHdrWords, a.s);
    if (a.nk) {
        // (a failed rank sends whatever its buffers hold: every rank fails below)
        comm_group_start(c);
        comm_all_gather(c, c->local_ids.p, c->all_ids.p, sizeof(int64_t) * a.nk, a.s);
        comm_all_gather(c, c->local_dist.p, c->all_dist.p, sizeof(float) * a.nk, a.s);
        comm_group_end(c);
    }
    if (have) merge_out(c, a, b);
    MQVS_HIP(hipMemcpyAsync(ht, hd, sizeof(int64_t) * kHdrWords * c->nranks, hipMemcpyDeviceToHost, a.s));
    host_wait(a.s);
    if (have && a.nk) search_collect_stats(c->device);
    try {
        for (int r = 0; r < c->nranks; ++r)
            if (!row(ht, r)[kHdrFast])
                fail(MQVS_ERR_BAD_ARGUMENTS, "ranks disagree on the call: rank " + std::to_string(r) +
                                                 " called with other arguments than the last sharded search");
        check_table(c, ht, local_code, local_err);
    } catch (...) {
        c->last.valid = false;
        throw;
    }
    bool redo = false;
    int64_t base = 0;
    for (int r = 0; r < c->nranks; ++r) {
        if ((int32_t)(uint32_t)(uint64_t)row(ht, r)[kHdrFlags] != 0) redo = true;
        if (a.cos) {
            if (row(ht, r)[kHdrOrd] != base) redo = true;
            base += row(ht, r)[kHdrChunks];
        }
    }
    if (redo) return Fast::kRedo;
    return Fast::kDone;
}

// The validated path: argument checks and every allocation first, then a
// header exchange and one host sync (shard order, agreement on the call, each
// rank's status and cosine chunk count, hence its exact ordinal base), the
// local search with its host-driven fallbacks, one exchange of the lists and
// the statuses, the merge and a second sync.  A rank that fails at any step
// still joins every exchange, so all ranks return the same error.
void slow_search(mqvs_comm *c, const CallArgs &a, const ShardCall &call) {
    mqvs_segment *shard = a.shard;
    c->last.valid = false;
    auto *hd = (int64_t *)c->hdr.p;
    int64_t *mine = hd + (size_t)kHdrWords * c->nranks;
    int64_t *hm = c->h_hdr, *ht = c->h_hdr + kHdrWords;
    std::string local_err;
    int local_code = MQVS_OK;
    const float *dq = nullptr;
    const uint8_t *dfilter = nullptr, *dexists = nullptr;
    Bufs b;
    try {
        stage_inputs(c, a, dq, dfilter, dexists);
        b = get_bufs(c, a, a.nk);
    } catch (const Error &e) {
        local_err = e.msg;
        local_code = e.code;
    }
    // 1. header exchange
    fill_header(hm, shard, a.nq, a.k, a.metric, false, -1, (int64_t)a.nk, local_code);
    MQVS_HIP(hipMemcpyAsync(mine, hm, sizeof(int64_t) * kHdrWords, hipMemcpyHostToDevice, a.s));
    if (a.cos && local_code == MQVS_OK)
        launch_count_active_chunks(dfilter, shard->nonempty_bits, dexists, shard->n, shard->granule, b.chunk_flags,
                                   mine + kHdrChunks, a.s);
    comm_all_gather(c, mine, hd, sizeof(int64_t) * kHdrWords, a.s);
    MQVS_HIP(hipMemcpyAsync(ht, hd, sizeof(int64_t) * kHdrWords * c->nranks, hipMemcpyDeviceToHost, a.s));
    host_wait(a.s);
    for (int r = 0; r < c->nranks; ++r) {
        if (!row(ht, r)[kHdrFast]) continue;
        // A rank on the fast path (its call equals the last validated one)
        // already waits in that call's exchange of nk_fast results: join it
        // with this rank's buffers (sized for that call, so nothing is
        // allocated), then every rank fails.
        const size_t nkf = (size_t)row(ht, r)[kHdrNk];
        if (nkf) {
            auto *li = c->local_ids.get(sizeof(int64_t) * nkf), *ld = c->local_dist.get(sizeof(float) * nkf);
            auto *ai = c->all_ids.get(sizeof(int64_t) * nkf * c->nranks);
            auto *ad = c->all_dist.get(sizeof(float) * nkf * c->nranks);
            comm_group_start(c);
            comm_all_gather(c, li, ai, sizeof(int64_t) * nkf, a.s);
            comm_all_gather(c, ld, ad, sizeof(float) * nkf, a.s);
            comm_group_end(c);
            host_wait(a.s);
        }
        fail(MQVS_ERR_BAD_ARGUMENTS, "ranks disagree on the call: rank " + std::to_string(r) +
                                         " repeated the last sharded search, this rank did not");
    }
    check_table(c, ht, local_code, local_err);
    int64_t ord_base = -1;
    if (a.cos) {
        ord_base = 0;
        for (int r = 0; r < c->rank; ++r) ord_base += row(ht, r)[kHdrChunks];
    }
    if (a.nk) {
        // 2. local top-k (ids part-global: the shard's row_offset applied)
        try {
            search_segment(shard, dq, a.nq, a.k, a.metric, dfilter, dexists, b.li, b.ld, a.search_flags, a.s,
                           ord_base);
        } catch (const Error &e) {
            local_err = e.msg;
            local_code = e.code;
        }
        // 3. one exchange: (ids, distances) of every rank, rank-major, and
        // each rank's status (in the header table)
        fill_header(hm, shard, a.nq, a.k, a.metric, false, ord_base, (int64_t)a.nk, local_code);
        MQVS_HIP(hipMemcpyAsync(mine, hm, sizeof(int64_t) * kHdrWords, hipMemcpyHostToDevice, a.s));
        comm_group_start(c);
        comm_all_gather(c, b.li, b.ai, sizeof(int64_t) * a.nk, a.s);
        comm_all_gather(c, b.ld, b.ad, sizeof(float) * a.nk, a.s);
        comm_all_gather(c, mine, hd, sizeof(int64_t) * kHdrWords, a.s);
        comm_group_end(c);
        if (local_code == MQVS_OK) merge_out(c, a, b);
        MQVS_HIP(hipMemcpyAsync(ht, hd, sizeof(int64_t) * kHdrWords * c->nranks, hipMemcpyDeviceToHost, a.s));
        host_wait(a.s);
        for (int r = 0; r < c->nranks; ++r)
            if (!row(ht, r)[kHdrOk])
                fail(r == c->rank ? local_code : (int)row(ht, r)[kHdrCode],
                     r == c->rank ? local_err : "sharded search failed on rank " + std::to_string(r));
    }
    // every rank validated this call together: the next equal call takes the
    // fast path on every rank
    c->last = call;
    c->last.ord_base = a.cos && !a.filter ? ord_base : -1;
}

}  // namespace

extern "C" {

int mqvs_sharded_search(mqvs_comm_t c, mqvs_segment_t shard, const float *queries, int32_t nq, int32_t k,
                        int32_t metric, const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids,
                        float *out_dist, uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        // (a call that cannot take part in the exchange fails alone)
        if (!c || !shard) fail(MQVS_ERR_BAD_ARGUMENTS, "null communicator or shard");
        if (shard->device != c->device) fail(MQVS_ERR_BAD_ARGUMENTS, "shard and communicator on different devices");
        std::lock_guard<std::mutex> lock(c->mu);
        DeviceGuard guard(c->device);
        WaitScope wsc{6, (uint64_t)(uintptr_t)c, (uint64_t)(uintptr_t)shard, (uint64_t)nq, (uint64_t)k,
                      (uint64_t)metric, filter != nullptr, row_exists != nullptr, flags};
        CallArgs a{shard, queries, nq, k, metric, filter, row_exists, out_ids, out_dist,
                   flags & ~(MQVS_F_ASYNC | MQVS_F_DEVICE_PTRS), (flags & MQVS_F_DEVICE_PTRS) != 0,
                   stream ? (hipStream_t)stream : c->stream,
                   (size_t)std::max(nq, 0) * (size_t)std::max(k, 0),
                   metric == MQVS_METRIC_COSINE && c->nranks > 1};
        ShardCall call;
        call.valid = true;
        call.shard = shard;
        call.row_offset = shard->row_offset;
        call.rows = shard->n;
        call.nq = nq;
        call.k = k;
        call.metric = metric;
        call.d = shard->d;
        call.filter = filter != nullptr;
        call.exists = row_exists != nullptr;
        call.dev = a.dev;
        if (c->last.same(call)) {
            c->fast_calls++;
            if (fast_search(c, a) == Fast::kDone) return;
            // every rank read the same table and re-runs together
            c->redo_calls++;
        }
        slow_search(c, a, call);
    });
}

int mqvs_comm_stats(mqvs_comm_t c, int64_t *fast_calls, int64_t *redo_calls) {
    return guarded([&] {
        if (!c) fail(MQVS_ERR_BAD_ARGUMENTS, "null communicator");
        std::lock_guard<std::mutex> lock(c->mu);
        if (fast_calls) *fast_calls = c->fast_calls;
        if (redo_calls) *redo_calls = c->redo_calls;
    });
}

}  // extern "C"
