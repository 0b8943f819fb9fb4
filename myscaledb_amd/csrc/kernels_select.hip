// kernels_select.hip -- top-k selection for gfx950.
//
// Replaces the faiss result heap (per granule chunk) plus the two-pointer
// merge of MergeTreeVSManager::searchWrapper (MergeTreeVSManager.cpp:1653-1679)
// and the cross-part multimap merge (MergeTreeBaseSearchManager.cpp:207-297).
// The reference's cumulative result is the k best rows under one total order
// (mqvs_internal.h key32 + tie rules); here it is found in three steps:
//   k_probe_select  radix select (4 x 8-bit digits) of the k-th key over the
//                   dense probe values -> per-query threshold tau, and the
//                   probe rows with key <= tau become the first candidates;
//   (scan kernels append every later row with key <= tau)
//   k_final_select  bitonic sort of the candidates in LDS by the full key
//                   (L2/IP: key, row; cosine: 1-ip, chunk, ip desc, row) and
//                   emit the first k in the reference's output layout.

#include "select_common.h"

namespace mqvs {



// 1024 threads, 16 probe values in flight per thread (as k_probe_select_wide)
constexpr int kProbeThreads = 1024;

template <int METRIC>
__global__ __launch_bounds__(kProbeThreads) void k_probe_select(const float *probe, int64_t P,
                                                             int64_t ld, int k, uint32_t *tau,
                                                             int *cand_count, Cand *cand,
                                                             int cap, int64_t row_base,
                                                             const int32_t *row_list) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    const int q = blockIdx.x;
    const float *row = probe + (int64_t)q * ld;
    const uint32_t th = block_radix_select_rows<METRIC, kProbeThreads>(row, P, k, hist, sh);
    if (threadIdx.x == 0) tau[q] = th;
    for_each_f4<kProbeThreads>(row, P, [&](int64_t i, float raw) {
        const uint32_t key = key32<METRIC>(raw);
        if (key != 0xFFFFFFFFu && key <= th) {
            const int pos = atomicAdd(&cand_count[q], 1);
            if (pos < cap) {
                Cand c;
                c.raw = raw;
                // probe column = scan position; gather mode maps it to the row
                c.row = row_list ? (uint32_t)row_list[row_base + i] : (uint32_t)(row_base + i);
                cand[(int64_t)q * cap + pos] = c;
            }
        }
    });
}

// Tighten tau for queries whose candidate list overflowed: the k-th key among
// the `cap` stored candidates (a subset of rows) bounds the true k-th key.
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_cand_tau(const Cand *cand, const int *cand_count,
                                                         int cap, int k, uint32_t *tau) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    const int q = blockIdx.x;
    if (cand_count[q] <= cap) return;  // uniform per block
    const Cand *c = cand + (int64_t)q * cap;
    auto keyof = [&](int64_t i) { return key32<METRIC>(c[i].raw); };
    const uint32_t th = block_radix_select(keyof, cap, k, hist, sh);
    if (threadIdx.x == 0 && th < tau[q]) tau[q] = th;
}


// scratch (k > kSortCap): 2 kLargeCap records per query in global memory;
// the records to sort then may exceed the LDS sort (global_sort).
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_final_select(const Cand *cand,
                                                             const int *cand_count, int cap,
                                                             int k, int64_t chunk_rows,
                                                             int64_t id_offset, int64_t *out_ids,
                                                             float *out_dist, int *overflow,
                                                             uint4 *scratch) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];  // kSortCap records
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_cnt;
    const int q = blockIdx.x;
    uint4 *g = scratch ? scratch + (int64_t)q * 2 * kLargeCap : nullptr;
    const int lcap = g ? kLargeCap : kSortCap;  // records this call can sort
    int n = cand_count[q];
    if (n > cap) {
        if (threadIdx.x == 0) atomicOr(overflow, 1);
        n = cap;
    }
    const Cand *c = cand + (int64_t)q * cap;
    auto make_rec = [&](const Cand &e) {
        uint4 r;
        r.x = key32<METRIC>(e.raw);
        r.w = e.row;
        if (METRIC == MQVS_METRIC_COSINE) {
            // ties on 1-ip: earlier granule chunk first (merge keeps `final`
            // on equality), then ip descending within a chunk (faiss IP
            // order), then row (MergeTreeVSManager.cpp:1653-1679)
            r.y = chunk_rows > 0 ? (uint32_t)((int64_t)e.row / chunk_rows) : 0u;
            r.z = ~ord_asc(e.raw);
        } else {
            r.y = 0;
            r.z = 0;
        }
        return r;
    };
    int m = n;
    if (n <= kSortCap) {
        for (int i = threadIdx.x; i < n; i += SEL_THREADS) recs[i] = make_rec(c[i]);
    } else {
        // long list: k-th primary key first, then sort only key <= it (k + ties)
        auto keyof = [&](int64_t i) { return key32<METRIC>(c[i].raw); };
        const uint32_t th = block_radix_select(keyof, n, k, hist, sh);
        // rows tying at the k-th key rank by row (L2 / IP / binary: the key
        // then the row is the whole order), so when more than kSortCap rows
        // reach the k-th key only the smallest rows of the tie are kept (the
        // (k - #below)-th smallest tied row bounds them); cosine ties also
        // rank by chunk and ip and keep the plain path
        uint32_t rth = 0xFFFFFFFFu;
        if (METRIC != MQVS_METRIC_COSINE && th != 0xFFFFFFFEu) {
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            int below = 0, tie = 0;
            for (int i = threadIdx.x; i < n; i += SEL_THREADS) {
                const uint32_t key = keyof(i);
                below += key < th;
                tie += key == th;
            }
            atomicAdd(&s_cnt, below);
            __syncthreads();
            const int nbelow = s_cnt;
            __syncthreads();
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            atomicAdd(&s_cnt, tie);
            __syncthreads();
            const int ntie = s_cnt;
            __syncthreads();
            if (nbelow + ntie > lcap) {
                auto rowof = [&](int64_t i) {
                    const Cand e = c[i];
                    return key32<METRIC>(e.raw) == th ? e.row : 0xFFFFFFFFu;
                };
                rth = block_radix_select(rowof, n, k - nbelow, hist, sh);
            }
        }
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += SEL_THREADS) {
            const Cand e = c[i];
            const uint32_t key = key32<METRIC>(e.raw);
            if (key != 0xFFFFFFFFu && (key < th || (key == th && e.row <= rth))) {
                const int pos = atomicAdd(&s_cnt, 1);
                const uint4 r = make_rec(e);
                if (pos < kSortCap) recs[pos] = r;
                if (g && pos < kLargeCap) g[pos] = r;
            }
        }
        __syncthreads();
        m = s_cnt;
        if (m > lcap) {  // more than lcap rows tie at the k-th key
            if (threadIdx.x == 0) atomicOr(overflow, 2);
            m = lcap;
        }
    }
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f
                      : (METRIC == kMetricIpRaw) ? -3.40282347e+38f
                                                 : 3.40282347e+38f;
    if (m > kSortCap) {
        __syncthreads();
        const uint4 *sorted = global_sort(g, g + kLargeCap, m, recs);
        for (int i = threadIdx.x; i < k; i += SEL_THREADS) {
            int64_t id = -1;
            float dist = pad;
            if (i < m) {
                id = (int64_t)sorted[i].w + id_offset;
                dist = key_to_value(METRIC, sorted[i].x);
            }
            out_ids[(int64_t)q * k + i] = id;
            out_dist[(int64_t)q * k + i] = dist;
        }
        return;
    }
    int N = 1;
    while (N < m) N <<= 1;
    for (int i = m + threadIdx.x; i < N; i += SEL_THREADS)
        recs[i] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    __syncthreads();
    block_bitonic_sort(recs, N);
    for (int i = threadIdx.x; i < k; i += SEL_THREADS) {
        int64_t id = -1;
        float dist = pad;
        if (i < N && recs[i].x != 0xFFFFFFFFu) {
            id = (int64_t)recs[i].w + id_offset;
            dist = key_to_value(METRIC, recs[i].x);
        }
        out_ids[(int64_t)q * k + i] = id;
        out_dist[(int64_t)q * k + i] = dist;
    }
}

// Merge of per-list results: key (distance, list, position).  rev_ties (IP
// cross-PART merge, MergeTreeBaseSearchManager.cpp:207-297): the reference
// walks its insertion-ordered multimap backwards for DESC, so equal scores
// come out last-inserted first -> key (distance, ~list, ~position).
// scratch: 2 nshards k records per query when nshards k > kSortCap (the
// records are sorted through global memory), else null.
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_merge_shards(int nshards, int nq, int k,
                                                             const int64_t *in_ids,
                                                             const float *in_dist,
                                                             int64_t *out_ids, float *out_dist,
                                                             int rev_ties, uint4 *scratch) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];
    const int q = blockIdx.x;
    const int n = nshards * k;
    auto record = [&](int i) {
        uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        const int s = i / k, pos = i % k;
        const int64_t off = ((int64_t)s * nq + q) * k + pos;
        if (in_ids[off] >= 0) {
            const float v = in_dist[off];
            r.x = (METRIC == MQVS_METRIC_IP || METRIC == kMetricIpRaw) ? ~ord_asc(v) : ord_asc(v);
            r.y = rev_ties ? ~(uint32_t)s : (uint32_t)s;
            r.z = rev_ties ? ~(uint32_t)pos : (uint32_t)pos;
        }
        r.w = (uint32_t)i;  // (unique: empty slots sort last, by position)
        return r;
    };
    const uint4 *sorted = recs;
    int N = 1;
    if (n > kSortCap) {
        uint4 *g = scratch + (int64_t)q * 2 * n;
        for (int i = threadIdx.x; i < n; i += SEL_THREADS) g[i] = record(i);
        __syncthreads();
        sorted = global_sort(g, g + n, n, recs);
        N = n;
    } else {
        while (N < n) N <<= 1;
        for (int i = threadIdx.x; i < N; i += SEL_THREADS)
            recs[i] = i < n ? record(i) : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        __syncthreads();
        block_bitonic_sort(recs, N);
    }
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f : 3.40282347e+38f;
    for (int i = threadIdx.x; i < k; i += SEL_THREADS) {
        int64_t id = -1;
        float dist = pad;
        if (i < N && sorted[i].x != 0xFFFFFFFFu) {
            const int src = (int)sorted[i].w;
            const int s = src / k, pos = src % k;
            const int64_t off = ((int64_t)s * nq + q) * k + pos;
            id = in_ids[off];
            dist = in_dist[off];
        }
        out_ids[(int64_t)q * k + i] = id;
        out_dist[(int64_t)q * k + i] = dist;
    }
}

// ---------------------------------------------------------------------------
#define MQVS_DISPATCH_METRIC(metric, KERNEL, ...)                                         \
    switch (metric) {                                                                     \
        case MQVS_METRIC_L2: KERNEL<MQVS_METRIC_L2> __VA_ARGS__; break;                 \
        case MQVS_METRIC_IP: KERNEL<MQVS_METRIC_IP> __VA_ARGS__; break;                 \
        case MQVS_METRIC_COSINE: KERNEL<MQVS_METRIC_COSINE> __VA_ARGS__; break;         \
        default: KERNEL<kMetricIpRaw> __VA_ARGS__; break;                                 \
    }

template <int M>
static void probe_select_t(const float *probe, int64_t P, int64_t ld, int nq, int k,
                           uint32_t *tau, int *cc, Cand *cand, int cap, int64_t row_base,
                           const int32_t *row_list, hipStream_t s) {
    hipLaunchKernelGGL(k_probe_select<M>, dim3(nq), dim3(kProbeThreads), 0, s, probe, P, ld, k, tau,
                       cc, cand, cap, row_base, row_list);
}

void launch_probe_select(const float *probe, int64_t P, int64_t ld, int nq, int k, int metric,
                         uint32_t *tau, int *cand_count, Cand *cand, int cand_cap,
                         int64_t row_base, const int32_t *row_list, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, probe_select_t,
                         (probe, P, ld, nq, k, tau, cand_count, cand, cand_cap, row_base, row_list, s));
}

template <int M>
static void cand_tau_t(const Cand *cand, const int *cc, int cap, int nq, int k, uint32_t *tau,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_cand_tau<M>, dim3(nq), dim3(SEL_THREADS), 0, s, cand, cc, cap, k, tau);
}

void launch_cand_tau(const Cand *cand, const int *cand_count, int cand_cap, int nq, int k,
                     int metric, uint32_t *tau, const int *, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, cand_tau_t, (cand, cand_count, cand_cap, nq, k, tau, s));
}

static size_t sort_lds(int n) {
    int N = 1;
    while (N < n) N <<= 1;
    return (size_t)N * sizeof(uint4);
}

template <int M>
static void final_select_t(const Cand *cand, const int *cc, int cap, int nq, int k,
                           int64_t chunk_rows, int64_t id_offset, int64_t *out_ids,
                           float *out_dist, int *overflow, uint4 *scratch, hipStream_t s) {
    hipLaunchKernelGGL(k_final_select<M>, dim3(nq), dim3(SEL_THREADS), sort_lds(kSortCap), s, cand, cc,
                       cap, k, chunk_rows, id_offset, out_ids, out_dist, overflow, scratch);
}

void launch_final_select(const Cand *cand, const int *cand_count, int cand_cap, int nq, int k,
                         int metric, int64_t chunk_rows, int64_t id_offset, int64_t *out_ids,
                         float *out_dist, int *overflow, uint4 *scratch, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, final_select_t, (cand, cand_count, cand_cap, nq, k, chunk_rows,
                                                  id_offset, out_ids, out_dist, overflow, scratch, s));
}

template <int M>
static void merge_shards_t(int nshards, int nq, int k, const int64_t *in_ids, const float *in_dist,
                           int64_t *out_ids, float *out_dist, int rev_ties, uint4 *scratch, hipStream_t s) {
    hipLaunchKernelGGL(k_merge_shards<M>, dim3(nq), dim3(SEL_THREADS),
                       sort_lds(nshards * k > kSortCap ? kSortCap : nshards * k), s, nshards, nq, k, in_ids, in_dist,
                       out_ids, out_dist, rev_ties, scratch);
}

void launch_merge_shards(int nshards, int nq, int k, int metric, const int64_t *in_ids,
                         const float *in_dist, int64_t *out_ids, float *out_dist, bool part_merge,
                         uint4 *scratch, hipStream_t s) {
    if (nq <= 0) return;
    const int rev = part_merge && (metric == MQVS_METRIC_IP || metric == kMetricIpRaw);
    MQVS_DISPATCH_METRIC(metric, merge_shards_t,
                         (nshards, nq, k, in_ids, in_dist, out_ids, out_dist, rev, scratch, s));
}

// ---------------------------------------------------------------------------
// Between scan segments: tighten the per-query threshold from the candidates
// collected so far and compact the list into the other buffer.
//   exact (APPROX = false): tau = min(tau, k-th key32 of the candidates)
//   approx (bf16):          thr = tighter(thr, widen(k-th approximate value))
// Every row of the exact top-k seen so far passes the new threshold (same
// argument as the probe threshold), so nothing the final select needs is lost.
// Up to `stage` candidates (the launch's LDS) are first copied into LDS with
// four loads in flight per thread, and the three radix passes and the
// compaction read them there: from global memory each pass waited one load
// per 256 candidates in turn (nq 1: ~3000 candidates, 9-16 us per refine).
constexpr int kRefineStage = 8192;

template <int METRIC, bool APPROX>
__global__ __launch_bounds__(SEL_THREADS) void k_refine(const Cand *cin, const int *cnt_in, int cap,
                                                       int k, const float *bq, uint32_t *tau,
                                                       float *thr, Cand *cout, int *cnt_out, int stage) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_cnt;
    extern __shared__ Cand s_cand[];
    const int q = blockIdx.x;
    int n = cnt_in[q];
    if (n > cap) n = cap;  // overflowed lists keep their overflow: count stays > cap
    const Cand *c = cin + (int64_t)q * cap;
    if (n <= stage) {
        int i = threadIdx.x;
        for (; i + 3 * SEL_THREADS < n; i += 4 * SEL_THREADS) {
            const Cand a = c[i], b = c[i + SEL_THREADS], d = c[i + 2 * SEL_THREADS], e = c[i + 3 * SEL_THREADS];
            s_cand[i] = a;
            s_cand[i + SEL_THREADS] = b;
            s_cand[i + 2 * SEL_THREADS] = d;
            s_cand[i + 3 * SEL_THREADS] = e;
        }
        for (; i < n; i += SEL_THREADS) s_cand[i] = c[i];
        __syncthreads();
        c = s_cand;
    }
    uint32_t tk = 0;
    float tf = 0.f;
    // (k <= 256: the bound from the threads' 4 smallest keys, kept_kth_bound)
    __shared__ uint32_t skeys[4 * SEL_THREADS];
    const bool kept = k <= SEL_THREADS;
    if (APPROX) {
        auto keyof = [&](int64_t i) { return okey<METRIC>(c[i].raw); };
        const uint32_t th = kept ? kept_kth_bound<SEL_THREADS, 4>(keyof, n, k, skeys, hist, sh)
                                 : block_radix_select<3>(keyof, n, k, hist, sh);  // (a bound: 3 passes)
        tf = thr[q];
        if (th != 0xFFFFFFFEu) {
            const float w = widen<METRIC>(okey_bound_value<METRIC>(th), bq[q]);
            tf = (METRIC == MQVS_METRIC_L2) ? fminf(tf, w) : fmaxf(tf, w);
        }
    } else {
        auto keyof = [&](int64_t i) { return key32<METRIC>(c[i].raw); };
        const uint32_t th = kept ? kept_kth_bound<SEL_THREADS, 4>(keyof, n, k, skeys, hist, sh)
                                 : block_radix_select<3>(keyof, n, k, hist, sh);
        tk = tau[q];
        if (th < tk) tk = th;
    }
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Cand *o = cout + (int64_t)q * cap;
    for (int i = threadIdx.x; i < n; i += SEL_THREADS) {
        const Cand e = c[i];
        bool take;
        if (APPROX) {
            take = (METRIC == MQVS_METRIC_L2) ? (e.raw <= tf) : (e.raw >= tf);
        } else {
            const uint32_t key = key32<METRIC>(e.raw);
            take = key != 0xFFFFFFFFu && key <= tk;
        }
        if (take) o[atomicAdd(&s_cnt, 1)] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // an overflowed input stays flagged as overflowed (its lost rows are unknown)
        cnt_out[q] = cnt_in[q] > cap ? cnt_in[q] : s_cnt;
        if (APPROX) thr[q] = tf;
        else tau[q] = tk;
    }
}

template <int M, bool A>
static void refine_t(const Cand *cin, const int *cnt_in, int cap, int nq, int k, const float *bq,
                     uint32_t *tau, float *thr, Cand *cout, int *cnt_out, hipStream_t s) {
    // (small batches stage up to 8192 candidates; a batch, whose thousand
    // workgroups need occupancy more, 2048: ~2k appends per segment)
    const int stage = std::min(cap, nq <= 16 ? kRefineStage : kRefineStage / 4);
    hipLaunchKernelGGL((k_refine<M, A>), dim3(nq), dim3(SEL_THREADS), sizeof(Cand) * (size_t)stage, s, cin, cnt_in,
                       cap, k, bq, tau, thr, cout, cnt_out, stage);
}

void launch_refine(const Cand *cin, const int *cnt_in, int cap, int nq, int k, int metric,
                   bool approx, const float *bq, uint32_t *tau, float *thr, Cand *cout, int *cnt_out,
                   hipStream_t s) {
    if (nq <= 0) return;
#define MQVS_REFINE(M)                                                                      \
    (approx ? refine_t<M, true>(cin, cnt_in, cap, nq, k, bq, tau, thr, cout, cnt_out, s)   \
            : refine_t<M, false>(cin, cnt_in, cap, nq, k, bq, tau, thr, cout, cnt_out, s))
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_REFINE(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_REFINE(MQVS_METRIC_IP); break;
        case MQVS_METRIC_COSINE: MQVS_REFINE(MQVS_METRIC_COSINE); break;
        default: MQVS_REFINE(kMetricIpRaw); break;
    }
#undef MQVS_REFINE
}

}  // namespace mqvs
