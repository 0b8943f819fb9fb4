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
#include "mqvs_internal.h"

namespace mqvs {

constexpr int SEL_THREADS = 256;

// Histogram update with run-length aggregation: a thread keeps a running
// (bucket, count) pair and only flushes to LDS when the bucket changes, which
// removes the LDS-atomic pile-up on the few buckets that the high digits of
// clustered float keys fall into.
struct RunHist {
    uint32_t cur = 0xFFFFFFFFu, cnt = 0;
    __device__ void add(uint32_t *hist, uint32_t b) {
        if (b == cur) {
            ++cnt;
        } else {
            if (cnt) atomicAdd(&hist[cur], cnt);
            cur = b;
            cnt = 1;
        }
    }
    __device__ void flush(uint32_t *hist) {
        if (cnt) atomicAdd(&hist[cur], cnt);
        cnt = 0;
        cur = 0xFFFFFFFFu;
    }
};

// k-th smallest valid key (1-based rank k) among `count` values produced by
// load(i); 0xFFFFFFFE when fewer than k values are valid.  Block-wide.
template <typename KeyFn>
__device__ uint32_t block_radix_select(KeyFn keyof, int64_t count, int k, uint32_t *hist,
                                       uint32_t *sh) {
    const int t = threadIdx.x;
    uint32_t prefix = 0, mask = 0, kk = (uint32_t)k;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        for (int i = t; i < 256; i += SEL_THREADS) hist[i] = 0;
        __syncthreads();
        RunHist rh;
        for (int64_t i = t; i < count; i += SEL_THREADS) {
            const uint32_t key = keyof(i);
            if (key == 0xFFFFFFFFu) continue;
            if ((key & mask) != prefix) continue;
            rh.add(hist, (key >> shift) & 255u);
        }
        rh.flush(hist);
        __syncthreads();
        if (t == 0) {
            uint32_t total = 0;
            for (int b = 0; b < 256; ++b) total += hist[b];
            uint32_t done = 0, cum = 0, bsel = 0;
            if (pass == 0 && total < kk) {
                done = 1;  // fewer than k valid: every valid value qualifies
            } else {
                for (int b = 0; b < 256; ++b) {
                    if (cum + hist[b] >= kk) {
                        bsel = (uint32_t)b;
                        break;
                    }
                    cum += hist[b];
                }
            }
            sh[0] = done;
            sh[1] = bsel;
            sh[2] = cum;
        }
        __syncthreads();
        if (sh[0]) {
            __syncthreads();
            return 0xFFFFFFFEu;
        }
        prefix |= sh[1] << shift;
        mask |= 255u << shift;
        kk -= sh[2];
        __syncthreads();
    }
    return prefix;
}

template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_probe_select(const float *probe, int64_t P,
                                                             int64_t ld, int k, uint32_t *tau,
                                                             int *cand_count, Cand *cand,
                                                             int cap, int64_t row_base) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    const int q = blockIdx.x;
    const float *row = probe + (int64_t)q * ld;
    auto keyof = [&](int64_t i) { return key32<METRIC>(row[i]); };
    const uint32_t th = block_radix_select(keyof, P, k, hist, sh);
    if (threadIdx.x == 0) tau[q] = th;
    for (int64_t i = threadIdx.x; i < P; i += SEL_THREADS) {
        const float raw = row[i];
        const uint32_t key = key32<METRIC>(raw);
        if (key != 0xFFFFFFFFu && key <= th) {
            const int pos = atomicAdd(&cand_count[q], 1);
            if (pos < cap) {
                Cand c;
                c.raw = raw;
                c.row = (uint32_t)(row_base + i);
                cand[(int64_t)q * cap + pos] = c;
            }
        }
    }
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

// ---------------------------------------------------------------------------
// Bitonic sort of up to kSortCap 16-byte records in LDS, lexicographic on
// (x, y, z, w) ascending.
__device__ inline bool rec_less(const uint4 &a, const uint4 &b) {
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.z != b.z) return a.z < b.z;
    return a.w < b.w;
}

__device__ void block_bitonic_sort(uint4 *recs, int N) {
    for (int size = 2; size <= N; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < (N >> 1); i += SEL_THREADS) {
                const int lo = 2 * stride * (i / stride) + (i % stride);
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                uint4 a = recs[lo], b = recs[hi];
                if (rec_less(b, a) == up) {
                    recs[lo] = b;
                    recs[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ inline float key_to_value(int metric, uint32_t k1) {
    // inverse of ord_asc / ~ord_asc
    uint32_t u = (metric == MQVS_METRIC_IP || metric == kMetricIpRaw) ? ~k1 : k1;
    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    return __builtin_bit_cast(float, u);
}

template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_final_select(const Cand *cand,
                                                             const int *cand_count, int cap,
                                                             int k, int64_t chunk_rows,
                                                             int64_t id_offset, int64_t *out_ids,
                                                             float *out_dist, int *overflow) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];
    const int q = blockIdx.x;
    int n = cand_count[q];
    if (n > cap) {
        if (threadIdx.x == 0) atomicOr(overflow, 1);
        n = cap;
    }
    int N = 1;
    while (N < n) N <<= 1;
    const Cand *c = cand + (int64_t)q * cap;
    for (int i = threadIdx.x; i < N; i += SEL_THREADS) {
        uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (i < n) {
            const Cand e = c[i];
            r.x = key32<METRIC>(e.raw);
            r.w = e.row;
            if (METRIC == MQVS_METRIC_COSINE) {
                // ties on 1-ip: earlier granule chunk first (merge keeps
                // `final` on equality), then ip descending within a chunk
                // (faiss IP order), then row (MergeTreeVSManager.cpp:1653-1679)
                r.y = chunk_rows > 0 ? (uint32_t)((int64_t)e.row / chunk_rows) : 0u;
                r.z = ~ord_asc(e.raw);
            } else {
                r.y = 0;
                r.z = 0;
            }
        }
        recs[i] = r;
    }
    __syncthreads();
    block_bitonic_sort(recs, N);
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f
                      : (METRIC == kMetricIpRaw) ? -3.40282347e+38f
                                                 : 3.40282347e+38f;
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

// Merge of per-shard result lists: key (distance, shard, position).
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_merge_shards(int nshards, int nq, int k,
                                                             const int64_t *in_ids,
                                                             const float *in_dist,
                                                             int64_t *out_ids, float *out_dist) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];
    const int q = blockIdx.x;
    const int n = nshards * k;
    int N = 1;
    while (N < n) N <<= 1;
    for (int i = threadIdx.x; i < N; i += SEL_THREADS) {
        uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (i < n) {
            const int s = i / k, pos = i % k;
            const int64_t off = ((int64_t)s * nq + q) * k + pos;
            if (in_ids[off] >= 0) {
                const float v = in_dist[off];
                r.x = (METRIC == MQVS_METRIC_IP || METRIC == kMetricIpRaw) ? ~ord_asc(v) : ord_asc(v);
                r.y = (uint32_t)s;
                r.z = (uint32_t)pos;
                r.w = (uint32_t)i;
            }
        }
        recs[i] = r;
    }
    __syncthreads();
    block_bitonic_sort(recs, N);
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f : 3.40282347e+38f;
    for (int i = threadIdx.x; i < k; i += SEL_THREADS) {
        int64_t id = -1;
        float dist = pad;
        if (i < N && recs[i].x != 0xFFFFFFFFu) {
            const int src = (int)recs[i].w;
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
                           hipStream_t s) {
    hipLaunchKernelGGL(k_probe_select<M>, dim3(nq), dim3(SEL_THREADS), 0, s, probe, P, ld, k, tau,
                       cc, cand, cap, row_base);
}

void launch_probe_select(const float *probe, int64_t P, int64_t ld, int nq, int k, int metric,
                         uint32_t *tau, int *cand_count, Cand *cand, int cand_cap,
                         int64_t row_base, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, probe_select_t,
                         (probe, P, ld, nq, k, tau, cand_count, cand, cand_cap, row_base, s));
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
                           float *out_dist, int *overflow, hipStream_t s) {
    hipLaunchKernelGGL(k_final_select<M>, dim3(nq), dim3(SEL_THREADS), sort_lds(cap), s, cand, cc,
                       cap, k, chunk_rows, id_offset, out_ids, out_dist, overflow);
}

void launch_final_select(const Cand *cand, const int *cand_count, int cand_cap, int nq, int k,
                         int metric, int64_t chunk_rows, int64_t id_offset, int64_t *out_ids,
                         float *out_dist, int *overflow, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, final_select_t, (cand, cand_count, cand_cap, nq, k, chunk_rows,
                                                  id_offset, out_ids, out_dist, overflow, s));
}

template <int M>
static void merge_shards_t(int nshards, int nq, int k, const int64_t *in_ids, const float *in_dist,
                           int64_t *out_ids, float *out_dist, hipStream_t s) {
    hipLaunchKernelGGL(k_merge_shards<M>, dim3(nq), dim3(SEL_THREADS), sort_lds(nshards * k), s,
                       nshards, nq, k, in_ids, in_dist, out_ids, out_dist);
}

void launch_merge_shards(int nshards, int nq, int k, int metric, const int64_t *in_ids,
                         const float *in_dist, int64_t *out_ids, float *out_dist, hipStream_t s) {
    if (nq <= 0) return;
    MQVS_DISPATCH_METRIC(metric, merge_shards_t,
                         (nshards, nq, k, in_ids, in_dist, out_ids, out_dist, s));
}

}  // namespace mqvs
