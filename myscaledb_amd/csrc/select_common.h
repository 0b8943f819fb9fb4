// select_common.h -- block-wide radix select, float-row visitor and LDS bitonic
// sort shared by the selection kernels (kernels_select.hip, kernels_bf16.hip).
#pragma once
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

// Bucket holding the kk-th smallest key (1-based) of a 256-bucket histogram,
// found by wave 0 in parallel (4 buckets per lane + a lane prefix sum).
// Writes sh[0] = done (total < kk on the first pass), sh[1] = bucket,
// sh[2] = count below the bucket.  Caller syncs before and after.
__device__ inline void hist_pick(const uint32_t *hist, uint32_t kk, bool first, uint32_t *sh) {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
    const uint32_t mine = h0 + h1 + h2 + h3;
    uint32_t inc = mine;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    const uint32_t total = __shfl(inc, 63);
    const uint32_t before = inc - mine;
    if (first && total < kk) {
        if (lane == 0) {
            sh[0] = 1;
            sh[1] = 0;
            sh[2] = 0;
        }
        return;
    }
    // the first lane whose inclusive count reaches kk holds the bucket
    const uint64_t hit = __ballot(inc >= kk);
    const int L = __ffsll((long long)hit) - 1;
    if (lane == L) {
        uint32_t cum = before, b = 4 * lane;
        const uint32_t hs[4] = {h0, h1, h2, h3};
        for (int j = 0; j < 4; ++j) {
            if (cum + hs[j] >= kk) {
                b = 4 * lane + j;
                break;
            }
            cum += hs[j];
        }
        sh[0] = 0;
        sh[1] = b;
        sh[2] = cum;
    }
}

// k-th smallest valid key (1-based rank k) among `count` values produced by
// load(i); 0xFFFFFFFE when fewer than k values are valid.  Block-wide.
// PASSES = 3 (thresholds only): the top 24 bits of the k-th key, the low byte
// set -- an upper bound on the k-th key (every key <= it passes a "<= bound"
// test, so a threshold built from it keeps every row the exact one keeps;
// 2^-16 relative looser) without the fourth histogram pass.
template <int PASSES = 4, typename KeyFn>
__device__ inline uint32_t block_radix_select(KeyFn keyof, int64_t count, int k, uint32_t *hist,
                                       uint32_t *sh) {
    const int t = threadIdx.x;
    uint32_t prefix = 0, mask = 0, kk = (uint32_t)k;
    for (int pass = 0; pass < PASSES; ++pass) {
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
        hist_pick(hist, kk, pass == 0, sh);  // fewer than k valid on pass 0: sh[0] = done
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
    return PASSES == 4 ? prefix : prefix | (0xFFFFFFFFu >> (8 * PASSES));
}

// block_radix_select with the bucket search in parallel and 4 keys in
// flight per thread (keyof(i) may read global memory).
template <int NT = SEL_THREADS, int PASSES = 4, typename KeyFn>
__device__ inline uint32_t block_radix_select_mlp(KeyFn keyof, int64_t count, int k, uint32_t *hist, uint32_t *sh) {
    constexpr int SEL_THREADS = NT;  // block size of the caller
    const int t = threadIdx.x;
    uint32_t prefix = 0, mask = 0, kk = (uint32_t)k;
    for (int pass = 0; pass < PASSES; ++pass) {
        const int shift = 24 - 8 * pass;
        for (int i = t; i < 256; i += SEL_THREADS) hist[i] = 0;
        __syncthreads();
        RunHist rh;
        int64_t i = t;
        for (; i + 3 * SEL_THREADS < count; i += 4 * SEL_THREADS) {
            const uint32_t k0 = keyof(i), k1 = keyof(i + SEL_THREADS), k2 = keyof(i + 2 * SEL_THREADS),
                           k3 = keyof(i + 3 * SEL_THREADS);
            if (k0 != 0xFFFFFFFFu && (k0 & mask) == prefix) rh.add(hist, (k0 >> shift) & 255u);
            if (k1 != 0xFFFFFFFFu && (k1 & mask) == prefix) rh.add(hist, (k1 >> shift) & 255u);
            if (k2 != 0xFFFFFFFFu && (k2 & mask) == prefix) rh.add(hist, (k2 >> shift) & 255u);
            if (k3 != 0xFFFFFFFFu && (k3 & mask) == prefix) rh.add(hist, (k3 >> shift) & 255u);
        }
        for (; i < count; i += SEL_THREADS) {
            const uint32_t key = keyof(i);
            if (key != 0xFFFFFFFFu && (key & mask) == prefix) rh.add(hist, (key >> shift) & 255u);
        }
        rh.flush(hist);
        __syncthreads();
        hist_pick(hist, kk, pass == 0, sh);
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
    return PASSES == 4 ? prefix : prefix | (0xFFFFFFFFu >> (8 * PASSES));
}

// An upper bound on the k-th smallest valid key of count keys: each thread
// keeps its KEEP smallest in registers, and block_radix_select_mlp's three
// passes (the low byte set) run over those NT * KEEP keys in LDS (skeys).
// The k-th smallest of a subset is >= the k-th of all, and equal unless a
// thread held more than KEEP of the k best -- a threshold needs no more.
// 0xFFFFFFFE when the subset holds fewer than k valid keys (then the caller
// keeps its threshold: every row passes it).  One pass over the keys with no
// LDS atomics per key (the full radix passes serialised on the few buckets
// clustered keys share).
template <int NT, int KEEP, typename KeyFn>
__device__ inline uint32_t kept_kth_bound(KeyFn keyof, int64_t count, int k, uint32_t *skeys, uint32_t *hist,
                                          uint32_t *sh) {
    const int t = threadIdx.x;
    uint32_t best[KEEP];
#pragma unroll
    for (int j = 0; j < KEEP; ++j) best[j] = 0xFFFFFFFFu;
    auto insert = [&](uint32_t key) {
        if (key >= best[KEEP - 1]) return;
#pragma unroll
        for (int j = 0; j < KEEP; ++j) {
            if (key < best[j]) {
                const uint32_t o = best[j];
                best[j] = key;
                key = o;
            }
        }
    };
    int64_t i = t;
    for (; i + 3 * NT < count; i += 4 * NT) {
        const uint32_t k0 = keyof(i), k1 = keyof(i + NT), k2 = keyof(i + 2 * NT), k3 = keyof(i + 3 * NT);
        insert(k0);
        insert(k1);
        insert(k2);
        insert(k3);
    }
    for (; i < count; i += NT) insert(keyof(i));
#pragma unroll
    for (int j = 0; j < KEEP; ++j) skeys[j * NT + t] = best[j];
    __syncthreads();
    return block_radix_select_mlp<NT, 3>([&](int64_t x) { return skeys[x]; }, (int64_t)KEEP * NT, k, hist, sh);
}

// The k smallest valid keys for small k (k <= kSelSmallK): each thread keeps
// its k smallest (key, index) pairs (insertion into registers), then k rounds
// of a block minimum over the threads' heads (wave shuffles + one LDS
// exchange), the owner popping its head.  Writes the popped indices in order
// to idx_out[0 ..) and returns their count (< k: fewer valid keys);
// *kth_out = the k-th pair (key << 32 | index), or ~0 when fewer than k.
// 0xFFFFFFFF keys are never taken; indices < 2^32.  No histogram passes.
// red: 2 * (NT / 64) words of LDS.
// KMAX (>= k): the registers kept per thread -- the insertion costs KMAX
// compare-and-swaps per key, so a k = 1 pick with KMAX 8 spent ~8x the VALU
// instructions of a minimum (the coarse pick runs 4 workgroups per CU: VALU-
// bound there, 7-15 us of ~25 per query).
constexpr int kSelSmallK = 8;
template <int NT = SEL_THREADS, int KMAX = kSelSmallK, typename KeyFn>
__device__ inline int block_topk_small(KeyFn keyof, int64_t count, int k, uint64_t *red, int *idx_out,
                                       uint64_t *kth_out) {
    static_assert(KMAX >= 1 && KMAX <= kSelSmallK, "KMAX");
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t loc[KMAX];  // (key << 32 | index), ascending
#pragma unroll
    for (int j = 0; j < KMAX; ++j) loc[j] = ~0ull;
    uint64_t worst = ~0ull;  // loc[k - 1]
    for (int64_t i = t; i < count; i += NT) {
        const uint32_t key = keyof(i);
        if (key == 0xFFFFFFFFu) continue;
        uint64_t v = ((uint64_t)key << 32) | (uint64_t)(uint32_t)i;
        if (v >= worst) continue;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {  // sorted insertion; the largest falls off
            if (j < k && v < loc[j]) {
                const uint64_t o = loc[j];
                loc[j] = v;
                v = o;
            }
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (j == k - 1) worst = loc[j];
    }
    int head = 0, n = 0;
    uint64_t last = ~0ull;
    for (int r = 0; r < k; ++r) {
        uint64_t h = ~0ull;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (j == head) h = loc[j];
        uint64_t m = h;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(m, off);
            m = o < m ? o : m;
        }
        uint64_t *slot = red + (r & 1) * (NT / 64);
        if (lane == 0) slot[wv] = m;
        __syncthreads();
        m = slot[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) m = slot[w] < m ? slot[w] : m;
        if (m == ~0ull) break;  // fewer than k valid keys
        if (h == m) ++head;     // (pairs are unique: one owner)
        if (t == 0) idx_out[r] = (int)(uint32_t)m;
        last = m;
        ++n;
    }
    __syncthreads();  // (idx_out and red are read / reused by the caller)
    *kth_out = n == k ? last : ~0ull;
    return n;
}

// Visit every element of a float row: float4 loads, 4 in flight per thread
// (the probe rows are megabytes; a scalar loop leaves HBM idle).
template <int NT = SEL_THREADS, typename F>
__device__ inline void for_each_f4(const float *row, int64_t P, F &&f) {
    constexpr int SEL_THREADS = NT;  // block size of the caller
    const int t = threadIdx.x;
    const bool al = ((uintptr_t)row & 15) == 0;
    int64_t head = 0;
    if (al) {
        const int64_t n4 = P / 4;
        const float4 *r4 = reinterpret_cast<const float4 *>(row);
        int64_t i = t;
        for (; i + 3 * SEL_THREADS < n4; i += 4 * SEL_THREADS) {
            const float4 a = r4[i], b = r4[i + SEL_THREADS], c = r4[i + 2 * SEL_THREADS],
                         e = r4[i + 3 * SEL_THREADS];
            f(4 * i, a.x); f(4 * i + 1, a.y); f(4 * i + 2, a.z); f(4 * i + 3, a.w);
            const int64_t ib = i + SEL_THREADS, ic = i + 2 * SEL_THREADS, ie = i + 3 * SEL_THREADS;
            f(4 * ib, b.x); f(4 * ib + 1, b.y); f(4 * ib + 2, b.z); f(4 * ib + 3, b.w);
            f(4 * ic, c.x); f(4 * ic + 1, c.y); f(4 * ic + 2, c.z); f(4 * ic + 3, c.w);
            f(4 * ie, e.x); f(4 * ie + 1, e.y); f(4 * ie + 2, e.z); f(4 * ie + 3, e.w);
        }
        for (; i < n4; i += SEL_THREADS) {
            const float4 a = r4[i];
            f(4 * i, a.x); f(4 * i + 1, a.y); f(4 * i + 2, a.z); f(4 * i + 3, a.w);
        }
        head = n4 * 4;
    }
    for (int64_t i = head + t; i < P; i += SEL_THREADS) f(i, row[i]);
}

template <int METRIC, int NT = SEL_THREADS>
__device__ inline uint32_t block_radix_select_rows(const float *row, int64_t P, int k, uint32_t *hist,
                                            uint32_t *sh) {
    const int t = threadIdx.x;
    uint32_t prefix = 0, mask = 0, kk = (uint32_t)k;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        for (int i = t; i < 256; i += SEL_THREADS) hist[i] = 0;
        __syncthreads();
        RunHist rh;
        for_each_f4<NT>(row, P, [&](int64_t, float raw) {
            const uint32_t key = key32<METRIC>(raw);
            if (key != 0xFFFFFFFFu && (key & mask) == prefix) rh.add(hist, (key >> shift) & 255u);
        });
        rh.flush(hist);
        __syncthreads();
        hist_pick(hist, kk, pass == 0, sh);
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

// ---------------------------------------------------------------------------
// Bitonic sort of up to kSortCap 16-byte records in LDS, lexicographic on
// (x, y, z, w) ascending.
__device__ inline bool rec_less(const uint4 &a, const uint4 &b) {
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.z != b.z) return a.z < b.z;
    return a.w < b.w;
}

__device__ inline void block_bitonic_sort(uint4 *recs, int N) {
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

// ---------------------------------------------------------------------------
// Large result sets (k above kSortCap, up to kMaxK; shard merges of more than
// kSortCap records): the records live in a global scratch of the query; runs
// of kSortCap are sorted in LDS by the bitonic network above, then merged in
// passes of doubling width.  Every record's key is unique (it ends with the
// row / list position), so a record's place in the merged run is its place
// in its own run plus the count of smaller records in the partner run (a
// binary search).  Equal records (the all-ones padding, a candidate listed
// twice) are merged stably -- left run first: a right-run record counts the
// left run's records <= it -- so no two records ever claim the same slot.
template <bool OR_EQUAL = false>
__device__ inline int count_less(const uint4 *a, int n, const uint4 &e) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (OR_EQUAL ? !rec_less(e, a[mid]) : rec_less(a[mid], e))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Sorts g[0, m) (tmp: m more records of scratch); recs: kSortCap records of
// LDS.  Returns the buffer that holds the sorted records (g or tmp).
__device__ inline uint4 *global_sort(uint4 *g, uint4 *tmp, int m, uint4 *recs) {
    for (int r0 = 0; r0 < m; r0 += kSortCap) {
        const int len = m - r0 < kSortCap ? m - r0 : kSortCap;
        int N = 1;
        while (N < len) N <<= 1;
        for (int i = threadIdx.x; i < N; i += SEL_THREADS)
            recs[i] = i < len ? g[r0 + i] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        __syncthreads();
        block_bitonic_sort(recs, N);
        for (int i = threadIdx.x; i < len; i += SEL_THREADS) g[r0 + i] = recs[i];
        __syncthreads();
    }
    uint4 *src = g, *dst = tmp;
    for (int w = kSortCap; w < m; w *= 2) {
        for (int i = threadIdx.x; i < m; i += SEL_THREADS) {
            const int base = i / (2 * w) * (2 * w);
            const int a1 = base + w < m ? base + w : m;
            const int b1 = base + 2 * w < m ? base + 2 * w : m;
            const uint4 e = src[i];
            const int pos = i < a1 ? (i - base) + count_less<false>(src + a1, b1 - a1, e)
                                   : (i - a1) + count_less<true>(src + base, a1 - base, e);
            dst[base + pos] = e;
        }
        __syncthreads();
        uint4 *t = src;
        src = dst;
        dst = t;
    }
    return src;
}

__device__ inline float key_to_value(int metric, uint32_t k1) {
    // inverse of ord_asc / ~ord_asc
    uint32_t u = (metric == MQVS_METRIC_IP || metric == kMetricIpRaw) ? ~k1 : k1;
    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    return __builtin_bit_cast(float, u);
}

// Approximate ordering key: smaller = better, NaN last; no validity cut (the
// exact value decides validity after the re-rank).
template <int METRIC>
__device__ inline uint32_t okey(float v) {
    if (v != v) return 0xFFFFFFFFu;
    const uint32_t o = ord_asc(v);
    return (METRIC == MQVS_METRIC_L2) ? o : ~o;
}

template <int METRIC>
__device__ inline float okey_value(uint32_t k) {
    uint32_t u = (METRIC == MQVS_METRIC_L2) ? k : ~k;
    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    return __builtin_bit_cast(float, u);
}

// the value of an upper bound on a k-th key (block_radix_select<3>: its low
// byte set): past the worst infinity the bound's bits decode to a NaN, which
// would fail every test -- the k-th value was that infinity, so use it
template <int METRIC>
__device__ inline float okey_bound_value(uint32_t k) {
    const float v = okey_value<METRIC>(k);
    if (v == v) return v;
    return METRIC == MQVS_METRIC_L2 ? __builtin_inff() : -__builtin_inff();
}

// threshold on the approximate value that keeps every row of the exact top-k
template <int METRIC>
__device__ inline float widen(float kth, float b) {
    if (METRIC == MQVS_METRIC_L2) {
        const float t = kth + 2.0f * b;
        return t + fabsf(t) * 2.4e-7f + 1e-30f;
    }
    const float t = kth - 2.0f * b;
    return t - fabsf(t) * 2.4e-7f - 1e-30f;
}


}  // namespace mqvs
