// kernels_ivf.hip -- kernels of the index path (mqvs_index_*, index.hip):
// the MSTG-type index (the reference's Search::VectorIndex behind
// VIWithColumnInPart::search, VIWithDataPart.cpp:858-957) laid out for HBM.
//
// Layout.  The part's rows are partitioned into `nlist` lists by a k-means
// coarse quantizer.  The lists are stored back to back as one bf16 plane in
// list order (each list padded to a multiple of 16 positions; blocked as
// [npos / 16][dpad / 32][16][32], 1 KiB pieces like the FLAT plane),
// with perm[pos] = segment row (-1 = padding) and pnorm[pos] = |y|^2.
//
// Search (one batch of nq queries, each probing nprobe lists):
//   k_plan_*      group the nq*nprobe (query, probe) pairs by list, cut each
//                 list's queries into 16-query work items, and give every
//                 pair its region of the candidate buffer
//   k_ivf_scan    per work item: stream the list's bf16 rows from HBM straight
//                 into MFMA A fragments (v_mfma_f32_16x16x32_bf16), the 16
//                 queries as B from LDS; approximate values to the regions
//   k_ivf_select  per query: radix-select the num_reorder best approximate
//                 values, ordered compaction, bitonic sort in LDS
// then the exact fp32 re-rank (k_rerank_ids, kernels_rerank.hip).
#include <cstdlib>

#include "mqvs_internal.h"
#include "select_common.h"

namespace mqvs {

typedef __bf16 ivf_bf16x8 __attribute__((ext_vector_type(8)));
typedef float ivf_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPlanThreads = 1024;
constexpr int kIvfWin = 4;      // 64-column windows loaded per group in the scan

// Exclusive scan of `n` int64 values produced by val(i) into out(i, prefix);
// returns the total.  One workgroup of kPlanThreads; each thread owns a
// contiguous run, run sums are scanned in LDS.
template <class Val, class Out>
__device__ int64_t block_exclusive_scan(int64_t n, Val val, Out out, int64_t *sh) {
    const int t = threadIdx.x;
    const int64_t per = (n + kPlanThreads - 1) / kPlanThreads;
    const int64_t b = t * per, e = min(n, b + per);
    int64_t s = 0;
    for (int64_t i = b; i < e; ++i) s += val(i);
    // block prefix of the run sums: wave scans, then the 16 wave totals
    const int lane = t & 63, wv = t >> 6;
    int64_t inc = s;
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    if (t == 0) {
        int64_t acc = 0;
        for (int w = 0; w < kPlanThreads / 64; ++w) {
            const int64_t v = sh[w];
            sh[w] = acc;
            acc += v;
        }
        sh[kPlanThreads] = acc;
    }
    __syncthreads();
    int64_t run = sh[wv] + inc - s;
    for (int64_t i = b; i < e; ++i) {
        const int64_t v = val(i);
        out(i, run);
        run += v;
    }
    const int64_t total = sh[kPlanThreads];
    __syncthreads();
    return total;
}

// Plan, in four launches (the pairs are spread over the grid; only the two
// prefix sums run in a single workgroup):
//   count    lcount[l] = pairs probing list l
//   lists    exclusive scans over the lists: lstart (pairs), work items
//   scatter  pairs grouped by list; per query, probe offsets inside its region
//   queries  exclusive scan of the query regions (qstart)
__global__ __launch_bounds__(256) void k_plan_count(IvfParams p) {
    const int64_t E = (int64_t)p.nq * p.nprobe;
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < E; e += (int64_t)gridDim.x * 256) {
        const int64_t l = p.probes[e];
        if (l >= 0 && l < p.nlist) atomicAdd(&p.lcount[l], 1);
    }
}

// Workgroup b owns lists [b 16 kPlanThreads, (b + 1) 16 kPlanThreads): wave
// w of it owns S of them (S a multiple of 64) and walks them 64 at a time,
// lane l on list w S + 64 s + l, so every load is coalesced; the (pair count,
// length) of its <= 16 steps stay in registers.  The three prefix sums (pairs,
// work items, streamed rows) are wave scans with a carry, then one combine
// over the 16 wave totals and, with more than one workgroup, the totals of the
// workgroups before (bsum, written by the SUMS pass of the same kernel).
// (One workgroup walking 39063 lists took 0.074 ms; three take ~0.01.)
template <bool SUMS>
__global__ __launch_bounds__(kPlanThreads) void k_plan_lists_reg(IvfParams p) {
    constexpr int ST = 16;
    constexpr int NWV = kPlanThreads / 64;
    __shared__ int64_t sh[3][NWV];
    const int base = blockIdx.x * ST * kPlanThreads;
    const int L = min(p.nlist - base, ST * kPlanThreads);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int S = ((L + NWV - 1) / NWV + 63) / 64 * 64;
    const int qs = p.qg == 64 ? 6 : p.qg == 32 ? 5 : 4;  // qg is 16, 32 or 64
    int cnt[ST], len[ST];
#pragma unroll
    for (int u = 0; u < ST; ++u) {
        const int i = wv * S + 64 * u + lane;
        const bool in = 64 * u < S && i < L;
        cnt[u] = in ? p.lcount[base + i] : 0;
        len[u] = in ? (int)(p.list_off[base + i + 1] - p.list_off[base + i]) : 0;
    }
    auto items_of = [&](int u) { return (int64_t)((cnt[u] + p.qg - 1) >> qs) * ((len[u] + p.chunk - 1) / p.chunk); };
    auto rows_of = [&](int u) { return (int64_t)((cnt[u] + p.qg - 1) >> qs) * len[u]; };
    int64_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
    for (int u = 0; u < ST; ++u) {
        w0 += cnt[u];
        w1 += items_of(u);
        w2 += rows_of(u);
    }
    for (int o = 32; o > 0; o >>= 1) {
        w0 += __shfl_xor(w0, o);
        w1 += __shfl_xor(w1, o);
        w2 += __shfl_xor(w2, o);
    }
    if (lane == 0) {
        sh[0][wv] = w0;
        sh[1][wv] = w1;
        sh[2][wv] = w2;
    }
    __syncthreads();
    if (SUMS) {
        if (t < 3) {
            int64_t v = 0;
            for (int w = 0; w < NWV; ++w) v += sh[t][w];
            p.bsum[3 * blockIdx.x + t] = v;
        }
        return;
    }
    int64_t c0 = 0, c1 = 0, t1 = 0, t2 = 0;
    for (int w = 0; w < NWV; ++w) {
        if (w < wv) {
            c0 += sh[0][w];
            c1 += sh[1][w];
        }
        t1 += sh[1][w];
        t2 += sh[2][w];
    }
    if (gridDim.x > 1) {
        t1 = t2 = 0;
        for (int b = 0; b < (int)gridDim.x; ++b) {
            if (b < (int)blockIdx.x) {
                c0 += p.bsum[3 * b];
                c1 += p.bsum[3 * b + 1];
            }
            t1 += p.bsum[3 * b + 1];
            t2 += p.bsum[3 * b + 2];
        }
    }
#pragma unroll
    for (int u = 0; u < ST; ++u) {
        if (64 * u >= S) break;  // wave-uniform
        const int64_t v0 = cnt[u], v1 = items_of(u);
        int64_t i0 = v0, i1 = v1;
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y0 = __shfl_up(i0, o), y1 = __shfl_up(i1, o);
            if (lane >= o) {
                i0 += y0;
                i1 += y1;
            }
        }
        const int i = wv * S + 64 * u + lane;
        if (i < L) {
            p.lstart[base + i] = c0 + i0 - v0;
            p.lfill[base + i] = 0;  // the scatter's cursors (no memset of their own)
            int64_t r1 = c1 + i1 - v1;
            const int g = (cnt[u] + p.qg - 1) >> qs;
            const int nc = (len[u] + p.chunk - 1) / p.chunk;
            for (int j = 0; j < g; ++j)
                for (int cc = 0; cc < nc; ++cc) {
                    p.item_list[r1] = base + i;
                    p.item_grp[r1] = j;
                    p.item_chk[r1] = cc;
                    ++r1;
                }
        }
        c0 += __shfl(i0, 63);
        c1 += __shfl(i1, 63);
    }
    if (t == 0 && blockIdx.x == 0) {
        *p.nitems = (int)t1;
        p.stats[1] = t1;
        p.stats[2] = t2 * p.dpad * 2;
        p.stats[3] = (int64_t)p.nq * p.nprobe;
    }
}

// Workgroup b owns kPlanBlk lists: their (pair count, length) are staged in
// LDS by coalesced loads, then thread t walks lists [kPlanPer t, kPlanPer (t +
// 1)) sequentially, so the block does one wave scan per prefix sum instead of
// one per 64 lists (the register walk above: 35 us for 39063 lists in 3
// workgroups).  Multi-workgroup carries as above (bsum, SUMS pass).
constexpr int kPlanPer = 4;
constexpr int kPlanBlk = kPlanPer * kPlanThreads;

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    return v;
}

template <bool SUMS>
__global__ __launch_bounds__(kPlanThreads) void k_plan_lists_blk(IvfParams p) {
    constexpr int NWV = kPlanThreads / 64;
    __shared__ int s_cnt[kPlanBlk], s_len[kPlanBlk];
    __shared__ int64_t sh[3][NWV];
    const int base = blockIdx.x * kPlanBlk;
    const int L = min(p.nlist - base, kPlanBlk);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int qs = p.qg == 64 ? 6 : p.qg == 32 ? 5 : 4;  // qg is 16, 32 or 64
    for (int i = t; i < kPlanBlk; i += kPlanThreads) {
        const bool in = i < L;
        s_cnt[i] = in ? p.lcount[base + i] : 0;
        s_len[i] = in ? (int)(p.list_off[base + i + 1] - p.list_off[base + i]) : 0;
    }
    __syncthreads();
    int64_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
    for (int r = 0; r < kPlanPer; ++r) {
        const int c = s_cnt[kPlanPer * t + r], l = s_len[kPlanPer * t + r];
        const int64_t g = (c + p.qg - 1) >> qs;
        a0 += c;
        a1 += g * ((l + p.chunk - 1) / p.chunk);
        a2 += g * l;
    }
    const int64_t i0 = wave_incl_scan(a0), i1 = wave_incl_scan(a1), i2 = wave_incl_scan(a2);
    if (lane == 63) {
        sh[0][wv] = i0;
        sh[1][wv] = i1;
        sh[2][wv] = i2;
    }
    __syncthreads();
    if (SUMS) {
        if (t < 3) {
            int64_t v = 0;
            for (int w = 0; w < NWV; ++w) v += sh[t][w];
            p.bsum[3 * blockIdx.x + t] = v;
        }
        return;
    }
    int64_t c0 = i0 - a0, c1 = i1 - a1, t1 = 0, t2 = 0;
    for (int w = 0; w < NWV; ++w) {
        if (w < wv) {
            c0 += sh[0][w];
            c1 += sh[1][w];
        }
        t1 += sh[1][w];
        t2 += sh[2][w];
    }
    if (gridDim.x > 1) {
        t1 = t2 = 0;
        for (int b = 0; b < (int)gridDim.x; ++b) {
            if (b < (int)blockIdx.x) {
                c0 += p.bsum[3 * b];
                c1 += p.bsum[3 * b + 1];
            }
            t1 += p.bsum[3 * b + 1];
            t2 += p.bsum[3 * b + 2];
        }
    }
#pragma unroll
    for (int r = 0; r < kPlanPer; ++r) {
        const int li = kPlanPer * t + r;
        if (li >= L) break;
        const int c = s_cnt[li], l = s_len[li];
        const int g = (c + p.qg - 1) >> qs;
        const int nc = (l + p.chunk - 1) / p.chunk;
        p.lstart[base + li] = c0;
        p.lfill[base + li] = 0;  // the scatter's cursors (no memset of their own)
        for (int j = 0; j < g; ++j)
            for (int cc = 0; cc < nc; ++cc) {
                p.item_list[c1] = base + li;
                p.item_grp[c1] = j;
                p.item_chk[c1] = cc;
                ++c1;
            }
        c0 += c;
    }
    if (t == 0 && blockIdx.x == 0) {
        *p.nitems = (int)t1;
        p.stats[1] = t1;
        p.stats[2] = t2 * p.dpad * 2;
        p.stats[3] = (int64_t)p.nq * p.nprobe;
    }
}

// One workgroup for any nlist: the same wave-strided layout with the per-list
// values loaded again in the second pass instead of kept in registers.  Kept
// for A/B (MQVS_IVF_PLAN=1, measurement build); the default is
// k_plan_lists_blk above.  (A contiguous run of lists per
// thread made every load of a wave touch 64 different lines: 0.27 ms of plan
// at 39063 lists against 0.05 at 10000.)
__global__ __launch_bounds__(kPlanThreads) void k_plan_lists(IvfParams p) {
    constexpr int NWV = kPlanThreads / 64;
    __shared__ int64_t sh[3][NWV];
    const int L = p.nlist;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int S = ((L + NWV - 1) / NWV + 63) / 64 * 64;
    const int qs = p.qg == 64 ? 6 : p.qg == 32 ? 5 : 4;  // qg is 16, 32 or 64
    auto load = [&](int u, int &cnt, int &len) {
        const int i = wv * S + 64 * u + lane;
        const bool in = i < L;
        cnt = in ? p.lcount[i] : 0;
        len = in ? (int)(p.list_off[i + 1] - p.list_off[i]) : 0;
    };
    auto items_of = [&](int cnt, int len) {
        return (int64_t)((cnt + p.qg - 1) >> qs) * ((len + p.chunk - 1) / p.chunk);
    };
    int64_t w0 = 0, w1 = 0, w2 = 0;
    const int steps = S / 64;
#pragma unroll 8
    for (int u = 0; u < steps; ++u) {
        int cnt, len;
        load(u, cnt, len);
        w0 += cnt;
        w1 += items_of(cnt, len);
        w2 += (int64_t)((cnt + p.qg - 1) >> qs) * len;
    }
    for (int o = 32; o > 0; o >>= 1) {
        w0 += __shfl_xor(w0, o);
        w1 += __shfl_xor(w1, o);
        w2 += __shfl_xor(w2, o);
    }
    if (lane == 0) {
        sh[0][wv] = w0;
        sh[1][wv] = w1;
        sh[2][wv] = w2;
    }
    __syncthreads();
    int64_t c0 = 0, c1 = 0, t1 = 0, t2 = 0;
    for (int w = 0; w < NWV; ++w) {
        if (w < wv) {
            c0 += sh[0][w];
            c1 += sh[1][w];
        }
        t1 += sh[1][w];
        t2 += sh[2][w];
    }
    for (int u = 0; u < steps; ++u) {
        int cnt, len;
        load(u, cnt, len);
        const int64_t v0 = cnt, v1 = items_of(cnt, len);
        int64_t i0 = v0, i1 = v1;
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y0 = __shfl_up(i0, o), y1 = __shfl_up(i1, o);
            if (lane >= o) {
                i0 += y0;
                i1 += y1;
            }
        }
        const int i = wv * S + 64 * u + lane;
        if (i < L) {
            p.lstart[i] = c0 + i0 - v0;
            p.lfill[i] = 0;
            int64_t r1 = c1 + i1 - v1;
            const int g = (cnt + p.qg - 1) >> qs;
            const int nc = (len + p.chunk - 1) / p.chunk;
            for (int j = 0; j < g; ++j)
                for (int cc = 0; cc < nc; ++cc) {
                    p.item_list[r1] = i;
                    p.item_grp[r1] = j;
                    p.item_chk[r1] = cc;
                    ++r1;
                }
        }
        c0 += __shfl(i0, 63);
        c1 += __shfl(i1, 63);
    }
    if (t == 0) {
        *p.nitems = (int)t1;
        p.stats[1] = t1;
        p.stats[2] = t2 * p.dpad * 2;
        p.stats[3] = (int64_t)p.nq * p.nprobe;
    }
}

__global__ __launch_bounds__(256) void k_plan_scatter(IvfParams p) {
    const int64_t E = (int64_t)p.nq * p.nprobe;
    const int64_t gt = blockIdx.x * 256ll + threadIdx.x, gs = (int64_t)gridDim.x * 256;
    // pairs grouped by list (order inside a list is free: every pair owns
    // its output region, so results do not depend on it)
    for (int64_t e = gt; e < E; e += gs) {
        const int64_t l = p.probes[e];
        if (l >= 0 && l < p.nlist) {
            const int slot = atomicAdd(&p.lfill[l], 1);
            p.lq[p.lstart[l] + slot] = (int)e;
        }
    }
    // per query: its probes' regions back to back in probe order (offsets
    // relative to the query's region; qstart added by the scan)
    for (int64_t q = gt; q < p.nq; q += gs) {
        int64_t tot = 0;
        for (int r = 0; r < p.nprobe; ++r) {
            const int64_t e = q * p.nprobe + r;
            const int64_t l = p.probes[e];
            p.qbase[e] = tot;
            if (l >= 0 && l < p.nlist) tot += p.list_off[l + 1] - p.list_off[l];
        }
        p.qstart[q] = tot;
    }
}

__global__ __launch_bounds__(kPlanThreads) void k_plan_queries(IvfParams p) {
    __shared__ int64_t sh[kPlanThreads + 1];
    const int64_t total = block_exclusive_scan(
        p.nq, [&](int64_t i) { return p.qstart[i]; }, [&](int64_t i, int64_t v) { p.qstart[i] = v; }, sh);
    if (threadIdx.x == 0) {
        p.qstart[p.nq] = total;
        p.stats[0] = total;  // approximate values written
    }
}

// Plan for few pairs (E = nq * nprobe <= kPlanSmallE; nprobe 1..4 at nq
// 1000), in ONE workgroup: the (list, pair) keys are sorted in LDS, so the
// lists a query batch actually probes are runs of the sorted keys -- the
// general plan above scans every list of the index (39063: zero-fill, count,
// two passes over the lists, scatter, query scan = six launches, ~43 us at
// nq 1000, nprobe 1).  Outputs are the general plan's: lstart / lcount of the
// probed lists (the scan reads no other), the pairs grouped by list in lq,
// items in list order, the query regions (qbase, qstart) and the stats.
constexpr int kPlanSmallE = 4096;
__global__ __launch_bounds__(kPlanThreads) void k_plan_small(IvfParams p) {
    __shared__ uint64_t key[kPlanSmallE];
    __shared__ int64_t sh[kPlanThreads + 1];
    __shared__ unsigned long long s_rows;
    const int t = threadIdx.x;
    const int E = p.nq * p.nprobe;
    const int qs = p.qg == 64 ? 6 : p.qg == 32 ? 5 : 4;  // qg is 16, 32 or 64
    int N = 1;
    while (N < E) N <<= 1;
    for (int i = t; i < N; i += kPlanThreads) {
        uint64_t k = ~0ull;
        if (i < E) {
            const int64_t l = p.probes[i];
            if (l >= 0 && l < p.nlist) k = ((uint64_t)l << 32) | (uint32_t)i;
        }
        key[i] = k;
    }
    if (t == 0) s_rows = 0;
    __syncthreads();
    for (int size = 2; size <= N; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < (N >> 1); i += kPlanThreads) {
                const int lo = 2 * stride * (i / stride) + (i % stride), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint64_t a = key[lo], b = key[hi];
                if ((b < a) == up) {
                    key[lo] = b;
                    key[hi] = a;
                }
            }
            __syncthreads();
        }
    // valid keys [0, Ev); a run of one list starts where the list changes
    auto list_at = [&](int i) { return (int)(key[i] >> 32); };
    auto valid = [&](int i) { return key[i] != ~0ull; };
    auto head = [&](int i) { return valid(i) && (i == 0 || list_at(i - 1) != list_at(i)); };
    // run length: the first position of a larger list (binary search)
    auto run_len = [&](int i) {
        const uint64_t bound = ((uint64_t)(uint32_t)list_at(i) + 1) << 32;
        int lo = i + 1, hi = N;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (key[mid] < bound) lo = mid + 1;
            else hi = mid;
        }
        return lo - i;
    };
    auto list_len = [&](int l) { return (int)(p.list_off[l + 1] - p.list_off[l]); };
    const int64_t nitems = block_exclusive_scan(
        N,
        [&](int64_t i) -> int64_t {
            if (!head((int)i)) return 0;
            const int g = (run_len((int)i) + p.qg - 1) >> qs;
            return (int64_t)g * ((list_len(list_at((int)i)) + p.chunk - 1) / p.chunk);
        },
        [&](int64_t i, int64_t r1) {
            if (!valid((int)i)) return;
            const int l = list_at((int)i);
            p.lq[i] = (int)(uint32_t)key[i];
            if (!head((int)i)) return;
            const int c = run_len((int)i), len = list_len(l);
            const int g = (c + p.qg - 1) >> qs, nc = (len + p.chunk - 1) / p.chunk;
            p.lstart[l] = i;
            p.lcount[l] = c;
            atomicAdd(&s_rows, (unsigned long long)g * (unsigned long long)len);
            for (int j = 0; j < g; ++j)
                for (int cc = 0; cc < nc; ++cc) {
                    p.item_list[r1] = l;
                    p.item_grp[r1] = j;
                    p.item_chk[r1] = cc;
                    ++r1;
                }
        },
        sh);
    // per query: its probes' regions back to back in probe order, then the
    // exclusive scan of the query totals
    for (int q = t; q < p.nq; q += kPlanThreads) {
        int64_t tot = 0;
        for (int r = 0; r < p.nprobe; ++r) {
            const int64_t e = (int64_t)q * p.nprobe + r;
            const int64_t l = p.probes[e];
            p.qbase[e] = tot;
            if (l >= 0 && l < p.nlist) tot += p.list_off[l + 1] - p.list_off[l];
        }
        p.qstart[q] = tot;
    }
    __syncthreads();
    const int64_t total = block_exclusive_scan(
        p.nq, [&](int64_t i) { return p.qstart[i]; }, [&](int64_t i, int64_t v) { p.qstart[i] = v; }, sh);
    if (t == 0) {
        p.qstart[p.nq] = total;
        *p.nitems = (int)nitems;
        p.stats[0] = total;
        p.stats[1] = nitems;
        p.stats[2] = (int64_t)s_rows * p.dpad * 2;
        p.stats[3] = E;
    }
}

// Plan for the dense case (every query probes every list, probe r = list r:
// the coarse quantizer's centroid chunks), in one grid kernel.
__global__ __launch_bounds__(256) void k_plan_dense(IvfParams p, int64_t npos) {
    const int L = p.nlist, G = (p.nq + p.qg - 1) / p.qg;
    const int64_t E = (int64_t)p.nq * L;
    const int64_t gt = blockIdx.x * 256ll + threadIdx.x, gs = (int64_t)gridDim.x * 256;
    for (int64_t e = gt; e < E; e += gs) {
        const int64_t q = e / L, l = e - q * L;
        p.lq[l * p.nq + q] = (int)e;
        p.qbase[e] = p.list_off[l];
    }
    // items (list, group, slice): lists here are centroid chunks of equal
    // length, so every list has the same slices
    const int NC = (int)((p.list_off[1] - p.list_off[0] + p.chunk - 1) / p.chunk);
    for (int64_t i = gt; i < (int64_t)L * G * NC; i += gs) {
        p.item_list[i] = (int)(i / ((int64_t)G * NC));
        p.item_grp[i] = (int)((i / NC) % G);
        p.item_chk[i] = (int)(i % NC);
    }
    for (int64_t l = gt; l < L; l += gs) {
        p.lcount[l] = p.nq;
        p.lstart[l] = l * p.nq;
    }
    for (int64_t q = gt; q <= p.nq; q += gs) p.qstart[q] = q * npos;
    if (gt == 0) {
        *p.nitems = L * G * NC;
        p.stats[0] = (int64_t)p.nq * npos;
        p.stats[1] = (int64_t)L * G * NC;
        p.stats[2] = (int64_t)G * npos * p.dpad * 2;
        p.stats[3] = E;
    }
}

// query q's candidate region (start, length)
__device__ inline void ivf_region(const IvfRegions &g, int q, int64_t &start, int64_t &T) {
    if (g.qstart) {
        start = g.qstart[q];
        T = g.qstart[q + 1] - start;
        return;
    }
    start = (int64_t)q * g.stride;
    T = 0;
    for (int r = 0; r < g.nprobe; ++r) {
        const int64_t l = g.probes[(int64_t)q * g.nprobe + r];
        if (l >= 0 && l < g.nlist) T += g.list_off[l + 1] - g.list_off[l];
    }
}

// pair mode's stats (the plan's in the grouped mode), by the select: query
// q's [values, items, plane bytes, pairs] to stats[4 q ..] (summed by the
// final copy, k_words_to_host: 4 atomics per query on the same 4 words
// serialised the select, 26 -> 75 us at nq 1000)
__device__ inline void ivf_pair_stats(const IvfRegions &g, int q, int64_t T, bool leader) {
    if (g.qstart || !g.stats || !leader) return;
    int64_t items = 0, pairs = 0;
    for (int r = 0; r < g.nprobe; ++r) {
        const int64_t l = g.probes[(int64_t)q * g.nprobe + r];
        if (l < 0 || l >= g.nlist) continue;
        items += (g.list_off[l + 1] - g.list_off[l] + g.chunk - 1) / g.chunk;
        ++pairs;
    }
    int64_t *o = g.stats + 4 * (int64_t)q;
    o[0] = T;
    o[1] = items;
    o[2] = T * g.dpad * 2;
    o[3] = pairs;
}

// Scan work item = one list x up to 16 QB queries (QB MFMA B blocks).  The
// query tile sits in LDS (row stride 2 dpad + 16 B: the 16 rows of a B block
// hit distinct bank groups).  Each wave takes 16-row blocks of the list; lane
// (l16, c) streams row l16 straight from HBM into A fragments: per 64-column
// window, k-step 1 = bytes [16c, 16c + 16), k-step 2 = [64 + 16c, ...), so
// one load instruction covers a contiguous 64-B half-window of 16 rows.
// kIvfWin windows are in flight per lane and the next group is prefetched
// while the current one feeds the MFMAs; every A fragment serves QB MFMAs.
template <int METRIC, int QB, bool NTL>
__global__ __launch_bounds__(256) void k_ivf_scan(IvfParams p) {
    constexpr int QG = 16 * QB;
    // plane reads: each probed list's rows are read once per query group
    // (NTL: non-temporal, kept out of the caches' retention)
    auto ldp = [](const uint16_t *a) __attribute__((always_inline)) {
        typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
        if (NTL)
            return __builtin_bit_cast(ivf_bf16x8, __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(a)));
        return *reinterpret_cast<const ivf_bf16x8 *>(a);
    };
    extern __shared__ __attribute__((aligned(16))) unsigned char qtile[];  // QG x (2 dpad + 16) B
    __shared__ int s_ent[QG];
    __shared__ int64_t s_base[QG];
    __shared__ float s_qn[QG];
    const int64_t qstr = 2 * p.dpad + 16;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int l16 = lane & 15, c = lane >> 4;
    const int nitems = p.pair_stride ? p.nq * p.nprobe * p.pair_nch : *p.nitems;
    const int cpr = (int)(p.dpad / 8);  // 16-B chunks per query row
    const int ngrp = (int)((p.dpad / 64 + kIvfWin - 1) / kIvfWin);
    for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
        int l, g, chk, pe = -1;
        if (p.pair_stride) {
            // pair mode: one query's probe; slices past its list's end are
            // empty.  Slice-major (slice 0 of every pair first): pair-major
            // gave the workgroups of the first slices two items each and the
            // rest none (scan 82 -> 169 us at nq 1000, nprobe 1)
            const int E = p.nq * p.nprobe;
            chk = it / E;
            pe = it - chk * E;
            g = 0;
            const int64_t ll = p.probes[pe];
            if (ll < 0 || ll >= p.nlist) continue;  // (uniform over the workgroup)
            l = (int)ll;
            if ((int64_t)chk * p.chunk >= p.list_off[l + 1] - p.list_off[l]) continue;
        } else {
            l = p.item_list[it];
            g = p.item_grp[it];
            chk = p.item_chk[it];
        }
        const int64_t pos0 = p.list_off[l];
        const int cb = p.chunk / 16;  // 16-position blocks per work item
        const int nb = (int)min<int64_t>((p.list_off[l + 1] - pos0) / 16, (int64_t)(chk + 1) * cb);
        // the wave's blocks b0, b0 + 4, ... as one sequence of (block, window
        // group) steps: the next step's loads -- the next block's first group
        // included -- are in flight while a step feeds the MFMAs
        const int b0 = chk * cb + w;
        const int nsteps = b0 < nb ? (nb - b0 + 3) / 4 * ngrp : 0;
        // the plane is blocked like the FLAT pre-filter plane: 16 positions x
        // 32 columns = 1 KiB per piece (k_ivf_pack), so each fragment load of a
        // wave reads one contiguous KiB (8 whole 128-B lines)
        const uint16_t *rp0 = p.plane + ((pos0 >> 4) + (int64_t)b0) * 16 * p.dpad + l16 * 32 + c * 8;
        const int64_t bstride = 4 * 16 * p.dpad;  // 4 blocks on
        auto load = [&](int st, ivf_bf16x8 *dst) {
            const int bi = st / ngrp, grp = st - bi * ngrp;
            const uint16_t *rp = rp0 + bi * bstride;
#pragma unroll
            for (int u = 0; u < kIvfWin; ++u) {
                const int64_t kw = ((int64_t)grp * kIvfWin + u) * 64;
                if (kw < p.dpad) {
                    dst[2 * u] = ldp(rp + (kw >> 5) * 512);
                    dst[2 * u + 1] = ldp(rp + ((kw >> 5) + 1) * 512);
                }
            }
        };
        // the first step's rows are requested before the query tile is staged
        // (its chain of dependent loads: pairs, regions, query rows): at ~256
        // positions per list the item setup is a large part of an item
        ivf_bf16x8 cur[2 * kIvfWin], nxt[2 * kIvfWin];
        if (nsteps > 0) load(0, cur);
        const int cnt = p.pair_stride ? 1 : min(QG, p.lcount[l] - g * QG);
        __syncthreads();  // the previous item's readers are done with qtile
        if (threadIdx.x < QG) {
            const int j = threadIdx.x;
            int e = -1;
            int64_t base = 0;
            if (p.pair_stride) {
                // the pair's region: its query's stride, after the lists of
                // the query's earlier probes
                if (j == 0) {
                    e = pe;
                    const int q = e / p.nprobe, r = e - q * p.nprobe;
                    base = (int64_t)q * p.pair_stride;
                    for (int r2 = 0; r2 < r; ++r2) {
                        const int64_t l2 = p.probes[(int64_t)q * p.nprobe + r2];
                        if (l2 >= 0 && l2 < p.nlist) base += p.list_off[l2 + 1] - p.list_off[l2];
                    }
                }
            } else {
                e = j < cnt ? p.lq[p.lstart[l] + (int64_t)g * QG + j] : -1;
                base = e >= 0 ? p.qstart[e / p.nprobe] + p.qbase[e] : 0;
            }
            s_ent[j] = e;
            s_base[j] = base;
            s_qn[j] = (e >= 0 && METRIC == MQVS_METRIC_L2) ? p.qnorm[e / p.nprobe] : 0.f;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < QG * cpr; i += 256) {
            const int j = i / cpr, cc = i - j * cpr;
            const int e = s_ent[j];
            uint4 v = make_uint4(0, 0, 0, 0);
            if (e >= 0) v = reinterpret_cast<const uint4 *>(p.q_hi + (int64_t)(e / p.nprobe) * p.dpad)[cc];
            *reinterpret_cast<uint4 *>(qtile + j * qstr + cc * 16) = v;
        }
        __syncthreads();
        const unsigned char *qp = qtile + l16 * qstr + c * 16;
        int ent[QB];
#pragma unroll
        for (int j = 0; j < QB; ++j) ent[j] = s_ent[16 * j + l16];
        ivf_f32x4 acc[QB];
        int32_t rows[4];
        float pn[4];
        for (int st = 0; st < nsteps; ++st) {
            const int bi = st / ngrp, grp = st - bi * ngrp;
            const int64_t lp = (int64_t)(b0 + 4 * bi) * 16 + 4 * c;
            if (grp == 0) {
#pragma unroll
                for (int j = 0; j < QB; ++j) acc[j] = ivf_f32x4{0.f, 0.f, 0.f, 0.f};
                // the block's position records, ahead of the next step's loads
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    rows[r] = p.perm[pos0 + lp + r];
                    pn[r] = METRIC == MQVS_METRIC_L2 ? p.pnorm[pos0 + lp + r] : 0.f;
                }
            }
            if (st + 1 < nsteps) load(st + 1, nxt);
#pragma unroll
            for (int u = 0; u < kIvfWin; ++u) {
                const int64_t kw = ((int64_t)grp * kIvfWin + u) * 64;
                if (kw < p.dpad) {
#pragma unroll
                    for (int j = 0; j < QB; ++j) {
                        const unsigned char *qj = qp + 16 * j * qstr + 2 * kw;
                        const ivf_bf16x8 q0 = *reinterpret_cast<const ivf_bf16x8 *>(qj);
                        const ivf_bf16x8 q1 = *reinterpret_cast<const ivf_bf16x8 *>(qj + 64);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[2 * u], q0, acc[j], 0, 0, 0);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[2 * u + 1], q1, acc[j], 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 2 * kIvfWin; ++u) cur[u] = nxt[u];
            if (grp != ngrp - 1) continue;
            // C: lane (l16, c) holds rows 4c..4c+3 of the block for query slot 16 j + l16
            int32_t rr[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int32_t row = rows[r];
                if (row >= 0 && p.filter && !bit_test(p.filter, row)) row = -1;
                if (row >= 0 && p.exists && !bit_test(p.exists, row)) row = -1;
                rr[r] = row;
            }
#pragma unroll
            for (int j = 0; j < QB; ++j) {
                if (ent[j] < 0) continue;
                Cand out[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float raw = acc[j][r];
                    if (METRIC == MQVS_METRIC_L2) raw = (s_qn[16 * j + l16] + pn[r]) - 2.0f * raw;
                    out[r].raw = rr[r] >= 0 ? raw : __builtin_nanf("");
                    out[r].row = rr[r] >= 0 ? (uint32_t)rr[r] : 0xFFFFFFFFu;
                }
                uint4 *dst = reinterpret_cast<uint4 *>(p.cand + s_base[16 * j + l16] + lp);
                dst[0] = *reinterpret_cast<const uint4 *>(&out[0]);
                dst[1] = *reinterpret_cast<const uint4 *>(&out[2]);
            }
        }
    }
}

// Per query: the R best approximate values, sorted by (key, row); at the R-th
// key the lowest rows win (every row of the region is distinct).  Writes the
// rows (for the exact re-rank) and, for first-stage-only searches, ids + the
// approximate distance.  NT threads per query; regions up to `keycap` values
// keep their keys in LDS for the four radix passes, longer ones stream them
// (4 loads in flight per thread).  The records below the R-th key and those at
// it are gathered in one pass with LDS atomics (their order does not matter:
// they are sorted); more ties at the R-th key than kTieCap, or than the
// record array has room for, fall back to a position-ordered pass for them.
constexpr int kTieCap = 64;  // <= every NT the kernel is launched with

// LARGE (R above kSortCap, num_reorder / k up to kLargeCap): the records go to
// 2 R records of global scratch per query (gscr) and are sorted there by
// global_sort (LDS runs of kSortCap, then merge passes); NT = SEL_THREADS.
template <int METRIC, int NT, bool LARGE = false>
__global__ __launch_bounds__(NT) void k_ivf_select(const Cand *cand, IvfRegions rg, int R,
                                                   int64_t *out_rows, int64_t id_offset, float *out_approx,
                                                   int keycap, uint4 *gscr, float *out_raw) {
    // pow2 >= R records (LARGE: kSortCap, the sort runs), then the key cache
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];
    __shared__ uint4 ties[kTieCap];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_wave[NT / 64];
    __shared__ int s_m, s_tie;
    static_assert(!LARGE || NT == SEL_THREADS, "global_sort strides by SEL_THREADS");
    int N = 1;
    while (N < R) N <<= 1;
    uint32_t *kc = reinterpret_cast<uint32_t *>(recs + (LARGE ? kSortCap : N));
    const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint4 *rr = LARGE ? gscr + (int64_t)q * 2 * R : recs;  // the records (LARGE: [0, R); [R, 2R) sort scratch)
    const int mcap = LARGE ? R : N;                        // room for records below th + ties
    int64_t rs0 = 0, T = 0;
    ivf_region(rg, q, rs0, T);
    ivf_pair_stats(rg, q, T, threadIdx.x == 0);
    const Cand *c = cand + rs0;
    auto gkey = [&](int64_t i) {
        const Cand e = c[i];
        return e.row == 0xFFFFFFFFu ? 0xFFFFFFFFu : okey<METRIC>(e.raw);
    };
    const bool cached = T <= keycap;
    if (t == 0) {
        s_m = 0;
        s_tie = 0;
    }
    uint32_t th;
    if (cached) {
        int64_t i = t;
        for (; i + 3 * NT < T; i += 4 * NT) {
            const uint32_t k0 = gkey(i), k1 = gkey(i + NT), k2 = gkey(i + 2 * NT), k3 = gkey(i + 3 * NT);
            kc[i] = k0;
            kc[i + NT] = k1;
            kc[i + 2 * NT] = k2;
            kc[i + 3 * NT] = k3;
        }
        for (; i < T; i += NT) kc[i] = gkey(i);
        __syncthreads();
        th = block_radix_select_mlp<NT>([&](int64_t j) { return kc[j]; }, T, R, hist, sh);
    } else {
        th = block_radix_select_mlp<NT>(gkey, T, R, hist, sh);
    }
    // fewer than R valid keys: every valid one; else those below th (fewer
    // than R) + the ties at th (at most kTieCap kept)
    const bool all = th == 0xFFFFFFFEu;
    auto visit = [&](int64_t i, uint32_t key) {
        if (key == 0xFFFFFFFFu) return;
        if (all || key < th) {
            const Cand e = c[i];
            const int pos = atomicAdd(&s_m, 1);
            if (pos < R) rr[pos] = make_uint4(key, e.row, __builtin_bit_cast(uint32_t, e.raw), 0u);
        } else if (key == th) {
            const Cand e = c[i];
            const int pos = atomicAdd(&s_tie, 1);
            if (pos < kTieCap) ties[pos] = make_uint4(key, e.row, __builtin_bit_cast(uint32_t, e.raw), 0u);
        }
    };
    {
        int64_t i = t;
        for (; i + 3 * NT < T; i += 4 * NT) {
            const uint32_t k0 = cached ? kc[i] : gkey(i), k1 = cached ? kc[i + NT] : gkey(i + NT),
                           k2 = cached ? kc[i + 2 * NT] : gkey(i + 2 * NT),
                           k3 = cached ? kc[i + 3 * NT] : gkey(i + 3 * NT);
            visit(i, k0);
            visit(i + NT, k1);
            visit(i + 2 * NT, k2);
            visit(i + 3 * NT, k3);
        }
        for (; i < T; i += NT) visit(i, cached ? kc[i] : gkey(i));
    }
    __syncthreads();
    const int below = min(s_m, R);
    int m = below;
    if (!all) {
        const int nt = s_tie;
        if (nt <= kTieCap && below + nt <= mcap) {
            // the ties after the records below th (kTieCap <= NT)
            if (t < nt) rr[below + t] = ties[t];
            m = below + nt;
        } else {
            // mass ties: the first R - below of them by position
            if (t == 0) s_m = below;
            __syncthreads();
            for (int64_t base = 0; base < T; base += NT) {
                const int m0 = s_m;
                if (m0 >= R) break;
                const int64_t i = base + t;
                bool flag = false;
                uint32_t key = 0xFFFFFFFFu;
                if (i < T) {
                    key = cached ? kc[i] : gkey(i);
                    flag = key == th;
                }
                const uint64_t bal = __ballot(flag);
                if (lane == 0) s_wave[wv] = __popcll(bal);
                __syncthreads();
                int off = m0;
                for (int x = 0; x < wv; ++x) off += s_wave[x];
                off += __popcll(bal & ((1ull << lane) - 1ull));
                if (flag && off < R) {
                    const Cand e = c[i];
                    rr[off] = make_uint4(key, e.row, __builtin_bit_cast(uint32_t, e.raw), 0u);
                }
                __syncthreads();
                if (t == 0) {
                    int tot = 0;
                    for (int x = 0; x < NT / 64; ++x) tot += s_wave[x];
                    s_m = min(R, m0 + tot);
                }
                __syncthreads();
            }
            m = s_m;
        }
    }
    __syncthreads();
    const uint4 *sorted = recs;
    if constexpr (LARGE) {
        sorted = global_sort(rr, rr + R, m, recs);
    } else {
    int Nm = 1;
    while (Nm < m) Nm <<= 1;
    for (int i = m + t; i < Nm; i += NT) recs[i] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    __syncthreads();
    // bitonic sort of recs[0, Nm) (block-wide, NT threads)
    for (int size = 2; size <= Nm; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < (Nm >> 1); i += NT) {
                const int lo = 2 * stride * (i / stride) + (i % stride);
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint4 a = recs[lo], b2 = recs[hi];
                if (rec_less(b2, a) == up) {
                    recs[lo] = b2;
                    recs[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    }
    for (int i = t; i < R; i += NT) {
        const bool ok = i < m;
        const uint4 r = ok ? sorted[i] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (out_approx) {
            out_rows[(int64_t)q * R + i] = ok ? (int64_t)r.y + id_offset : -1;
            const float raw = __builtin_bit_cast(float, r.z);
            float dist = (METRIC == MQVS_METRIC_COSINE) ? cos_dist(raw) : raw;
            if (!ok) dist = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f : 3.40282347e+38f;
            out_approx[(int64_t)q * R + i] = dist;
        } else {
            out_rows[(int64_t)q * R + i] = ok ? (int64_t)r.y : -1;
        }
        // (the re-rank's bound pruning: the raw approximate values, NaN past the valid ones)
        if (out_raw) out_raw[(int64_t)q * R + i] = ok ? __builtin_bit_cast(float, r.z) : __builtin_nanf("");
    }
}

// Small R (the coarse quantizer: R = nprobe <= 16): one wave per query.  Each
// lane keeps its RM best (key, row) in registers over a strided slice of the
// region (8 loads in flight); the wave then pops the R smallest heads (64-bit
// min over the lanes per pop).  Order = (key, row), like k_ivf_select for a
// monotone perm.
template <int METRIC, int RM>
__global__ __launch_bounds__(256) void k_ivf_select_small(const Cand *cand, IvfRegions rg, int nq, int R,
                                                         int64_t *out_rows, int64_t id_offset, float *out_approx) {
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;  // wave-uniform
    int64_t rs0 = 0, T = 0;
    ivf_region(rg, q, rs0, T);
    ivf_pair_stats(rg, q, T, lane == 0);
    const Cand *c = cand + rs0;
    uint64_t best[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) best[i] = ~0ull;
    auto insert = [&](uint64_t x) {
        if (x >= best[RM - 1]) return;
#pragma unroll
        for (int j = 0; j < RM; ++j) {
            const uint64_t lo = x < best[j] ? x : best[j];
            const uint64_t hi = x < best[j] ? best[j] : x;
            best[j] = lo;
            x = hi;
        }
    };
    for (int64_t i0 = lane; i0 < T; i0 += 64 * U) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + 64 * u;
            const Cand e = i < T ? c[i] : Cand{0.f, 0xFFFFFFFFu};
            v[u] = e.row == 0xFFFFFFFFu ? ~0ull : ((uint64_t)okey<METRIC>(e.raw) << 32) | e.row;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) insert(v[u]);
    }
    // the R smallest over the wave: pop the smallest head R times
    int head = 0;
    for (int i = 0; i < R; ++i) {
        uint64_t mine = ~0ull;
#pragma unroll
        for (int j = 0; j < RM; ++j)
            if (j == head) mine = best[j];
        uint64_t m = mine;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t y = __shfl_xor(m, o);
            m = y < m ? y : m;
        }
        if (mine == m && m != ~0ull) ++head;  // (key, row) pairs are distinct
        if (lane == 0) {
            const bool ok = m != ~0ull && (uint32_t)(m >> 32) != 0xFFFFFFFFu;
            out_rows[(int64_t)q * R + i] = ok ? (int64_t)(uint32_t)m + (out_approx ? id_offset : 0) : -1;
        }
    }
}

// ---- build kernels ---------------------------------------------------------

// plane[pos] = bf16(rows[perm[pos]]) (zero for padding and columns >= d),
// pnorm[pos] = |y|^2
__global__ __launch_bounds__(256) void k_ivf_pack(const float *rows, const float *norms, int d,
                                                  const int32_t *perm, int64_t npos, int64_t dpad,
                                                  uint16_t *plane, float *pnorm) {
    const int64_t c8 = dpad / 8;
    const int64_t total = npos * c8;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t pos = i / c8, cc = i - pos * c8;
        const int32_t row = perm[pos];
        uint16_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t col = cc * 8 + j;
            const float x = (row >= 0 && col < d) ? rows[(int64_t)row * d + col] : 0.f;
            v[j] = f32_to_bf16_rn(x);
        }
        uint4 o;
        o.x = v[0] | ((uint32_t)v[1] << 16);
        o.y = v[2] | ((uint32_t)v[3] << 16);
        o.z = v[4] | ((uint32_t)v[5] << 16);
        o.w = v[6] | ((uint32_t)v[7] << 16);
        // 16-position blocks of 32-column pieces (1 KiB each): see k_ivf_scan
        const int64_t col0 = cc * 8;
        *reinterpret_cast<uint4 *>(plane + ((pos >> 4) * (dpad / 32) + (col0 >> 5)) * 512 + (pos & 15) * 32 +
                                   (col0 & 31)) = o;
        if (cc == 0) pnorm[pos] = row >= 0 ? norms[row] : 0.f;
    }
}

// dst[i] = src[idx[i]] (rows of d floats, source row stride src_ld; idx null = identity)
__global__ __launch_bounds__(256) void k_gather_rows(const float *src, int64_t src_ld, int d, const int64_t *idx,
                                                     int64_t m, float *dst) {
    const int64_t total = m * d;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / d, col = i - r * d;
        dst[i] = src[(idx ? idx[r] : r) * src_ld + col];
    }
}

// k-means update: centroid c = mean of its members (rows order[off[c]..off[c+1]),
// summed in that order, so the result is deterministic); empty clusters keep
// their centroid.
__global__ __launch_bounds__(256) void k_centroid_mean(const float *rows, int d, const int32_t *order,
                                                       const int64_t *off, float *cent) {
    const int c = blockIdx.x;
    const int64_t b = off[c], e = off[c + 1];
    if (e <= b) return;
    const float inv = 1.0f / (float)(e - b);
    for (int j = threadIdx.x; j < d; j += 256) {
        float s = 0.f;
        for (int64_t i = b; i < e; ++i) s += rows[(int64_t)order[i] * d + j];
        cent[(int64_t)c * d + j] = s * inv;
    }
}

// probes[q][j] = j: every query probes every list (the coarse quantizer's
// centroid chunks)
__global__ __launch_bounds__(256) void k_iota_probes(int64_t *probes, int64_t E, int np) {
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < E; e += (int64_t)gridDim.x * 256) probes[e] = e % np;
}

// ---- launchers -------------------------------------------------------------

void launch_ivf_plan_dense(const IvfParams &p, int64_t npos, hipStream_t s) {
    const int64_t E = (int64_t)p.nq * p.nlist;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((E + 255) / 256, 2048));
    hipLaunchKernelGGL(k_plan_dense, dim3(grid), dim3(256), 0, s, p, npos);
}

void launch_iota_probes(int64_t *probes, int nq, int np, hipStream_t s) {
    const int64_t E = (int64_t)nq * np;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((E + 255) / 256, 1024));
    hipLaunchKernelGGL(k_iota_probes, dim3(grid), dim3(256), 0, s, probes, E, np);
}

void launch_ivf_plan(const IvfParams &p, hipStream_t s) {
    const int64_t E = (int64_t)p.nq * p.nprobe;
    if (E <= kPlanSmallE && tune_int("MQVS_IVF_PLAN", 0) == 0) {
        hipLaunchKernelGGL(k_plan_small, dim3(1), dim3(kPlanThreads), 0, s, p);
        return;
    }
    // (lfill: zeroed by the list pass; a fill kernel, not hipMemsetAsync: the
    // runtime's fill took two launches)
    launch_fill2(reinterpret_cast<uint32_t *>(p.lcount), p.nlist, 0u, nullptr, 0, 0u, s);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((std::max(E, (int64_t)p.nq) + 255) / 256, 2048));
    hipLaunchKernelGGL(k_plan_count, dim3(grid), dim3(256), 0, s, p);
    // A/B (measurement build): 1 one workgroup, 2 register walk, 3 the list
    // kernels even for few pairs (k_plan_small above otherwise)
    const int plan = tune_int("MQVS_IVF_PLAN", 0);
    if (plan == 1) {
        hipLaunchKernelGGL(k_plan_lists, dim3(1), dim3(kPlanThreads), 0, s, p);
    } else if (plan == 2) {
        const int nb = (p.nlist + 16 * kPlanThreads - 1) / (16 * kPlanThreads);
        if (nb > 1) hipLaunchKernelGGL(k_plan_lists_reg<true>, dim3(nb), dim3(kPlanThreads), 0, s, p);
        hipLaunchKernelGGL(k_plan_lists_reg<false>, dim3(std::max(nb, 1)), dim3(kPlanThreads), 0, s, p);
    } else {
        const int nb = (p.nlist + kPlanBlk - 1) / kPlanBlk;
        if (nb > 1) hipLaunchKernelGGL(k_plan_lists_blk<true>, dim3(nb), dim3(kPlanThreads), 0, s, p);
        hipLaunchKernelGGL(k_plan_lists_blk<false>, dim3(std::max(nb, 1)), dim3(kPlanThreads), 0, s, p);
    }
    hipLaunchKernelGGL(k_plan_scatter, dim3(grid), dim3(256), 0, s, p);
    hipLaunchKernelGGL(k_plan_queries, dim3(1), dim3(kPlanThreads), 0, s, p);
}

template <int QB, bool NTL>
static void ivf_scan_t(const IvfParams &p, int metric, int grid, hipStream_t s) {
    const size_t lds = (size_t)16 * QB * (2 * p.dpad + 16);
    if (lds > 65536) {  // 64-query tiles of wide rows: opt in to more than 64 KiB of LDS
        MQVS_HIP(hipFuncSetAttribute((const void *)k_ivf_scan<MQVS_METRIC_L2, QB, NTL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        MQVS_HIP(hipFuncSetAttribute((const void *)k_ivf_scan<MQVS_METRIC_IP, QB, NTL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        MQVS_HIP(hipFuncSetAttribute((const void *)k_ivf_scan<MQVS_METRIC_COSINE, QB, NTL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }
    switch (metric) {
        case MQVS_METRIC_L2:
            hipLaunchKernelGGL((k_ivf_scan<MQVS_METRIC_L2, QB, NTL>), dim3(grid), dim3(256), lds, s, p);
            break;
        case MQVS_METRIC_IP:
            hipLaunchKernelGGL((k_ivf_scan<MQVS_METRIC_IP, QB, NTL>), dim3(grid), dim3(256), lds, s, p);
            break;
        default:
            hipLaunchKernelGGL((k_ivf_scan<MQVS_METRIC_COSINE, QB, NTL>), dim3(grid), dim3(256), lds, s, p);
            break;
    }
}

template <bool NTL>
static void ivf_scan_nt(const IvfParams &p, int metric, int grid, hipStream_t s) {
    if (p.qg == 64)
        ivf_scan_t<4, NTL>(p, metric, grid, s);
    else if (p.qg == 32)
        ivf_scan_t<2, NTL>(p, metric, grid, s);
    else
        ivf_scan_t<1, NTL>(p, metric, grid, s);
}

void launch_ivf_scan(const IvfParams &p, int metric, int grid, hipStream_t s) {
    if (tune_int("MQVS_IVF_NT", 1) == 1)
        ivf_scan_nt<true>(p, metric, grid, s);
    else
        ivf_scan_nt<false>(p, metric, grid, s);
}

void launch_ivf_select(const Cand *cand, const IvfRegions &rg, int nq, int R, int metric, int64_t *out_rows,
                       int64_t id_offset, float *out_approx, int64_t expect_len, hipStream_t s, uint4 *gscr,
                       float *out_raw) {
    if (R <= 16 && !out_approx && !out_raw) {
        const dim3 grid((unsigned)((nq + 3) / 4));
#define MQVS_SMALL(M, RM_) \
    hipLaunchKernelGGL((k_ivf_select_small<M, RM_>), grid, dim3(256), 0, s, cand, rg, nq, R, out_rows, id_offset, \
                       out_approx)
#define MQVS_SMALL_M(M)              \
    if (R <= 2) MQVS_SMALL(M, 2);      \
    else if (R <= 4) MQVS_SMALL(M, 4); \
    else if (R <= 8) MQVS_SMALL(M, 8); \
    else MQVS_SMALL(M, 16);
        switch (metric) {
            case MQVS_METRIC_L2: MQVS_SMALL_M(MQVS_METRIC_L2); break;
            case MQVS_METRIC_IP: MQVS_SMALL_M(MQVS_METRIC_IP); break;
            default: MQVS_SMALL_M(MQVS_METRIC_COSINE); break;
        }
#undef MQVS_SMALL_M
#undef MQVS_SMALL
        return;
    }
    const bool large = R > kSortCap;
    if (large && !gscr) fail(MQVS_ERR_LOGICAL, "ivf select: no scratch for num_reorder above 4096");
    int N = 1;
    while (N < R) N <<= 1;
    if (large) N = kSortCap;  // LDS: the sort runs
    // LDS key cache sized for the expected region length (<= 64 KiB, and
    // within the LDS left beside the records); long regions (many probed
    // lists) get 1024 threads per query
    int keycap = 1024;
    while (keycap < expect_len && keycap < 16384) keycap <<= 1;
    while (keycap > 0 && sizeof(uint4) * N + sizeof(uint32_t) * keycap > 144 * 1024) keycap >>= 1;
    const size_t lds = sizeof(uint4) * N + sizeof(uint32_t) * keycap;
    const bool wide = expect_len > 16384;
#define MQVS_SEL(M)                                                                                                 \
    do {                                                                                                            \
        if (large)                                                                                                  \
            hipLaunchKernelGGL((k_ivf_select<M, SEL_THREADS, true>), dim3(nq), dim3(SEL_THREADS), lds, s, cand,     \
                               rg, R, out_rows, id_offset, out_approx, keycap, gscr, out_raw);                  \
        else if (wide)                                                                                              \
            hipLaunchKernelGGL((k_ivf_select<M, 1024>), dim3(nq), dim3(1024), lds, s, cand, rg, R, out_rows,    \
                               id_offset, out_approx, keycap, nullptr, out_raw);                                    \
        else                                                                                                        \
            hipLaunchKernelGGL((k_ivf_select<M, SEL_THREADS>), dim3(nq), dim3(SEL_THREADS), lds, s, cand, rg, R, \
                               out_rows, id_offset, out_approx, keycap, nullptr, out_raw);                          \
    } while (0)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_SEL(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_SEL(MQVS_METRIC_IP); break;
        default: MQVS_SEL(MQVS_METRIC_COSINE); break;
    }
#undef MQVS_SEL
}

void launch_ivf_pack(const float *rows, const float *norms, int d, const int32_t *perm, int64_t npos, int64_t dpad,
                     uint16_t *plane, float *pnorm, hipStream_t s) {
    const int64_t total = npos * (dpad / 8);
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 65536);
    if (grid > 0) hipLaunchKernelGGL(k_ivf_pack, dim3(grid), dim3(256), 0, s, rows, norms, d, perm, npos, dpad, plane, pnorm);
}

void launch_gather_rows(const float *src, int64_t src_ld, int d, const int64_t *idx, int64_t m, float *dst,
                        hipStream_t s) {
    const int64_t total = m * d;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 65536);
    if (grid > 0) hipLaunchKernelGGL(k_gather_rows, dim3(grid), dim3(256), 0, s, src, src_ld, d, idx, m, dst);
}

void launch_centroid_mean(const float *rows, int d, const int32_t *order, const int64_t *off, int nlist, float *cent,
                          hipStream_t s) {
    if (nlist > 0) hipLaunchKernelGGL(k_centroid_mean, dim3(nlist), dim3(256), 0, s, rows, d, order, off, cent);
}

// ---------------------------------------------------------------------------
// The coarse step's pick (index.hip): per query, from the batch probe's best
// approximate value of every group of 2^gs_log2 centroids (kernels_p4.hip,
// GRP 16 or 8), the
// exact fp32 value of each centroid of a few groups and the nprobe best.
// The group maxima are bf16 values within bq (the query's bound on |approx -
// exact|, k_query_bound) of the exact ones.
//  1. core: the T best groups (by (key, group); large T: its ties included,
//     up to Tcap), scored exactly;
//     they hold T >= nprobe centroids, so the nprobe-th best exact value of
//     the core, v, is a bound the final nprobe-th best cannot be worse than.
//  2. extras: a group outside the core can hold a centroid better than v only
//     if its maximum is within bq of v (its centroids' exact values are at
//     most maximum + bq); those groups are scored too, up to Tcap groups in
//     all.
//  3. overflow (more than Tcap groups in the core's ties or within bq of v:
//     near-ties, e.g. a query about equidistant from many centroids): every
//     group that passes is scored, in batches of Tcap taken in group order by
//     an ordered compaction, each batch merged into a running top-nprobe; the
//     query is counted in *ovf (mqvs_index_search_stats.pick_overflow).  The
//     probes stay the exact top-nprobe; only the time grows.
// Step 2 compares with the core's exact v, not with the T-th approximate
// maximum: usually no group passes (round 5 first took every group within
// 2 bq of the T-th maximum -- 8 more groups per query at nprobe 1, the pick
// 50 -> ~100 us at 39063 lists).  The probes are the exact top-nprobe of the
// centroids (in this pick's fp32 dot order).  One workgroup per query;
// Tcap <= kCoarsePickMaxT.  qn: L2 only, |q|^2 (the group values are full
// distances, the records |y|^2 - 2 ip).
//
// The group keys are staged in LDS once (up to kPickStage groups: 131072
// lists), so the four radix passes read LDS, not L2.  The exact values are
// computed a wave per kPickU centroids with float4 loads (kPickU x d/256
// independent 16-B loads per lane in flight; the pick is latency-bound, not
// bandwidth-bound: 48-160 centroids x 3 KB per query).  The nprobe best are
// placed by rank counting (M <= 256) or the LDS bitonic sort.
constexpr int kPickStage = 8192;
constexpr int kPickU = 4;
constexpr int kPickBest = kCoarsePickMaxT;  // running top-nprobe records of an overflowing pick (nprobe <= it)

template <int METRIC, bool STAGED>  // METRIC: MQVS_METRIC_L2 or kMetricIpRaw (the coarse metric)
__global__ __launch_bounds__(SEL_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_coarse_pick(const float *gmax, int64_t gld, int64_t ngroups, int T,
                                                             int Tcap, int nprobe, const float *q, int64_t qld,
                                                             const float *cent, const float *cnorm, int64_t ncent,
                                                             int d, const float *bq, const float *qnorms,
                                                             int gs_log2, int64_t *probes,
                                                             unsigned long long *ovf, int trace) {
    // (measurement build: trace = 1 prints phase timestamps of three workgroups)
    const bool tr = kDebugTuning && trace && threadIdx.x == 0 &&
                    (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2 || blockIdx.x == gridDim.x - 1);
    uint64_t ts[6] = {0, 0, 0, 0, 0, 0};
    if (tr) ts[0] = wall_clock64();
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_grp[kCoarsePickCap];
    __shared__ int s_wc[SEL_THREADS / 64];
    __shared__ int s_ng, s_valid, s_cur;
    __shared__ uint32_t s_knp;
    __shared__ uint64_t s_red[2 * (SEL_THREADS / 64)];
    // dynamic LDS: recs [pow2 >= kPickBest + GS Tcap] then (STAGED) keys
    // [ngroups], sized per launch so small pickups keep many workgroups per CU
    extern __shared__ uint4 dyn[];
    uint4 *recs = dyn;
    int NR = 1;
    const int GS = 1 << gs_log2;  // centroids per group
    while (NR < kPickBest + GS * Tcap) NR <<= 1;
    uint32_t *keys = reinterpret_cast<uint32_t *>(dyn + NR);
    const int qi = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const float *row = gmax + (int64_t)qi * gld;
    // T = 1 (nprobe 1): the best (key, group) kept while staging -- one pass
    // and a block minimum instead of a second pass over the keys
    uint64_t best = ~0ull;
    if (STAGED) {
        for_each_f4(row, ngroups, [&](int64_t i, float v) {
            const uint32_t k = okey<METRIC>(v);
            keys[i] = k;
            const uint64_t pr = ((uint64_t)k << 32) | (uint64_t)(uint32_t)i;
            if (k != 0xFFFFFFFFu && pr < best) best = pr;
        });
        __syncthreads();
    }
    if (tr) ts[1] = wall_clock64();
    auto keyof = [&](int64_t i) { return STAGED ? keys[i] : okey<METRIC>(row[i]); };
    // (the core's T groups come straight from the select for T <= kSelSmallK)
    uint64_t tpair = ~0ull;  // the T-th (key << 32 | group)
    int ncore = 0;
    uint32_t th = 0xFFFFFFFEu;
    if (T == 1 && STAGED) {
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(best, off);
            best = o < best ? o : best;
        }
        if (lane == 0) s_red[wv] = best;
        __syncthreads();
        best = s_red[0];
#pragma unroll
        for (int w = 1; w < SEL_THREADS / 64; ++w) best = s_red[w] < best ? s_red[w] : best;
        if (best != ~0ull) {
            ncore = 1;
            tpair = best;
            if (t == 0) s_grp[0] = (int)(uint32_t)best;
        }
        th = tpair == ~0ull ? 0xFFFFFFFEu : (uint32_t)(tpair >> 32);
        __syncthreads();  // (s_red, s_grp)
    } else if (T <= 2) {
        ncore = block_topk_small<SEL_THREADS, 2>(keyof, ngroups, T, s_red, s_grp, &tpair);
        th = tpair == ~0ull ? 0xFFFFFFFEu : (uint32_t)(tpair >> 32);
    } else if (T <= 4) {
        ncore = block_topk_small<SEL_THREADS, 4>(keyof, ngroups, T, s_red, s_grp, &tpair);
        th = tpair == ~0ull ? 0xFFFFFFFEu : (uint32_t)(tpair >> 32);
    } else if (T <= kSelSmallK) {
        ncore = block_topk_small(keyof, ngroups, T, s_red, s_grp, &tpair);
        th = tpair == ~0ull ? 0xFFFFFFFEu : (uint32_t)(tpair >> 32);
    } else {
        th = block_radix_select_mlp(keyof, ngroups, T, hist, sh);
    }
    if (t == 0) {
        s_ng = ncore;
        s_valid = 0;
        s_knp = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (tr) ts[2] = wall_clock64();
    // the groups whose key passes take(key, group), appended to s_grp (up to Tcap)
    auto collect = [&](auto take) {
        for (int64_t i = t; i < ngroups; i += SEL_THREADS) {
            const uint32_t k = keyof(i);
            if (k == 0xFFFFFFFFu || !take(k, i)) continue;
            const int slot = atomicAdd(&s_ng, 1);
            if (slot < Tcap) s_grp[slot] = (int)i;
        }
        __syncthreads();
    };
    // exact values of centroids c in [cb, ce) (GS per taken group) into
    // recs[ro + c]: wave wv scores centroids c0 .. c0 + kPickU - 1, lanes over
    // float4 columns (scalar columns when d or the rows are not 16-B aligned)
    const float *qv = q + (int64_t)qi * qld;
    const bool v4 = (d & 3) == 0 && (((uintptr_t)cent | (uintptr_t)qv) & 15) == 0;
    auto score = [&](int cb, int ce, int ro) {
        for (int c0 = cb + wv * kPickU; c0 < ce; c0 += (SEL_THREADS / 64) * kPickU) {
            int64_t r[kPickU];
            float dot[kPickU];
#pragma unroll
            for (int u = 0; u < kPickU; ++u) {
                const int c = c0 + u;
                r[u] = c < ce ? ((int64_t)s_grp[c >> gs_log2] << gs_log2) + (c & (GS - 1)) : ncent;
                if (r[u] >= ncent) r[u] = -1;
                dot[u] = 0.f;
            }
            if (v4) {
                const float4 *q4 = reinterpret_cast<const float4 *>(qv);
                // three column steps per round: 3 kPickU independent 16-B loads
                // per lane in flight (d = 768 is one round)
                const int n4 = d >> 2;
                for (int j0 = lane; j0 < n4; j0 += 3 * 64) {
                    float4 x[3], y[3][kPickU];
#pragma unroll
                    for (int tt = 0; tt < 3; ++tt) {
                        const int j = j0 + 64 * tt;
                        const bool in = j < n4;
                        x[tt] = in ? q4[j] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int u = 0; u < kPickU; ++u)
                            y[tt][u] = in && r[u] >= 0 ? reinterpret_cast<const float4 *>(cent + r[u] * d)[j]
                                                       : float4{0.f, 0.f, 0.f, 0.f};
                    }
#pragma unroll
                    for (int tt = 0; tt < 3; ++tt)
#pragma unroll
                        for (int u = 0; u < kPickU; ++u) {
                            dot[u] = fmaf(x[tt].x, y[tt][u].x, dot[u]);
                            dot[u] = fmaf(x[tt].y, y[tt][u].y, dot[u]);
                            dot[u] = fmaf(x[tt].z, y[tt][u].z, dot[u]);
                            dot[u] = fmaf(x[tt].w, y[tt][u].w, dot[u]);
                        }
                }
            } else {
                for (int e = lane; e < d; e += 64) {
                    const float x = qv[e];
#pragma unroll
                    for (int u = 0; u < kPickU; ++u)
                        if (r[u] >= 0) dot[u] = fmaf(x, cent[r[u] * d + e], dot[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < kPickU; ++u) {
                float v = dot[u];
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
                dot[u] = v;
            }
            if (lane < kPickU) {
                float dv = dot[0];
                int64_t rv = r[0];
#pragma unroll
                for (int u = 1; u < kPickU; ++u)
                    if (lane == u) {
                        dv = dot[u];
                        rv = r[u];
                    }
                const int c = c0 + lane;
                if (c < ce) {
                    uint32_t key = 0xFFFFFFFFu;
                    if (rv >= 0) key = okey<METRIC>(METRIC == MQVS_METRIC_L2 ? cnorm[rv] - 2.0f * dv : dv);
                    recs[ro + c] = uint4{key, (uint32_t)(rv >= 0 ? rv : 0xFFFFFFFFu), 0u, 0u};
                    if (key != 0xFFFFFFFFu) atomicAdd(&s_valid, 1);
                }
            }
        }
        __syncthreads();
    };
    // 1. core: the T best (key, group) pairs (large T: the groups better than
    // the T-th key, then its ties)
    if (T > kSelSmallK) {
        collect([&](uint32_t k, int64_t) { return th == 0xFFFFFFFEu || k < th; });
        if (th != 0xFFFFFFFEu) collect([&](uint32_t k, int64_t) { return k == th; });
        tpair = th == 0xFFFFFFFEu ? ~0ull : ((uint64_t)th << 32) | 0xFFFFFFFFull;  // (every tie is in)
    }
    const int ng0 = min(s_ng, Tcap);
    // (a core with more ties than Tcap groups: overflow)
    bool over = s_ng > Tcap;
    score(0, GS * ng0, 0);
    if (tr) ts[3] = wall_clock64();
    int ng = ng0;
    uint32_t kx = th;  // every group that can hold a top-nprobe centroid has key <= max(kx, th)
    // 2. extras (needs the bound and a full core; fewer than T valid groups:
    // every group is in the core already).  The collect counts every group
    // that passes, so a working set that cannot hold them shows as s_ng > Tcap.
    if (bq && tpair != ~0ull) {
        const int M0 = GS * ng0;
        for (int c = t; c < M0; c += SEL_THREADS) {
            const uint4 e = recs[c];
            if (e.x == 0xFFFFFFFFu) continue;
            int rank = 0;
            for (int o = 0; o < M0; ++o) rank += rec_less(recs[o], e) ? 1 : 0;
            if (rank == nprobe - 1) s_knp = e.x;
        }
        __syncthreads();
        if (s_knp != 0xFFFFFFFFu) {
            // the approximate maximum a group needs: v -/+ bq (rounding slack
            // as widen's), v a full distance for L2
            float v = okey_value<METRIC>(s_knp);
            if (METRIC == MQVS_METRIC_L2) v = qnorms[qi] + v;
            const float b = bq[qi];
            float w;
            if (METRIC == MQVS_METRIC_L2) {
                w = v + b;
                w = w + fabsf(w) * 2.4e-7f + 1e-30f;
            } else {
                w = v - b;
                w = w - fabsf(w) * 2.4e-7f - 1e-30f;
            }
            kx = w == w ? okey<METRIC>(w) : th;
        } else {
            // fewer than nprobe valid centroids in the core: every group
            // within 2 bq of the T-th maximum
            const float w = widen<METRIC>(okey_value<METRIC>(th), bq[qi]);
            kx = w == w ? okey<METRIC>(w) : th;
        }
        if (kx >= th && !over) {
            collect([&](uint32_t k, int64_t i) {
                return k <= kx && (((uint64_t)k << 32) | (uint64_t)(uint32_t)i) > tpair;
            });
            over = s_ng > Tcap;
            ng = min(s_ng, Tcap);
            if (!over && ng > ng0) score(M0, GS * ng, 0);
        }
    }
    if (over) {
        // 3. every group with key <= max(kx, th), Tcap groups at a time in
        // group order; recs[0, nprobe) keeps the best so far (sorted), the
        // batch's records follow at kPickBest
        if (t == 0 && ovf) atomicAdd(ovf, 1ull);
        const uint32_t kall = kx > th ? kx : th;
        for (int c = t; c < kPickBest; c += SEL_THREADS) recs[c] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        int64_t cursor = 0;
        while (cursor < ngroups) {
            // ordered compaction of the next Tcap passing groups from `cursor`
            int nb = 0;
            int64_t i0 = cursor;
            while (i0 < ngroups && nb < Tcap) {
                const int64_t i = i0 + t;
                bool pass = false;
                if (i < ngroups) {
                    const uint32_t kk = keyof(i);
                    pass = kk != 0xFFFFFFFFu && kk <= kall;
                }
                const uint64_t bal = __ballot(pass);
                if (lane == 0) s_wc[wv] = __popcll(bal);
                __syncthreads();
                int before = 0, tot = 0;
                for (int x = 0; x < SEL_THREADS / 64; ++x) {
                    before += x < wv ? s_wc[x] : 0;
                    tot += s_wc[x];
                }
                const int pos = nb + before + __popcll(bal & ((1ull << lane) - 1ull));
                if (pass && pos < Tcap) s_grp[pos] = (int)i;
                if (pass && pos == Tcap - 1) s_cur = (int)(i + 1);
                __syncthreads();
                if (nb + tot >= Tcap) {
                    i0 = s_cur;
                    nb = Tcap;
                } else {
                    nb += tot;
                    i0 += SEL_THREADS;
                }
                __syncthreads();  // (s_wc, s_cur reused)
            }
            cursor = i0;
            if (nb == 0) break;
            score(0, GS * nb, kPickBest);
            int N = 1;
            while (N < kPickBest + GS * nb) N <<= 1;
            for (int c = kPickBest + GS * nb + t; c < N; c += SEL_THREADS)
                recs[c] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            __syncthreads();
            block_bitonic_sort(recs, N);
            for (int c = nprobe + t; c < kPickBest; c += SEL_THREADS)
                recs[c] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            __syncthreads();
        }
        for (int j = t; j < nprobe; j += SEL_THREADS) {
            const uint4 e = recs[j];
            probes[(int64_t)qi * nprobe + j] = e.x == 0xFFFFFFFFu ? -1 : (int64_t)e.y;
        }
        return;
    }
    const int M = GS * ng;
    __syncthreads();
    if (tr) ts[4] = wall_clock64();
    auto trace_out = [&]() {
        if (tr)
            printf("pick q %d ng0 %d ng %d stage %llu select %llu core %llu extras %llu place %llu (x10ns)\n", qi,
                   ng0, ng, (unsigned long long)(ts[1] - ts[0]), (unsigned long long)(ts[2] - ts[1]),
                   (unsigned long long)(ts[3] - ts[2]), (unsigned long long)(ts[4] - ts[3]),
                   (unsigned long long)(wall_clock64() - ts[4]));
    };
    const int nvalid = s_valid;
    if (M <= 256) {
        // rank counting: valid records are unique (key, centroid), so each
        // lands on its own rank; the invalid ones are not placed
        for (int c = t; c < M; c += SEL_THREADS) {
            const uint4 e = recs[c];
            if (e.x == 0xFFFFFFFFu) continue;
            int rank = 0;
            for (int o = 0; o < M; ++o) rank += rec_less(recs[o], e) ? 1 : 0;
            if (rank < nprobe) probes[(int64_t)qi * nprobe + rank] = (int64_t)e.y;
        }
        for (int j = nvalid + t; j < nprobe; j += SEL_THREADS) probes[(int64_t)qi * nprobe + j] = -1;
        trace_out();
        return;
    }
    int N = 1;
    while (N < M) N <<= 1;
    for (int c = M + t; c < N; c += SEL_THREADS) recs[c] = uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    __syncthreads();
    block_bitonic_sort(recs, N);
    for (int j = t; j < nprobe; j += SEL_THREADS) {
        const uint4 e = j < M ? recs[j] : uint4{0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u};
        probes[(int64_t)qi * nprobe + j] = e.x == 0xFFFFFFFFu ? -1 : (int64_t)e.y;
    }
    trace_out();
}

void launch_coarse_pick(const float *gmax, int64_t gld, int64_t ngroups, int T, int nprobe, int metric,
                        const float *q, int64_t qld, const float *cent, const float *cnorm, int64_t ncent, int d,
                        const float *bq, const float *qnorms, int gs_log2, int nq, int64_t *probes,
                        unsigned long long *ovf, hipStream_t s) {
    if (nq <= 0) return;
    if (T > kCoarsePickMaxT || nprobe > kPickBest) fail(MQVS_ERR_LOGICAL, "coarse pick: nprobe above its cap");
    // room for the groups within the bound of the core's nprobe-th value
    // (near-ties): as many as a core of nprobe + 2 groups had (a smaller core
    // leaves more of the near groups to the extras); more are the overflow
    // path's (exact, batched)
    const int Tcap = std::min(kCoarsePickCap, std::max(T, nprobe + 2) + std::max(std::max(T, nprobe + 2), 8));
    const int trace = tune_int("MQVS_PICK_TRACE", 0);
#define MQVS_PICK(M, ST)                                                                                         \
    hipLaunchKernelGGL((k_coarse_pick<M, ST>), dim3(nq), dim3(SEL_THREADS), lds, s, gmax, gld, ngroups, T, Tcap, \
                       nprobe, q, qld, cent, cnorm, ncent, d, bq, qnorms, gs_log2, probes, ovf, trace)
    const bool staged = ngroups <= kPickStage;
    size_t nr = 1;
    while (nr < kPickBest + ((size_t)1 << gs_log2) * Tcap) nr <<= 1;
    const size_t lds = nr * sizeof(uint4) + (staged ? sizeof(uint32_t) * (size_t)ngroups : 0);
    if (metric == MQVS_METRIC_L2) {
        if (staged) MQVS_PICK(MQVS_METRIC_L2, true); else MQVS_PICK(MQVS_METRIC_L2, false);
    } else {
        if (staged) MQVS_PICK(kMetricIpRaw, true); else MQVS_PICK(kMetricIpRaw, false);
    }
#undef MQVS_PICK
}

}  // namespace mqvs
