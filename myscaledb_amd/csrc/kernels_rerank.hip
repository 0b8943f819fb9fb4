// kernels_rerank.hip -- exact distances to given candidate rows + top-k
// (mqvs_rerank, the computeTopDistanceSubset contract of
// VIWithDataPart.cpp:838-856 / MergeTreeVSManager.cpp:511-631).
//
// One workgroup per query: gather the query's candidate rows, compute each
// distance with the brute-force formula the same batch size selects in
// mqvs_search (nq < 20: faiss fvec product-then-add; nq >= 20: BLAS form with
// an fma-chain inner product; cosine with the chunk's query variant), then
// sort (key, chunk, ip, row) in LDS exactly like the search's final select.
// With every row of the segment as candidates the result equals mqvs_search.
#include "mqvs_internal.h"
#include "select_common.h"

namespace mqvs {

template <int METRIC, bool DIRECT>
__device__ inline float cand_value(const ScanParams &p, int q, int64_t row) {
    const int64_t chunk = p.chunk_rows > 0 ? row / p.chunk_rows : 0;
    const int ord = chunk_ordinal(p, chunk);
    const int v = variant_of(p, q, ord < 0 ? 0 : ord);
    const int64_t qs = (int64_t)((p.d + 31) / 32 * 32);
    const float *x = p.qvars + ((int64_t)q * p.maxv + v) * qs;
    const float *y = p.rows + row * p.d;
    float acc = 0.0f;
    if (DIRECT) {
        // kernels_scan.hip k_scan_small order: sequential, product then add
        auto step = [&](float a, float b) {
            if (METRIC == MQVS_METRIC_L2) {
                const float e = a - b;
                acc = acc + e * e;
            } else {
                acc = acc + a * b;
            }
        };
        if ((p.d & 3) == 0) {
            const float4 *x4 = reinterpret_cast<const float4 *>(x);
            const float4 *y4 = reinterpret_cast<const float4 *>(y);
            for (int i = 0; i < (p.d >> 2); ++i) {
                const float4 a = y4[i], b = x4[i];
                step(a.x, b.x);
                step(a.y, b.y);
                step(a.z, b.z);
                step(a.w, b.w);
            }
        } else {
            for (int i = 0; i < p.d; ++i) step(y[i], x[i]);
        }
        return acc;
    }
    for (int i = 0; i < p.d; ++i) acc = fmaf(x[i], y[i], acc);
    if (METRIC == MQVS_METRIC_L2) {
        float d = (p.qnorms[q] + p.row_norms[row]) - 2.0f * acc;
        if (d < 0) d = 0;
        return d;
    }
    return acc;
}

// candidate record -> top-k outputs (shared by both re-rank kernels)
template <int METRIC>
__device__ inline uint4 rerank_rec(const ScanParams &p, int64_t row, float raw) {
    uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    if (row < 0) return r;
    r.x = key32<METRIC>(raw);
    r.w = (uint32_t)row;
    if (METRIC == MQVS_METRIC_COSINE) {
        r.y = p.chunk_rows > 0 ? (uint32_t)(row / p.chunk_rows) : 0u;
        r.z = ~ord_asc(raw);
    } else {
        r.y = 0;
        r.z = 0;
    }
    if (r.x == 0xFFFFFFFFu) r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    return r;
}

// Sort the query's candidate records and write its top k.  g == null: the
// records are recs[0, ncand) in LDS (ncand <= kSortCap); else they are
// g[0, ncand) in the query's global scratch (2 ncand records) and recs is
// kSortCap records of LDS for global_sort.
template <int METRIC>
__device__ inline void rerank_emit(uint4 *recs, uint4 *g, int ncand, int k, int q, int64_t id_offset,
                                   int64_t *out_ids, float *out_dist) {
    const uint4 *sorted = recs;
    int N = ncand;
    if (g) {
        __syncthreads();
        sorted = global_sort(g, g + ncand, ncand, recs);
    } else {
        N = 1;
        while (N < ncand) N <<= 1;
        for (int i = ncand + threadIdx.x; i < N; i += SEL_THREADS)
            recs[i] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        __syncthreads();
        block_bitonic_sort(recs, N);
    }
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f
                      : (METRIC == kMetricIpRaw) ? -3.40282347e+38f
                                                 : 3.40282347e+38f;
    for (int i = threadIdx.x; i < k; i += SEL_THREADS) {
        int64_t id = -1;
        float dist = pad;
        if (i < N && sorted[i].x != 0xFFFFFFFFu) {
            id = (int64_t)sorted[i].w + id_offset;
            dist = key_to_value(METRIC, sorted[i].x);
        }
        out_ids[(int64_t)q * k + i] = id;
        out_dist[(int64_t)q * k + i] = dist;
    }
}

// Bound pruning (index re-rank; RerankPrune in mqvs_internal.h): how many of
// query q's candidates -- sorted by their approximate value a -- can reach the
// exact top k.  With B the bound on |a - exact| (k_query_bound for query
// variant 0, plus |x_v - x_0| |y|max for the cosine variant x_v the exact
// value of a row uses), the k best candidates have exact values within B of
// a_k, the k-th approximate value, so the k-th exact value is at most a_k + B
// (L2; at least a_k - B for IP / cosine, larger better); a candidate with a >
// a_k + 2B has an exact value strictly worse, and so has every later one.
// The output is the same as re-ranking all of them.  No pruning (m = ncand)
// when a_k is not a valid value, B is not finite, or for IP the k best could
// fall under the FLT_MIN cut (searchWrapper's init) and leave fewer than k.
// wave_prune_cut: the cut of query q, computed by one wave (its 64 lanes
// share the cosine variant distances); returns whether pruning applies and
// the cut w on the approximate raw value (keep a <= w for L2, a >= w else),
// uniform over the wave.
template <int METRIC>
__device__ inline bool wave_prune_cut(const ScanParams &p, const RerankPrune &pr, int q, int ncand, int k, float &w) {
    const int lane = threadIdx.x & 63;
    // cosine: the largest distance of a used variant from variant 0, in fp64
    // (from the query prep when it measured it)
    double dmax = 0.0;
    if (METRIC == MQVS_METRIC_COSINE && pr.qdelta) {
        const double dq = (double)pr.qdelta[q];
        dmax = dq * dq;
    } else if (METRIC == MQVS_METRIC_COSINE && p.maxv > 1) {
        const int mu = p.qmu[q], lam = p.qlam[q];
        const int nv = (lam >= 1 && mu >= 0 && mu + lam <= p.maxv) ? mu + lam : p.maxv;
        const int64_t qs = (int64_t)((p.d + 31) / 32 * 32);
        const float *x0 = p.qvars + (int64_t)q * p.maxv * qs;
        for (int v = 1; v < nv; ++v) {
            const float *xv = x0 + (int64_t)v * qs;
            double ss = 0.0;
            for (int i = lane; i < p.d; i += 64) {
                const double e = (double)xv[i] - (double)x0[i];
                ss += e * e;
            }
            for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
            dmax = ss > dmax ? ss : dmax;
        }
    }
    const float ak = pr.raw[(int64_t)q * ncand + k - 1];
    const float ym = *pr.ymax;
    const float dv = dmax > 0.0 ? (float)(sqrt(dmax) * (1.0 + 1e-6)) * ym * 1.0001f : 0.f;
    const float b = pr.bq[q] + dv + 1e-30f;
    bool ok = ak == ak && b < 1e30f && ym < 1e30f;
    if (METRIC == MQVS_METRIC_L2) {
        w = ak + 2.0f * b;
        w = w + fabsf(w) * 2.4e-7f + 1e-30f;
    } else {
        w = ak - 2.0f * b;
        w = w - fabsf(w) * 2.4e-7f - 1e-30f;
        if (METRIC == MQVS_METRIC_IP) {
            float lo = ak - b;
            lo = lo - fabsf(lo) * 2.4e-7f;
            ok = ok && lo > 1.17549435e-38f;
        }
    }
    return ok && w == w;
}

// Block-uniform result; s_m: one int of LDS.
template <int METRIC>
__device__ inline int rerank_keep(const ScanParams &p, const RerankPrune &pr, int q, int ncand, int k, int *s_m) {
    if (!pr.raw || k >= ncand) return ncand;
    const float *raw = pr.raw + (int64_t)q * ncand;
    const int t = threadIdx.x;
    if (t == 0) *s_m = ncand;
    __shared__ float s_cut;
    __shared__ int s_ok;
    if (t < 64) {
        float w = 0.f;
        const bool ok = wave_prune_cut<METRIC>(p, pr, q, ncand, k, w);
        if (t == 0) {
            s_cut = w;
            s_ok = ok ? 1 : 0;
        }
    }
    __syncthreads();
    if (s_ok) {
        const float w = s_cut;
        // the first candidate past the cut (NaN: no candidate) ends the prefix
        for (int i = t; i < ncand; i += SEL_THREADS) {
            const float a = raw[i];
            const bool keep = METRIC == MQVS_METRIC_L2 ? a <= w : a >= w;
            if (!keep) {
                atomicMin(s_m, i);
                break;
            }
        }
    }
    __syncthreads();
    return *s_m;
}

// Generic form (any d): one thread per candidate walks its row.
template <int METRIC, bool DIRECT>
__global__ __launch_bounds__(SEL_THREADS) void k_rerank_ids(ScanParams p, const int64_t *cand, int ncand,
                                                           int k, int64_t id_offset, int64_t *out_ids,
                                                           float *out_dist, uint4 *scratch, RerankPrune pr) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];  // pow2 >= ncand (or kSortCap) records
    __shared__ int s_m;
    const int q = blockIdx.x;
    const int64_t *c = cand + (int64_t)q * ncand;
    uint4 *g = scratch ? scratch + (int64_t)q * 2 * ncand : nullptr;
    uint4 *dst = g ? g : recs;
    const int m = rerank_keep<METRIC>(p, pr, q, ncand, k, &s_m);
    if (threadIdx.x == 0 && pr.count) atomicAdd(pr.count, (unsigned long long)m);
    for (int i = threadIdx.x; i < ncand; i += SEL_THREADS) {
        int64_t row = i < m ? c[i] : -1;
        if (!(row >= 0 && row < p.n && row_valid(p, row))) row = -1;
        dst[i] = rerank_rec<METRIC>(p, row, row >= 0 ? cand_value<METRIC, DIRECT>(p, q, row) : 0.f);
    }
    rerank_emit<METRIC>(recs, g, ncand, k, q, id_offset, out_ids, out_dist);
}

// d % 4 == 0: the same per-candidate sequential chain (bit-identical), with
// the rows streamed cooperatively: per 32-column tile a wave loads its 64
// candidates' 128-B row slices with float4 loads (8 lanes per row, full
// cache lines), prefetching the next tile into registers, and stages them
// in LDS (row stride 33 floats: conflict-free column reads); each lane then
// runs its chain from LDS.  Lanes of a wave run in lockstep, so the wave's
// own LDS tile needs no barrier.  row < 0: no candidate (returns 0).
// tile: this wave's 64 x kRrStride floats of LDS.
constexpr int kRrStride = 33;

template <int METRIC, bool DIRECT>
__device__ inline float wave_exact(const ScanParams &p, int q, int64_t row, float *tile) {
    const int lane = threadIdx.x & 63;
    const int d = p.d;
    const int64_t qs = (int64_t)((d + 31) / 32 * 32);
    const int ntiles = (d + 31) / 32;
    const float *x = p.qvars;
    if (row >= 0) {
        const int64_t chunk = p.chunk_rows > 0 ? row / p.chunk_rows : 0;
        const int ord = chunk_ordinal(p, chunk);
        const int v = variant_of(p, q, ord < 0 ? 0 : ord);
        x = p.qvars + ((int64_t)q * p.maxv + v) * qs;
    }
    float acc = 0.0f;
    if (__ballot(row >= 0)) {
        // rows this lane loads: slot j*8 + lane/8, float4 column lane%8
        int64_t lrow[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) lrow[j] = __shfl(row, j * 8 + (lane >> 3));
        float4 ry[8], rx[8];
        auto load = [&](int t) {
            const int col = t * 32 + (lane & 7) * 4;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                ry[j] = (lrow[j] >= 0 && col < d) ? *reinterpret_cast<const float4 *>(p.rows + lrow[j] * d + col)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
            // the lane's own query slice (variant of its row's chunk)
#pragma unroll
            for (int j = 0; j < 8; ++j) rx[j] = *reinterpret_cast<const float4 *>(x + t * 32 + 4 * j);
        };
        load(0);
        for (int t = 0; t < ntiles; ++t) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float *dst = tile + (j * 8 + (lane >> 3)) * kRrStride + (lane & 7) * 4;
                dst[0] = ry[j].x;
                dst[1] = ry[j].y;
                dst[2] = ry[j].z;
                dst[3] = ry[j].w;
            }
            float xt[32];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                xt[4 * j] = rx[j].x;
                xt[4 * j + 1] = rx[j].y;
                xt[4 * j + 2] = rx[j].z;
                xt[4 * j + 3] = rx[j].w;
            }
            if (t + 1 < ntiles) load(t + 1);
            __builtin_amdgcn_wave_barrier();
            const float *mine = tile + lane * kRrStride;
            const int cols = min(32, d - t * 32);
            if (cols == 32) {
#pragma unroll
                for (int cc = 0; cc < 32; ++cc) {
                    const float a = mine[cc], b = xt[cc];
                    if (DIRECT) {
                        if (METRIC == MQVS_METRIC_L2) {
                            const float e = a - b;
                            acc = acc + e * e;
                        } else {
                            acc = acc + a * b;
                        }
                    } else {
                        acc = fmaf(b, a, acc);
                    }
                }
            } else {
                for (int cc = 0; cc < cols; ++cc) {
                    const float a = mine[cc], b = x[t * 32 + cc];
                    if (DIRECT) {
                        if (METRIC == MQVS_METRIC_L2) {
                            const float e = a - b;
                            acc = acc + e * e;
                        } else {
                            acc = acc + a * b;
                        }
                    } else {
                        acc = fmaf(b, a, acc);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    float raw = acc;
    if (!DIRECT && METRIC == MQVS_METRIC_L2 && row >= 0) {
        raw = (p.qnorms[q] + p.row_norms[row]) - 2.0f * acc;
        if (raw < 0) raw = 0;
    }
    return raw;
}

// d = 32 NT (NT a compile-time tile count; the common d = 768 is NT = 24):
// the same chain and staging, the tile loop fully unrolled and the row
// slices of kRrPF tiles in flight in a register ring.  Every load is
// unconditional (a lane without a candidate streams row 0, its result is
// discarded; the ring's refills past the last tile re-read it), so the
// compiler counts each wait exactly: wave_exact waits a full random-row load
// latency per tile (one tile ahead), ~24 latencies per wave at d = 768.
constexpr int kRrPF = 3;
// XPF: tiles of the query slice in flight.  1 (the index re-rank: registers
// are its occupancy) waits an L2 round trip for the query slice every tile --
// the whole chain at small nq, where one workgroup's 24 tiles are the exact
// stage (k_exact_records at nq 1: ~23 us); 3 keeps it in a ring like the rows.
template <int METRIC, bool DIRECT, int NT, int XPF = 1>
__device__ inline float wave_exact_nt(const ScanParams &p, int q, int64_t row, float *tile) {
    constexpr int d = 32 * NT;
    const int lane = threadIdx.x & 63;
    const float *x = p.qvars;
    if (row >= 0) {
        const int64_t chunk = p.chunk_rows > 0 ? row / p.chunk_rows : 0;
        const int ord = chunk_ordinal(p, chunk);
        const int v = variant_of(p, q, ord < 0 ? 0 : ord);
        x = p.qvars + ((int64_t)q * p.maxv + v) * d;
    }
    float acc = 0.0f;
    if (__ballot(row >= 0)) {
        // rows this lane loads: slot j*8 + lane/8, float4 column lane%8
        const float *base[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t r = __shfl(row, j * 8 + (lane >> 3));
            base[j] = p.rows + (r >= 0 ? r : 0) * d + (lane & 7) * 4;
        }
        float4 ry[kRrPF][8], rx[XPF][8];
        auto load_y = [&](int t, float4(&dst)[8]) __attribute__((always_inline)) {
            const int tt = t < NT ? t : NT - 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) dst[j] = *reinterpret_cast<const float4 *>(base[j] + tt * 32);
        };
        auto load_x = [&](int t, float4(&dst)[8]) __attribute__((always_inline)) {
            const int tt = t < NT ? t : NT - 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) dst[j] = *reinterpret_cast<const float4 *>(x + tt * 32 + 4 * j);
        };
#pragma unroll
        for (int sl = 0; sl < kRrPF; ++sl) load_y(sl, ry[sl]);
#pragma unroll
        for (int sl = 0; sl < XPF; ++sl) load_x(sl, rx[sl]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            float4(&cur)[8] = ry[t % kRrPF];
            float4(&curx)[8] = rx[t % XPF];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float *dst = tile + (j * 8 + (lane >> 3)) * kRrStride + (lane & 7) * 4;
                dst[0] = cur[j].x;
                dst[1] = cur[j].y;
                dst[2] = cur[j].z;
                dst[3] = cur[j].w;
            }
            float xt[32];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                xt[4 * j] = curx[j].x;
                xt[4 * j + 1] = curx[j].y;
                xt[4 * j + 2] = curx[j].z;
                xt[4 * j + 3] = curx[j].w;
            }
            load_y(t + kRrPF, cur);
            load_x(t + XPF, curx);
            __builtin_amdgcn_wave_barrier();
            const float *mine = tile + lane * kRrStride;
#pragma unroll
            for (int cc = 0; cc < 32; ++cc) {
                const float a = mine[cc], b = xt[cc];
                if (DIRECT) {
                    if (METRIC == MQVS_METRIC_L2) {
                        const float e = a - b;
                        acc = acc + e * e;
                    } else {
                        acc = acc + a * b;
                    }
                } else {
                    acc = fmaf(b, a, acc);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    float raw = acc;
    if (!DIRECT && METRIC == MQVS_METRIC_L2 && row >= 0) {
        raw = (p.qnorms[q] + p.row_norms[row]) - 2.0f * acc;
        if (raw < 0) raw = 0;
    }
    return raw;
}

// wave_exact_nt for d = 768, wave_exact otherwise
template <int METRIC, bool DIRECT, int XPF = 1>
__device__ inline float wave_exact_any(const ScanParams &p, int q, int64_t row, float *tile) {
    if (p.d == 768) return wave_exact_nt<METRIC, DIRECT, 24, XPF>(p, q, row, tile);
    return wave_exact<METRIC, DIRECT>(p, q, row, tile);
}

template <int METRIC, bool DIRECT, int XPF = 1>
__global__ __launch_bounds__(SEL_THREADS) void k_rerank_ids_tiled(ScanParams p, const int64_t *cand, int ncand,
                                                                 int k, int64_t id_offset, int64_t *out_ids,
                                                                 float *out_dist, int nrec, uint4 *scratch,
                                                                 RerankPrune pr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int s_m;
    uint4 *recs = reinterpret_cast<uint4 *>(smem);
    uint4 *g = scratch ? scratch + (int64_t)blockIdx.x * 2 * ncand : nullptr;
    uint4 *dst = g ? g : recs;
    const int wv = threadIdx.x >> 6;
    float *tile = reinterpret_cast<float *>(smem + (size_t)nrec * sizeof(uint4)) + wv * 64 * kRrStride;
    const int q = blockIdx.x;
    const int64_t *c = cand + (int64_t)q * ncand;
    const int m = rerank_keep<METRIC>(p, pr, q, ncand, k, &s_m);
    if (threadIdx.x == 0 && pr.count) atomicAdd(pr.count, (unsigned long long)m);
    for (int cb = 0; cb < ncand; cb += SEL_THREADS) {
        const int i = cb + threadIdx.x;
        int64_t row = -1;
        if (i < m) {
            row = c[i];
            if (!(row >= 0 && row < p.n && row_valid(p, row))) row = -1;
        }
        const float raw = wave_exact_any<METRIC, DIRECT, XPF>(p, q, row, tile);
        if (i < ncand) dst[i] = rerank_rec<METRIC>(p, row, raw);
    }
    rerank_emit<METRIC>(recs, g, ncand, k, q, id_offset, out_ids, out_dist);
}

// Two queries per workgroup (waves 0-1: query 2 b, waves 2-3: query 2 b + 1),
// for up to kRrPairMax candidates: k_rerank_ids_tiled's chain and records,
// each query's candidates 128 at a time over its two waves.  At ~233 VGPRs
// two waves per SIMD fit -- two workgroups per CU: one query per workgroup
// took two rounds of 1000 workgroups at nq 1000, each as long as a 24-tile
// random-row chain, and after pruning (~120 of 200 candidates kept) half of
// its waves had no rows; here 500 workgroups are one round.  The top k is
// placed by rank counting over the kept prefix (records are unique: key, then
// row; equal records -- a row listed twice -- rank by position, as a stable
// sort), the same output as rerank_emit's sort.  Measured slower (mode 3,
// nprobe 1, k 100: re-rank 127 -> 140 us; the rows arrive at ~2.9 TB/s either
// way -- a torch index_select of the same rows runs at 2.5-2.8 TB/s,
// tools/gather_tlb_probe.py -- so the random-row read rate bounds it, not the
// rounds): MQVS_RR_PAIR=1, measurement build only.
constexpr int kRrPairMax = 512;

template <int METRIC, bool DIRECT>
__global__ __launch_bounds__(SEL_THREADS) void k_rerank_ids_pair(ScanParams p, const int64_t *cand, int ncand,
                                                                int k, int64_t id_offset, int64_t *out_ids,
                                                                float *out_dist, RerankPrune pr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int s_m[2], s_ok[2], s_nv[2];
    __shared__ float s_cut[2];
    const int h = threadIdx.x >> 7, ht = threadIdx.x & 127, wv = threadIdx.x >> 6;
    const int q = blockIdx.x * 2 + h;
    const bool act = q < p.nq;
    const int qq = act ? q : 0;
    uint4 *recs = reinterpret_cast<uint4 *>(smem) + (size_t)h * ncand;
    float *tile = reinterpret_cast<float *>(smem + 2 * (size_t)ncand * sizeof(uint4)) + wv * 64 * kRrStride;
    if (ht == 0) {
        s_m[h] = act ? ncand : 0;
        s_ok[h] = 0;
        s_nv[h] = 0;
    }
    // the cut (rerank_keep, per half): its first wave
    if (act && pr.raw && k < ncand && ht < 64) {
        float w = 0.f;
        const bool ok = wave_prune_cut<METRIC>(p, pr, q, ncand, k, w);
        if (ht == 0) {
            s_cut[h] = w;
            s_ok[h] = ok ? 1 : 0;
        }
    }
    __syncthreads();
    if (act && s_ok[h]) {
        const float w = s_cut[h];
        const float *raw = pr.raw + (int64_t)q * ncand;
        for (int i = ht; i < ncand; i += 128) {
            const float a = raw[i];
            const bool keep = METRIC == MQVS_METRIC_L2 ? a <= w : a >= w;
            if (!keep) {
                atomicMin(&s_m[h], i);
                break;
            }
        }
    }
    __syncthreads();
    const int m = s_m[h];
    if (act && ht == 0 && pr.count) atomicAdd(pr.count, (unsigned long long)m);
    const int64_t *c = cand + (int64_t)qq * ncand;
    for (int cb = 0; cb < ncand; cb += 128) {
        const int i = cb + ht;
        int64_t row = -1;
        if (i < m) {
            row = c[i];
            if (!(row >= 0 && row < p.n && row_valid(p, row))) row = -1;
        }
        const float raw = cb < m ? wave_exact_any<METRIC, DIRECT>(p, qq, row, tile) : 0.f;
        if (i < ncand) recs[i] = rerank_rec<METRIC>(p, row, raw);
    }
    __syncthreads();
    // records at m and later are invalid (all ones: never less than a valid one)
    if (act) {
        for (int i = ht; i < m; i += 128) {
            const uint4 e = recs[i];
            if (e.x == 0xFFFFFFFFu) continue;
            int rank = 0;
            for (int o = 0; o < m; ++o) {
                const uint4 f = recs[o];
                rank += (rec_less(f, e) || (o < i && f.x == e.x && f.y == e.y && f.z == e.z && f.w == e.w)) ? 1 : 0;
            }
            atomicAdd(&s_nv[h], 1);
            if (rank < k) {
                out_ids[(int64_t)q * k + rank] = (int64_t)e.w + id_offset;
                out_dist[(int64_t)q * k + rank] = key_to_value(METRIC, e.x);
            }
        }
    }
    __syncthreads();
    if (act) {
        const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f
                          : (METRIC == kMetricIpRaw) ? -3.40282347e+38f
                                                     : 3.40282347e+38f;
        for (int i = s_nv[h] + ht; i < k; i += 128) {
            out_ids[(int64_t)q * k + i] = -1;
            out_dist[(int64_t)q * k + i] = pad;
        }
    }
}

// ---------------------------------------------------------------------------
// Exact re-rank of the pre-filter's survivors, spread over the whole chip
// (mqvs_search path 2): query q's cnt[q] survivor rows are surv[q * rs + i];
// their records go to recs[q * rs + i].  Work items (chunk of 256
// survivors, query), chunk-major, walked grid-stride.
template <int METRIC, bool DIRECT, bool XPF3 = true>
__global__ __launch_bounds__(SEL_THREADS) void k_exact_records(ScanParams p, const uint32_t *surv, const int *cnt,
                                                              int64_t rs, int chunks, uint4 *recs) {
    __shared__ float tiles[(SEL_THREADS / 64) * 64 * kRrStride];
    float *tile = tiles + (threadIdx.x >> 6) * 64 * kRrStride;
    const int items = p.nq * chunks;
    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        const int c = it / p.nq, q = it - c * p.nq;
        const int m = cnt[q];
        if (c * SEL_THREADS >= m) continue;  // uniform over the block
        const int i = c * SEL_THREADS + threadIdx.x;
        const int64_t row = i < m ? (int64_t)surv[(int64_t)q * rs + i] : -1;
        float raw;
        if ((p.d & 3) == 0)
            raw = XPF3 ? wave_exact_any<METRIC, DIRECT, 3>(p, q, row, tile) : wave_exact_any<METRIC, DIRECT>(p, q, row, tile);
        else
            raw = row >= 0 ? cand_value<METRIC, DIRECT>(p, q, row) : 0.f;
        if (i < m) recs[(int64_t)q * rs + i] = rerank_rec<METRIC>(p, row, raw);
    }
}

// Small batches: one wave per workgroup, work items of (64 survivors, query).
// At nq 1 the ~240 survivors of k_exact_records's one 256-thread workgroup
// were 24 tiles of random rows pulled through ONE CU (~780 KB at the per-CU
// read rate: ~23 us; a deeper query-slice prefetch did not help); here their
// 4 waves run on 4 CUs.  Same chain, same records.
template <int METRIC, bool DIRECT>
__global__ __launch_bounds__(64) void k_exact_records_1w(ScanParams p, const uint32_t *surv, const int *cnt,
                                                         int64_t rs, int chunks, uint4 *recs) {
    __shared__ float tile[64 * kRrStride];
    const int lane = threadIdx.x;
    const int64_t items = (int64_t)p.nq * chunks;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int c = (int)(it / p.nq), q = (int)(it - (int64_t)c * p.nq);
        const int m = cnt[q];
        if (c * 64 >= m) continue;  // (uniform over the wave)
        const int i = c * 64 + lane;
        const int64_t row = i < m ? (int64_t)surv[(int64_t)q * rs + i] : -1;
        const float raw = wave_exact_any<METRIC, DIRECT>(p, q, row, tile);
        if (i < m) recs[(int64_t)q * rs + i] = rerank_rec<METRIC>(p, row, raw);
    }
}

// Sort each query's cnt[q] records (recs[q * rs ...]; above kSortCap through
// global_sort with the next cnt[q] records as the second buffer) and write
// its top k.
// Top k of up to kSortCap records without sorting them all: the k-th
// smallest distance key X by radix select (LDS reads), the records with key
// <= X (k plus ties at X) compacted, and each of those placed by counting the
// smaller ones (full record order; keys are unique per row).  More than
// kSelCap records at <= X (mass ties): the bitonic sort of all of them.
constexpr int kSelCap = SEL_THREADS;

// rcap: the records' LDS room (a power of two <= kSortCap; kSortCap when a
// query may hold more records -- the global_sort path needs all of it)
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_sort_emit(uint4 *recs, const int *cnt, int64_t rs, int k,
                                                          int64_t id_offset, int64_t *out_ids, float *out_dist,
                                                          int rcap, const int *fl, int *host_fl) {
    extern __shared__ __attribute__((aligned(16))) uint4 lrec[];  // rcap + kSelCap records
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_c;
    const int q = blockIdx.x;
    if (host_fl && q == 0 && threadIdx.x < 8) {
        // the search's status words (final: written by earlier kernels)
        *reinterpret_cast<volatile int *>(host_fl + threadIdx.x) = fl[threadIdx.x];
        __threadfence_system();
    }
    const int m = cnt[q];
    uint4 *g = recs + (int64_t)q * rs;
    if (m > rcap) {
        rerank_emit<METRIC>(lrec, g, m, k, q, id_offset, out_ids, out_dist);
        return;
    }
    uint4 *sel = lrec + rcap;
    if (threadIdx.x == 0) s_c = 0;
    for (int i = threadIdx.x; i < m; i += SEL_THREADS) lrec[i] = g[i];
    __syncthreads();
    // X: the k-th key, or (k <= 256) an upper bound on it from the threads'
    // 4 smallest keys (kept_kth_bound: one pass, no per-key LDS atomics) --
    // the records <= X still hold the top k, and are placed by rank below
    __shared__ uint32_t skeys[4 * SEL_THREADS];
    const uint32_t X = k <= SEL_THREADS
                           ? kept_kth_bound<SEL_THREADS, 4>([&](int64_t i) { return lrec[i].x; }, m, k, skeys, hist, sh)
                           : block_radix_select([&](int64_t i) { return lrec[i].x; }, m, k, hist, sh);
    // (0xFFFFFFFE: fewer than k valid records -- all valid ones qualify)
    for (int i = threadIdx.x; i < m; i += SEL_THREADS) {
        const uint4 r = lrec[i];
        if (r.x != 0xFFFFFFFFu && r.x <= X) {
            const int pos = atomicAdd(&s_c, 1);
            if (pos < kSelCap) sel[pos] = r;
        }
    }
    __syncthreads();
    const int c = s_c;
    if (c > kSelCap) {
        rerank_emit<METRIC>(lrec, nullptr, m, k, q, id_offset, out_ids, out_dist);
        return;
    }
    if ((int)threadIdx.x < c) {
        const uint4 r = sel[threadIdx.x];
        int rank = 0, j = 0;
        for (; j + 4 <= c; j += 4) {
            const uint4 a0 = sel[j], a1 = sel[j + 1], a2 = sel[j + 2], a3 = sel[j + 3];
            rank += (rec_less(a0, r) ? 1 : 0) + (rec_less(a1, r) ? 1 : 0) + (rec_less(a2, r) ? 1 : 0) +
                    (rec_less(a3, r) ? 1 : 0);
        }
        for (; j < c; ++j) rank += rec_less(sel[j], r) ? 1 : 0;
        if (rank < k) {
            out_ids[(int64_t)q * k + rank] = (int64_t)r.w + id_offset;
            out_dist[(int64_t)q * k + rank] = key_to_value(METRIC, r.x);
        }
    }
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f
                      : (METRIC == kMetricIpRaw) ? -3.40282347e+38f
                                                 : 3.40282347e+38f;
    for (int i = c + threadIdx.x; i < k; i += SEL_THREADS) {
        out_ids[(int64_t)q * k + i] = -1;
        out_dist[(int64_t)q * k + i] = pad;
    }
}

void launch_exact_rerank(const ScanParams &p, int metric, const uint32_t *surv, const int *cnt, int64_t rs,
                         int cap, uint4 *recs, int k, int64_t id_offset, int64_t *out_ids, float *out_dist,
                         hipStream_t s, const int *fl, int *host_fl) {
    const int chunks = (cap + SEL_THREADS - 1) / SEL_THREADS;
    const int items = p.nq * chunks;
    const int grid = std::max(1, std::min(items, 4096));
    const bool direct = !blas_formula(p);
    // small batches (d % 4 == 0): one wave per workgroup over 64-survivor items
    const bool one_wave = (p.d & 3) == 0 && p.nq <= tune_int("MQVS_RR_1W_NQ", 16);
    const int chunks64 = (cap + 63) / 64;
    const int grid64 = std::max(1, std::min(p.nq * chunks64, 16384));
    // (measurement build A/B: MQVS_RR_XPF=1, the query slice one tile ahead)
    // (query slice three tiles ahead measured slower: nq 1 23.2 -> 25.2 us,
    // the index re-rank 124 -> 167 us)
    const bool xpf1 = tune_int("MQVS_RR_XPF", 1) == 1;
#define MQVS_ER(M)                                                                                                \
    do {                                                                                                          \
        if (one_wave && direct)                                                                                   \
            hipLaunchKernelGGL((k_exact_records_1w<M, true>), dim3(grid64), dim3(64), 0, s, p, surv, cnt, rs,      \
                               chunks64, recs);                                                                   \
        else if (one_wave)                                                                                        \
            hipLaunchKernelGGL((k_exact_records_1w<M, false>), dim3(grid64), dim3(64), 0, s, p, surv, cnt, rs,     \
                               chunks64, recs);                                                                   \
        else if (xpf1 && direct)                                                                                  \
            hipLaunchKernelGGL((k_exact_records<M, true, false>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv, cnt, \
                               rs, chunks, recs);                                                                 \
        else if (xpf1)                                                                                            \
            hipLaunchKernelGGL((k_exact_records<M, false, false>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv,  \
                               cnt, rs, chunks, recs);                                                            \
        else if (direct)                                                                                          \
            hipLaunchKernelGGL((k_exact_records<M, true>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv, cnt, rs, \
                               chunks, recs);                                                                     \
        else                                                                                                      \
            hipLaunchKernelGGL((k_exact_records<M, false>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv, cnt,    \
                               rs, chunks, recs);                                                                 \
        hipLaunchKernelGGL((k_sort_emit<M>), dim3(p.nq), dim3(SEL_THREADS), (kSortCap + kSelCap) * sizeof(uint4), s, \
                           recs, cnt, rs, k, id_offset, out_ids, out_dist, kSortCap, fl, host_fl);                 \
    } while (0)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_ER(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_ER(MQVS_METRIC_IP); break;
        case MQVS_METRIC_COSINE: MQVS_ER(MQVS_METRIC_COSINE); break;
        default: MQVS_ER(kMetricIpRaw); break;
    }
#undef MQVS_ER
}

// ---------------------------------------------------------------------------
// The index re-rank spread over waves instead of one workgroup per query
// (R <= kSortCap, d % 4 == 0).  k_rerank_ids_tiled keeps every query's
// candidates in one 4-wave workgroup: at ~233 VGPRs two waves per SIMD fit,
// so 1000 queries took two rounds of workgroups and a workgroup lasts as long
// as its slowest wave's 24-tile chain whether the bound pruned half its
// candidates or not.  Here:
//   k_rerank_plan      one wave per query: the pruned prefix (wave_prune_cut)
//                      and its valid rows, compacted in candidate order;
//   k_exact_records_w  work items of (64 candidates, query), chunk-major over
//                      the queries, one per wave (the waves of a workgroup
//                      take 4 consecutive queries' same chunk);
//   k_sort_emit        the top k of each query's records, as mqvs_search.
// Records and order are the ones k_rerank_ids_tiled produces.
template <int METRIC>
__global__ __launch_bounds__(256) void k_rerank_plan(ScanParams p, const int64_t *cand, int ncand, int k,
                                                     RerankPrune pr, uint32_t *surv, int *cnt) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (q >= p.nq) return;
    float w = 0.f;
    const bool ok = pr.raw && k < ncand && wave_prune_cut<METRIC>(p, pr, q, ncand, k, w);
    const int64_t *c = cand + (int64_t)q * ncand;
    const float *raw = pr.raw ? pr.raw + (int64_t)q * ncand : nullptr;
    uint32_t *out = surv + (int64_t)q * ncand;
    int n = 0, m = ncand;
    for (int i0 = 0; i0 < ncand; i0 += 64) {
        const int i = i0 + lane;
        bool keep = i < ncand;
        if (ok && keep) {
            const float a = raw[i];
            keep = METRIC == MQVS_METRIC_L2 ? a <= w : a >= w;
        }
        const uint64_t km = __ballot(keep);
        // the sorted candidates: the first one past the cut ends the prefix
        const int stop = km == ~0ull ? 64 : __builtin_ctzll(~km);
        const int64_t row = (i < ncand && lane < stop) ? c[i] : -1;
        const bool v = row >= 0 && row < p.n && row_valid(p, row);
        const uint64_t vm = __ballot(v);
        if (v) out[n + __popcll(vm & ((1ull << lane) - 1ull))] = (uint32_t)row;
        n += __popcll(vm);
        if (stop < 64) {
            m = i0 + stop;
            break;
        }
    }
    if (lane == 0) {
        cnt[q] = n;
        if (pr.count) atomicAdd(pr.count, (unsigned long long)m);
    }
}

template <int METRIC, bool DIRECT>
__global__ __launch_bounds__(SEL_THREADS) void k_exact_records_w(ScanParams p, const uint32_t *surv, const int *cnt,
                                                                int64_t rs, int chunks, uint4 *recs) {
    __shared__ float tiles[(SEL_THREADS / 64) * 64 * kRrStride];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *tile = tiles + wv * 64 * kRrStride;
    const int64_t items = (int64_t)p.nq * chunks;
    const int64_t nw = (int64_t)gridDim.x * (SEL_THREADS / 64);
    for (int64_t it = (int64_t)blockIdx.x * (SEL_THREADS / 64) + wv; it < items; it += nw) {
        const int c = (int)(it / p.nq), q = (int)(it - (int64_t)c * p.nq);
        const int m = cnt[q];
        if (c * 64 >= m) continue;  // (uniform over the wave)
        const int i = c * 64 + lane;
        const int64_t row = i < m ? (int64_t)surv[(int64_t)q * rs + i] : -1;
        const float raw = wave_exact_any<METRIC, DIRECT>(p, q, row, tile);
        if (i < m) recs[(int64_t)q * rs + i] = rerank_rec<METRIC>(p, row, raw);
    }
}

bool launch_rerank_ids_wide(const ScanParams &p, int metric, const int64_t *cand, int ncand, int k,
                            int64_t id_offset, int64_t *out_ids, float *out_dist, const RerankPrune &pr,
                            uint32_t *surv, int *cnt, uint4 *recs, hipStream_t s) {
    if (ncand > kSortCap || (p.d & 3) || p.nq <= 0) return false;
    const bool direct = !blas_formula(p);
    const int chunks = (ncand + 63) / 64;
    const int64_t items = (int64_t)p.nq * chunks;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((items + 3) / 4, 8192));
    int rcap = 1;  // (every query holds at most ncand records: LDS for that many)
    while (rcap < ncand) rcap <<= 1;
#define MQVS_RW(M)                                                                                                  \
    do {                                                                                                            \
        hipLaunchKernelGGL((k_rerank_plan<M>), dim3((p.nq + 3) / 4), dim3(256), 0, s, p, cand, ncand, k, pr, surv,  \
                           cnt);                                                                                    \
        if (direct)                                                                                                 \
            hipLaunchKernelGGL((k_exact_records_w<M, true>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv, cnt,      \
                               (int64_t)ncand, chunks, recs);                                                       \
        else                                                                                                        \
            hipLaunchKernelGGL((k_exact_records_w<M, false>), dim3(grid), dim3(SEL_THREADS), 0, s, p, surv, cnt,     \
                               (int64_t)ncand, chunks, recs);                                                       \
        hipLaunchKernelGGL((k_sort_emit<M>), dim3(p.nq), dim3(SEL_THREADS), (rcap + kSelCap) * sizeof(uint4), s,     \
                           recs, cnt, (int64_t)ncand, k, id_offset, out_ids, out_dist, rcap, nullptr, nullptr);     \
    } while (0)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_RW(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_RW(MQVS_METRIC_IP); break;
        default: MQVS_RW(MQVS_METRIC_COSINE); break;
    }
#undef MQVS_RW
    return true;
}

template <int M, bool DIRECT>
static void rerank_ids_t(const ScanParams &p, const int64_t *cand, int ncand, int k, int64_t id_offset,
                         int64_t *ids, float *dist, uint4 *scratch, hipStream_t s, const RerankPrune &pr) {
    int N = 1;
    while (N < ncand) N <<= 1;
    if (scratch) N = kSortCap;  // LDS records of global_sort
    if ((p.d & 3) == 0 && !scratch && ncand <= kRrPairMax && tune_int("MQVS_RR_PAIR", 0) == 1) {
        const size_t lds = 2 * (size_t)ncand * sizeof(uint4) + (SEL_THREADS / 64) * 64 * kRrStride * sizeof(float);
        hipLaunchKernelGGL((k_rerank_ids_pair<M, DIRECT>), dim3((p.nq + 1) / 2), dim3(SEL_THREADS), lds, s, p, cand,
                           ncand, k, id_offset, ids, dist, pr);
    } else if ((p.d & 3) == 0) {
        const size_t lds = N * sizeof(uint4) + (SEL_THREADS / 64) * 64 * kRrStride * sizeof(float);
        // (measurement build A/B: MQVS_IDX_XPF=3, the query slice three tiles ahead)
        if (tune_int("MQVS_IDX_XPF", 1) == 3)
            hipLaunchKernelGGL((k_rerank_ids_tiled<M, DIRECT, 3>), dim3(p.nq), dim3(SEL_THREADS), lds, s, p, cand,
                               ncand, k, id_offset, ids, dist, N, scratch, pr);
        else
            hipLaunchKernelGGL((k_rerank_ids_tiled<M, DIRECT>), dim3(p.nq), dim3(SEL_THREADS), lds, s, p, cand,
                               ncand, k, id_offset, ids, dist, N, scratch, pr);
    } else {
        hipLaunchKernelGGL((k_rerank_ids<M, DIRECT>), dim3(p.nq), dim3(SEL_THREADS), N * sizeof(uint4), s, p, cand,
                           ncand, k, id_offset, ids, dist, scratch, pr);
    }
}

void launch_rerank_ids(const ScanParams &p, int metric, const int64_t *cand, int ncand, int k,
                       int64_t id_offset, int64_t *out_ids, float *out_dist, uint4 *scratch, hipStream_t s,
                       const RerankPrune &pr) {
    const bool direct = !blas_formula(p);
#define MQVS_RR(M)                                                                                   \
    direct ? rerank_ids_t<M, true>(p, cand, ncand, k, id_offset, out_ids, out_dist, scratch, s, pr) \
           : rerank_ids_t<M, false>(p, cand, ncand, k, id_offset, out_ids, out_dist, scratch, s, pr)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_RR(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_RR(MQVS_METRIC_IP); break;
        default: MQVS_RR(MQVS_METRIC_COSINE); break;
    }
#undef MQVS_RR
}

}  // namespace mqvs
