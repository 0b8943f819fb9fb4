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

template <int METRIC, bool DIRECT>
__global__ __launch_bounds__(SEL_THREADS) void k_rerank_ids(ScanParams p, const int64_t *cand, int ncand,
                                                           int k, int64_t id_offset, int64_t *out_ids,
                                                           float *out_dist) {
    extern __shared__ __attribute__((aligned(16))) uint4 recs[];  // kSortCap records
    const int q = blockIdx.x;
    const int64_t *c = cand + (int64_t)q * ncand;
    for (int i = threadIdx.x; i < ncand; i += SEL_THREADS) {
        const int64_t row = c[i];
        uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (row >= 0 && row < p.n && row_valid(p, row)) {
            const float raw = cand_value<METRIC, DIRECT>(p, q, row);
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
        }
        recs[i] = r;
    }
    int N = 1;
    while (N < ncand) N <<= 1;
    for (int i = ncand + threadIdx.x; i < N; i += SEL_THREADS)
        recs[i] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    __syncthreads();
    block_bitonic_sort(recs, N);
    const float pad = (METRIC == MQVS_METRIC_IP) ? 1.17549435e-38f : 3.40282347e+38f;
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

template <int M, bool DIRECT>
static void rerank_ids_t(const ScanParams &p, const int64_t *cand, int ncand, int k, int64_t id_offset,
                         int64_t *ids, float *dist, hipStream_t s) {
    hipLaunchKernelGGL((k_rerank_ids<M, DIRECT>), dim3(p.nq), dim3(SEL_THREADS), kSortCap * sizeof(uint4), s,
                       p, cand, ncand, k, id_offset, ids, dist);
}

void launch_rerank_ids(const ScanParams &p, int metric, const int64_t *cand, int ncand, int k,
                       int64_t id_offset, int64_t *out_ids, float *out_dist, hipStream_t s) {
    const bool direct = p.nq < kBlasThreshold;
#define MQVS_RR(M)                                                                  \
    direct ? rerank_ids_t<M, true>(p, cand, ncand, k, id_offset, out_ids, out_dist, s) \
           : rerank_ids_t<M, false>(p, cand, ncand, k, id_offset, out_ids, out_dist, s)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_RR(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_RR(MQVS_METRIC_IP); break;
        default: MQVS_RR(MQVS_METRIC_COSINE); break;
    }
#undef MQVS_RR
}

}  // namespace mqvs
