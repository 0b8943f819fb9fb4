// kernels_binary.hip -- brute-force scan of binary vectors (FixedString(N)
// columns): tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110),
// i.e. faiss::hammings_knn_mc (Hamming) and jaccard_knn (Jaccard) under
// vectorScanWithoutIndex<BinaryVector> (MergeTreeVSManager.cpp:1188-1273,
// 1395-1425).
//
// Popcount work is integer and HBM-bound (one 16-B code slice per lane per
// step, a handful of v_xor / v_bcnt per slice and query), so it stays on the
// VALU; no reshaping into MFMA.  A 256-thread workgroup owns a 256-row tile,
// one row per lane; code rows are 16-B aligned (stride code_words * 4 B, zero
// padded -- zero bytes add nothing to xor / and / or popcounts).  Queries are
// wave-uniform and come in through scalar loads, QC per pass; rows of up to
// 8 x 16 B (1024 bits) stay in registers across query passes, longer rows
// are re-read per pass (L1/L2 hits after the first).
//
// The value each row gets (the "raw" of the shared select pipeline):
//   Hamming  popcount(q ^ y) as a float; rows at distance == d bits are never
//            returned (hammings_knn_mc emits distances b < nBit only)
//   Jaccard  (den - num) / den in fp32, 1.0 when num == 0 (KAT 00038 pins the
//            division form)
// Both are ascending and finite, so probe / refine / final select run with
// the L2 ordering key (ord_asc) and the (key, row) tie rule of
// hammings_knn_mc's per-distance arrival order and searchWrapper's strict
// merge.  APPEND with tau_strict: after the probe (rows [0, P)) and every
// refine, the candidates hold every row scanned so far with key <= tau, and
// later segments only contain larger rows, so a row with key == tau can never
// beat the k-th candidate: strict `key < tau` keeps integer ties (Hamming)
// from flooding the candidate lists.
#include "mqvs_internal.h"

namespace mqvs {

template <int METRIC, bool PROBE, bool REG>
__global__ __launch_bounds__(256) void k_scan_binary(ScanParams p) {
    constexpr int QC = 8;   // queries per pass (accumulators in registers)
    constexpr int RW = 8;   // 16-B slices kept in registers (REG: rows <= 1024 bits)
    const int t = threadIdx.x;
    const int W4 = p.code_words / 4;
    const int nbits = p.nbits;
    for (int64_t ti = blockIdx.x; ti < p.tiles; ti += gridDim.x) {
        int64_t r0, r1, chunk;
        tile_range(p, ti, r0, r1, chunk);
        const int64_t pos = r0 + t;
        const bool inrange = pos < r1;
        const int64_t row = pos;
        const bool valid_row = inrange && row_valid(p, row);
        const uint4 *yr = reinterpret_cast<const uint4 *>(p.codes + (inrange ? row : 0) * p.code_words);
        uint4 yc[RW];
        if (REG) {
#pragma unroll
            for (int u = 0; u < RW; ++u)
                yc[u] = (u < W4 && inrange) ? yr[u] : make_uint4(0u, 0u, 0u, 0u);
        }
        for (int j0 = 0; j0 < p.nq; j0 += QC) {
            uint32_t a[QC], b[QC];
#pragma unroll
            for (int jj = 0; jj < QC; ++jj) a[jj] = b[jj] = 0u;
            auto step = [&](const uint4 y, int u) {
#pragma unroll
                for (int jj = 0; jj < QC; ++jj) {
                    if (j0 + jj < p.nq) {  // wave-uniform
                        const uint4 q = reinterpret_cast<const uint4 *>(p.qcodes + (int64_t)(j0 + jj) * p.code_words)[u];
                        if (METRIC == MQVS_METRIC_HAMMING) {
                            a[jj] += __builtin_popcount(q.x ^ y.x) + __builtin_popcount(q.y ^ y.y) +
                                     __builtin_popcount(q.z ^ y.z) + __builtin_popcount(q.w ^ y.w);
                        } else {
                            a[jj] += __builtin_popcount(q.x & y.x) + __builtin_popcount(q.y & y.y) +
                                     __builtin_popcount(q.z & y.z) + __builtin_popcount(q.w & y.w);
                            b[jj] += __builtin_popcount(q.x | y.x) + __builtin_popcount(q.y | y.y) +
                                     __builtin_popcount(q.z | y.z) + __builtin_popcount(q.w | y.w);
                        }
                    }
                }
            };
            if (REG) {
#pragma unroll
                for (int u = 0; u < RW; ++u)
                    if (u < W4) step(yc[u], u);
            } else {
                for (int u = 0; u < W4; ++u) step(inrange ? yr[u] : make_uint4(0u, 0u, 0u, 0u), u);
            }
#pragma unroll
            for (int jj = 0; jj < QC; ++jj) {
                const int j = j0 + jj;
                if (j >= p.nq) break;  // wave-uniform
                float raw;
                bool valid = valid_row;
                if (METRIC == MQVS_METRIC_HAMMING) {
                    raw = (float)a[jj];
                    valid = valid && (int)a[jj] < nbits;
                } else {
                    raw = a[jj] == 0u ? 1.0f : (float)(b[jj] - a[jj]) / (float)b[jj];
                }
                if (PROBE) {
                    if (inrange) p.probe[(int64_t)j * p.probe_ld + (pos - p.row_begin)] = valid ? raw : __builtin_nanf("");
                    continue;
                }
                const uint32_t key = ord_asc(raw);
                const uint32_t tau = p.tau[j];
                const bool take = valid && (p.tau_strict ? key < tau : key <= tau);
                const unsigned long long m = __ballot(take);
                if (m == 0) continue;
                const int lane = t & 63;
                const int leader = __ffsll((long long)m) - 1;
                int base = 0;
                if (lane == leader) base = atomicAdd(&p.cand_count[j], __popcll(m));
                base = __shfl(base, leader);
                if (take) {
                    const int slot = base + __popcll(m & ((1ull << lane) - 1ull));
                    if (slot < p.cand_cap) {
                        Cand c;
                        c.raw = raw;
                        c.row = (uint32_t)row;
                        p.cand[(int64_t)j * p.cand_cap + slot] = c;
                    }
                }
            }
        }
    }
}

template <int METRIC, bool PROBE>
static void scan_binary_t(const ScanParams &p, hipStream_t s) {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(p.tiles, 4096));
    if (p.code_words <= 32)
        hipLaunchKernelGGL((k_scan_binary<METRIC, PROBE, true>), dim3(grid), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((k_scan_binary<METRIC, PROBE, false>), dim3(grid), dim3(256), 0, s, p);
}

void launch_scan_binary(const ScanParams &p, int metric, bool probe, hipStream_t s) {
    if (metric == MQVS_METRIC_HAMMING)
        probe ? scan_binary_t<MQVS_METRIC_HAMMING, true>(p, s) : scan_binary_t<MQVS_METRIC_HAMMING, false>(p, s);
    else
        probe ? scan_binary_t<MQVS_METRIC_JACCARD, true>(p, s) : scan_binary_t<MQVS_METRIC_JACCARD, false>(p, s);
}

// Hamming results of the faiss contract (mqvs_knn_binary_raw): float counts
// -> int32 in place (the reference's reinterpret_cast<int32_t*>(distance)),
// padding INT32_MAX.
__global__ void k_hamming_to_int(const int64_t *ids, float *dist, int64_t m) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) {
        const int32_t v = ids[i] >= 0 ? (int32_t)dist[i] : 2147483647;
        reinterpret_cast<int32_t *>(dist)[i] = v;
    }
}

void launch_hamming_to_int(const int64_t *ids, float *dist, int64_t m, hipStream_t s) {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 1024));
    hipLaunchKernelGGL(k_hamming_to_int, dim3(grid), dim3(256), 0, s, ids, dist, m);
}

}  // namespace mqvs
