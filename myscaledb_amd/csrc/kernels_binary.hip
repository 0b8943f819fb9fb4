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
#include <cstdlib>

#include "mqvs_internal.h"

namespace mqvs {

template <int METRIC, bool PROBE, bool REG>
__global__ __launch_bounds__(256) void k_scan_binary(ScanParams p) {
    constexpr int QC = 8;   // queries per pass (accumulators in registers)
    constexpr int RW = 8;   // 16-B slices kept in registers (REG: rows <= 1024 bits)
    const int t = threadIdx.x;
    const int W4 = p.code_words / 4;
    const int nbits = p.nbits;
    // REG: the next tile's row is loaded before this tile's popcounts, so two
    // rows per lane are in flight (HBM latency x bandwidth needs ~64 KB per CU)
    uint4 yn[RW];
    auto load_row = [&](int64_t ti, uint4 *dst) {
        int64_t r0, r1, chunk;
        tile_range(p, ti, r0, r1, chunk);
        const int64_t pos = r0 + t;
        const uint4 *src = reinterpret_cast<const uint4 *>(p.codes + (pos < r1 ? pos : 0) * p.code_words);
#pragma unroll
        for (int u = 0; u < RW; ++u) dst[u] = (u < W4 && pos < r1) ? src[u] : make_uint4(0u, 0u, 0u, 0u);
    };
    if (REG && blockIdx.x < p.tiles) load_row(blockIdx.x, yn);
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
            for (int u = 0; u < RW; ++u) yc[u] = yn[u];
            if (ti + gridDim.x < p.tiles) load_row(ti + gridDim.x, yn);
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
                if (PROBE) {
                    float raw;
                    bool valid = valid_row;
                    if (METRIC == MQVS_METRIC_HAMMING) {
                        raw = (float)a[jj];
                        valid = valid && (int)a[jj] < nbits;
                    } else {
                        raw = a[jj] == 0u ? 1.0f : (float)(b[jj] - a[jj]) / (float)b[jj];
                    }
                    if (inrange) p.probe[(int64_t)j * p.probe_ld + (pos - p.row_begin)] = valid ? raw : __builtin_nanf("");
                    continue;
                }
                // APPEND: the threshold as a value (wave-uniform); keys of the
                // non-negative values are ord_asc = bits | 2^31, and a tau of
                // 0xFFFFFFFE / 0xFFFFFFFF (fewer than k rows so far) takes all
                const uint32_t tau = p.tau[j];
                const bool all = tau >= 0xFFFFFFFEu;
                const float tf = __builtin_bit_cast(float, tau & 0x7FFFFFFFu);
                bool take;
                float raw = 0.f;
                if (METRIC == MQVS_METRIC_HAMMING) {
                    // integer limit: h < ceil(tf) (strict) or h <= floor(tf)
                    int lim = nbits;
                    if (!all && tf < (float)nbits) lim = p.tau_strict ? (int)ceilf(tf) : (int)floorf(tf) + 1;
                    take = valid_row && (int)a[jj] < lim;
                    raw = (float)a[jj];
                } else {
                    // cheap superset test first, exact fp32 division for the few that pass
                    const float dn = (float)(b[jj] - a[jj]), dd = (float)b[jj];
                    take = valid_row && (all || a[jj] == 0u || dn <= tf * dd * 1.0000005f);
                    if (take) {
                        raw = a[jj] == 0u ? 1.0f : dn / dd;
                        const uint32_t key = ord_asc(raw);
                        take = p.tau_strict ? key < tau : key <= tau;
                    }
                }
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

// Small batches (nq <= 8) are HBM-bound: lanes read consecutive 16-B slices
// of the tile (fully coalesced) instead of one row each.  With W4 slices per
// row (W4 = 1, 2, 4, 8), lane t always holds slice u = t % W4 of rows
// (s * 256 + t) / W4, s = 0 .. W4-1; its query slices sit in registers for
// the whole launch, partial popcounts are summed over the W4 lanes of a row
// by xor-shuffles, and lane u == 0 emits the row.
template <int METRIC, bool PROBE, int W4>
__global__ __launch_bounds__(256) void k_scan_binary_co(ScanParams p) {
    constexpr int QC = 8;
    const int t = threadIdx.x;
    const int u = t & (W4 - 1);
    const int nbits = p.nq > 0 ? p.nbits : 0;
    uint4 qv[QC];
#pragma unroll
    for (int jj = 0; jj < QC; ++jj)
        qv[jj] = jj < p.nq ? reinterpret_cast<const uint4 *>(p.qcodes + (int64_t)jj * p.code_words)[u]
                           : make_uint4(0u, 0u, 0u, 0u);
    // per-query integer limits / value thresholds of APPEND (wave-uniform)
    int lim[QC];
    float tfv[QC];
    bool allv[QC];
#pragma unroll
    for (int jj = 0; jj < QC; ++jj) {
        lim[jj] = nbits;
        tfv[jj] = 0.f;
        allv[jj] = true;
        if (!PROBE && jj < p.nq) {
            const uint32_t tau = p.tau[jj];
            allv[jj] = tau >= 0xFFFFFFFEu;
            tfv[jj] = __builtin_bit_cast(float, tau & 0x7FFFFFFFu);
            if (!allv[jj] && tfv[jj] < (float)nbits)
                lim[jj] = p.tau_strict ? (int)ceilf(tfv[jj]) : (int)floorf(tfv[jj]) + 1;
        }
    }
    const uint4 *base = reinterpret_cast<const uint4 *>(p.codes);
    for (int64_t ti = blockIdx.x; ti < p.tiles; ti += gridDim.x) {
        int64_t r0, r1, chunk;
        tile_range(p, ti, r0, r1, chunk);
        uint4 y[W4];
#pragma unroll
        for (int sidx = 0; sidx < W4; ++sidx) {
            const int64_t row = r0 + (sidx * 256 + t) / W4;
            y[sidx] = row < r1 ? base[r0 * W4 + sidx * 256 + t] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int sidx = 0; sidx < W4; ++sidx) {
            const int64_t row = r0 + (sidx * 256 + t) / W4;
            const bool inrange = row < r1;
            const bool lead = u == 0;
            const bool valid_row = lead && inrange && row_valid(p, row);
#pragma unroll
            for (int jj = 0; jj < QC; ++jj) {
                if (jj >= p.nq) break;  // wave-uniform
                const uint4 q = qv[jj], yy = y[sidx];
                uint32_t a, b = 0u;
                if (METRIC == MQVS_METRIC_HAMMING) {
                    a = __builtin_popcount(q.x ^ yy.x) + __builtin_popcount(q.y ^ yy.y) +
                        __builtin_popcount(q.z ^ yy.z) + __builtin_popcount(q.w ^ yy.w);
                } else {
                    a = __builtin_popcount(q.x & yy.x) + __builtin_popcount(q.y & yy.y) +
                        __builtin_popcount(q.z & yy.z) + __builtin_popcount(q.w & yy.w);
                    b = __builtin_popcount(q.x | yy.x) + __builtin_popcount(q.y | yy.y) +
                        __builtin_popcount(q.z | yy.z) + __builtin_popcount(q.w | yy.w);
                }
#pragma unroll
                for (int o = 1; o < W4; o <<= 1) {
                    a += __shfl_xor(a, o);
                    if (METRIC == MQVS_METRIC_JACCARD) b += __shfl_xor(b, o);
                }
                if (PROBE) {
                    if (lead && inrange) {
                        float raw;
                        bool valid = valid_row;
                        if (METRIC == MQVS_METRIC_HAMMING) {
                            raw = (float)a;
                            valid = valid && (int)a < nbits;
                        } else {
                            raw = a == 0u ? 1.0f : (float)(b - a) / (float)b;
                        }
                        p.probe[(int64_t)jj * p.probe_ld + (row - p.row_begin)] = valid ? raw : __builtin_nanf("");
                    }
                    continue;
                }
                bool take;
                float raw = 0.f;
                if (METRIC == MQVS_METRIC_HAMMING) {
                    take = valid_row && (int)a < lim[jj];
                    raw = (float)a;
                } else {
                    const float dn = (float)(b - a), dd = (float)b;
                    take = valid_row && (allv[jj] || a == 0u || dn <= tfv[jj] * dd * 1.0000005f);
                    if (take) {
                        raw = a == 0u ? 1.0f : dn / dd;
                        const uint32_t key = ord_asc(raw);
                        const uint32_t tau = p.tau[jj];
                        take = p.tau_strict ? key < tau : key <= tau;
                    }
                }
                const unsigned long long m = __ballot(take);
                if (m == 0) continue;
                const int lane = t & 63;
                const int leader = __ffsll((long long)m) - 1;
                int cbase = 0;
                if (lane == leader) cbase = atomicAdd(&p.cand_count[jj], __popcll(m));
                cbase = __shfl(cbase, leader);
                if (take) {
                    const int slot = cbase + __popcll(m & ((1ull << lane) - 1ull));
                    if (slot < p.cand_cap) {
                        Cand c;
                        c.raw = raw;
                        c.row = (uint32_t)row;
                        p.cand[(int64_t)jj * p.cand_cap + slot] = c;
                    }
                }
            }
        }
    }
}

static int64_t bin_grid_cap() {
    static const int64_t cap = [] {
        const char *e = tune_env("MQVS_BIN_GRID");  // tuning knob (tools/binary_sweep.py)
        return e ? std::max<int64_t>(64, std::atoll(e)) : (int64_t)4096;
    }();
    return cap;
}

template <int METRIC, bool PROBE>
static void scan_binary_t(const ScanParams &p, hipStream_t s) {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(p.tiles, bin_grid_cap()));
    if (p.nq <= 8 && !tune_env("MQVS_BIN_NOCO")) {
        switch (p.code_words / 4) {
            case 1: hipLaunchKernelGGL((k_scan_binary_co<METRIC, PROBE, 1>), dim3(grid), dim3(256), 0, s, p); return;
            case 2: hipLaunchKernelGGL((k_scan_binary_co<METRIC, PROBE, 2>), dim3(grid), dim3(256), 0, s, p); return;
            case 4: hipLaunchKernelGGL((k_scan_binary_co<METRIC, PROBE, 4>), dim3(grid), dim3(256), 0, s, p); return;
            case 8: hipLaunchKernelGGL((k_scan_binary_co<METRIC, PROBE, 8>), dim3(grid), dim3(256), 0, s, p); return;
            default: break;
        }
    }
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
