// scan_emit.h -- epilogue of the approximate (bf16 / MX) scan kernels: PROBE
// stores dense approximate values, APPEND keeps rows over the threshold.
#pragma once

#include "mqvs_internal.h"

namespace mqvs {

// AGG = false: one atomic per taker -- the batch kernels (kernels_p4.hip),
// whose appends are rare and spread over many queries: the aggregated form
// there made the whole nq 1000 main scan 7 % slower (12.6 -> 13.5 ms, same-box
// library A/B, profiles/r05/emit_agg_ab.txt: its end-of-launch queue flush
// walks up to 64 queries per ballot round)
template <int METRIC, bool PROBE, bool AGG = true>
__device__ inline void emit_approx(const ScanParams &p, int j, int64_t pos, int64_t row, bool valid,
                                   float raw) {
    if (PROBE) {
        p.probe[(int64_t)j * p.probe_ld + (pos - p.row_begin)] = valid ? raw : __builtin_nanf("");
        return;
    }
    if constexpr (!AGG) {
        if (!valid) return;
        const float t = p.thr[j];
        if ((METRIC == MQVS_METRIC_L2) ? (raw <= t) : (raw >= t)) {
            const int slot = atomicAdd(&p.cand_count[j], 1);
            if (slot < p.cand_cap) {
                Cand c;
                c.raw = raw;
                c.row = (uint32_t)row;
                p.cand[(int64_t)j * p.cand_cap + slot] = c;
            }
        }
        return;
    }
    const bool take = valid && ((METRIC == MQVS_METRIC_L2) ? (raw <= p.thr[j]) : (raw >= p.thr[j]));
    // Wave-aggregated append: one atomic per query among the wave's takers
    // (the active lanes of this call).  With few queries -- nq = 1, or a
    // loose threshold early in a scan -- every taker of a wave hits the same
    // counter, and per-lane atomics on it serialised the first main segment
    // of a 1 %-selective gathered scan (6.6k appends: 129 us for 66k rows).
    uint64_t pend = __ballot(take);
    if (pend == 0) return;
    const int lane = (int)__lane_id();
    while (pend) {
        const int leader = __builtin_ctzll(pend);
        const int jl = __shfl(j, leader);
        const bool mine = take && j == jl;
        const uint64_t same = __ballot(mine);
        int base = 0;
        if (lane == leader) base = atomicAdd(&p.cand_count[jl], (int)__popcll(same));
        base = __shfl(base, leader);
        if (mine) {
            const int slot = base + (int)__popcll(same & ((1ull << lane) - 1ull));
            if (slot < p.cand_cap) {
                Cand c;
                c.raw = raw;
                c.row = (uint32_t)row;
                p.cand[(int64_t)j * p.cand_cap + slot] = c;
            }
        }
        pend &= ~same;
    }
}

// pos: scan position (probe column); row: its row, -1 = gather padding
template <int METRIC, bool PROBE>
__device__ inline void emit_ip(const ScanParams &p, int j, int64_t pos, int64_t row, float ip) {
    if (row < 0) {
        if (PROBE) emit_approx<METRIC, true>(p, j, pos, row, false, 0.f);
        return;
    }
    float raw = ip;
    if (METRIC == MQVS_METRIC_L2) {
        raw = (p.qnorms[j] + p.row_norms[row]) - 2.0f * ip;
        if (raw < 0) raw = 0;
    }
    emit_approx<METRIC, PROBE>(p, j, pos, row, row_valid(p, row), raw);
}

// Epilogue for NV accumulator values of query j (scan positions pos_of(0..NV-1)).
// APPEND: candidates are rare, so the fast path only compares every value
// with the query's threshold (no row bounds, no bitmaps, no branches); the
// values of a wave with any lane over it take the exact per-row path.
template <int METRIC, bool PROBE, int NV, class RowFn, class ValFn>
__device__ inline void emit_vals(const ScanParams &p, int j, int64_t r1, RowFn pos_of, ValFn val) {
    if (PROBE) {
#pragma unroll
        for (int r = 0; r < NV; ++r) {
            const int64_t pos = pos_of(r);
            if (pos < r1) emit_ip<METRIC, true>(p, j, pos, row_at(p, pos), val(r));
        }
        return;
    }
    const float t = p.thr[j];
    const float qn = (METRIC == MQVS_METRIC_L2) ? p.qnorms[j] : 0.f;
    bool any = false;
#pragma unroll
    for (int r = 0; r < NV; ++r) {
        float raw = val(r);
        if (METRIC == MQVS_METRIC_L2) {
            const int64_t row = max(row_at(p, min(pos_of(r), r1 - 1)), (int64_t)0);
            raw = (qn + p.row_norms[row]) - 2.0f * raw;
            if (raw < 0) raw = 0;
            any |= raw <= t;
        } else {
            any |= raw >= t;
        }
    }
    if (any) {
#pragma unroll
        for (int r = 0; r < NV; ++r) {
            const int64_t pos = pos_of(r);
            if (pos < r1) emit_ip<METRIC, false>(p, j, pos, row_at(p, pos), val(r));
        }
    }
}

}  // namespace mqvs
