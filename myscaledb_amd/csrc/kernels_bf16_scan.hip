// kernels_bf16_scan.hip -- split-precision bf16 MFMA scan (the nq >= 20
// pre-filter of kernels_bf16.hip).
//
// SPLIT = 3: x = xh + xl (two bf16 roundings) and
//     x.y ~ xh.yh + xh.yl + xl.yh
// accumulated in one fp32 accumulator: 3 bf16 MFMAs per block-step, 3/16 of
// the f32 MFMA cost.  Error vs the exact fp32 chain (bound in
// kernels_bf16.hip, k_query_bound):
//     (3.1 2^-16 + 4.1 d 2^-24 + 1.2e-7) |x| |y|
// SPLIT = 1: hi planes only, bound (2^-7 + 2^-16 + 2.1 d 2^-24) |x| |y|.
//
// Workgroup tile: 256 rows x QT queries, 4 x WQ waves, each wave 64 rows x
// (32 QB) queries:
//     nq <= 64 : 256 x  64  (8 waves, QB 1)   LDS 2 x 40 KiB
//     nq <= 128: 256 x 128  (8 waves, QB 2)   LDS 2 x 48 KiB
//     else     : 256 x 256  (8 waves, QB 4)   LDS 2 x 64 KiB
// K is staged 32 bf16 (64 B per row per plane) deep; one stage is the
// contiguous image [Y hi | Y lo | Q hi | Q lo] filled by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB = 16 image rows per instruction), double
// buffered.  The large tile gives each 64 KiB stage ~3k cycles of MFMA work,
// enough for a one-stage prefetch to cover the load latency.
//
// Schedule variants (VAR bits, chosen per shape in launch_split):
//   1  s_setprio(1) around the stage's MFMA work, so the waves of a SIMD
//      keep the matrix pipe fed while another wave issues loads
//   2  the next stage's LDS-DMA issue split in two halves placed between the
//      MFMA groups (instead of one burst after the barrier, where every wave
//      of the workgroup issues at once and the matrix pipe idles)
//   4  v_mfma_f32_16x16x32_bf16 (4 x 2QB blocks of 16 x 16 per wave) instead
//      of v_mfma_f32_32x32x16_bf16 (2 x QB blocks of 32 x 32)
//   128 Y-early ring (16x16x32 only): the Y part of stage s+2 is issued right
//      after a mid-stage barrier (default for the nq <= 128 shapes)
// Diagnostic builds, reachable only through MQVS_BF16_TUNE: 64 s_memtime
// stage stamps; 256 / 512 drop the per-stage load wait / all per-stage sync
// (WRONG results, timing only -- they showed the 256 x 256 shape is bound by
// its MFMA + ds_read + LDS-DMA issue stream, not by load latency: no change
// without the wait, +3.5% without any barrier).
// Chunk c (16 B) of image row r sits at slot c ^ f(r): f(r) = (r >> 2) & 3 for
// the 32x32 fragment reads, 2 ((r >> 2) & 1) for the 16x16 reads; either way
// every ds_read_b128 lane group hits 16 distinct 16-B bank slots.
#include <cstdio>
#include <cstdlib>

#include "mqvs_internal.h"
#include "scan_emit.h"

namespace mqvs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BS_K = 32;          // bf16 per row per stage
constexpr int BS_ROWB = BS_K * 2; // 64 B: 4 chunks of 16 B
constexpr int BS_RT = kBfRows;    // rows per workgroup tile (all shapes)

template <bool M16>
__device__ inline int swz(int r, int c) {
    return M16 ? (c ^ (((r >> 2) & 1) << 1)) : (c ^ ((r >> 2) & 3));
}

template <int METRIC, bool PROBE, int SPLIT, int WQ, int QB, int VAR>
__global__ __launch_bounds__(256 * WQ) void k_scan_bf16(ScanParams p) {
    constexpr bool PRIO = VAR & 1, SPLIT_ISSUE = VAR & 2, M16 = VAR & 4, STAMPS = VAR & 64,
                   YEARLY = (VAR & 128) && M16;
    constexpr int WR = 4;                   // row waves
    constexpr int NW = WR * WQ;             // waves per workgroup
    constexpr int QT = 32 * QB * WQ;        // queries per workgroup
    constexpr int PL = (SPLIT == 3) ? 2 : 1;// planes per operand
    constexpr int GY = BS_RT / 16;          // 1-KiB groups per Y plane
    constexpr int GQ = QT / 16;             // 1-KiB groups per Q plane
    constexpr int G = PL * (GY + GQ);       // groups per stage
    constexpr int GPW = G / NW;             // groups per wave
    static_assert(G % NW == 0, "stage groups must split evenly over the waves");
    constexpr int STAGE = G * 1024;         // bytes per stage
    constexpr int YPW = (PL * GY) / NW;     // Y-plane groups per wave: src[0, YPW)
    static_assert((PL * GY) % NW == 0, "Y groups must split evenly over the waves");
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][STAGE];

    const int64_t L = p.tiles * p.num_qblocks;
    const int64_t cpx = (L + 7) / 8;
    const int64_t b = blockIdx.x;
    const int64_t l = (b % 8) * cpx + b / 8;  // query blocks of a row tile on one XCD
    if (l >= L) return;
    const int64_t ti = l / p.num_qblocks;
    const int qb = (int)(l % p.num_qblocks);
    int64_t r0, r1, chunk;
    tile_range(p, ti, r0, r1, chunk);
    if (r0 >= r1) return;  // tile past the end of a partial last granule
    const int ord = chunk_ordinal(p, chunk);
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int wr = w % WR, wq = w / WR;
    const int q0 = qb * QT;

    if (ord < 0) {
        if (PROBE) {
            for (int i = t; i < BS_RT * QT; i += 64 * NW) {
                const int64_t row = r0 + (i % BS_RT);
                const int j = q0 + i / BS_RT;
                if (row < r1 && j < p.nq) emit_approx<METRIC, true>(p, j, row, -1, false, 0.f);
            }
        }
        return;
    }

    // LDS-DMA sources: group g = wave w + i*NW (i < GPW) fills 16 image rows
    // of one plane; lane -> (row lane/4, slot lane%4) holds chunk swz(row, slot)
    const uint16_t *src[GPW];
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        const int g = w + i * NW;
        int pl, rbase;  // plane 0..3 = Yh, Yl, Qh, Ql
        if (g < PL * GY) {
            pl = g / GY;
            rbase = (g % GY) * 16;
        } else {
            pl = 2 + (g - PL * GY) / GQ;
            rbase = ((g - PL * GY) % GQ) * 16;
        }
        const int r = rbase + (lane >> 2);
        const int c = swz<M16>(r, lane & 3);
        if (pl < 2) {
            const int64_t gp = r0 + r;
            int64_t gr = gp < r1 ? row_at(p, gp) : -1;
            if (gr < 0) gr = row_at(p, r0);  // padding: any real row, results discarded
            src[i] = (pl == 0 ? p.rows_hi : p.rows_lo) + gr * p.dpad + c * 8;
        } else {
            int j = q0 + r;
            if (j >= p.nq) j = 0;
            const int64_t qo = ((int64_t)j * p.maxv + variant_of(p, j, ord)) * p.dpad + c * 8;
            src[i] = (pl == 2 ? p.q_hi : p.q_lo) + qo;
        }
    }
    auto issue = [&](int s, int bf, int i0, int i1) {
        const int64_t k0 = (int64_t)s * BS_K;
#pragma unroll
        for (int i = 0; i < GPW; ++i)
            if (i >= i0 && i < i1)
                __builtin_amdgcn_global_load_lds((const void *)(src[i] + k0),
                                                 (lds_void *)&lds[bf][(w + i * NW) * 1024], 16, 0, 0);
    };
    // split issue: half `part` of the next stage's pieces, pinned in place
    auto issue_part = [&](bool more, int s, int part) {
        if (!SPLIT_ISSUE || !more) return;
        __builtin_amdgcn_sched_barrier(0);
        issue(s + 1, (s + 1) & 1, part * (GPW / 2), part == 0 ? GPW / 2 : GPW);
        __builtin_amdgcn_sched_barrier(0);
    };

    // plane byte offsets inside a stage
    constexpr int OFF_YH = 0;
    constexpr int OFF_YL = GY * 1024;
    constexpr int OFF_QH = PL * GY * 1024;
    constexpr int OFF_QL = OFF_QH + GQ * 1024;
    auto frag = [&](const unsigned char *st, int off, int r, int c) {
        return *reinterpret_cast<const bf16x8 *>(st + off + r * BS_ROWB + swz<M16>(r, c) * 16);
    };
    auto mma32 = [](bf16x8 a, bf16x8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    };
    auto mma16 = [](bf16x8 a, bf16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    };

    const int nst = (int)(p.dpad / BS_K);
    if constexpr (!YEARLY) {
        issue(0, 0, 0, GPW);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    if constexpr (!M16) {
        const int h = lane >> 5, l32 = lane & 31;
        f32x16 acc[2][QB];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < QB; ++j) acc[i][j] = f32x16{0};
        const int ra0 = wr * 64 + l32;
        const int rq0 = wq * 32 * QB + l32;
        for (int s = 0; s < nst; ++s) {
            const bool more = s + 1 < nst;
            if (!SPLIT_ISSUE && more) issue(s + 1, (s + 1) & 1, 0, GPW);
            const unsigned char *st = lds[s & 1];
            if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < BS_K / 16; ++kk) {
                const int c = 2 * kk + h;
                bf16x8 ah[2], al[2], bh[QB], bl[QB];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    ah[i] = frag(st, OFF_YH, ra0 + 32 * i, c);
                    if (SPLIT == 3) al[i] = frag(st, OFF_YL, ra0 + 32 * i, c);
                }
#pragma unroll
                for (int j = 0; j < QB; ++j) {
                    bh[j] = frag(st, OFF_QH, rq0 + 32 * j, c);
                    if (SPLIT == 3) bl[j] = frag(st, OFF_QL, rq0 + 32 * j, c);
                }
                issue_part(more, s, kk);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < QB; ++j) {
                        acc[i][j] = mma32(ah[i], bh[j], acc[i][j]);
                        if (SPLIT == 3) {
                            acc[i][j] = mma32(ah[i], bl[j], acc[i][j]);
                            acc[i][j] = mma32(al[i], bh[j], acc[i][j]);
                        }
                    }
            }
            if (PRIO) __builtin_amdgcn_s_setprio(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int jb = 0; jb < QB; ++jb) {
                const int j = q0 + rq0 + jb * 32;
                if (j >= p.nq) continue;
                const int64_t rbase = r0 + wr * 64 + rb * 32 + 4 * h;
                emit_vals<METRIC, PROBE, 16>(
                    p, j, r1, [&](int r) { return rbase + (r & 3) + 8 * (r >> 2); },
                    [&](int r) { return acc[rb][jb][r]; });
            }
    } else {
        // 16x16x32: lane -> row (lane & 15) of a 16-row block, chunk lane >> 4
        constexpr int QB16 = 2 * QB;  // 16-query blocks per wave
        const int l16 = lane & 15, c = lane >> 4;
        f32x4 acc[4][QB16];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < QB16; ++j) acc[i][j] = f32x4{0};
        const int ra0 = wr * 64 + l16;
        const int rq0 = wq * 32 * QB + l16;
        // diagnostic build only (VAR bit 64): per-wave s_memtime stamps
        uint64_t sum_read = 0, sum_mfma = 0, sum_sync = 0, tp = 0;
        auto stamp = [&]() -> uint64_t {
            uint64_t tt = 0;
            if constexpr (STAMPS) {
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt)::"memory");
                __builtin_amdgcn_sched_barrier(0);
            }
            return tt;
        };
        if constexpr (STAMPS) tp = stamp();
        if constexpr (YEARLY) {
            // Y-early ring (VAR bit 128): a stage's Y planes are consumed as
            // soon as every wave has its row fragments, so the Y part of stage
            // s+2 is issued into the current buffer right after a mid-stage
            // barrier (~1.9 stages of lead for the HBM-streamed rows); the Q
            // part of stage s+1 goes out at the top of stage s.  Issue order
            // per wave: Y(s+1) < Q(s+1) < Y(s+2), so the wait for stage s+1
            // is vmcnt(YPW).  Barriers are raw (no vmcnt(0) drain) and written
            // as one asm statement with a memory clobber, so no LDS access
            // moves across them.
            issue(0, 0, 0, GPW);
            if (nst > 1) {
                issue(1, 1, 0, YPW);
                asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(YPW) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            }
            for (int s = 0; s < nst; ++s) {
                const unsigned char *st = lds[s & 1];
                if (s + 1 < nst) {
                    __builtin_amdgcn_sched_barrier(0);
                    issue(s + 1, (s + 1) & 1, YPW, GPW);  // Q(s+1): its buffer part is free
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (PRIO) __builtin_amdgcn_s_setprio(1);
                bf16x8 ah[4], al[4], bh[QB], bl[QB];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    ah[i] = frag(st, OFF_YH, ra0 + 16 * i, c);
                    if (SPLIT == 3) al[i] = frag(st, OFF_YL, ra0 + 16 * i, c);
                }
#pragma unroll
                for (int jj = 0; jj < QB; ++jj) {
                    bh[jj] = frag(st, OFF_QH, rq0 + 16 * jj, c);
                    if (SPLIT == 3) bl[jj] = frag(st, OFF_QL, rq0 + 16 * jj, c);
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Y(s) consumed
                if (s + 2 < nst) {
                    __builtin_amdgcn_sched_barrier(0);
                    issue(s + 2, s & 1, 0, YPW);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    if (hf == 1) {
#pragma unroll
                        for (int jj = 0; jj < QB; ++jj) {
                            bh[jj] = frag(st, OFF_QH, rq0 + 16 * (QB + jj), c);
                            if (SPLIT == 3) bl[jj] = frag(st, OFF_QL, rq0 + 16 * (QB + jj), c);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int jj = 0; jj < QB; ++jj) {
                            f32x4 &a = acc[i][hf * QB + jj];
                            a = mma16(ah[i], bh[jj], a);
                            if (SPLIT == 3) {
                                a = mma16(ah[i], bl[jj], a);
                                a = mma16(al[i], bh[jj], a);
                            }
                        }
                }
                if (PRIO) __builtin_amdgcn_s_setprio(0);
                if (s + 2 < nst)
                    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(YPW) : "memory");
                else if (s + 1 < nst)
                    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            }
        }
        for (int s = 0; s < (YEARLY ? 0 : nst); ++s) {
            const bool more = s + 1 < nst;
            if (!SPLIT_ISSUE && more) issue(s + 1, (s + 1) & 1, 0, GPW);
            const unsigned char *st = lds[s & 1];
            if (PRIO) __builtin_amdgcn_s_setprio(1);
            bf16x8 ah[4], al[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ah[i] = frag(st, OFF_YH, ra0 + 16 * i, c);
                if (SPLIT == 3) al[i] = frag(st, OFF_YL, ra0 + 16 * i, c);
            }
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                bf16x8 bh[QB], bl[QB];
#pragma unroll
                for (int jj = 0; jj < QB; ++jj) {
                    bh[jj] = frag(st, OFF_QH, rq0 + 16 * (hf * QB + jj), c);
                    if (SPLIT == 3) bl[jj] = frag(st, OFF_QL, rq0 + 16 * (hf * QB + jj), c);
                }
                if constexpr (STAMPS) {
                    if (hf == 0) {
                        const uint64_t t1 = stamp();
                        sum_read += t1 - tp;
                        tp = t1;
                    }
                }
                issue_part(more, s, hf);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int jj = 0; jj < QB; ++jj) {
                        f32x4 &a = acc[i][hf * QB + jj];
                        a = mma16(ah[i], bh[jj], a);
                        if (SPLIT == 3) {
                            a = mma16(ah[i], bl[jj], a);
                            a = mma16(al[i], bh[jj], a);
                        }
                    }
            }
            if (PRIO) __builtin_amdgcn_s_setprio(0);
            if constexpr (STAMPS) {
                const uint64_t t2 = stamp();
                sum_mfma += t2 - tp;
                tp = t2;
            }
            if constexpr ((VAR & 512) != 0) {
                // diagnostic only (wrong results): no per-stage sync at all
            } else if constexpr ((VAR & 256) != 0) {
                asm volatile("s_barrier" ::: "memory");  // diagnostic only: barrier without the load wait
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            if constexpr (STAMPS) {
                const uint64_t t3 = stamp();
                sum_sync += t3 - tp;
                tp = t3;
            }
        }
        if constexpr (STAMPS) {
            if (lane == 0 && p.dbg) {
                atomicAdd(&p.dbg[0], (unsigned long long)sum_read);
                atomicAdd(&p.dbg[1], (unsigned long long)sum_mfma);
                atomicAdd(&p.dbg[2], (unsigned long long)sum_sync);
                atomicAdd(&p.dbg[3], 1ull);
                atomicAdd(&p.dbg[4], (unsigned long long)nst);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jb = 0; jb < QB16; ++jb) {
                const int j = q0 + rq0 + jb * 16;
                if (j >= p.nq) continue;
                const int64_t rbase = r0 + wr * 64 + i * 16 + 4 * c;
                emit_vals<METRIC, PROBE, 4>(
                    p, j, r1, [&](int r) { return rbase + r; }, [&](int r) { return acc[i][jb][r]; });
            }
    }
}

template <int METRIC, bool PROBE, int SPLIT, int WQ, int QB, int VAR>
static void launch_shape(ScanParams p, hipStream_t s) {
    constexpr int QT = 32 * QB * WQ;
    p.num_qblocks = (p.nq + QT - 1) / QT;
    const int64_t L = p.tiles * p.num_qblocks;
    if (L < 1) return;
    const int64_t grid = (L + 7) / 8 * 8;
    if constexpr ((VAR & 64) != 0) {
        // diagnostic build: per-wave stage-segment cycle sums, printed per launch
        static unsigned long long *dbg = nullptr;
        if (!dbg) (void)hipMalloc((void **)&dbg, 8 * sizeof(unsigned long long));
        (void)hipMemsetAsync(dbg, 0, 8 * sizeof(unsigned long long), s);
        p.dbg = dbg;
        hipLaunchKernelGGL((k_scan_bf16<METRIC, PROBE, SPLIT, WQ, QB, VAR>), dim3((unsigned)grid),
                           dim3(256 * WQ), 0, s, p);
        unsigned long long h[8] = {0};
        (void)hipMemcpyAsync(h, dbg, sizeof(h), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const double stages = h[4] ? (double)h[4] : 1.0;
        std::fprintf(stderr, "stamps waves=%llu stages=%llu cycles/stage: read %.0f mfma %.0f sync %.0f\n", h[3],
                     h[4], h[0] / stages, h[1] / stages, h[2] / stages);
        return;
    }
    hipLaunchKernelGGL((k_scan_bf16<METRIC, PROBE, SPLIT, WQ, QB, VAR>), dim3((unsigned)grid),
                       dim3(256 * WQ), 0, s, p);
}

// Tuning override (tools/tune_bf16.py, cosine APPEND split-3 launches only):
// MQVS_BF16_TUNE="WQ,QB,VAR" picks the workgroup shape and schedule variant.
static bool tune_override(int &wq, int &qb, int &var) {
    const char *e = tune_env("MQVS_BF16_TUNE");
    if (!e || !*e) return false;
    return std::sscanf(e, "%d,%d,%d", &wq, &qb, &var) == 3;
}

template <int METRIC, bool PROBE, int SPLIT>
static bool launch_tuned(const ScanParams &p, hipStream_t s) {
    int wq, qb, var;
    if (!tune_override(wq, qb, var)) return false;
    const int key = (wq * 10 + qb) * 1000 + var;
    switch (key) {
#define MQVS_TUNE_CASE(WQ_, QB_, V_) \
    case (WQ_ * 10 + QB_) * 1000 + V_:launch_shape<METRIC, PROBE, SPLIT, WQ_, QB_, V_>(p, s); return true;
        MQVS_TUNE_CASE(1, 2, 0) MQVS_TUNE_CASE(1, 2, 4) MQVS_TUNE_CASE(1, 2, 7)
        MQVS_TUNE_CASE(2, 1, 0) MQVS_TUNE_CASE(2, 1, 4) MQVS_TUNE_CASE(2, 1, 7)
        MQVS_TUNE_CASE(1, 4, 0) MQVS_TUNE_CASE(1, 4, 4) MQVS_TUNE_CASE(1, 4, 7)
        MQVS_TUNE_CASE(2, 2, 0) MQVS_TUNE_CASE(2, 2, 4) MQVS_TUNE_CASE(2, 2, 7)
        MQVS_TUNE_CASE(2, 4, 0) MQVS_TUNE_CASE(2, 4, 4) MQVS_TUNE_CASE(2, 4, 7) MQVS_TUNE_CASE(2, 4, 71)
        MQVS_TUNE_CASE(2, 4, 132) MQVS_TUNE_CASE(2, 4, 133) MQVS_TUNE_CASE(2, 2, 133) MQVS_TUNE_CASE(2, 1, 133)
        MQVS_TUNE_CASE(2, 4, 263) MQVS_TUNE_CASE(2, 4, 519)
#undef MQVS_TUNE_CASE
        default: return false;
    }
}

template <int METRIC, bool PROBE, int SPLIT>
static void launch_split(const ScanParams &p, hipStream_t s) {
    if constexpr (METRIC == MQVS_METRIC_COSINE && !PROBE && SPLIT == 3)
        if (launch_tuned<METRIC, PROBE, SPLIT>(p, s)) return;
    // shapes and variants measured with tools/tune_bf16.py (10M x 768 cosine,
    // profiles/r01/tune_bf16_*.jsonl): nq 64: 5.86 ms (Y-early ring, HBM
    // ~5.2 TB/s), nq 128: 7.33 ms (Y-early), nq 1000: 36.1 ms (1.27 PF/s; the
    // Y-early ring's extra barrier costs 5% on this MFMA-bound shape)
    constexpr int kSmallVar = SPLIT == 3 ? 133 : 7;
    if (p.nq <= 64)  // (split 1 has 20 pieces per stage: 4 waves)
        launch_shape<METRIC, PROBE, SPLIT, SPLIT == 3 ? 2 : 1, SPLIT == 3 ? 1 : 2, kSmallVar>(p, s);
    else if (p.nq <= 128)
        launch_shape<METRIC, PROBE, SPLIT, 2, 2, kSmallVar>(p, s);
    else
        launch_shape<METRIC, PROBE, SPLIT, 2, 4, 7>(p, s);
}

template <int METRIC, bool PROBE>
static void launch_bf16_t(const ScanParams &p, int split, hipStream_t s) {
    if (split == 3)
        launch_split<METRIC, PROBE, 3>(p, s);
    else
        launch_split<METRIC, PROBE, 1>(p, s);
}

void launch_scan_bf16(const ScanParams &p, int metric, bool probe, int split, hipStream_t s) {
    switch (metric) {
        case MQVS_METRIC_L2:
            probe ? launch_bf16_t<MQVS_METRIC_L2, true>(p, split, s)
                  : launch_bf16_t<MQVS_METRIC_L2, false>(p, split, s);
            break;
        case MQVS_METRIC_IP:
            probe ? launch_bf16_t<MQVS_METRIC_IP, true>(p, split, s)
                  : launch_bf16_t<MQVS_METRIC_IP, false>(p, split, s);
            break;
        case MQVS_METRIC_COSINE:
            probe ? launch_bf16_t<MQVS_METRIC_COSINE, true>(p, split, s)
                  : launch_bf16_t<MQVS_METRIC_COSINE, false>(p, split, s);
            break;
        default:
            probe ? launch_bf16_t<kMetricIpRaw, true>(p, split, s)
                  : launch_bf16_t<kMetricIpRaw, false>(p, split, s);
            break;
    }
}

}  // namespace mqvs
