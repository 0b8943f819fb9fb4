// kernels_hi.hip -- bf16-hi pre-filter (split 2, the default): ONE bf16 MFMA
// per block-step on the bf16 roundings of rows and queries, a rigorous error
// bound from norms measured at quantisation, and the exact fp32 re-rank of the
// survivors (kernels_bf16.hip, k_rerank_select).
//
// Why one product is enough.  With h = bf16_rn(v) and r = v - h (exact),
//     x.y - xh.yh = xh.ry + rx.yh + rx.ry
// so |x.y - xh.yh| <= |xh||ry| + |rx||yh| + |rx||ry| (Cauchy-Schwarz), where
// |r| / |v| is ~2^-9 for any vector (round-to-nearest to 8 significant bits).
// The margin this leaves around the k-th value (~0.004 of |x||y|) admits a
// few hundred extra rows per query on the Gaussian / mixture parts measured;
// every one of them is re-ranked with the exact fp32 chain, so the output is
// bit-identical to the fp32 path.  (Rounds 1-2 also kept a hi + lo split and
// a bf16 + fp6-MX split; both streamed more bytes per element for the same
// survivors and were removed in round 3.)
//
// Planes are row-blocked in groups of 16 vectors (mqvs_internal.h,
// kPlaneSlab): vector u, stage s (32 columns) at byte (u >> 4) nst 1024 +
// plane_step_off(s) + plane_vec_off(u & 15); a stage's 16-vector piece is
// 1 KiB contiguous (kPlaneSlab 32).
//
// Scan pipeline: a ring of NBUF LDS stages (stage = 32 columns of the 256-row
// tile and of the QT-query tile, filled by global_load_lds_dwordx4 in 1 KiB
// pieces), NBUF - 1 stages in flight.  Per stage: a counted vmcnt for this
// wave's pieces of the stage being consumed (later stages stay in flight), ONE
// raw s_barrier (every wave's pieces have landed; every wave is done with the
// stage consumed before, whose buffer is re-issued right after the barrier),
// then the MFMA work.  No __syncthreads() in the loop: its fence would drain
// the in-flight LDS-DMA (cdna_hip_programming.md, "Pipelining across barriers").
#include <cstdio>
#include <atomic>
#include <cstdlib>

#include "mqvs_internal.h"
#include "scan_emit.h"
#include "tuning.h"

namespace mqvs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int bf16x4x2 __attribute__((ext_vector_type(4)));  // 8 bf16 as 4 dwords (16-B loads)
typedef __attribute__((address_space(3))) void lds_void;

constexpr int HI_K = 32;  // columns per stage

// sqrt(s) rounded up to float
__device__ inline float hi_sqrt_up(double s) { return (float)(sqrt(s) * (1.0 + 1e-7)); }

// ---------------------------------------------------------------------------
// quantisation: source vector v -> plane vector u = (v % vgroup) vpad + v / vgroup
// record (kMxRec floats, the MX record's slots): [0] |h|, [1] |r|, [6] |x|
// One wave per vector, grid-stride over the vectors; the segment maxima of
// |h|, |r|, |x| are reduced per workgroup and published with three atomics
// per workgroup (one atomic per vector on the same three words serialised:
// 340 ms for 10M x 768, profiles/r03/bench_kernel_stats.csv).
__global__ __launch_bounds__(256) void k_to_hi(const float *src, int64_t rows, int d, int64_t sstride, int64_t dpad,
                                               int64_t vgroup, int64_t vpad, uint16_t *hi, float *rec,
                                               float *maxrec) {
    __shared__ unsigned smax[4][3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nb = (int)(dpad / HI_K);
    unsigned m[3] = {0u, 0u, 0u};  // running maxima (bit patterns of non-negative floats; NaN -> +inf)
    for (int64_t v = (int64_t)blockIdx.x * 4 + w; v < rows; v += (int64_t)gridDim.x * 4) {
        const float *x = src + v * sstride;
        const int64_t u = (v % vgroup) * vpad + v / vgroup;
        uint16_t *hu = hi ? hi + (u >> 4) * nb * 512 + plane_vec_off((uint32_t)(u & 15)) / 2 : nullptr;  // (null: records only)
        double nx = 0, nh = 0, nr = 0;
        for (int64_t i = lane; i < dpad; i += 64) {
            const float xv = i < d ? x[i] : 0.f;
            const uint16_t hb = f32_to_bf16_rn(xv);
            const float hv = __builtin_bit_cast(float, (uint32_t)hb << 16);
            const float rv = xv - hv;  // exact
            if (hi) hu[plane_step_off((uint32_t)(i >> 5)) / 2 + (i & 31)] = hb;
            nx += (double)xv * xv;
            nh += (double)hv * hv;
            nr += (double)rv * rv;
        }
        for (int off = 32; off > 0; off >>= 1) {
            nx += __shfl_xor(nx, off);
            nh += __shfl_xor(nh, off);
            nr += __shfl_xor(nr, off);
        }
        const float r[kMxRec] = {hi_sqrt_up(nh), hi_sqrt_up(nr), 0.f, 0.f, 0.f, 0.f, hi_sqrt_up(nx), 0.f};
        if (rec && lane < kMxRec) {
            float rv = 0.f;
#pragma unroll
            for (int t = 0; t < kMxRec; ++t)
                if (lane == t) rv = r[t];
            rec[v * kMxRec + lane] = rv;
        }
        const int slot[3] = {0, 1, 6};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const float f = r[slot[t]];
            const unsigned bits = (f == f) ? __builtin_bit_cast(unsigned, f) : 0x7F800000u;
            m[t] = bits > m[t] ? bits : m[t];
        }
    }
    if (!maxrec) return;
    if (lane == 0)
        for (int t = 0; t < 3; ++t) smax[w][t] = m[t];
    __syncthreads();
    if (threadIdx.x < 3) {
        const int t = threadIdx.x;
        unsigned b = smax[0][t];
        for (int ww = 1; ww < 4; ++ww) b = smax[ww][t] > b ? smax[ww][t] : b;
        atomicMax(reinterpret_cast<unsigned *>(maxrec) + (t == 2 ? 6 : t), b);
    }
}

void launch_to_hi(const float *src, int64_t rows, int d, int64_t src_stride, int64_t dpad, int64_t vgroup,
                  int64_t vpad, uint16_t *hi, float *rec, float *maxrec, hipStream_t s) {
    if (rows <= 0) return;
    const int cus = device_cus();
    const int64_t blocks = std::min<int64_t>((rows + 3) / 4, (int64_t)cus * 16);
    hipLaunchKernelGGL(k_to_hi, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, d, src_stride, dpad, vgroup, vpad,
                       hi, rec, maxrec);
}

// ---------------------------------------------------------------------------
// scan

__device__ inline int hswz(int r, int c) { return c ^ ((r >> 2) & 3); }

// s_waitcnt vmcnt(N) + raw s_barrier, N a compile-time count
template <int N>
__device__ inline void wait_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// raw s_barrier, no memory-op or MFMA movement across it
__device__ inline void raw_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(pend * P), pend in [0, DMAX - 1] (a runtime count: the tail
// of a loop issues fewer stages)
template <int P, int DMAX>
__device__ inline void wait_vm(int pend) {
    __builtin_amdgcn_sched_barrier(0);
    if (DMAX >= 4 && pend >= 3)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * 3) : "memory");
    else if (DMAX >= 3 && pend >= 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * 2) : "memory");
    else if (DMAX >= 2 && pend >= 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P * 1) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int GPW, int NBUF>
__device__ inline void wait_stage(int pending) {
    // pending: stages issued after the one about to be consumed (0 .. NBUF-2)
    static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
    if (NBUF >= 4 && pending >= 2) {
        wait_barrier<GPW * 2>();
    } else if (NBUF >= 3 && pending >= 1) {
        wait_barrier<GPW * 1>();
    } else {
        wait_barrier<0>();
    }
}

// Workgroup tile 256 rows x QT queries (QT = 32 QB WQ), 4 x WQ waves of 64
// rows x 32 QB queries, 32x32x16 bf16 MFMA blocks; workgroup -> (row tile,
// query block) with the query blocks of a row tile on one XCD (its L2 serves
// the tile's re-reads).
//
// PP (ping-pong): the two waves of a SIMD (waves w and w + 4: the query halves
// wq = 0 / 1) run one barrier apart, so that while one computes its 16 MFMAs of
// a stage the other reads its fragments of the next stage from LDS and issues
// its LDS-DMA pieces; the MFMA pipe then never waits for a wave's own reads /
// DMA issue (the lock-step loop leaves it idle during both: 18 ms compute-only
// against 6.6 ms of MFMA cycles at 10M x 768, nq 1000).  Every barrier is a
// raw s_barrier; a stage is ready for reading after a barrier that every
// issuing wave reached past a counted vmcnt covering its pieces; a buffer is
// re-issued only after the barrier that follows the last MFMA phase reading
// it.  Stages are issued D = NBUF - 2 ahead.
// DIAG (diagnostic builds, wrong results): 1 = row pieces read from the first
// 8 tiles only (an L2-resident row stream), 2 = query pieces from query
// group 0 only, 4 = query pieces not issued, 8 = row pieces not issued (the
// stage then holds stale bytes; the waits count only the issued pieces).
template <int METRIC, bool PROBE, int WQ, int QB, int NBUF, int PP = 0, int DIAG = 0>
__global__ __launch_bounds__(256 * WQ) void k_scan_hi(ScanParams p) {
    constexpr int WR = 4;
    constexpr int NW = WR * WQ;
    constexpr int QT = 32 * QB * WQ;
    constexpr int RT = kBfRows;     // 256
    constexpr int GY = RT / 16;     // 1-KiB pieces of the Y image
    constexpr int GQ = QT / 16;     // 1-KiB pieces of the Q image
    constexpr int G = GY + GQ;
    static_assert(G % NW == 0, "stage pieces must split evenly over the waves");
    constexpr int GPW = G / NW;
    constexpr int STAGE = G * 1024;
    __shared__ __attribute__((aligned(16))) unsigned char lds[NBUF * STAGE];

    const int64_t L = p.tiles * p.num_qblocks;
    const int64_t cpx = (L + 7) / 8;
    const int64_t b = blockIdx.x;
    const int64_t l = (b % 8) * cpx + b / 8;  // query blocks of a row tile on one XCD
    if (l >= L) return;
    const int64_t ti = l / p.num_qblocks;
    const int qb = (int)(l % p.num_qblocks);
    int64_t r0, r1, chunk;
    tile_range(p, ti, r0, r1, chunk);
    if (r0 >= r1) return;
    const int ord = chunk_ordinal(p, chunk);
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int wr = w % WR, wq = w / WR;
    const int q0 = qb * QT;

    if (ord < 0) {
        if (PROBE) {
            for (int i = t; i < RT * QT; i += 64 * NW) {
                const int64_t row = r0 + (i % RT);
                const int j = q0 + i / RT;
                if (row < r1 && j < p.nq) emit_approx<METRIC, true>(p, j, row, -1, false, 0.f);
            }
        }
        return;
    }

    const int nb = (int)(p.dpad / HI_K);
    // piece g = w + i NW fills 16 image rows; lane -> (image row lane / 4,
    // slot lane % 4) holds chunk hswz(row, slot)
    const unsigned char *src[GPW];
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        const int g = w + i * NW;
        const bool isy = g < GY;
        const int r = (isy ? g : g - GY) * 16 + (lane >> 2);
        const int c = hswz(r, lane & 3);
        int64_t u;
        const uint16_t *plane;
        if (isy) {
            const int64_t gp = r0 + r;
            u = gp < r1 ? row_at(p, gp) : -1;
            if (u < 0) u = row_at(p, r0);  // padding: any real row, results discarded
            if (DIAG & 1) u = (ti & 7) * RT + r;
            plane = p.rows_hi;
        } else {
            int j = q0 + r;
            if (j >= p.nq) j = 0;
            if (DIAG & 2) j = r & 15;
            u = (int64_t)variant_of(p, j, ord) * p.q_vpad + j;
            plane = p.q_hi;
        }
        src[i] = reinterpret_cast<const unsigned char *>(plane) +
                 ((u >> 4) * nb * 1024 + plane_vec_off((uint32_t)(u & 15)) + c * 16);
    }
    static_assert(GY % NW == 0, "row pieces: whole rounds of the waves");
    constexpr int YPW = GY / NW;  // pieces i < YPW are row pieces, the rest query pieces
    auto issue = [&](int s) {
        unsigned char *dst = lds + (s % NBUF) * STAGE;
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            if ((DIAG & 8) && i < YPW) continue;
            if ((DIAG & 4) && i >= YPW) continue;
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + plane_step_off((uint32_t)s)),
                                             (lds_void *)(dst + (w + i * NW) * 1024), 16, 0, 0);
        }
    };

    constexpr int OFF_Q = GY * 1024;
    const int h = lane >> 5, l32 = lane & 31;
    auto frag = [&](const unsigned char *st, int r, int c) {
        return *reinterpret_cast<const bf16x8 *>(st + r * 64 + hswz(r, c) * 16);
    };
    const int ra0 = wr * 64 + l32;
    const int rq0 = wq * 32 * QB + l32;

    f32x16 acc[2][QB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jb = 0; jb < QB; ++jb) acc[i][jb] = f32x16{0};

    const int nst = (int)(p.dpad / HI_K);
    constexpr int NPW = GPW - ((DIAG & 8) ? YPW : 0) - ((DIAG & 4) ? GPW - YPW : 0);  // pieces per wave, stage
    if constexpr (PP) {
        static_assert(WQ == 2 && NBUF >= 3, "ping-pong: two query halves, stages issued NBUF - 2 ahead");
        constexpr int D = NBUF - 2;
        const int grp = wq;  // waves w and w + 4 share a SIMD
        auto stage_frags = [&](int s, bf16x8 (&ah)[2][2], bf16x8 (&bh)[2][QB]) {
            const unsigned char *st = lds + (s % NBUF) * STAGE;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int c = 2 * kk + h;
#pragma unroll
                for (int i = 0; i < 2; ++i) ah[kk][i] = frag(st, ra0 + 32 * i, c);
#pragma unroll
                for (int jb = 0; jb < QB; ++jb) bh[kk][jb] = frag(st + OFF_Q, rq0 + 32 * jb, c);
            }
        };
        // prologue: stages 0 .. D-1 issued, stage 0 landed for everyone
#pragma unroll
        for (int s = 0; s < D; ++s)
            if (s < nst) issue(s);
        wait_vm<NPW, D>(nst - 1 < D - 1 ? nst - 1 : D - 1);
        raw_barrier();
        if (grp == 1) raw_barrier();
        for (int s = 0; s < nst; ++s) {
            bf16x8 ah[2][2], bh[2][QB];
            // read phase (the partner wave computes meanwhile)
            stage_frags(s, ah, bh);
            if (s + D < nst) issue(s + D);
            // pieces younger than stage s+1's, which the barrier after the
            // partner's next read phase must find landed
            const int pend = (nst - 2 - s) < D - 1 ? (nst - 2 - s) : D - 1;
            if (grp == 1 && s + 1 < nst) wait_vm<NPW, D>(pend);
            raw_barrier();
            // MFMA phase (the partner reads meanwhile)
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jb = 0; jb < QB; ++jb)
                        acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kk][i], bh[kk][jb], acc[i][jb], 0, 0,
                                                                             0);
            __builtin_amdgcn_s_setprio(0);
            if (grp == 0 && s + 1 < nst) wait_vm<NPW, D>(pend);
            raw_barrier();
        }
        if (grp == 0) raw_barrier();
    } else {
#pragma unroll
        for (int s = 0; s < NBUF - 1; ++s)
            if (s < nst) issue(s);
        for (int s = 0; s < nst; ++s) {
            const int after = nst - 1 - s;  // stages after s
            wait_stage<NPW, NBUF>(after < NBUF - 2 ? after : NBUF - 2);
            // every wave is past its reads of stage s-1: its buffer takes stage s+NBUF-1
            if (s + NBUF - 1 < nst) {
                __builtin_amdgcn_sched_barrier(0);
                issue(s + NBUF - 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            const unsigned char *st = lds + (s % NBUF) * STAGE;
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int c = 2 * kk + h;
                bf16x8 ah[2], bh[QB];
#pragma unroll
                for (int i = 0; i < 2; ++i) ah[i] = frag(st, ra0 + 32 * i, c);
#pragma unroll
                for (int jb = 0; jb < QB; ++jb) bh[jb] = frag(st + OFF_Q, rq0 + 32 * jb, c);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jb = 0; jb < QB; ++jb)
                        acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[jb], acc[i][jb], 0, 0, 0);
            }
            __builtin_amdgcn_s_setprio(0);
            // (the next iteration's barrier orders these reads before the buffer
            // is re-issued: the MFMAs consumed every fragment, so the reads retired)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
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
}

// Small batches (nq <= 32): HBM-bound, so no LDS staging at all.  The 256-row
// tile is 16 row blocks of 16 rows; wave w takes blocks w, w+4, w+8, w+12.  A
// row block's 32-column stage is ONE contiguous KiB of the row-blocked plane
// and exactly the A operand of v_mfma_f32_16x16x32_bf16 (lane l: row l & 15,
// columns 8 (l >> 4) .. +8), so each stage is one global_load_dwordx4 straight
// into the fragment; a block's whole row (nst loads, 24 KiB at d = 768) is in
// flight while the previous block feeds the MFMAs.  The query tile (NQB blocks
// of 16 queries, every stage's B fragment: 4 VGPRs each) stays in registers.
// NBLK: row blocks per wave -- 4 (256-row tiles), or 1 (kBfRowsSmall-row
// tiles: short scans such as a few queries' probe, where 256-row tiles leave
// most CUs idle and each wave's four blocks in a row set the time)
template <int METRIC, bool PROBE, int NQB, int NST, bool NT = false, int NBLK = 4>
__global__ __launch_bounds__(256) void k_scan_hi_reg(ScanParams p) {
    constexpr int RT = 64 * NBLK;
    const int64_t ti = blockIdx.x / p.num_qblocks;
    const int qb = (int)(blockIdx.x % p.num_qblocks);
    if (ti >= p.tiles) return;
    int64_t r0, r1, chunk;
    tile_range(p, ti, r0, r1, chunk);
    if (r0 >= r1) return;
    // (a gathered chunk run is padded to whole 256-row tiles: a shorter tile
    // may hold padding only -- no row, as an unsearched chunk)
    const int ord = (NBLK < 4 && p.row_list && p.row_list[r0] < 0) ? -1 : chunk_ordinal(p, chunk);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int l16 = lane & 15, c = lane >> 4;
    const int q0 = qb * 16 * NQB;
    if (ord < 0) {
        if (PROBE) {
            for (int i = t; i < RT * 16 * NQB; i += 256) {
                const int64_t row = r0 + (i % RT);
                const int j = q0 + i / RT;
                if (row < r1 && j < p.nq) emit_approx<METRIC, true>(p, j, row, -1, false, 0.f);
            }
        }
        return;
    }
    const int nb = (int)(p.dpad / HI_K);  // == NST (template: registers)
    bf16x4x2 qf[NQB][NST];
#pragma unroll
    for (int jb = 0; jb < NQB; ++jb) {
        int j = q0 + 16 * jb + l16;
        if (j >= p.nq) j = 0;
        const int64_t u = (int64_t)variant_of(p, j, ord) * p.q_vpad + j;
        const unsigned char *qs = reinterpret_cast<const unsigned char *>(p.q_hi) + (u >> 4) * nb * 1024 +
                                  plane_vec_off((uint32_t)(u & 15)) + c * 16;
#pragma unroll
        for (int s = 0; s < NST; ++s) qf[jb][s] = *reinterpret_cast<const bf16x4x2 *>(qs + plane_step_off(s));
    }
    auto rowsrc = [&](int rb) {
        const int64_t gp = r0 + 16 * rb + l16;
        int64_t u = gp < r1 ? row_at(p, gp) : -1;
        if (u < 0) u = row_at(p, r0);  // padding: any real row, results discarded
        return reinterpret_cast<const unsigned char *>(p.rows_hi) + (u >> 4) * nb * 1024 +
               plane_vec_off((uint32_t)(u & 15)) + c * 16;
    };
    bf16x4x2 a[2][NST];
    auto load = [&](int buf, int rb) {
        const unsigned char *src = rowsrc(rb);
#pragma unroll
        for (int s = 0; s < NST; ++s) {
            const bf16x4x2 *ps = reinterpret_cast<const bf16x4x2 *>(src + plane_step_off(s));
            if constexpr (NT) {
                // streaming rows (read once per search): non-temporal loads
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                a[buf][s] = __builtin_bit_cast(bf16x4x2, __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(ps)));
            } else {
                a[buf][s] = *ps;
            }
        }
    };
    load(0, w);
#pragma unroll
    for (int i = 0; i < NBLK; ++i) {
        const int rb = w + 4 * i;
        if (i + 1 < NBLK) load((i + 1) & 1, rb + 4);
        f32x4 acc[NQB];
#pragma unroll
        for (int jb = 0; jb < NQB; ++jb) acc[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NST; ++s)
#pragma unroll
            for (int jb = 0; jb < NQB; ++jb)
                acc[jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[i & 1][s]),
                                                                 __builtin_bit_cast(bf16x8, qf[jb][s]), acc[jb],
                                                                 0, 0, 0);
        // C: lane (l16, c) holds rows 4c .. 4c+3 of the block for query l16
#pragma unroll
        for (int jb = 0; jb < NQB; ++jb) {
            const int j = q0 + 16 * jb + l16;
            if (j >= p.nq) continue;
            const int64_t rbase = r0 + 16 * rb + 4 * c;
            emit_vals<METRIC, PROBE, 4>(
                p, j, r1, [&](int r) { return rbase + r; }, [&](int r) { return acc[jb][r]; });
        }
    }
}

template <int METRIC, bool PROBE, int NQB>
static void launch_hi_reg(ScanParams p, hipStream_t s) {
    p.num_qblocks = (p.nq + 16 * NQB - 1) / (16 * NQB);
    const int64_t grid = p.tiles * p.num_qblocks;
    if (grid < 1) return;
    // rows streamed with non-temporal loads: 10M x 768 cosine main scan
    // 2.55 -> 2.28 ms at nq 1 (6.0 -> 6.7 TB/s), 2.80 -> 2.55 ms at nq 16,
    // bit-identical (profiles/r02/smallnq/nt_ab.jsonl).  A/B switch
    // (tools/ab_split.py): MQVS_HI_NT=0 = plain loads
    const char *nte = tune_env("MQVS_HI_NT");
    const bool nt = !(nte && nte[0] == '0');
    switch (p.dpad / HI_K) {
#define MQVS_HI_REG(N_)                                                                                        \
    case N_:                                                                                                   \
        if (p.tile_rows == kBfRowsSmall)                                                                       \
            hipLaunchKernelGGL((k_scan_hi_reg<METRIC, PROBE, NQB, N_, true, 1>), dim3((unsigned)grid), dim3(256), \
                               0, s, p);                                                                       \
        else if (nt)                                                                                           \
            hipLaunchKernelGGL((k_scan_hi_reg<METRIC, PROBE, NQB, N_, true>), dim3((unsigned)grid), dim3(256), 0, s, \
                               p);                                                                             \
        else                                                                                                   \
            hipLaunchKernelGGL((k_scan_hi_reg<METRIC, PROBE, NQB, N_>), dim3((unsigned)grid), dim3(256), 0, s, p); \
        return;
        MQVS_HI_REG(2) MQVS_HI_REG(4) MQVS_HI_REG(6) MQVS_HI_REG(8) MQVS_HI_REG(10) MQVS_HI_REG(12)
        MQVS_HI_REG(14) MQVS_HI_REG(16) MQVS_HI_REG(18) MQVS_HI_REG(20) MQVS_HI_REG(22) MQVS_HI_REG(24)
#undef MQVS_HI_REG
        default: break;
    }
    fail(MQVS_ERR_DEVICE, "k_scan_hi_reg: no build for dpad " + std::to_string(p.dpad));
}

// dpad (d rounded to 64) of the register kernel's builds
constexpr int kHiRegMaxDpad = 24 * HI_K;

// A scan of nq queries that launch_scan_hi runs with k_scan_hi_reg<NQB = 1>,
// which also takes kBfRowsSmall-row tiles (PROBE scans always reach it; main
// scans when no tuned or batch kernel takes them first)
bool scan_hi_small_tiles_ok(int nq, int64_t dpad) {
    const char *reg = tune_env("MQVS_HI_REG");
    const bool use_reg = !(reg && reg[0] == '0');
    return use_reg && tune_int("MQVS_HI_SMALL_TILES", 1) == 1 && nq <= 16 && dpad <= kHiRegMaxDpad &&
           dpad % (2 * HI_K) == 0 && dpad >= 2 * HI_K;
}

template <int METRIC, bool PROBE, int WQ, int QB, int NBUF, int PP = 0, int DIAG = 0>
static void launch_hi_shape(ScanParams p, hipStream_t s) {
    constexpr int QT = 32 * QB * WQ;
    p.num_qblocks = (p.nq + QT - 1) / QT;
    const int64_t L = p.tiles * p.num_qblocks;
    if (L < 1) return;
    const int64_t grid = (L + 7) / 8 * 8;
    hipLaunchKernelGGL((k_scan_hi<METRIC, PROBE, WQ, QB, NBUF, PP, DIAG>), dim3((unsigned)grid), dim3(256 * WQ), 0, s,
                       p);
}

// Tuning override (tools/ab_split.py --tunes): MQVS_HI_TUNE="WQ,QB,NBUF[,PP[,DIAG]]"
template <int METRIC, bool PROBE>
static bool launch_hi_tuned(const ScanParams &p, hipStream_t s) {
    const char *e = tune_env("MQVS_HI_TUNE");
    int wq, qb, nbuf, pp = 0, diag = 0;
    if (!e || !*e || std::sscanf(e, "%d,%d,%d,%d,%d", &wq, &qb, &nbuf, &pp, &diag) < 3) return false;
    switch ((((wq * 10 + qb) * 10 + nbuf) * 100 + pp) * 100 + diag) {
#define MQVS_HI_CASE(WQ_, QB_, NB_, PP_, DG_)                                         \
    case (((WQ_ * 10 + QB_) * 10 + NB_) * 100 + PP_) * 100 + DG_:                     \
        launch_hi_shape<METRIC, PROBE, WQ_, QB_, NB_, PP_, DG_>(p, s);                \
        return true;
        MQVS_HI_CASE(2, 4, 3, 0, 0) MQVS_HI_CASE(2, 4, 4, 0, 0)
        MQVS_HI_CASE(2, 4, 4, 0, 2) MQVS_HI_CASE(2, 4, 4, 0, 12)
        MQVS_HI_CASE(2, 4, 4, 1, 0) MQVS_HI_CASE(2, 4, 3, 1, 0) MQVS_HI_CASE(2, 4, 4, 1, 12)
        MQVS_HI_CASE(2, 2, 3, 0, 0) MQVS_HI_CASE(2, 2, 4, 1, 0) MQVS_HI_CASE(2, 2, 3, 1, 0)
        MQVS_HI_CASE(1, 2, 3, 0, 0)
#undef MQVS_HI_CASE
        default: return false;
    }
}

// set when a main-scan launch of this thread took the batch kernel
// (mqvs_search_stats.batch_kernel)
static thread_local int g_batch_kernel_used = 0;
int take_batch_kernel_flag() {
    const int v = g_batch_kernel_used;
    g_batch_kernel_used = 0;
    return v;
}

template <int METRIC, bool PROBE>
static void launch_hi_t(const ScanParams &p, hipStream_t s) {
    if constexpr (!PROBE)
        if (launch_hi_tuned<METRIC, PROBE>(p, s)) return;
    if constexpr (!PROBE) {
        // batches: the one-wave-per-SIMD persistent scan (kernels_p4.hip) for
        // contiguous rows and identity chunk ordinals (measurement builds:
        // MQVS_HI_PP=0 selects k_scan_hi instead).  (Round 2's 8-wave
        // ping-pong kernel k_scan_hi_pp, 16.7 ms at nq 1000 against 13.5, is
        // retired; profiles/r03/baseline_r02_kernels_ab.jsonl.)
        const int pp = tune_int("MQVS_HI_PP", 2);
        if (p.nq > 128 && pp == 2 && launch_scan_p4(p, METRIC, s)) {
            g_batch_kernel_used = 1;
            return;
        }
    }
    const char *reg = tune_env("MQVS_HI_REG");  // A/B switch (tools/ab_split.py): 0 = LDS kernel only
    const bool use_reg = !(reg && reg[0] == '0');
    if (use_reg && p.nq <= 32 && p.dpad <= kHiRegMaxDpad) {
        if (p.nq <= 16)
            launch_hi_reg<METRIC, PROBE, 1>(p, s);
        else
            launch_hi_reg<METRIC, PROBE, 2>(p, s);
        return;
    }
    if (p.nq <= 64)
        launch_hi_shape<METRIC, PROBE, 1, 2, 3>(p, s);
    else if (p.nq <= 128)
        launch_hi_shape<METRIC, PROBE, 2, 2, 3>(p, s);
    else
        launch_hi_shape<METRIC, PROBE, 2, 4, 4>(p, s);
}

void launch_scan_hi(const ScanParams &p, int metric, bool probe, hipStream_t s) {
    switch (metric) {
        case MQVS_METRIC_L2:
            probe ? launch_hi_t<MQVS_METRIC_L2, true>(p, s) : launch_hi_t<MQVS_METRIC_L2, false>(p, s);
            break;
        case MQVS_METRIC_IP:
            probe ? launch_hi_t<MQVS_METRIC_IP, true>(p, s) : launch_hi_t<MQVS_METRIC_IP, false>(p, s);
            break;
        case MQVS_METRIC_COSINE:
            probe ? launch_hi_t<MQVS_METRIC_COSINE, true>(p, s) : launch_hi_t<MQVS_METRIC_COSINE, false>(p, s);
            break;
        default:
            probe ? launch_hi_t<kMetricIpRaw, true>(p, s) : launch_hi_t<kMetricIpRaw, false>(p, s);
            break;
    }
}

}  // namespace mqvs
