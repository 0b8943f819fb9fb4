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
// Planes are row-blocked (16 vectors x 32 columns = 1 KiB contiguous):
// vector u, stage s at byte ((u >> 4) nst + s) 1024 + (u & 15) 64.
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
__global__ __launch_bounds__(256) void k_to_hi(const float *src, int64_t rows, int d, int64_t sstride, int64_t dpad,
                                               int64_t vgroup, int64_t vpad, uint16_t *hi, float *rec,
                                               float *maxrec) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= rows) return;  // whole wave
    const float *x = src + v * sstride;
    const int nb = (int)(dpad / HI_K);
    const int64_t u = (v % vgroup) * vpad + v / vgroup;
    uint16_t *hu = hi + (u >> 4) * nb * 512 + (u & 15) * 32;
    double nx = 0, nh = 0, nr = 0;
    for (int64_t i = lane; i < dpad; i += 64) {
        const float xv = i < d ? x[i] : 0.f;
        const uint16_t hb = f32_to_bf16_rn(xv);
        const float hv = __builtin_bit_cast(float, (uint32_t)hb << 16);
        const float rv = xv - hv;  // exact
        hu[(i >> 5) * 512 + (i & 31)] = hb;
        nx += (double)xv * xv;
        nh += (double)hv * hv;
        nr += (double)rv * rv;
    }
    for (int off = 32; off > 0; off >>= 1) {
        nx += __shfl_xor(nx, off);
        nh += __shfl_xor(nh, off);
        nr += __shfl_xor(nr, off);
    }
    if (lane == 0) {
        float r[kMxRec] = {hi_sqrt_up(nh), hi_sqrt_up(nr), 0.f, 0.f, 0.f, 0.f, hi_sqrt_up(nx), 0.f};
#pragma unroll
        for (int t = 0; t < kMxRec; ++t) {
            if (rec) rec[v * kMxRec + t] = r[t];
            if (maxrec && (t < 2 || t == 6)) {
                // non-negative floats order as their bit patterns; NaN -> +inf
                const unsigned b = (r[t] == r[t]) ? __builtin_bit_cast(unsigned, r[t]) : 0x7F800000u;
                atomicMax(reinterpret_cast<unsigned *>(maxrec) + t, b);
            }
        }
    }
}

void launch_to_hi(const float *src, int64_t rows, int d, int64_t src_stride, int64_t dpad, int64_t vgroup,
                  int64_t vpad, uint16_t *hi, float *rec, float *maxrec, hipStream_t s) {
    if (rows <= 0) return;
    const int64_t blocks = (rows + 3) / 4;
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
        src[i] = reinterpret_cast<const unsigned char *>(plane) + ((u >> 4) * nb * 1024 + (u & 15) * 64 + c * 16);
    }
    static_assert(GY % NW == 0, "row pieces: whole rounds of the waves");
    constexpr int YPW = GY / NW;  // pieces i < YPW are row pieces, the rest query pieces
    auto issue = [&](int s) {
        unsigned char *dst = lds + (s % NBUF) * STAGE;
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            if ((DIAG & 8) && i < YPW) continue;
            if ((DIAG & 4) && i >= YPW) continue;
            __builtin_amdgcn_global_load_lds((const void *)(src[i] + (int64_t)s * 1024),
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

// ---------------------------------------------------------------------------
// Persistent ping-pong scan (batch APPEND, Cosine / IP, contiguous rows).
//
// Measured on k_scan_hi (10M rows, nq 1000, d 256 .. 1536): main-scan time
// = ~6 ms + ~5 ms per 256 dimensions, i.e. every workgroup pays ~10 us outside
// its K loop (a cold prologue that waits for its first stages, the epilogue,
// the launch), a third of the search at d = 768.  Here one workgroup per CU
// walks a sequence of (row tile, query block) items, and the LDS-DMA stage
// ring runs ACROSS items: the next item's first stages are in flight while
// the current item's last stages and epilogue run.  The two waves of each
// SIMD (query halves wq = 0 / 1) run one barrier apart (read phase of one
// against MFMA phase of the other, see k_scan_hi's PP notes).
//
// Epilogue without global memory: values over the query's threshold go to an
// LDS queue (ds atomics only), flushed to the candidate lists once at the end
// of the launch -- a global atomic's returned slot would make the wave wait
// for every LDS-DMA piece issued before it.  Thresholds and the cosine
// variant cycle of the workgroup's queries are loaded once (a workgroup keeps
// one query block).  A full queue falls back to the global append.
//
// Items: XCD x = blockIdx % 8 holds the tiles t = x (mod 8); its S slots split
// into S / nqb groups of nqb query blocks, group g taking tiles
// x + 8 (g + (S / nqb) i): the query blocks of a tile run together on one XCD
// and share its rows through that L2.
constexpr int kPpQueue = 1984;  // LDS candidate queue entries (16 B)

struct PpEntry {
    float raw;
    uint32_t row;
    int j;
    int pad;
};

// LDS queue append by inline asm: a compiler-visible LDS access here would
// get a wait for every LDS-DMA piece in flight (the waitcnt pass cannot tell
// that the queue and the stage ring do not overlap)
__device__ inline int lds_add_rtn(const void *addr, int v) {
    int r;
    const unsigned a = (unsigned)(size_t)(lds_void *)addr;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a), "v"(v) : "memory");
    return r;
}
__device__ inline void lds_store_b128(const void *addr, float x, uint32_t y, int z) {
    const unsigned a = (unsigned)(size_t)(lds_void *)addr;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {__builtin_bit_cast(unsigned, x), y, (unsigned)z, 0u};
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// DIAG (diagnostic builds, wrong results; MQVS_HI_PPDIAG): 1 = row pieces
// from the first 8 tiles only (L2-resident rows), 4 = query pieces not
// issued, 8 = row pieces not issued, 16 = a trivial epilogue (the MFMAs stay
// live: one compare of an accumulator sum per item), 32 = the threshold
// pre-check as OR-ed compares instead of a max tree (an A/B variant: exact),
// 64 = row pieces with the non-temporal policy (aux nt; an A/B variant: exact),
// 256 = SYNC: the query blocks of a row tile kept within kPpLag items of each
// other (an A/B variant: exact).  They run on different CUs of one XCD and
// share the tile through its L2 only while they stream it at about the same
// time; left alone they drift apart over the ~600 items of a launch and each
// re-reads the rows from beyond the L2 (PMC: 53 GB per search from the L2's
// misses against 15.2 GB of plane).  Every kPpSyncEvery items wave 0 reads its
// siblings' progress words (scalar loads: lgkmcnt, so no wait on the LDS-DMA
// ring) and sleeps while one is more than kPpLag items behind -- for at most
// kPpSpin rounds, so the result never depends on it and nothing can deadlock.
constexpr int kPpSyncEvery = 4, kPpLag = 1, kPpSpin = 64;
__device__ unsigned g_pp_prog[2048];  // per workgroup: epoch << 16 | items done

__device__ inline unsigned sload_glc(const unsigned *ptr) {
    unsigned v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(ptr) : "memory");
    return v;
}

template <int METRIC, int NBUF, int DIAG = 0>
__global__ __launch_bounds__(512) void k_scan_hi_pp(ScanParams p, int slots, unsigned epoch) {
    constexpr int WR = 4, WQ = 2, QB = 4, NW = 8;
    constexpr int QT = 32 * QB * WQ;  // 256
    constexpr int RT = kBfRows;       // 256
    constexpr int GY = RT / 16, GQ = QT / 16, G = GY + GQ;
    constexpr int GPW = G / NW;       // 4 pieces per wave and stage
    constexpr int YPW = GY / NW;      // 2 of them row pieces
    constexpr int STAGE = G * 1024;
    constexpr int D = NBUF - 2;       // stages in flight ahead of the one read
    static_assert(D >= 1 && GY % NW == 0, "shape");
    constexpr int NPW = GPW - ((DIAG & 8) ? YPW : 0) - ((DIAG & 4) ? GPW - YPW : 0);  // pieces per wave, stage
    // ONE __shared__ object: the stage ring, the candidate queue and its
    // counter (an LDS access to a second object after an LDS-DMA makes the
    // compiler wait for every DMA in flight, cdna_hip_programming.md)
    __shared__ __attribute__((aligned(16))) unsigned char lds[NBUF * STAGE + kPpQueue * 16 + 16];
    PpEntry *queue = reinterpret_cast<PpEntry *>(lds + NBUF * STAGE);
    int &qcount = *reinterpret_cast<int *>(lds + NBUF * STAGE + kPpQueue * 16);

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w % WR, wq = w / WR;
    const int grp = wq;  // waves w and w + 4 share a SIMD
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nqb = p.num_qblocks;
    const int ngroups = slots / nqb;
    if (slot >= ngroups * nqb) return;  // whole workgroup, before any barrier
    const int qb = slot % nqb, tg = slot / nqb;
    const int q0 = qb * QT;
    const int64_t tstride = 8 * (int64_t)ngroups;
    const int nb = (int)(p.dpad / HI_K);
    const int nst = nb;
    if (t == 0) qcount = 0;

    // per-lane constants: the two query rows of this wave's Q pieces (their
    // variant cycle), the four query columns of its accumulators (thresholds)
    int qj[2], qmu[2] = {0, 0}, qlam[2] = {1, 1};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int j = q0 + (w + i * NW) * 16 + (lane >> 2);
        if (j >= p.nq) j = 0;
        qj[i] = j;
        if (p.maxv > 1) {
            qmu[i] = p.qmu[j];
            qlam[i] = p.qlam[j];
        }
        asm volatile("" : "+v"(qmu[i]), "+v"(qlam[i]));  // (the loads' waits land here, before the ring)
    }
    const int h = lane >> 5, l32 = lane & 31;
    const int ra0 = wr * 64 + l32;
    const int rq0 = wq * 32 * QB + l32;
    float thr[QB];
#pragma unroll
    for (int jb = 0; jb < QB; ++jb) {
        const int j = q0 + rq0 + jb * 32;
        thr[jb] = j < p.nq ? p.thr[j] : __builtin_inff();  // (never taken)
        asm volatile("" : "+v"(thr[jb]));
    }

    // item cursor helpers (items are tiles of this slot's sequence)
    // 32-bit tile arithmetic when the part allows it: tile_range's 64-bit
    // divisions are software sequences of ~120 instructions, three per call,
    // and an item boundary runs two of these calls (the issue cursor in a read
    // phase, the compute cursor after the epilogue), exposed to the partner
    // wave at the barrier.  (DIAG & 1024: tile_range, an A/B variant.)
    const bool t32 = (DIAG & 1024) == 0 && p.row_end + p.chunk_rows + p.tile_rows <= 0x7FFFFFFF &&
                     p.tiles <= 0x7FFFFFFF && p.row_begin >= 0;
    const uint32_t c0_32 = (t32 && p.tiles_per_chunk > 0) ? (uint32_t)p.row_begin / (uint32_t)p.chunk_rows : 0u;
    auto item_range = [&](int64_t ti, int64_t &r0, int64_t &r1, int &ord) -> bool {
        int64_t chunk;
        if (t32) {
            const uint32_t tt = (uint32_t)ti, tr = (uint32_t)p.tile_rows;
            if (p.tiles_per_chunk > 0) {
                const uint32_t tpc = (uint32_t)p.tiles_per_chunk, cr = (uint32_t)p.chunk_rows;
                const uint32_t qd = tt / tpc, rem = tt - qd * tpc;
                const uint32_t c = c0_32 + qd, cs = c * cr;
                const uint32_t a = cs + rem * tr;
                const uint32_t e = a + tr < cs + cr ? a + tr : cs + cr;
                r0 = a;
                r1 = e;
                chunk = c;
            } else {
                const uint32_t a = (uint32_t)p.row_begin + tt * tr;
                r0 = a;
                r1 = (int64_t)a + tr;
                chunk = p.chunk_rows > 0 ? a / (uint32_t)p.chunk_rows : 0;
            }
            if (r1 > p.row_end) r1 = p.row_end;
        } else {
            tile_range(p, ti, r0, r1, chunk);
        }
        ord = (int)chunk + p.ord_base;  // (no chunk_ord table on this path)
        return r0 < r1;
    };
    auto next_item = [&](int64_t ti, int64_t &r0, int64_t &r1, int &ord) -> int64_t {
        for (; ti < p.tiles; ti += tstride)
            if (item_range(ti, r0, r1, ord)) return ti;
        return -1;
    };

    // issue cursor: item ti_i (rows [ir0, ir1), ordinal iord), next stage si
    int64_t ir0 = 0, ir1 = 0;
    int iord = 0;
    int64_t ti_i = next_item(xcd + 8 * (int64_t)tg, ir0, ir1, iord);
    if (ti_i < 0) return;  // no work (uniform)
    const unsigned char *src[GPW];
    auto set_src = [&]() {
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            const int g = w + i * NW;
            const int r = (i < YPW ? g : g - GY) * 16 + (lane >> 2);
            const int c = hswz(r, lane & 3);
            int64_t u;
            const uint16_t *plane;
            if (i < YPW) {
                u = ir0 + r < ir1 ? ir0 + r : ir0;  // padding rows: any real row, discarded
                if (DIAG & 1) u = ((ir0 / RT) & 7) * RT + r;
                plane = p.rows_hi;
            } else {
                const int k = i - YPW;
                const int var = p.maxv <= 1 ? 0 : (iord < qmu[k] ? iord : qmu[k] + (iord - qmu[k]) % qlam[k]);
                u = (int64_t)var * p.q_vpad + qj[k];
                plane = p.q_hi;
            }
            src[i] = reinterpret_cast<const unsigned char *>(plane) + ((u >> 4) * nb * 1024 + (u & 15) * 64 + c * 16);
        }
    };
    set_src();
    int si = 0;
    int64_t issued = 0;  // stages issued so far (global stage counter)
    auto issue_next = [&]() {
        if (ti_i < 0) return;
        unsigned char *dst = lds + (int)(issued % NBUF) * STAGE;
#pragma unroll
        for (int i = 0; i < GPW; ++i) {
            if ((DIAG & 8) && i < YPW) continue;
            if ((DIAG & 4) && i >= YPW) continue;
            if ((DIAG & 64) && i < YPW)
                __builtin_amdgcn_global_load_lds((const void *)(src[i] + (int64_t)si * 1024),
                                                 (lds_void *)(dst + (w + i * NW) * 1024), 16, 0, 2);
            else
                __builtin_amdgcn_global_load_lds((const void *)(src[i] + (int64_t)si * 1024),
                                                 (lds_void *)(dst + (w + i * NW) * 1024), 16, 0, 0);
        }
        ++issued;
        if (++si == nst) {
            si = 0;
            ti_i = next_item(ti_i + tstride, ir0, ir1, iord);
            if (ti_i >= 0) set_src();
        }
    };

    // compute cursor: item rows [cr0, cr1), stage sc, global stage gc
    int64_t cr0 = ir0, cr1 = ir1;
    int64_t ti_c = ti_i;
    int sc = 0;
    int64_t gc = 0;
    unsigned done = 0;  // items finished (SYNC)

    constexpr int OFF_Q = GY * 1024;
    auto frag = [&](const unsigned char *st, int r, int c) {
        return *reinterpret_cast<const bf16x8 *>(st + r * 64 + hswz(r, c) * 16);
    };
    f32x16 acc[2][QB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jb = 0; jb < QB; ++jb) acc[i][jb] = f32x16{0};

    // prologue: D stages in flight, the first landed for everyone
    for (int s = 0; s < D; ++s) issue_next();
    {
        const int64_t pend = issued - 1 < D - 1 ? issued - 1 : D - 1;
        wait_vm<NPW, D>((int)pend);
    }
    __syncthreads();  // (qcount = 0 visible; no DMA wait hidden in it: all waited above)
    if (grp == 1) raw_barrier();
    while (true) {
        // read phase (the partner wave computes meanwhile): the first half
        // (16 columns) of the stage's fragments; the second half is read
        // inside the MFMA phase, after the first half's MFMAs have issued
        // (keeps the fragments at 24 VGPRs: acc takes 128)
        const unsigned char *st = lds + (int)(gc % NBUF) * STAGE;
        bf16x8 ah[2], bh[QB];
#pragma unroll
        for (int i = 0; i < 2; ++i) ah[i] = frag(st, ra0 + 32 * i, h);
#pragma unroll
        for (int jb = 0; jb < QB; ++jb) bh[jb] = frag(st + OFF_Q, rq0 + 32 * jb, h);
        __builtin_amdgcn_sched_barrier(0);
        issue_next();
        const bool has_next = gc + 1 < issued;
        // pieces issued after stage gc+1 may stay in flight
        const int pend = has_next ? (int)(issued - gc - 2) : 0;
        if (grp == 1 && has_next) wait_vm<NPW, D>(pend);
        raw_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jb = 0; jb < QB; ++jb)
                acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[jb], acc[i][jb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i) ah[i] = frag(st, ra0 + 32 * i, 2 + h);
#pragma unroll
        for (int jb = 0; jb < QB; ++jb) bh[jb] = frag(st + OFF_Q, rq0 + 32 * jb, 2 + h);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jb = 0; jb < QB; ++jb)
                acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[jb], acc[i][jb], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (++sc == nst) {
            // item epilogue: values over the threshold -> LDS queue.  A
            // candidate is rare (a few per item and query block), so each
            // block of 16 values of a query column is first tested with ONE
            // compare of their max (v_max3 chains); only a block over the
            // threshold walks its values (per-value branches everywhere cost
            // 4 ms at 10M x 768, nq 1000, as much as the LDS-DMA stream; a
            // ballot-compacted walk measured slower than this one)
            if (!(DIAG & 16)) {
                const int crn = (int)(cr1 - cr0);  // rows of the item (<= RT)
#pragma unroll
                for (int jb = 0; jb < QB; ++jb)
#pragma unroll
                    for (int rb = 0; rb < 2; ++rb) {
                        // any of the 16 over the threshold (DIAG & 32: 16
                        // compares OR-ed as lane masks; else an fmaxf tree)
                        bool any = false;
                        if constexpr ((DIAG & 32) != 0) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) any |= acc[rb][jb][r] >= thr[jb];
                        } else {
                            float mx = acc[rb][jb][0];
#pragma unroll
                            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[rb][jb][r]);
                            any = mx >= thr[jb];
                        }
                        if (any) {
                            // (row offsets in the tile as 32-bit values, the
                            // 64-bit row formed only under the branch behind
                            // an opaque copy: otherwise the compiler shares
                            // the rows' addresses in the candidate bitmaps
                            // across the jb blocks, hoisting 32 of them out
                            // of the walk and spilling them at every item)
                            const int j = q0 + rq0 + jb * 32;
                            const int rlb = wr * 64 + rb * 32 + 4 * h;
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const float raw = acc[rb][jb][r];
                                const int rl = rlb + (r & 3) + 8 * (r >> 2);
                                if (raw >= thr[jb] && rl < crn && j < p.nq) {
                                    int rlo = rl;
                                    asm volatile("" : "+v"(rlo));
                                    const int64_t row = cr0 + rlo;
                                    const int pos = lds_add_rtn(&qcount, 1);
                                    if (pos < kPpQueue)
                                        lds_store_b128(queue + pos, raw, (uint32_t)row, j);
                                    else
                                        emit_approx<METRIC, false>(p, j, row, row, row_valid(p, row), raw);
                                }
                            }
                        }
                    }
            }
            if (DIAG & 16) {
                float sum = 0.f;
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                    for (int jb = 0; jb < QB; ++jb)
#pragma unroll
                        for (int r = 0; r < 16; ++r) sum += acc[rb][jb][r];
                if (sum == -1.2345e-30f) lds_add_rtn(&qcount, 1);
            }
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int jb = 0; jb < QB; ++jb) acc[rb][jb] = f32x16{0};
            sc = 0;
            int cord;
            ti_c = next_item(ti_c + tstride, cr0, cr1, cord);
            if constexpr ((DIAG & 256) != 0) {
                ++done;
                if (w == 0) {
                    if (lane == 0)
                        __hip_atomic_store(&g_pp_prog[blockIdx.x], (epoch << 16) | done, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    if (done % kPpSyncEvery == 0 && nqb > 1) {
                        for (int it = 0; it < kPpSpin; ++it) {
                            bool behind = false;
                            for (int b = 0; b < nqb; ++b) {
                                if (b == qb) continue;
                                const unsigned v = sload_glc(&g_pp_prog[xcd + 8 * (tg * nqb + b)]);
                                if ((v >> 16) != epoch || (v & 0xFFFFu) + kPpLag < done) behind = true;
                            }
                            if (!behind) break;
                            __builtin_amdgcn_s_sleep(8);
                        }
                    }
                }
            }
        }
        ++gc;
        if (grp == 0 && has_next) wait_vm<NPW, D>(pend);
        raw_barrier();
        if (!has_next) break;
    }
    if (grp == 0) raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (asm queue stores retired)
    __syncthreads();
    const int nqueue = qcount < kPpQueue ? qcount : kPpQueue;
    for (int e = t; e < nqueue; e += 512) {
        const PpEntry en = queue[e];
        emit_approx<METRIC, false>(p, en.j, en.row, en.row, row_valid(p, en.row), en.raw);
    }
}

template <int METRIC>
static bool launch_hi_pp(ScanParams p, hipStream_t s) {
    constexpr int QT = 256;
    p.num_qblocks = (p.nq + QT - 1) / QT;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        MQVS_HIP(hipGetDevice(&dev));
        MQVS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int per_xcd = cus / 8;
    if (p.num_qblocks > per_xcd || p.tiles < 1) return false;
    const int slots = per_xcd / p.num_qblocks * p.num_qblocks;
    const char *dg = tune_env("MQVS_HI_PPDIAG");
    const int diag = dg ? std::atoi(dg) : 0;
    static std::atomic<unsigned> launches{0};
    const unsigned epoch = (launches.fetch_add(1, std::memory_order_relaxed) + 1) & 0xFFFFu;
    // (the decomposition builds 17 / 20 / 24 / 28 of profiles/r02/pp_decomposition.jsonl
    // are template arguments too: add their case to run them again)
#define MQVS_PP(DG_)                                                                                             \
    hipLaunchKernelGGL((k_scan_hi_pp<METRIC, 4, DG_>), dim3((unsigned)(8 * per_xcd)), dim3(512), 0, s, p, slots, \
                       epoch)
    if constexpr (kDebugTuning) {  // (diagnostic variants: measurement builds only)
        switch (diag) {
            case 16: MQVS_PP(16); break;
            case 32: MQVS_PP(32); break;
            case 64: MQVS_PP(64); break;
            case 256: MQVS_PP(256); break;
            case 1024: MQVS_PP(1024); break;
            default: MQVS_PP(0); break;
        }
    } else {
        MQVS_PP(0);
    }
#undef MQVS_PP
    return true;
}

// Small batches (nq <= 32): HBM-bound, so no LDS staging at all.  The 256-row
// tile is 16 row blocks of 16 rows; wave w takes blocks w, w+4, w+8, w+12.  A
// row block's 32-column stage is ONE contiguous KiB of the row-blocked plane
// and exactly the A operand of v_mfma_f32_16x16x32_bf16 (lane l: row l & 15,
// columns 8 (l >> 4) .. +8), so each stage is one global_load_dwordx4 straight
// into the fragment; a block's whole row (nst loads, 24 KiB at d = 768) is in
// flight while the previous block feeds the MFMAs.  The query tile (NQB blocks
// of 16 queries, every stage's B fragment: 4 VGPRs each) stays in registers.
template <int METRIC, bool PROBE, int NQB, int NST, bool NT = false>
__global__ __launch_bounds__(256) void k_scan_hi_reg(ScanParams p) {
    constexpr int RT = kBfRows;
    const int64_t ti = blockIdx.x / p.num_qblocks;
    const int qb = (int)(blockIdx.x % p.num_qblocks);
    if (ti >= p.tiles) return;
    int64_t r0, r1, chunk;
    tile_range(p, ti, r0, r1, chunk);
    if (r0 >= r1) return;
    const int ord = chunk_ordinal(p, chunk);
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
                                  (u & 15) * 64 + c * 16;
#pragma unroll
        for (int s = 0; s < NST; ++s) qf[jb][s] = *reinterpret_cast<const bf16x4x2 *>(qs + (int64_t)s * 1024);
    }
    auto rowsrc = [&](int rb) {
        const int64_t gp = r0 + 16 * rb + l16;
        int64_t u = gp < r1 ? row_at(p, gp) : -1;
        if (u < 0) u = row_at(p, r0);  // padding: any real row, results discarded
        return reinterpret_cast<const unsigned char *>(p.rows_hi) + (u >> 4) * nb * 1024 + (u & 15) * 64 + c * 16;
    };
    bf16x4x2 a[2][NST];
    auto load = [&](int buf, int rb) {
        const unsigned char *src = rowsrc(rb);
#pragma unroll
        for (int s = 0; s < NST; ++s) {
            const bf16x4x2 *ps = reinterpret_cast<const bf16x4x2 *>(src + (int64_t)s * 1024);
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
    for (int i = 0; i < 4; ++i) {
        const int rb = w + 4 * i;
        if (i + 1 < 4) load((i + 1) & 1, rb + 4);
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
        if (nt)                                                                                                \
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
        // contiguous rows and identity chunk ordinals; measurement builds can
        // select the 8-wave ping-pong kernel instead (MQVS_HI_PP=1) or neither
        // (MQVS_HI_PP=0)
        const int pp = tune_int("MQVS_HI_PP", 2);
        if (p.nq > 128 && pp == 2 && launch_scan_p4(p, METRIC, s)) {
            g_batch_kernel_used = 1;
            return;
        }
        if constexpr (METRIC != MQVS_METRIC_L2)
            if (p.nq > 128 && pp == 1 && !p.row_list && !p.chunk_ord && launch_hi_pp<METRIC>(p, s)) return;
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
