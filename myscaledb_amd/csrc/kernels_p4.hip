// kernels_p4.hip -- the batch pre-filter scan (split 2, nq > 128) at ONE wave
// per SIMD.  It replaces faiss's BLAS branch for large batches
// (BruteForceSearch.h:80-87, exhaustive_L2sqr_blas / exhaustive_inner_product_blas)
// as the first stage of kernels_hi.hip's bf16-hi pre-filter: the approximate
// values it appends are re-ranked exactly afterwards (kernels_rerank.hip).
//
// Shape.  A persistent workgroup of 4 waves per CU walks work items of 256
// rows x 256 queries.  Wave (wr, wq) owns 128 rows x 128 queries: 4 x 4
// accumulators of v_mfma_f32_32x32x16_bf16 = 256 AGPRs, the whole accumulator
// half of the register file.  Per 32-column stage a wave reads 16 fragments
// (ds_read_b128) for 32 MFMAs: half the LDS fragment traffic per MFMA of
// round 2's 8-wave 64 x 128 shape (k_scan_hi_pp: 12 reads per 16), and
// the stage's 32 KiB LDS-DMA image (256 rows + 256 queries x 64 B) is the same.
//
// Pipeline (per stage s, global stage counter over the whole launch): the
// k-step-0 fragments of stage s are in registers at the top.  Between its 16
// k-step-0 MFMAs the wave reads its k-step-1 fragments of stage s and issues
// its 8 LDS-DMA pieces of stage s + D; it then waits (counted vmcnt) for its
// own pieces of stage s + 1 and for its fragment reads (lgkmcnt(0)), and joins
// ONE raw s_barrier: stage s + 1 is complete for every wave, and every wave is
// done reading stage s, whose buffer the next phase re-fills (D = NBUF - 1).
// Between the 16 k-step-1 MFMAs it reads the k-step-0 fragments of stage
// s + 1.  The stage ring runs across item boundaries, so the next item's
// first stages are in flight during the current item's last stages and
// epilogue.
//
// First stage of an item: the k-step-0 MFMAs take C = 0 (an inline constant:
// no accumulator zeroing) -- or, for L2, C = -|y|^2 / 2 of the block's rows,
// read from a 1 KiB LDS copy of the item's row norms (one 4-B-per-lane
// LDS-DMA piece per wave).  The accumulator then holds ip - |y|^2 / 2, and
// the L2 append test qn - 2 acc <= t is a per-query threshold on acc, as for
// IP and cosine.  The row norm enters before the products instead of after,
// so the accumulation's error bound grows by |y|^2 / 2 per term
// (k_query_bound adds it for L2).
//
// Epilogue: per query column, the maximum of the wave's 64 values (v_max3
// chain) against the threshold; only a column over it walks its values.  A
// candidate goes to this wave's queue in global memory at a slot given by a
// ballot prefix count (no atomics, no LDS), flushed to the per-query lists at
// the end of the launch.  A global atomic with return inside the loop would
// make the wave wait for every LDS-DMA piece in flight; a full queue falls back
// to exactly that (correct, slower).
//
// PROBE (p.p4_gmax set; searches without a PREWHERE filter or deletes, whose
// group maxima could come from rows that do not count): the same scan over
// the probe rows, with no threshold tests: per query and 128-row half tile (one wave's rows of an item) the
// best approximate value is written to p4_gmax[q][2 t + wr] as a raw metric
// value (L2: fl(qn - 2 acc)).  The k-th best of those maxima is the k-th best
// of k actual rows, so k_probe_select_wide turns it into an append threshold
// with the same guarantee as the dense probe matrix it replaces (at nq 1000:
// 2.8 MB written instead of 360 MB); the main scan then covers the probe rows
// too.
//
// Items: XCD x = blockIdx % 8 takes tiles t = x (mod 8); its
// workgroups form groups of nqb query blocks that stream the same row tiles,
// so a tile's rows are shared through that XCD's L2.
#include <atomic>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "mqvs_internal.h"
#include "scan_emit.h"
#include "tuning.h"

namespace mqvs {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
}  // namespace

constexpr int kP4Tile = 256;       // rows and queries per work item
constexpr int kP4Stage = 32768;    // one stage: (256 rows + 256 queries) x 64 B
constexpr int kP4QOff = 16384;     // query image within a stage
constexpr int kP4HiK = 32;         // columns per stage

// LDS image swizzle: image row r keeps its 16-B chunk c at slot
// c ^ p4_g((r >> 2) & 3).  Conflict-free for the ds_read_b128 lane groups of
// both the 32x32x16 fragment (lane -> row l & 31, chunk 2 kk + (l >> 5)) and
// the 16x16x32 one (row l & 15, chunk l >> 4): in every 16-lane group the
// (row & 3, slot) pairs are distinct.
__device__ __host__ inline int p4_g(int x) { return (4 - x) & 3; }

// s_waitcnt vmcnt(P n), n in [0, 3] at run time (P: pieces a wave issues per
// stage; a stage that also carries a norm piece makes the wait stricter by
// one operation, never looser)
// (X: pieces of a half-issued stage on top, when any is wanted)
template <int P, int X = 0>
__device__ inline void p4_wait_vm(int n, bool any = true) {
    __builtin_amdgcn_sched_barrier(0);
    if (P > 0 && any && n >= 3)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * P + X) : "memory");
    else if (P > 0 && any && n == 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P + X) : "memory");
    else if (P > 0 && any && n == 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P + X) : "memory");
    else if (P > 0 && any && X > 0)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): compile-time
// indices without relying on the unroller (the epilogue is too large for it)
template <class F, int... I>
__device__ inline void p4_for_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ inline void p4_for(F &&f) {
    p4_for_impl(f, std::make_integer_sequence<int, N>{});
}

// v_max3_f32 (IEEE maxNum: a quiet NaN never wins, so a NaN value never
// passes a threshold, as in emit_approx)
__device__ inline float p4_max3(float a, float b, float c) {
    float r;
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// an accumulator value (in an AGPR) copied to a VGPR, in program order
__device__ inline float p4_aread(float a) {
    float r;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(a));
    return r;
}
// four of them in one ordered statement (the compiler pads every inline asm
// with a hazard s_nop; one per four reads)
__device__ inline f32x4 p4_aread4(float a, float b, float c, float d) {
    float x, y, z, w;
    asm volatile(
        "v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\t"
        "v_accvgpr_read_b32 %2, %6\n\tv_accvgpr_read_b32 %3, %7"
        : "=v"(x), "=v"(y), "=v"(z), "=v"(w)
        : "a"(a), "a"(b), "a"(c), "a"(d));
    return f32x4{x, y, z, w};
}

__device__ inline void p4_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// PL: where a stage's 8 LDS-DMA pieces go: 0 = k-step-0 phase slots 8..15;
// 1 = slots 8..11 of both phases; 2 = slots 8, 10, 12, 14 of both phases
// (the ds_read-free gaps)
// DIAG (measurement builds only; wrong results): 4 = query pieces not issued,
// 8 = row pieces not issued, 16 = no threshold tests (the accumulators are
// kept live by one read per block), 32 = threshold tests without walks,
// 128 = no stage barrier, 256 = no fragment-read wait before it, 512 = cosine
// query variant 0 for every chunk
template <int METRIC, int NBUF, int DIAG = 0, int PL = 0, bool PROBE = false>
__global__ __launch_bounds__(256, 1) void k_scan_p4(ScanParams p, int slots, u32x4 *queue, int qcap, int tmap) {
    constexpr bool L2 = METRIC == MQVS_METRIC_L2;
    // cache policy of the row / query pieces (PL bits 4 / 8: nt)
    constexpr int RPOL = (PL & 4) ? 2 : 0, QPOL = (PL & 8) ? 2 : 0;
    // stages in flight ahead of the one consumed: a buffer is re-filled one
    // barrier after its last fragment reads retired (lgkmcnt(0) before it)
    constexpr int D = NBUF - 1;
    static_assert(D >= 1 && D <= 4, "ring depth");
    constexpr int NORM = L2 ? 2048 : 0;  // two item-parity copies of 256 row norms
    constexpr int WSCR = 4 * 64 * 16 * 4;  // epilogue walk scratch: 16 values per lane and wave
    constexpr int NPW = 8 - ((DIAG & 8) ? 4 : 0) - ((DIAG & 4) ? 4 : 0);  // pieces per wave and stage
    // ONE __shared__ object (an LDS access to a second object after an
    // LDS-DMA makes the compiler wait for every DMA in flight)
    __shared__ __attribute__((aligned(16))) unsigned char lds[NBUF * kP4Stage + NORM + WSCR];
    unsigned char *norm_lds = lds + NBUF * kP4Stage;

    // (the wave index through readfirstlane: known wave-uniform, so branches
    // on it are scalar)
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = w & 1, wq = w >> 1;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nqb = p.num_qblocks;
    const int ngroups = slots / nqb;
    if (slot >= ngroups * nqb) return;  // whole workgroup, before any barrier
    const int qb = slot % nqb, tg = slot / nqb;
    const int q0 = qb * kP4Tile;
    const int tstride = 8 * ngroups;
    const int nst = (int)(p.dpad / kP4HiK);
    const int l32 = lane & 31, h = lane >> 5;
    float *wscr = reinterpret_cast<float *>(lds + NBUF * kP4Stage + NORM) + w * 1024;

    // per-lane query constants: the four query rows of this wave's query
    // pieces (variant cycles), the four query columns of its accumulators
    // Cosine variants: with the ordinal planes (p.q_ord, built when every
    // query's chain fits them) a chunk's queries are ONE contiguous plane,
    // chosen per item; otherwise each lane picks its query's variant.
    int om0 = 0, oln = 1;
    bool ordm = false;
    if (p.q_ord_desc) {
        om0 = __builtin_amdgcn_readfirstlane(p.q_ord_desc[0]);
        oln = __builtin_amdgcn_readfirstlane(p.q_ord_desc[1]);
        ordm = __builtin_amdgcn_readfirstlane(p.q_ord_desc[2]) != 0;
    }
    const bool pervar = p.maxv > 1 && !ordm;
    int qmu[4], qlam[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int j = q0 + (w + 4 * i) * 16 + (lane >> 2);
        if (j >= p.nq) j = 0;
        qmu[i] = 0;
        qlam[i] = 1;
        if (pervar) {
            qmu[i] = p.qmu[j];
            qlam[i] = p.qlam[j];
        }
    }
    // thresholds on the accumulator: IP / cosine acc >= t; L2 acc = ip - yn/2
    // and the append test fl(qn - 2 acc) <= t, pre-checked as acc >= (qn - t)/2
    // less a rounding slack (the walk applies the exact test)
    // (slack: if fl(qn - 2 acc) <= t then acc >= (qn - t) / 2 - t u / (2 - 2u);
    // the computed half may be u |qn - t| / 2 high; 8 u (|qn| + |t|) covers both)
    float thr[4], tl[4], qnl[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        const int j = q0 + wq * 128 + jb * 32 + l32;
        const float tj = j < p.nq && !PROBE ? p.thr[j] : 0.f;
        tl[jb] = tj;
        qnl[jb] = 0.f;
        if constexpr (L2) {
            const float qn = j < p.nq ? p.qnorms[j] : 0.f;
            qnl[jb] = qn;
            const float half = (qn - tj) * 0.5f;
            thr[jb] = half - 4.8e-7f * (fabsf(qn) + fabsf(tj)) - 1e-30f;
        } else {
            thr[jb] = tj;
        }
        if (j >= p.nq) thr[jb] = __builtin_inff();  // padding queries never pass
        asm volatile("" : "+v"(thr[jb]), "+v"(tl[jb]), "+v"(qnl[jb]));  // (the loads' waits land here)
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(qmu[i]), "+v"(qlam[i]));

    // item cursors (items are tiles of this slot's sequence), in 32-bit
    // arithmetic (the launcher checks the part allows it); every value is
    // wave-uniform and kept in scalar registers
    const uint32_t tr = (uint32_t)p.tile_rows, cr = (uint32_t)p.chunk_rows;
    const uint32_t tpc = (uint32_t)p.tiles_per_chunk;
    const uint32_t c0 = tpc > 0 ? (uint32_t)p.row_begin / cr : 0u;
    const uint32_t rbeg = (uint32_t)p.row_begin, rend = (uint32_t)p.row_end;
    const int ntiles = (int)p.tiles;
    auto item_at = [&](int ti, int &r0, int &r1, int &ord) __attribute__((always_inline)) -> bool {
        const uint32_t tt = (uint32_t)ti;
        uint32_t a, e, c;
        if (tpc > 0) {
            const uint32_t qd = tt / tpc, rem = tt - qd * tpc;
            c = c0 + qd;
            const uint32_t cs = c * cr;
            a = cs + rem * tr;
            e = a + tr < cs + cr ? a + tr : cs + cr;
        } else {
            a = rbeg + tt * tr;
            e = a + tr;
            c = a / cr;
        }
        if (e > rend) e = rend;
        r0 = __builtin_amdgcn_readfirstlane((int)a);
        r1 = __builtin_amdgcn_readfirstlane((int)e);
        ord = __builtin_amdgcn_readfirstlane((int)c) + p.ord_base;  // (no chunk_ord table on this path)
        return r0 < r1;
    };
    auto next_item = [&](int ti, int &r0, int &r1, int &ord) __attribute__((always_inline)) -> int {
        for (; ti < ntiles; ti += tstride)
            if (item_at(ti, r0, r1, ord)) return ti;
        return -1;
    };

    // issue cursor: item ti_i (rows [ir0, ir1), ordinal iord), next stage si
    int ir0 = 0, ir1 = 0;
    int iord = 0;
    // tile sequence of group tg of XCD x: t = start + 8 G j (G groups per
    // XCD).  tmap 1: start = x G + tg -- the XCD's groups work on G
    // consecutive tiles at a time (one chunk: one cosine query variant in the
    // XCD's L2); tmap 0: start = x + 8 tg
    int ti_i = next_item(tmap ? xcd * ngroups + tg : xcd + 8 * tg, ir0, ir1, iord);
    if (ti_i < 0) return;  // no work (uniform)
    const int nb = nst;
    const uint32_t blk = (uint32_t)nb * 1024u;  // bytes of one 16-vector block over all stages
    // DMA sources: a uniform base per stage + a 32-bit per-lane offset.
    // Piece i < 4 is row piece pc = w + 4 i (image rows 16 pc .. +16), i >= 4
    // query piece w + 4 (i - 4).  Lane -> image row lane >> 2 of the piece,
    // slot lane & 3, which holds chunk (lane & 3) ^ p4_g((lane >> 4) & 3).
    // Row tiles start on a 16-row block (the launcher checks), so row piece pc
    // of an item is plane block ir0 / 16 + pc; a piece past the item's rows
    // re-reads piece 0 (discarded).
    uint32_t roff[4], qoff[4];
    const unsigned char *rbase = nullptr;  // plane block of the item's first row (uniform)
    const unsigned char *qplane = reinterpret_cast<const unsigned char *>(ordm ? p.q_ord : p.q_hi);
    const uint64_t pstride = (uint64_t)(p.q_vpad >> 4) * blk;  // bytes of one ordinal plane
    uint32_t noff = 0;                      // L2: this lane's row norm, relative to the item's first row
    const unsigned char *nbase = nullptr;
    bool first_src = true;                  // query offsets: per item only for cosine variants
    // (the per-lane constants are re-derived from an opaque copy of the lane
    // index at every item: hoisted out of the item loop they were spilled,
    // and every reload from scratch waits for the whole LDS-DMA ring)
    auto set_src = [&]() __attribute__((always_inline)) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t lc = plane_vec_off((uint32_t)(ln >> 2)) + (uint32_t)((ln & 3) ^ p4_g((ln >> 4) & 3)) * 16u;
        rbase = reinterpret_cast<const unsigned char *>(p.rows_hi) + (uint64_t)(uint32_t)(ir0 >> 4) * blk;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = w + 4 * i;
            roff[i] = (ir0 + pc * 16 < ir1 ? (uint32_t)pc * blk : 0u) + lc;
        }
        if (ordm) {
            const int pl = iord < om0 ? iord : om0 + (iord - om0) % oln;
            qplane = reinterpret_cast<const unsigned char *>(p.q_ord) + (uint64_t)pl * pstride;
        }
        if (pervar || first_src) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int j = q0 + (w + 4 * i) * 16 + (ln >> 2);
                if (j >= p.nq) j = 0;
                int var = 0;
                if (pervar && (DIAG & 512) == 0) {
                    const int mu = qmu[i], lam = qlam[i];
                    var = iord < mu ? iord : mu + (iord - mu) % lam;
                }
                const uint32_t u = (uint32_t)var * (uint32_t)p.q_vpad + (uint32_t)j;
                qoff[i] = (u >> 4) * blk + plane_vec_off(u & 15) + (uint32_t)((ln & 3) ^ p4_g((ln >> 4) & 3)) * 16u;
            }
        }
        if constexpr (L2) {
            nbase = reinterpret_cast<const unsigned char *>(p.row_norms + ir0);
            const int last = ir1 - 1 - ir0;
            noff = (uint32_t)(64 * w + ln < last ? 64 * w + ln : last) * 4u;
        }
    };
    set_src();
    first_src = false;
    int si = 0;           // next stage of the issue item
    int issued = 0;       // stages issued (global counter)
    int ibuf = 0;         // ring buffer of the next issued stage
    int items_issued = 0;
    bool live = true;     // stages left to issue (else: dummy pieces, never read)
    // piece x of the next stage (x < 8; 8 = the L2 norm piece of an item's
    // first stage).  Once every stage is issued the pieces keep going to the
    // free buffer with the last sources (never read: the ring's counted waits
    // stay uniform)
    auto issue_piece = [&](int x) __attribute__((always_inline)) {
        if ((DIAG & 8) && x < 4) return;
        if ((DIAG & 4) && x >= 4 && x < 8) return;
        unsigned char *dst = lds + ibuf * kP4Stage;
        if (x < 4) {
            __builtin_amdgcn_global_load_lds((const void *)(rbase + plane_step_off((uint32_t)si) + roff[x]),
                                             (lds_void *)(dst + (w + 4 * x) * 1024), 16, 0, RPOL);
        } else if (x < 8) {
            // (a uniform base in SGPRs and one 32-bit lane offset: the
            // saddr form of the load, no 64-bit address add per piece)
            const uint32_t vo = plane_step_off((uint32_t)si) + qoff[x - 4];
            const uint64_t qb = (uint64_t)qplane;
            const unsigned char *qbase = reinterpret_cast<const unsigned char *>(
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(qb >> 32)) << 32) |
                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)qb));
            __builtin_amdgcn_global_load_lds((const void *)(qbase + vo),
                                             (lds_void *)(dst + kP4QOff + (w + 4 * (x - 4)) * 1024), 16, 0, QPOL);
        } else if constexpr (L2) {
            __builtin_amdgcn_global_load_lds((const void *)(nbase + noff),
                                             (lds_void *)(norm_lds + (items_issued & 1) * 1024 + w * 256), 4, 0, 0);
        }
    };
    auto issue_advance = [&]() __attribute__((always_inline)) {
        if (!live) return;
        ++issued;
        ibuf = ibuf + 1 == NBUF ? 0 : ibuf + 1;
        if (++si == nst) {
            si = 0;
            ++items_issued;
            int r0 = 0, r1 = 0, o = 0;
            const int tn = next_item(ti_i + tstride, r0, r1, o);
            if (tn >= 0) {
                ti_i = tn;
                ir0 = r0;
                ir1 = r1;
                iord = o;
                set_src();
            } else {
                live = false;
                si = nst - 1;  // dummy pieces re-read the last stage
            }
        }
    };
    auto issue_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < 8; ++x) issue_piece(x);
        if (L2 && si == 0 && live) issue_piece(8);
        issue_advance();
    };

    // compute cursor: item rows [cr0, cr1), stage sc, global stage gc
    int cr0 = ir0, cr1 = ir1;
    int ti_c = ti_i;
    int gc = 0;    // stages consumed (global counter)
    int cbuf = 0;  // ring buffer of stage gc
    int items_done = 0;

    // fragment offsets: image row R, chunk c at R * 64 + (c ^ p4_g((R >> 2) & 3)) * 16
    const int gl = p4_g((l32 >> 2) & 3);
    const int offa0 = l32 * 64 + ((0 + h) ^ gl) * 16;  // k-step 0: chunks 0 / 1
    const int offa1 = l32 * 64 + ((2 + h) ^ gl) * 16;  // k-step 1: chunks 2 / 3
    const int rowA = wr * 128 * 64, rowB = kP4QOff + wq * 128 * 64;
    auto frag = [&](const unsigned char *st, int off) __attribute__((always_inline)) { return *reinterpret_cast<const bf16x8 *>(st + off); };

    f32x16 acc[4][4];
    float gmx[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};  // PROBE
    int qcnt = 0;  // this wave's queue entries (wave-uniform)
    u32x4 *wq_base = queue + (int64_t)(blockIdx.x * 4 + w) * qcap;

    // prologue: D stages in flight, the first landed for everyone
    for (int s = 0; s < D; ++s) issue_stage();
    p4_wait_vm<NPW>(issued - 1);
    p4_barrier();
    bf16x8 a0[4], b0[4], a1[4], b1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a0[i] = frag(lds, rowA + i * 32 * 64 + offa0);
#pragma unroll
    for (int i = 0; i < 4; ++i) b0[i] = frag(lds, rowB + i * 32 * 64 + offa0);

    // The threshold test of one 32 x 32 block (rows rb, queries jb) of the
    // item whose rows start at ecr0 (ecrn of them): the maximum of the lane's
    // 16 values (v_maximum3_f32: no canonicalising max per value as with
    // fmaxf; a NaN value can only come from a NaN query, whose values all fail
    // the threshold either way) against its query's threshold; a block with
    // any lane over it walks its values.  The tests run in the MFMA gaps of
    // the stages around an item boundary (below), not as an epilogue of their
    // own.
    auto check_block = [&](auto RB, auto JB, int ecr0, int ecrn, int eti) __attribute__((always_inline)) {
        constexpr int rb = decltype(RB)::value, jb = decltype(JB)::value;
        if constexpr (PROBE) {
            // the lane's best value of the block (rows past the item: -inf),
            // folded into its query's running maximum; after the wave's last
            // row block the two half-waves' maxima combine and lanes 0..31
            // write one raw value per query
            const f32x16 blk = acc[rb][jb];
            f32x4 v4[4];
#pragma unroll
            for (int g = 0; g < 4; ++g)
                v4[g] = p4_aread4(blk[4 * g], blk[4 * g + 1], blk[4 * g + 2], blk[4 * g + 3]);
            if (ecrn < kP4Tile) {
                const int rbl = wr * 128 + rb * 32 + 4 * h;
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (rbl + (r & 3) + 8 * (r >> 2) >= ecrn) v4[r >> 2][r & 3] = -__builtin_inff();
            }
            float mx = v4[0][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mx = __builtin_elementwise_maximum(mx, v4[r >> 2][r & 3]);
            gmx[jb] = __builtin_elementwise_maximum(gmx[jb], mx);
            if constexpr (rb == 3) {
                const float o = __shfl_xor(gmx[jb], 32);
                const float v = __builtin_elementwise_maximum(gmx[jb], o);
                const int j = q0 + wq * 128 + jb * 32 + l32;
                if (h == 0 && j < p.nq) {
                    float raw = v;
                    if constexpr (L2) raw = qnl[jb] - 2.0f * v;
                    if (v == -__builtin_inff()) raw = __builtin_nanf("");
                    p.p4_gmax[(int64_t)j * p.p4_gld + 2 * eti + wr] = raw;
                }
                gmx[jb] = -__builtin_inff();
            }
            return;
        }
        if constexpr ((DIAG & 16) != 0) {
            // (diagnostic: keep the accumulators live, test nothing)
            const f32x16 blk = acc[rb][jb];
            if (p4_aread(blk[0]) == -1.2345e-30f) qcnt += 1;
            return;
        }
        const int j = q0 + wq * 128 + jb * 32 + l32;
        // (the block read in order, four values per statement: the compiler's
        // own reads are hoisted together and spill)
        const f32x16 blk = acc[rb][jb];
        f32x4 v4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) v4[g] = p4_aread4(blk[4 * g], blk[4 * g + 1], blk[4 * g + 2], blk[4 * g + 3]);
        float mx = v4[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = __builtin_elementwise_maximum(mx, v4[r >> 2][r & 3]);
        // (a wave-uniform branch: the queue count is wave state)
        if (__ballot(mx >= thr[jb]) == 0) return;
        if constexpr ((DIAG & 32) != 0) {  // (diagnostic: tests without walks)
            qcnt += 1;
            return;
        }
        // the walk (rare): each lane's mask of values at or over the
        // threshold; the values go to this wave's LDS scratch and a rolled loop
        // takes one set bit per lane and round (rounds = the largest count in
        // the wave, mostly 1).  (Unrolled over registers, the walks make the
        // compiler spill, and every reload from scratch memory waits for the
        // whole LDS-DMA ring.)
        const float th = thr[jb], tj = tl[jb], qn = qnl[jb];
        unsigned m16 = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) m16 |= (v4[r >> 2][r & 3] >= th ? 1u : 0u) << r;  // (padding: thr = +inf)
#pragma unroll
        for (int g = 0; g < 4; ++g) *reinterpret_cast<f32x4 *>(wscr + lane * 16 + 4 * g) = v4[g];
        const int rbl = wr * 128 + rb * 32 + 4 * h;
#pragma unroll 1
        while (__ballot(m16 != 0u) != 0) {
            bool pass = m16 != 0u;
            const int r = pass ? __builtin_ctz(m16) : 0;
            m16 &= m16 - 1u;
            const float x = wscr[lane * 16 + r];
            float raw = x;
            if constexpr (L2) {
                raw = qn - 2.0f * x;
                pass = pass && raw <= tj;
            }
            const int rl = rbl + (r & 3) + 8 * (r >> 2);
            pass = pass && rl < ecrn;
            const uint64_t m = __ballot(pass);
            if (m == 0) continue;
            const int pre =
                __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            if (pass) {
                const uint32_t row = (uint32_t)(ecr0 + rl);
                const int slot_ = qcnt + pre;
                if (slot_ < qcap)
                    wq_base[slot_] = u32x4{__builtin_bit_cast(unsigned, raw), row, (unsigned)j, 0u};
                else  // queue full: the direct append (its returned slot makes
                      // this wave wait for its LDS-DMA in flight: correct, slower)
                    emit_approx<METRIC, false, false>(p, j, row, row, row_valid(p, row), raw);
            }
            qcnt += __popcll(m);
        }
    };

    int pcr0 = 0, pcrn = 0, pti = 0;  // the previous item (its blocks 8..15 are tested in the next one)

    // k-step-0 phase: 16 MFMAs on (a0, b0); between them the k-step-1
    // fragments of this stage and the 8 LDS-DMA pieces of stage gc + D.
    // FIRST (the item's first stage): the MFMAs take C = 0, or -yn/2 of the
    // block's rows for L2, and with EPI2 the previous item's blocks 8..15 are
    // tested right before their first MFMA overwrites them.
    auto k0_phase = [&](const unsigned char *st, auto first_tag, auto epi_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value, EPI2 = decltype(epi_tag)::value;
        f32x16 cinit;
        p4_for<16>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value, rb = x >> 2, jb = x & 3;
            if constexpr (FIRST && EPI2 && x >= 8)
                check_block(std::integral_constant<int, rb>{}, std::integral_constant<int, jb>{}, pcr0, pcrn, pti);
            if constexpr (FIRST && L2 && jb == 0) {
                // C = -yn / 2 of the block's rows (the item's norms in LDS)
                const unsigned char *nb_ = norm_lds + (items_done & 1) * 1024;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 v = *reinterpret_cast<const f32x4 *>(nb_ + (wr * 128 + rb * 32 + 8 * g + 4 * h) * 4);
#pragma unroll
                    for (int e = 0; e < 4; ++e) cinit[4 * g + e] = -0.5f * v[e];
                }
            }
            if constexpr (FIRST && L2)
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[rb], b0[jb], cinit, 0, 0, 0);
            else if constexpr (FIRST)
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[rb], b0[jb], f32x16{0.f}, 0, 0, 0);
            else
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[rb], b0[jb], acc[rb][jb], 0, 0, 0);
            if constexpr (x < 4)
                a1[x] = frag(st, rowA + x * 32 * 64 + offa1);
            else if constexpr (x < 8)
                b1[x - 4] = frag(st, rowB + (x - 4) * 32 * 64 + offa1);
            else if constexpr ((PL & 3) == 0)
                issue_piece(x - 8);
            else if constexpr ((PL & 3) == 1 && x < 12)
                issue_piece(x - 8);
            else if constexpr ((PL & 3) == 2 && (x & 1) == 0)
                issue_piece((x - 8) >> 1);
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    // one stage: k-step-0 phase, the issue cursor, the barrier, k-step-1
    // phase.  LAST (the item's last stage): blocks 0..7 are tested two MFMAs
    // after their final one, in the k-step-1 phase's gaps.
    auto do_stage = [&](auto first_tag, auto epi_tag, auto last_tag) __attribute__((always_inline)) {
        constexpr bool LAST = decltype(last_tag)::value;
        const unsigned char *st = lds + cbuf * kP4Stage;
        const int nbuf_next = cbuf + 1 == NBUF ? 0 : cbuf + 1;
        k0_phase(st, first_tag, epi_tag);
        if (L2 && si == 0 && live) issue_piece(8);
        if constexpr ((PL & 3) == 0) issue_advance();
        // own pieces of stage gc + 1 landed (younger stages may stay in
        // flight); this stage's fragment reads retired (the next phase
        // re-fills its buffer); then the barrier: stage gc + 1 is complete
        // for every wave
        const bool has_next = gc + 1 < issued;
        // (PL > 0: the other half of stage gc + D is issued in the next phase;
        // its first half is younger than stage gc + 1's pieces)
        p4_wait_vm<NPW, (PL & 3) == 0 ? 0 : NPW / 2>(issued - gc - 2, has_next);
        if constexpr ((DIAG & 256) == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr ((DIAG & 128) == 0) p4_barrier();
        // k-step-1 phase: 16 MFMAs on (a1, b1); between them the k-step-0
        // fragments of stage gc + 1
        const unsigned char *sn = lds + nbuf_next * kP4Stage;
        const int crn = cr1 - cr0;
        p4_for<16>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value, rb = x >> 2, jb = x & 3;
            acc[rb][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[rb], b1[jb], acc[rb][jb], 0, 0, 0);
            // (the next stage's fragments are read unconditionally: past the
            // last stage they are stale ring bytes, never used; a branch per
            // gap cost 2.2 % of the main scan, profiles/r03/p4_next_reads_ab.jsonl)
            {
                if constexpr (x < 4)
                    a0[x] = frag(sn, rowA + x * 32 * 64 + offa0);
                else if constexpr (x < 8)
                    b0[x - 4] = frag(sn, rowB + (x - 4) * 32 * 64 + offa0);
            }
            if constexpr ((PL & 3) == 1 && x >= 8 && x < 12)
                issue_piece(x - 4);
            else if constexpr ((PL & 3) == 2 && x >= 8 && (x & 1) == 0)
                issue_piece(4 + ((x - 8) >> 1));
            if constexpr (LAST && x >= 2 && x < 10)
                check_block(std::integral_constant<int, ((x - 2) >> 2)>{}, std::integral_constant<int, (x - 2) & 3>{},
                            cr0, crn, ti_c);
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr ((PL & 3) != 0) issue_advance();
        ++gc;
        cbuf = nbuf_next;
    };

    // items: the first stage defines the accumulators (no phi with the last
    // item's: they stay in place), the other stages accumulate; nst >= 2
    using T = std::integral_constant<bool, true>;
    using F = std::integral_constant<bool, false>;
    bool first_item = true;
    while (true) {
        if (first_item)
            do_stage(T{}, F{}, F{});
        else
            do_stage(T{}, T{}, F{});
        for (int s = 1; s + 1 < nst; ++s) do_stage(F{}, F{}, F{});
        do_stage(F{}, F{}, T{});
        pcr0 = cr0;
        pcrn = cr1 - cr0;
        pti = ti_c;
        first_item = false;
        ++items_done;
        int cord;
        ti_c = next_item(ti_c + tstride, cr0, cr1, cord);
        if (ti_c < 0) break;
    }
    // blocks 8..15 of the last item
    p4_for<8>([&](auto X) __attribute__((always_inline)) {
        constexpr int x = decltype(X)::value + 8;
        check_block(std::integral_constant<int, (x >> 2)>{}, std::integral_constant<int, (x & 3)>{}, pcr0, pcrn, pti);
    });
    if constexpr (PROBE) return;
    // flush this wave's queue to the per-query candidate lists
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int nqueue = qcnt < qcap ? qcnt : qcap;
    for (int e = lane; e < nqueue; e += 64) {
        const u32x4 en = __builtin_nontemporal_load(wq_base + e);  // (bypasses L1)
        const uint32_t row = en[1];
        emit_approx<METRIC, false, false>(p, (int)en[2], row, row, row_valid(p, row), __builtin_bit_cast(float, en[0]));
    }
}

// ---------------------------------------------------------------------------
// k_scan_p4m: the same scan on v_mfma_f32_16x16x32_bf16.  Items, ring, DMA
// pieces, stage barrier and queue are those of k_scan_p4; only the tile inside
// a wave changes: its 128 rows x 128 queries are 8 x 8 blocks of 16 x 16 (64
// f32x4 accumulators = the same 256 AGPRs), and a 32-column stage is ONE
// k-step (lane l: row / query l & 15, chunk l >> 4 of the stage image).  The
// 64 MFMAs of a stage run as two phases of 32: phase 0 = row blocks 0..3
// (reading this stage's A fragments 4..7 and issuing the DMA pieces of stage
// s + D in its gaps), barrier, phase 1 = row blocks 4..7, query block by query
// block, each B fragment re-read for the next stage right after its last MFMA
// here (with A 0..3: the next stage's fragments, 16 x 4 VGPRs as before).
// Why: on random data the chip holds a higher clock on this shape than on
// 32x32x16 at the same cycles per flop (MI355X_MICROARCH.md, DVFS give-back
// item 7).  Threshold tests: per query block, the 16 values of four row blocks
// (row blocks 0..3 in the last stage's phase 1, 4..7 in the next item's first
// phase 0, before their first MFMA overwrites them).
// GRP (PROBE only): 0 = one value per (query, 128-row half tile) as k_scan_p4's
// probe; 16 = one per (query, 16-row block), p4_gmax[q][16 t + 8 wr + rb];
// 8 = one per (query, 8-row half block), p4_gmax[q][2 (16 t + 8 wr + rb) + h]
// (the index's coarse step, kernels_ivf.hip k_coarse_pick)
// (Measured and dropped, profiles/r04/p4m_l7_stg_ab.jsonl: the next stage's
// B fragment 7 read at the start of phase 0 instead of the end of phase 1,
// +0.4..2.4 % main scan; waves 2 and 3 issuing their DMA pieces in phase 1,
// +15 %.)
// DIAG (measurement builds only; 1, 2, 4: wrong results, timing only): 1 = no
// stage barrier, 2 = no DMA pieces issued, 4 = no threshold tests (the
// accumulators kept live by one read per block); 8 = the round-5 lane-major
// walk scratch (correct results; the A/B of its bank conflicts)
// PLM: where a stage's 8 DMA pieces (of stage s + D) go: 0 = phase 0 gaps
// 8, 11, .., 29; 1 = phase 0 gaps 0, 4, .., 28; 2 = the 4 row pieces in phase
// 0 (gaps 8, 14, 20, 26), the 4 query pieces in phase 1 (gaps 0, 8, 16, 24,
// after the barrier: stage s + D's buffer was last read before barrier
// s - 1); 3 = all 8 in phase 1 gaps 0, 4, .., 28
template <int METRIC, int NBUF, bool PROBE = false, int GRP = 0, int DIAG = 0, int PLM = 0>
__global__ __launch_bounds__(256, 1) void k_scan_p4m(ScanParams p, int slots, u32x4 *queue, int qcap, int tmap) {
    constexpr bool L2 = METRIC == MQVS_METRIC_L2;
    constexpr int D = NBUF - 1;
    static_assert(D >= 1 && D <= 4, "ring depth");
    constexpr int NORM = L2 ? 2048 : 0;
    constexpr int WSCR = 4 * 64 * 16 * 4;
    constexpr int QTAB = L2 ? kP4Tile * 8 : 0;  // L2: (threshold, |q|^2) of the item's queries for the walks
    constexpr int NPW = 8;
    __shared__ __attribute__((aligned(16))) unsigned char lds[NBUF * kP4Stage + NORM + WSCR + QTAB];
    unsigned char *norm_lds = lds + NBUF * kP4Stage;
    float *qtab = reinterpret_cast<float *>(lds + NBUF * kP4Stage + NORM + WSCR);

    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = w & 1, wq = w >> 1;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int nqb = p.num_qblocks;
    const int ngroups = slots / nqb;
    if (slot >= ngroups * nqb) return;
    const int qb = slot % nqb, tg = slot / nqb;
    const int q0 = qb * kP4Tile;
    const int tstride = 8 * ngroups;
    const int nst = (int)(p.dpad / kP4HiK);
    const int l16 = lane & 15, g4 = lane >> 4;
    float *wscr = reinterpret_cast<float *>(lds + NBUF * kP4Stage + NORM) + w * 1024;

    int om0 = 0, oln = 1;
    bool ordm = false;
    if (p.q_ord_desc) {
        om0 = __builtin_amdgcn_readfirstlane(p.q_ord_desc[0]);
        oln = __builtin_amdgcn_readfirstlane(p.q_ord_desc[1]);
        ordm = __builtin_amdgcn_readfirstlane(p.q_ord_desc[2]) != 0;
    }
    const bool pervar = p.maxv > 1 && !ordm;
    int qmu[4], qlam[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int j = q0 + (w + 4 * i) * 16 + (lane >> 2);
        if (j >= p.nq) j = 0;
        qmu[i] = 0;
        qlam[i] = 1;
        if (pervar) {
            qmu[i] = p.qmu[j];
            qlam[i] = p.qlam[j];
        }
    }
    // thresholds of the lane's query in each of the wave's 8 query blocks (as
    // k_scan_p4: L2 pre-checks acc >= (qn - t) / 2 less a rounding slack); the
    // L2 walk's exact test reads t and |q|^2 from an LDS table (registers are
    // scarce here, walks rare)
    float thr[8];
#pragma unroll
    for (int jb = 0; jb < 8; ++jb) {
        const int j = q0 + wq * 128 + jb * 16 + l16;
        const float tj = j < p.nq && !PROBE ? p.thr[j] : 0.f;  // (a probe has no thresholds)
        if constexpr (L2) {
            const float qn = j < p.nq ? p.qnorms[j] : 0.f;
            const float half = (qn - tj) * 0.5f;
            thr[jb] = half - 4.8e-7f * (fabsf(qn) + fabsf(tj)) - 1e-30f;
        } else {
            thr[jb] = tj;
        }
        if (j >= p.nq) thr[jb] = __builtin_inff();
        asm volatile("" : "+v"(thr[jb]));
    }
    if constexpr (L2) {
        // (written before the first LDS-DMA; the prologue barrier orders it)
        const int j = q0 + t;
        qtab[2 * t] = j < p.nq && !PROBE ? p.thr[j] : 0.f;
        qtab[2 * t + 1] = j < p.nq ? p.qnorms[j] : 0.f;
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(qmu[i]), "+v"(qlam[i]));

    const uint32_t tr = (uint32_t)p.tile_rows, cr = (uint32_t)p.chunk_rows;
    const uint32_t tpc = (uint32_t)p.tiles_per_chunk;
    const uint32_t c0 = tpc > 0 ? (uint32_t)p.row_begin / cr : 0u;
    const uint32_t rbeg = (uint32_t)p.row_begin, rend = (uint32_t)p.row_end;
    const int ntiles = (int)p.tiles;
    auto item_at = [&](int ti, int &r0, int &r1, int &ord) __attribute__((always_inline)) -> bool {
        const uint32_t tt = (uint32_t)ti;
        uint32_t a, e, c;
        if (tpc > 0) {
            const uint32_t qd = tt / tpc, rem = tt - qd * tpc;
            c = c0 + qd;
            const uint32_t cs = c * cr;
            a = cs + rem * tr;
            e = a + tr < cs + cr ? a + tr : cs + cr;
        } else {
            a = rbeg + tt * tr;
            e = a + tr;
            c = a / cr;
        }
        if (e > rend) e = rend;
        r0 = __builtin_amdgcn_readfirstlane((int)a);
        r1 = __builtin_amdgcn_readfirstlane((int)e);
        ord = __builtin_amdgcn_readfirstlane((int)c) + p.ord_base;
        return r0 < r1;
    };
    auto next_item = [&](int ti, int &r0, int &r1, int &ord) __attribute__((always_inline)) -> int {
        for (; ti < ntiles; ti += tstride)
            if (item_at(ti, r0, r1, ord)) return ti;
        return -1;
    };

    int ir0 = 0, ir1 = 0;
    int iord = 0;
    int ti_i = next_item(tmap ? xcd * ngroups + tg : xcd + 8 * tg, ir0, ir1, iord);
    if (ti_i < 0) return;
    const int nb = nst;
    const uint32_t blk = (uint32_t)nb * 1024u;
    uint32_t roff[4], qoff[4];
    const unsigned char *rbase = nullptr;
    const unsigned char *qplane = reinterpret_cast<const unsigned char *>(ordm ? p.q_ord : p.q_hi);
    const uint64_t pstride = (uint64_t)(p.q_vpad >> 4) * blk;
    uint32_t noff = 0;
    const unsigned char *nbase = nullptr;
    bool first_src = true;
    auto set_src = [&]() __attribute__((always_inline)) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t lc = plane_vec_off((uint32_t)(ln >> 2)) + (uint32_t)((ln & 3) ^ p4_g((ln >> 4) & 3)) * 16u;
        rbase = reinterpret_cast<const unsigned char *>(p.rows_hi) + (uint64_t)(uint32_t)(ir0 >> 4) * blk;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = w + 4 * i;
            roff[i] = (ir0 + pc * 16 < ir1 ? (uint32_t)pc * blk : 0u) + lc;
        }
        if (ordm) {
            const int pl = iord < om0 ? iord : om0 + (iord - om0) % oln;
            qplane = reinterpret_cast<const unsigned char *>(p.q_ord) + (uint64_t)pl * pstride;
        }
        if (pervar || first_src) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int j = q0 + (w + 4 * i) * 16 + (ln >> 2);
                if (j >= p.nq) j = 0;
                int var = 0;
                if (pervar) {
                    const int mu = qmu[i], lam = qlam[i];
                    var = iord < mu ? iord : mu + (iord - mu) % lam;
                }
                const uint32_t u = (uint32_t)var * (uint32_t)p.q_vpad + (uint32_t)j;
                qoff[i] = (u >> 4) * blk + plane_vec_off(u & 15) + (uint32_t)((ln & 3) ^ p4_g((ln >> 4) & 3)) * 16u;
            }
        }
        if constexpr (L2) {
            nbase = reinterpret_cast<const unsigned char *>(p.row_norms + ir0);
            const int last = ir1 - 1 - ir0;
            noff = (uint32_t)(64 * w + ln < last ? 64 * w + ln : last) * 4u;
        }
    };
    set_src();
    first_src = false;
    int si = 0, issued = 0, ibuf = 0, items_issued = 0;
    bool live = true;
    auto issue_piece = [&](int x) __attribute__((always_inline)) {
        if constexpr ((DIAG & 2) != 0) return;
        unsigned char *dst = lds + ibuf * kP4Stage;
        if (x < 4) {
            __builtin_amdgcn_global_load_lds((const void *)(rbase + plane_step_off((uint32_t)si) + roff[x]),
                                             (lds_void *)(dst + (w + 4 * x) * 1024), 16, 0, 0);
        } else if (x < 8) {
            const uint32_t vo = plane_step_off((uint32_t)si) + qoff[x - 4];
            const uint64_t qb_ = (uint64_t)qplane;
            const unsigned char *qbase = reinterpret_cast<const unsigned char *>(
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(qb_ >> 32)) << 32) |
                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)qb_));
            __builtin_amdgcn_global_load_lds((const void *)(qbase + vo),
                                             (lds_void *)(dst + kP4QOff + (w + 4 * (x - 4)) * 1024), 16, 0, 0);
        } else if constexpr (L2) {
            __builtin_amdgcn_global_load_lds((const void *)(nbase + noff),
                                             (lds_void *)(norm_lds + (items_issued & 1) * 1024 + w * 256), 4, 0, 0);
        }
    };
    auto issue_advance = [&]() __attribute__((always_inline)) {
        if (!live) return;
        ++issued;
        ibuf = ibuf + 1 == NBUF ? 0 : ibuf + 1;
        if (++si == nst) {
            si = 0;
            ++items_issued;
            int r0 = 0, r1 = 0, o = 0;
            const int tn = next_item(ti_i + tstride, r0, r1, o);
            if (tn >= 0) {
                ti_i = tn;
                ir0 = r0;
                ir1 = r1;
                iord = o;
                set_src();
            } else {
                live = false;
                si = nst - 1;
            }
        }
    };
    auto issue_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < 8; ++x) issue_piece(x);
        if (L2 && si == 0 && live) issue_piece(8);
        issue_advance();
    };

    int cr0 = ir0, cr1 = ir1;
    int ti_c = ti_i;
    int gc = 0, cbuf = 0, items_done = 0;

    // fragment offset: image row R = 16 i + (l & 15), chunk l >> 4
    const int offm = l16 * 64 + (g4 ^ p4_g((l16 >> 2) & 3)) * 16;
    const int rowA = wr * 128 * 64, rowB = kP4QOff + wq * 128 * 64;
    auto frag = [&](const unsigned char *st, int off) __attribute__((always_inline)) {
        return *reinterpret_cast<const bf16x8 *>(st + off);
    };

    f32x4 acc[8][8];
    float gmx[8];  // PROBE: the lane's running best per query block
#pragma unroll
    for (int jb = 0; jb < 8; ++jb) gmx[jb] = -__builtin_inff();
    int qcnt = 0;
    u32x4 *wq_base = queue + (int64_t)(blockIdx.x * 4 + w) * qcap;

    for (int s = 0; s < D; ++s) issue_stage();
    p4_wait_vm<NPW>(issued - 1);
    p4_barrier();
    bf16x8 a[8], b[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag(lds, rowA + i * 16 * 64 + offm);
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = frag(lds, rowB + i * 16 * 64 + offm);

    // the test of query block jb over row blocks 4 hf .. 4 hf + 3 (16 values
    // per lane, all of its query l & 15) of the item at rows ecr0 (ecrn rows)
    auto check = [&](auto HF, auto JB, int ecr0, int ecrn, int eti) __attribute__((always_inline)) {
        constexpr int hf = decltype(HF)::value, jb = decltype(JB)::value;
        f32x4 v4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 bk = acc[4 * hf + g][jb];
            v4[g] = p4_aread4(bk[0], bk[1], bk[2], bk[3]);
        }
        // value v4[g][i]: row wr 128 + (4 hf + g) 16 + 4 g4 + i
        const int rbl = wr * 128 + hf * 64 + 4 * g4;
        if constexpr (PROBE) {
            if (ecrn < kP4Tile) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (rbl + 16 * (r >> 2) + (r & 3) >= ecrn) v4[r >> 2][r & 3] = -__builtin_inff();
            }
        }
        const int j = q0 + wq * 128 + jb * 16 + l16;
        if constexpr (PROBE && (GRP == 16 || GRP == 8)) {
            // the four lanes of query l16 hold the block's 16 rows (lanes
            // g4 = 0, 1: rows 0..7; g4 = 2, 3: rows 8..15)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(v4[g][0], v4[g][1]),
                                                        __builtin_elementwise_maximum(v4[g][2], v4[g][3]));
                m = __builtin_elementwise_maximum(m, __shfl_xor(m, 16));
                if constexpr (GRP == 16) m = __builtin_elementwise_maximum(m, __shfl_xor(m, 32));
                if ((GRP == 16 ? g4 == 0 : (g4 & 1) == 0) && j < p.nq) {
                    float raw = m;
                    if constexpr (L2) raw = qtab[2 * (j - q0) + 1] - 2.0f * m;
                    if (m == -__builtin_inff()) raw = __builtin_nanf("");
                    const int64_t blk = 16 * eti + 8 * wr + 4 * hf + g;  // 16-row block of the part
                    p.p4_gmax[(int64_t)j * p.p4_gld + (GRP == 16 ? blk : 2 * blk + (g4 >> 1))] = raw;
                }
            }
            return;
        }
        if constexpr (!PROBE && (DIAG & 4) != 0) {
            if (v4[0][0] == -1.2345e-30f) qcnt += 1;  // (diagnostic: keep the accumulators live)
            return;
        }
        float mx = v4[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = __builtin_elementwise_maximum(mx, v4[r >> 2][r & 3]);
        if constexpr (PROBE) {
            gmx[jb] = __builtin_elementwise_maximum(gmx[jb], mx);
            if constexpr (hf == 1) {
                float v = __builtin_elementwise_maximum(gmx[jb], __shfl_xor(gmx[jb], 16));
                v = __builtin_elementwise_maximum(v, __shfl_xor(v, 32));
                if (g4 == 0 && j < p.nq) {
                    float raw = v;
                    if constexpr (L2) raw = qtab[2 * (j - q0) + 1] - 2.0f * v;
                    if (v == -__builtin_inff()) raw = __builtin_nanf("");
                    p.p4_gmax[(int64_t)j * p.p4_gld + 2 * eti + wr] = raw;
                }
                gmx[jb] = -__builtin_inff();
            }
            return;
        }
        if (__ballot(mx >= thr[jb]) == 0) return;
        const float th = thr[jb];
        float tj = 0.f, qn = 0.f;
        if constexpr (L2) {
            tj = qtab[2 * (j - q0)];
            qn = qtab[2 * (j - q0) + 1];
        }
        unsigned m16 = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) m16 |= (v4[r >> 2][r & 3] >= th ? 1u : 0u) << r;
        // walk scratch value-major (value r of lane l at r 64 + l): the walk's
        // reads of a per-lane value index hit 64 distinct banks; lane-major
        // (DIAG 8, round 5: lane stride 64 B) put every fourth lane on the
        // same bank -- 16-way conflicts on every read of the walk
        if constexpr ((DIAG & 8) != 0) {
#pragma unroll
            for (int g = 0; g < 4; ++g) *reinterpret_cast<f32x4 *>(wscr + lane * 16 + 4 * g) = v4[g];
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) wscr[r * 64 + lane] = v4[r >> 2][r & 3];
        }
#pragma unroll 1
        while (__ballot(m16 != 0u) != 0) {
            bool pass = m16 != 0u;
            const int r = pass ? __builtin_ctz(m16) : 0;
            m16 &= m16 - 1u;
            const float x = (DIAG & 8) != 0 ? wscr[lane * 16 + r] : wscr[r * 64 + lane];
            float raw = x;
            if constexpr (L2) {
                raw = qn - 2.0f * x;
                pass = pass && raw <= tj;
            }
            const int rl = rbl + 16 * (r >> 2) + (r & 3);
            pass = pass && rl < ecrn;
            const uint64_t m = __ballot(pass);
            if (m == 0) continue;
            const int pre =
                __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            if (pass) {
                const uint32_t row = (uint32_t)(ecr0 + rl);
                const int slot_ = qcnt + pre;
                if (slot_ < qcap)
                    wq_base[slot_] = u32x4{__builtin_bit_cast(unsigned, raw), row, (unsigned)j, 0u};
                else
                    emit_approx<METRIC, false, false>(p, j, row, row, row_valid(p, row), raw);
            }
            qcnt += __popcll(m);
        }
    };

    int pcr0 = 0, pcrn = 0, pti = 0;

    // C of an item's first MFMA on a row block: 0, or -|y|^2 / 2 of its rows
    auto cinit = [&](int rb) __attribute__((always_inline)) -> f32x4 {
        if constexpr (L2) {
            const unsigned char *nb_ = norm_lds + (items_done & 1) * 1024;
            const f32x4 v = *reinterpret_cast<const f32x4 *>(nb_ + (wr * 128 + rb * 16 + 4 * g4) * 4);
            return f32x4{-0.5f * v[0], -0.5f * v[1], -0.5f * v[2], -0.5f * v[3]};
        } else {
            return f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };

    // phase 0: row blocks 0..3 x query blocks 0..7; in its gaps this stage's
    // A fragments 4..7, the DMA pieces of stage gc + D and (EPI) the tests of
    // the previous item's row blocks 4..7
    auto phase0 = [&](const unsigned char *st, auto first_tag, auto epi_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value, EPI = decltype(epi_tag)::value;
        f32x4 ci = f32x4{0.f, 0.f, 0.f, 0.f};
        p4_for<32>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value, rb = x >> 3, jb = x & 7;
            if constexpr (FIRST && EPI && (x & 3) == 1)
                check(std::integral_constant<int, 1>{}, std::integral_constant<int, (x >> 2)>{}, pcr0, pcrn, pti);
            if constexpr (FIRST && jb == 0) ci = cinit(rb);
            if constexpr (FIRST)
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[jb], ci, 0, 0, 0);
            else
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[jb], acc[rb][jb], 0, 0, 0);
            if constexpr (x >= 2 && x < 6)
                a[2 + x] = frag(st, rowA + (2 + x) * 16 * 64 + offm);
            if constexpr (PLM == 0 && x >= 8 && (x - 8) % 3 == 0 && (x - 8) / 3 < 8)
                issue_piece((x - 8) / 3);
            else if constexpr (PLM == 1 && (x & 3) == 0)
                issue_piece(x >> 2);
            else if constexpr (PLM == 2 && x >= 8 && (x - 8) % 6 == 0)
                issue_piece((x - 8) / 6);
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    // phase 1: row blocks 4..7, query block by query block; the next stage's
    // B fragment jb right after its last MFMA here, its A fragments 0..3 in
    // between; LAST: the tests of this item's row blocks 0..3
    // (FIRST: row block by row block instead, so that one C value is live at
    // a time; the B fragments are then re-read in the last eight gaps)
    auto phase1 = [&](const unsigned char *sn, auto first_tag, auto last_tag, int crn) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value, LAST = decltype(last_tag)::value;
        f32x4 ci = f32x4{0.f, 0.f, 0.f, 0.f};
        p4_for<32>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            constexpr int jb = FIRST ? (x & 7) : (x >> 2), rb = FIRST ? 4 + (x >> 3) : 4 + (x & 3);
            if constexpr (FIRST && jb == 0) ci = cinit(rb);
            if constexpr (FIRST)
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[jb], ci, 0, 0, 0);
            else
                acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b[jb], acc[rb][jb], 0, 0, 0);
            if constexpr (FIRST ? rb == 7 : (x & 3) == 3)
                b[jb] = frag(sn, rowB + jb * 16 * 64 + offm);
            else if constexpr ((x & 3) == 1 && (x >> 2) < 4)
                a[x >> 2] = frag(sn, rowA + (x >> 2) * 16 * 64 + offm);
            if constexpr (LAST && (x & 3) == 2)
                check(std::integral_constant<int, 0>{}, std::integral_constant<int, jb>{}, cr0, crn, ti_c);
            if constexpr (PLM == 2 && (x & 7) == 0)
                issue_piece(4 + (x >> 3));
            else if constexpr (PLM == 3 && (x & 3) == 0)
                issue_piece(x >> 2);
            __builtin_amdgcn_sched_barrier(0);
        });
    };

    auto do_stage = [&](auto first_tag, auto epi_tag, auto last_tag) __attribute__((always_inline)) {
        const unsigned char *st = lds + cbuf * kP4Stage;
        const int nbuf_next = cbuf + 1 == NBUF ? 0 : cbuf + 1;
        phase0(st, first_tag, epi_tag);
        if constexpr (PLM < 2) {
            if (L2 && si == 0 && live) issue_piece(8);
            issue_advance();
        }
        const bool has_next = gc + 1 < issued;
        // (PLM 2: the row half of stage gc + D is issued and younger than
        // stage gc + 1's pieces; PLM 3: none of it yet)
        p4_wait_vm<NPW, PLM == 2 ? NPW / 2 : 0>(issued - gc - 2, has_next);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr ((DIAG & 1) == 0) p4_barrier();
        phase1(lds + nbuf_next * kP4Stage, first_tag, last_tag, cr1 - cr0);
        if constexpr (PLM >= 2) {
            if (L2 && si == 0 && live) issue_piece(8);
            issue_advance();
        }
        ++gc;
        cbuf = nbuf_next;
    };

    using T = std::integral_constant<bool, true>;
    using F = std::integral_constant<bool, false>;
    bool first_item = true;
    while (true) {
        if (first_item)
            do_stage(T{}, F{}, F{});
        else
            do_stage(T{}, T{}, F{});
        // (two stages per iteration: at a loop header the compiler drains
        // every LDS read in flight -- the next stage's last fragment, read in
        // the last gap -- so a stage boundary inside the body keeps counted
        // waits)
        int s = 1;
        for (; s + 2 < nst; s += 2) {
            do_stage(F{}, F{}, F{});
            do_stage(F{}, F{}, F{});
        }
        if (s + 1 < nst) do_stage(F{}, F{}, F{});
        do_stage(F{}, F{}, T{});
        pcr0 = cr0;
        pcrn = cr1 - cr0;
        pti = ti_c;
        first_item = false;
        ++items_done;
        int cord;
        ti_c = next_item(ti_c + tstride, cr0, cr1, cord);
        if (ti_c < 0) break;
    }
    // row blocks 4..7 of the last item
    p4_for<8>([&](auto X) __attribute__((always_inline)) {
        check(std::integral_constant<int, 1>{}, std::integral_constant<int, decltype(X)::value>{}, pcr0, pcrn, pti);
    });
    if constexpr (PROBE) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int nqueue = qcnt < qcap ? qcnt : qcap;
    for (int e = lane; e < nqueue; e += 64) {
        const u32x4 en = __builtin_nontemporal_load(wq_base + e);
        const uint32_t row = en[1];
        emit_approx<METRIC, false, false>(p, (int)en[2], row, row, row_valid(p, row), __builtin_bit_cast(float, en[0]));
    }
}

// queue entries per wave (16 B each): 4096 x 16 B x 4 waves x 256 CUs = 64 MiB
constexpr int kP4QueueCap = 4096;

// (the current device's CU count, queried per call: launch_p4 sizes its grid
// from the same query, so the queue always covers blockIdx * 4 + wave)
size_t p4_queue_bytes() {
    const int cus = device_cus();
    return (size_t)cus * 4 * kP4QueueCap * sizeof(u32x4);
}

// Cosine ordinal planes.  Query j uses variant v_j(o) = o < mu_j ? o :
// mu_j + (o - mu_j) % lam_j at chunk ordinal o.  With m0 = max mu_j and
// L = lcm(lam_j), every o >= m0 with (o - m0) % L = c uses the variants of
// o' = m0 + c, so m0 + L planes hold every chunk's queries contiguously
// (plane pl = o for o < m0, m0 + (o - m0) % L after).  desc = {m0, L, ok}.
__global__ void k_ord_desc(const int *qmu, const int *qlam, int nq, int pcap, int *desc) {
    __shared__ int smu;
    __shared__ unsigned long long slam;
    if (threadIdx.x == 0) {
        smu = 0;
        slam = 0;
    }
    __syncthreads();
    int mu = 0;
    unsigned long long lm = 0;
    for (int j = threadIdx.x; j < nq; j += blockDim.x) {
        mu = max(mu, qmu[j]);
        const int l = qlam[j];
        lm |= (l >= 1 && l <= 63) ? (1ull << l) : 1ull;  // (bit 0: a cycle too long to serve)
    }
    atomicMax(&smu, mu);
    atomicOr(&slam, lm);
    __syncthreads();
    if (threadIdx.x != 0) return;
    long long L = 1;
    bool ok = (slam & 1ull) == 0;
    for (int l = 2; l < 64 && ok; ++l) {
        if (!((slam >> l) & 1ull)) continue;
        long long a = L, b = l;
        while (b) {
            const long long t = a % b;
            a = b;
            b = t;
        }
        L = L / a * l;
        ok = L <= pcap;
    }
    ok = ok && (long long)smu + L <= pcap;
    desc[0] = smu;
    desc[1] = ok ? (int)L : 1;
    desc[2] = ok ? 1 : 0;
}

// one thread per 16 B of a plane vector's stage: (plane, vector, stage, quarter)
__global__ void k_ord_gather(const uint16_t *qhi, uint16_t *qord, const int *qmu, const int *qlam, int nq,
                             int64_t vpad, int nst, const int *desc) {
    if (!desc[2]) return;
    const int np = desc[0] + desc[1];
    const int64_t per_vec = (int64_t)nst * 4, per_plane = vpad * per_vec;
    const int64_t total = (int64_t)np * per_plane;
    const unsigned char *src = reinterpret_cast<const unsigned char *>(qhi);
    unsigned char *dst = reinterpret_cast<unsigned char *>(qord);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int pl = (int)(e / per_plane);
        const int64_t rem = e - (int64_t)pl * per_plane;
        const int64_t j = rem / per_vec;
        const int r2 = (int)(rem - j * per_vec), st = r2 >> 2, qt = r2 & 3;
        int v = 0;
        if (j < nq) {
            const int mu = qmu[j], lam = qlam[j];
            v = pl < mu ? pl : mu + (pl - mu) % lam;
        }
        const int64_t us = (int64_t)v * vpad + j, ud = (int64_t)pl * vpad + j;
        const int64_t os = (((us >> 4) * nst) << 10) + plane_step_off(st) + plane_vec_off((uint32_t)(us & 15)) + qt * 16;
        const int64_t od = (((ud >> 4) * nst) << 10) + plane_step_off(st) + plane_vec_off((uint32_t)(ud & 15)) + qt * 16;
        *reinterpret_cast<u32x4 *>(dst + od) = *reinterpret_cast<const u32x4 *>(src + os);
    }
}

void launch_ord_planes(const uint16_t *q_hi, uint16_t *q_ord, int *desc, const int *qmu, const int *qlam, int nq,
                       int64_t vpad, int64_t dpad, int pcap, hipStream_t s) {
    hipLaunchKernelGGL(k_ord_desc, dim3(1), dim3(256), 0, s, qmu, qlam, nq, pcap, desc);
    const int64_t total = (int64_t)pcap * vpad * (dpad / kP4HiK) * 4;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_ord_gather, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, q_hi, q_ord, qmu,
                       qlam, nq, vpad, (int)(dpad / kP4HiK), desc);
}

// the batch kernels' launch conditions (sets p.num_qblocks)
static bool p4_ok(ScanParams &p, bool need_queue = true) {
    if ((need_queue && !p.p4_queue) || p.row_list || p.chunk_ord || p.tiles < 1 || p.tile_rows != kP4Tile)
        return false;
    p.num_qblocks = (p.nq + kP4Tile - 1) / kP4Tile;
    const int cus = device_cus();
    if (p.num_qblocks > cus / 8 || p.dpad % kP4HiK) return false;
    if (p.row_begin % 16 || (p.tiles_per_chunk > 0 && p.chunk_rows % 16)) return false;
    if (p.row_begin < 0 || p.row_end + p.chunk_rows + p.tile_rows > 0x7FFFFFFF || p.tiles > 0x3FFFFFFF ||
        p.chunk_rows < 1)
        return false;
    if ((double)p.maxv * (double)p.q_vpad * (double)p.dpad * 2.0 >= 4294967296.0) return false;
    return true;
}

// true when the launch was taken (batch APPEND, contiguous rows, identity
// chunk ordinals, the queue workspace present)
template <int METRIC>
static bool launch_p4_t(ScanParams p, hipStream_t s) {
    if (!p.p4_queue || p.row_list || p.chunk_ord || p.tiles < 1 || p.tile_rows != kP4Tile) return false;
    p.num_qblocks = (p.nq + kP4Tile - 1) / kP4Tile;
    const int cus = device_cus();
    const int per_xcd = cus / 8;
    if (p.num_qblocks > per_xcd) return false;
    if (p.dpad % kP4HiK) return false;
    // row tiles start on 16-row plane blocks; query plane offsets fit 32 bits
    if (p.row_begin % 16 || (p.tiles_per_chunk > 0 && p.chunk_rows % 16)) return false;
    // 32-bit item arithmetic (rows, tiles, chunk starts)
    if (p.row_begin < 0 || p.row_end + p.chunk_rows + p.tile_rows > 0x7FFFFFFF || p.tiles > 0x3FFFFFFF ||
        p.chunk_rows < 1)
        return false;
    if ((double)p.maxv * (double)p.q_vpad * (double)p.dpad * 2.0 >= 4294967296.0) return false;
    if constexpr (METRIC == MQVS_METRIC_L2) {
        // the norm piece is a 4-B-per-lane DMA: any row alignment works
        if (!p.row_norms) return false;
    }
    const int slots = per_xcd / p.num_qblocks * p.num_qblocks;
    auto *q = reinterpret_cast<u32x4 *>(p.p4_queue);
    const dim3 grid((unsigned)(8 * per_xcd));
    const int tmap = tune_int("MQVS_P4_MAP", 1);
    if constexpr (kDebugTuning) {
        // measurement builds: ring depth and decomposition variants
        const int nbuf = tune_int("MQVS_P4_NBUF", 4);
        const int diag = tune_int("MQVS_P4_DIAG", 0);
        const int pl = tune_int("MQVS_P4_PL", 0);
#define MQVS_P4(NB_, DG_, PL_)                                                                                     \
    hipLaunchKernelGGL((k_scan_p4<METRIC, NB_, DG_, PL_>), grid, dim3(256), 0, s, p, slots, q, kP4QueueCap, tmap)
        if (diag == 4) MQVS_P4(4, 4, 0);
        else if (diag == 8) MQVS_P4(4, 8, 0);
        else if (diag == 12) MQVS_P4(4, 12, 0);
        else if (diag == 16) MQVS_P4(4, 16, 0);
        else if (diag == 28) MQVS_P4(4, 28, 0);
        else if (diag == 32) MQVS_P4(4, 32, 0);
        else if (diag == 128) MQVS_P4(4, 128, 0);
        else if (diag == 256) MQVS_P4(4, 256, 0);
        else if (diag == 384) MQVS_P4(4, 384, 0);
        else if (diag == 156) MQVS_P4(4, 156, 0);
        else if (diag == 512) MQVS_P4(4, 512, 0);
        else if (nbuf == 3) MQVS_P4(3, 0, 0);
        else if (pl == 1) MQVS_P4(4, 0, 1);
        else if (pl == 2) MQVS_P4(4, 0, 2);
        else if (pl == 4) MQVS_P4(4, 0, 4);
        else if (pl == 6) MQVS_P4(4, 0, 6);
        else if (pl == 8) MQVS_P4(4, 0, 8);
        else MQVS_P4(4, 0, 0);
#undef MQVS_P4
    } else {
        hipLaunchKernelGGL((k_scan_p4<METRIC, 4, 0>), grid, dim3(256), 0, s, p, slots, q, kP4QueueCap, tmap);
    }
    return true;
}

// the batch kernel actually launched: k_scan_p4 (32x32x16) or, with
// kP4M16, k_scan_p4m (16x16x32)
// 16x16x32 by default: main scan at nq 1000 -4.2 % (cosine) / -6.1 % (L2)
// against k_scan_p4, bit-identical results (profiles/r04/m16_ab.jsonl)
constexpr int kP4M16Default = 1;
template <int METRIC>
static bool launch_p4_any(const ScanParams &p, hipStream_t s) {
    if (tune_int("MQVS_P4_M16", kP4M16Default) == 0) return launch_p4_t<METRIC>(p, s);

    ScanParams c = p;
    if (!p4_ok(c)) return false;
    if (METRIC == MQVS_METRIC_L2 && !c.row_norms) return false;
    const int cus = device_cus();
    const int per_xcd = cus / 8;
    const int slots = per_xcd / c.num_qblocks * c.num_qblocks;
    const dim3 grid((unsigned)(8 * per_xcd));
    auto *qq = reinterpret_cast<u32x4 *>(c.p4_queue);
    const int tmap = tune_int("MQVS_P4_MAP", 1);
    if constexpr (kDebugTuning) {
        // measurement builds: decomposition variants (wrong results)
        const int diag = tune_int("MQVS_P4M_DIAG", 0);
        const int plm = tune_int("MQVS_P4M_PL", 0);
#define MQVS_P4M(DG_, PL_)                                                                                          \
    hipLaunchKernelGGL((k_scan_p4m<METRIC, 4, false, 0, DG_, PL_>), grid, dim3(256), 0, s, c, slots, qq, kP4QueueCap, \
                       tmap)
        if (diag == 1) MQVS_P4M(1, 0);
        else if (diag == 4) MQVS_P4M(4, 0);
        else if (diag == 8) MQVS_P4M(8, 0);
        else if (diag == 6) MQVS_P4M(6, 0);
        else if (plm == 1) MQVS_P4M(0, 1);
        else if (plm == 2) MQVS_P4M(0, 2);
        else if (plm == 3) MQVS_P4M(0, 3);
        else MQVS_P4M(0, 0);
#undef MQVS_P4M
        return true;
    }
    hipLaunchKernelGGL((k_scan_p4m<METRIC, 4>), grid, dim3(256), 0, s, c, slots, qq, kP4QueueCap, tmap);
    return true;
}

// the batch probe (PROBE above): the same launch conditions; false when the
// probe rows cannot take the batch kernel (the caller runs the dense probe)
template <int METRIC>
static bool launch_p4_probe_t(ScanParams p, hipStream_t s) {
    // Group maxima are taken over every row of a group: with a PREWHERE
    // filter or lightweight deletes the best row of a group may be one that
    // row_valid rejects, and the k-th maximum would then be tighter than the
    // k-th VALID row's value (true neighbours would fail the append test).
    // Such searches keep the dense probe, which masks invalid rows.
    if (p.filter || p.exists) return false;
    if (!p.p4_gmax || p.p4_gld < 2 * p.tiles || !p4_ok(p, false)) return false;
    if (METRIC == MQVS_METRIC_L2 && !p.row_norms) return false;
    const int cus = device_cus();
    const int per_xcd = cus / 8;
    const int slots = per_xcd / p.num_qblocks * p.num_qblocks;
    const dim3 grid((unsigned)(8 * per_xcd));
    auto *q = reinterpret_cast<u32x4 *>(p.p4_queue);
    if (tune_int("MQVS_P4_M16", kP4M16Default))
        hipLaunchKernelGGL((k_scan_p4m<METRIC, 4, true>), grid, dim3(256), 0, s, p, slots, q, kP4QueueCap, 1);
    else
        hipLaunchKernelGGL((k_scan_p4<METRIC, 4, 0, 0, true>), grid, dim3(256), 0, s, p, slots, q, kP4QueueCap, 1);
    return true;
}

template <int METRIC, int GRP>
static bool launch_p4_groups_t(ScanParams p, hipStream_t s) {
    if (!p.p4_gmax || p.p4_gld < (256 / GRP) * p.tiles || !p4_ok(p, false)) return false;
    if (METRIC == MQVS_METRIC_L2 && !p.row_norms) return false;
    const int cus = device_cus();
    const int per_xcd = cus / 8;
    const int slots = per_xcd / p.num_qblocks * p.num_qblocks;
    hipLaunchKernelGGL((k_scan_p4m<METRIC, 4, true, GRP>), dim3((unsigned)(8 * per_xcd)), dim3(256), 0, s, p, slots,
                       nullptr, kP4QueueCap, 1);
    return true;
}

// grp: centroids per group, 16 or 8 (p4_gmax[q][tiles * 256 / grp])
bool launch_scan_p4_groups(const ScanParams &p, int metric, int grp, hipStream_t s) {
    if (grp == 8)
        return metric == MQVS_METRIC_L2 ? launch_p4_groups_t<MQVS_METRIC_L2, 8>(p, s)
                                        : launch_p4_groups_t<kMetricIpRaw, 8>(p, s);
    return metric == MQVS_METRIC_L2 ? launch_p4_groups_t<MQVS_METRIC_L2, 16>(p, s)
                                    : launch_p4_groups_t<kMetricIpRaw, 16>(p, s);
}

bool launch_scan_p4_probe(const ScanParams &p, int metric, hipStream_t s) {
    switch (metric) {
        case MQVS_METRIC_L2: return launch_p4_probe_t<MQVS_METRIC_L2>(p, s);
        case MQVS_METRIC_IP: return launch_p4_probe_t<MQVS_METRIC_IP>(p, s);
        case MQVS_METRIC_COSINE: return launch_p4_probe_t<MQVS_METRIC_COSINE>(p, s);
        default: return launch_p4_probe_t<kMetricIpRaw>(p, s);
    }
}

bool launch_scan_p4(const ScanParams &p, int metric, hipStream_t s) {
    switch (metric) {
        case MQVS_METRIC_L2: return launch_p4_any<MQVS_METRIC_L2>(p, s);
        case MQVS_METRIC_IP: return launch_p4_any<MQVS_METRIC_IP>(p, s);
        case MQVS_METRIC_COSINE: return launch_p4_any<MQVS_METRIC_COSINE>(p, s);
        default: return launch_p4_any<kMetricIpRaw>(p, s);
    }
}

}  // namespace mqvs
