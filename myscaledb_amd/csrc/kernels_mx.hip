// kernels_mx.hip -- MX pre-filter: bf16 main term + block-scaled fp6 cross
// terms (the nq >= 8 pre-filter of mqvs_search, split 6).
//
// The split-3 pre-filter (kernels_bf16_scan.hip) spends three bf16 MFMAs per
// block-step: xh.yh + xh.yl + xl.yh.  The two cross terms are ~2^-9 of the
// main one and need only a few bits, so here they run on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with fp6 e2m3 operands, which issues in the
// cycles of one v_mfma_f32_32x32x16_bf16 while covering 4x the K: the pair
// (hi, residual) of 32 columns is ONE K=64 MX operand,
//
//     A (rows)    lanes 0-31: yr6 (residual), lanes 32-63: yh6 (hi)
//     B (queries) lanes 0-31: xh6 (hi),       lanes 32-63: xr6 (residual)
//     sum over K = xh6.yr6 + xr6.yh6
//
// so a 32-column stage costs 2 bf16 + 1 MX MFMA per 32x32 block (split 3: 6
// bf16), half the matrix-pipe cycles, and streams 3.5 B per element (split 3: 4).
// Lane layout, bit packing and per-lane scales of the MX instruction were
// measured on the hardware (tools/mx_probe.hip): lane l holds A[l & 31][32 (l >> 5)
// + j] as 6-bit element j at bit 6j of its six VGPRs, with its own E8M0 scale.
//
// Quantisation (k_to_mx): h = bf16_rn(x), r = x - h (exact); each of h, r is
// scaled by one power of two per vector (E8M0, max |.| -> <= 7.5) and rounded
// to e2m3.  The error is bounded RIGOROUSLY from norms measured during the
// quantisation (fp64), not from a format model:
//     x.y - [xh.yh + xh6.yr6 + xr6.yh6]
//       = (xh - xh6).yr + xh6.(yr - yr6) + (xr - xr6).yh + xr6.(yh - yh6) + xr.yr
// and Cauchy-Schwarz on each product with the query's norms and the segment's
// per-norm maxima (k_query_bound, split 6).
//
// Planes are row-blocked: 16 vectors x 32 columns are contiguous (bf16 hi:
// 1 KiB, fp6: 768 B), so one LDS-DMA instruction (16 image rows) reads whole
// cache lines instead of 16 partial ones -- the scan is bound by the L2 ->
// LDS stream (tools/tune_bf16.py diagnostics: the MFMA-free variant takes 88%
// of the full kernel's time).  Vector u, stage s (columns 32s..32s+31):
//     hi  byte ((u >> 4) nst + s) 1024 + (u & 15) 64
//     fp6 byte ((u >> 4) nst + s)  768 + (u & 15) 48
// Each lane addresses its own vector, so gathered rows and tiles that do not
// start on a 16-row boundary stay correct (only less contiguous).
// fp6 piece of a vector per stage, 48 bytes:
//     [h0 bytes 0-15][h1 bytes 0-15][h0 bytes 16-23 | h1 bytes 16-23]
// (tail halves swapped when bit 4 of the vector index is set)
// (h0/h1 = the 24-byte packed halves), so a lane's operand is one 16-B chunk
// (dwords 0-3) + one 8-B piece (dwords 4-5) whatever its half.  In LDS each
// vector's 3 chunks sit in a 64-B image row at slots c ^ ((r >> 2) & 3) (slot 3
// unused: its LDS-DMA lane is masked off), like the bf16 planes.
#include <cstdio>
#include <cstdlib>

#include "mqvs_internal.h"
#include "scan_emit.h"

namespace mqvs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int MX_K = 32;       // columns per stage
constexpr int MX_BLK = 48;     // fp6 plane bytes per vector per 32 columns
constexpr int MX_RT = kBfRows; // rows per workgroup tile

// ---------------------------------------------------------------------------
// quantisation

// e2m3 code of t (|t| <= 7.5), round to nearest even; q = its value
__device__ inline uint32_t e2m3_rn(float t, float &q) {
    const float a = fabsf(t);
    uint32_t code;
    float v;
    if (a < 1.0f) {  // subnormal: m/8 (m = 8 rolls into the first normal binade)
        const float m = rintf(a * 8.0f);
        code = (uint32_t)m;
        v = m * 0.125f;
    } else {
        const int e = a >= 4.0f ? 2 : a >= 2.0f ? 1 : 0;
        const float m = rintf(ldexpf(a, 3 - e));  // [8, 16]; 16 rolls into the next binade
        code = ((uint32_t)(e + 1) << 3) + (uint32_t)(m - 8.0f);
        v = ldexpf(m, e - 3);
    }
    const bool neg = t < 0.0f;
    q = neg ? -v : v;
    return code | (neg ? 32u : 0u);
}

// smallest e in [-127, 127] with m <= 7.5 * 2^e
__device__ inline int mx_scale_exp(float m) {
    if (!(m > 0.0f)) return -127;
    int e = (int)ceilf(log2f(m / 7.5f));
    e = e < -127 ? -127 : e > 127 ? 127 : e;
    while (e < 127 && m > ldexpf(7.5f, e)) ++e;
    while (e > -127 && m <= ldexpf(7.5f, e - 1)) --e;
    return e;
}

// sqrt(s) rounded up to float
__device__ inline float sqrt_up(double s) { return (float)(sqrt(s) * (1.0 + 1e-7)); }

// source vector v -> plane vector u = (v % vgroup) vpad + v / vgroup (rows:
// vgroup 1; query variants [nq][maxv]: vgroup maxv, vpad nq rounded to 16,
// so the 16 queries of a block share a variant plane)
template <bool RES_FIRST>
__global__ __launch_bounds__(256) void k_to_mx(const float *src, int64_t rows, int d, int64_t sstride,
                                               int64_t dpad, int64_t vgroup, int64_t vpad, uint16_t *hi,
                                               uint8_t *x6, uint8_t *sc, float *rec, float *maxrec) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= rows) return;  // whole wave
    const float *x = src + v * sstride;
    const int nb = (int)(dpad / MX_K);
    const int64_t u = (v % vgroup) * vpad + v / vgroup;
    uint16_t *hu = hi + (u >> 4) * nb * 512 + (u & 15) * 32;
    uint8_t *xu = x6 + (u >> 4) * nb * 768 + (u & 15) * MX_BLK;
    float mh = 0.f, mr = 0.f;
    for (int64_t i = lane; i < dpad; i += 64) {
        const float xv = i < d ? x[i] : 0.f;
        const uint16_t hb = f32_to_bf16_rn(xv);
        const float hv = __builtin_bit_cast(float, (uint32_t)hb << 16);
        hu[(i >> 5) * 512 + (i & 31)] = hb;
        mh = fmaxf(mh, fabsf(hv));
        mr = fmaxf(mr, fabsf(xv - hv));
    }
    for (int off = 32; off > 0; off >>= 1) {
        mh = fmaxf(mh, __shfl_xor(mh, off));
        mr = fmaxf(mr, __shfl_xor(mr, off));
    }
    const int eh = mx_scale_exp(mh), er = mx_scale_exp(mr);
    double nx = 0, nh = 0, nr = 0, nh6 = 0, neh = 0, nr6 = 0, ner = 0;
    for (int b = lane; b < nb; b += 64) {
        uint32_t wh[6] = {0, 0, 0, 0, 0, 0}, wr[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int i = MX_K * b + j;
            const float xv = i < d ? x[i] : 0.f;
            const float hv = __builtin_bit_cast(float, (uint32_t)f32_to_bf16_rn(xv) << 16);
            const float rv = xv - hv;  // exact
            float qh, qr;
            const uint32_t ch = e2m3_rn(ldexpf(hv, -eh), qh);
            const uint32_t cr = e2m3_rn(ldexpf(rv, -er), qr);
            const double dqh = ldexp((double)qh, eh), dqr = ldexp((double)qr, er);
            nx += (double)xv * xv;
            nh += (double)hv * hv;
            nr += (double)rv * rv;
            nh6 += dqh * dqh;
            nr6 += dqr * dqr;
            neh += ((double)hv - dqh) * ((double)hv - dqh);
            ner += ((double)rv - dqr) * ((double)rv - dqr);
            const int bit = 6 * j, w = bit >> 5, o = bit & 31;
            wh[w] |= ch << o;
            wr[w] |= cr << o;
            if (o > 26) {
                wh[w + 1] |= ch >> (32 - o);
                wr[w + 1] |= cr >> (32 - o);
            }
        }
        const uint32_t *h0 = RES_FIRST ? wr : wh, *h1 = RES_FIRST ? wh : wr;
        uint4 *blk = reinterpret_cast<uint4 *>(xu + (int64_t)b * 768);
        blk[0] = make_uint4(h0[0], h0[1], h0[2], h0[3]);
        blk[1] = make_uint4(h1[0], h1[1], h1[2], h1[3]);
        // tails swap halves on bit 4 of the plane vector: image rows r and
        // r + 16 then read different banks (conflict-free 8-B tail reads)
        blk[2] = ((u >> 4) & 1) ? make_uint4(h1[4], h1[5], h0[4], h0[5]) : make_uint4(h0[4], h0[5], h1[4], h1[5]);
    }
    double acc[7] = {nh, nr, nh6, neh, nr6, ner, nx};
#pragma unroll
    for (int t = 0; t < 7; ++t)
        for (int off = 32; off > 0; off >>= 1) acc[t] += __shfl_xor(acc[t], off);
    if (lane == 0) {
        sc[v * 2 + 0] = (uint8_t)(127 + (RES_FIRST ? er : eh));
        sc[v * 2 + 1] = (uint8_t)(127 + (RES_FIRST ? eh : er));
        // record: |h| |r| |h6| |h - h6| |r6| |r - r6| |x| (each rounded up)
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const float f = sqrt_up(acc[t]);
            if (rec) rec[v * kMxRec + t] = f;
            if (maxrec) {
                // non-negative floats order as their bit patterns; NaN -> +inf
                const unsigned u = (f == f) ? __builtin_bit_cast(unsigned, f) : 0x7F800000u;
                atomicMax(reinterpret_cast<unsigned *>(maxrec) + t, u);
            }
        }
        if (rec) rec[v * kMxRec + 7] = 0.f;
    }
}

void launch_to_mx(const float *src, int64_t rows, int d, int64_t src_stride, int64_t dpad, int64_t vgroup,
                  int64_t vpad, bool res_first, uint16_t *hi, uint8_t *x6, uint8_t *sc, float *rec, float *maxrec,
                  hipStream_t s) {
    if (rows <= 0) return;
    const int64_t blocks = (rows + 3) / 4;
    if (res_first)
        hipLaunchKernelGGL(k_to_mx<true>, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, d, src_stride, dpad,
                           vgroup, vpad, hi, x6, sc, rec, maxrec);
    else
        hipLaunchKernelGGL(k_to_mx<false>, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, d, src_stride, dpad,
                           vgroup, vpad, hi, x6, sc, rec, maxrec);
}

// ---------------------------------------------------------------------------
// scan
//
// Workgroup tile 256 rows x QT queries (QT = 32 QB WQ), 4 x WQ waves of 64 rows
// x 32 QB queries, 32x32 blocks.  Stage = 32 columns, LDS image
// [Y hi | Y fp6 | Q hi | Q fp6], 16 image rows (1 KiB) per LDS-DMA instruction,
// double buffered.  VAR bits: 1 s_setprio(1) around the MFMA work, 2 next
// stage's LDS-DMA issue split between the two column halves.

__device__ inline int swz4(int r, int c) { return c ^ ((r >> 2) & 3); }

// Workgroup -> (row tile, query block); workgroups are dispatched round-robin
// over the 8 XCDs (b % 8).  xcd_mode 0: all query blocks of a row tile on one
// XCD (its L2 serves the row tile's re-reads; every XCD's L2 holds every
// query block); xcd_mode g > 0 (g divides 8, num_qblocks a multiple of g... see
// launch_mx_shape): XCD x takes query blocks x % g (+ multiples of g) only, so
// an XCD's L2 holds num_qblocks / g query blocks while a row tile is read by g
// XCDs (its other reads come from the Infinity Cache).
__device__ inline bool mx_tile_of(const ScanParams &p, int64_t b, int64_t &ti, int &qb) {
    const int64_t L = p.tiles * p.num_qblocks;
    const int g = p.xcd_mode;
    if (g <= 1) {
        const int64_t cpx = (L + 7) / 8;
        const int64_t l = (b % 8) * cpx + b / 8;  // query blocks of a row tile on one XCD
        if (l >= L) return false;
        ti = l / p.num_qblocks;
        qb = (int)(l % p.num_qblocks);
        return true;
    }
    // g XCD groups; group x % g covers query blocks x % g, x % g + g, ...;
    // the 8 / g XCDs of a group split the (row tile, block) pairs round-robin
    const int x = (int)(b % 8), grp = x % g, sub = x / g, per = 8 / g;
    const int64_t i = b / 8;
    const int nqb_g = (p.num_qblocks - grp + g - 1) / g;  // query blocks of this group
    const int64_t Lg = p.tiles * nqb_g;
    const int64_t l = i * per + sub;
    if (l >= Lg || nqb_g <= 0) return false;
    ti = l / nqb_g;
    qb = grp + (int)(l % nqb_g) * g;
    return true;
}

template <int METRIC, bool PROBE, int WQ, int QB, int VAR>
__global__ __launch_bounds__(256 * WQ) void k_scan_mx(ScanParams p) {
    constexpr bool PRIO = VAR & 1, SPLIT_ISSUE = VAR & 2;
    // diagnostic builds (MQVS_MX_TUNE only, WRONG results, timing only):
    // 256 no LDS-DMA after the first stage, 512 no MFMA (LDS reads kept live),
    // 1024 no per-stage load wait (barrier only), 2048 no epilogue, 4096 no
    // LDS fragment reads (with 512)
    constexpr bool NO_DMA = VAR & 256, NO_MFMA = VAR & 512, NO_WAIT = VAR & 1024, NO_EMIT = VAR & 2048,
                   NO_READ = VAR & 4096;
    constexpr int WR = 4;
    constexpr int NW = WR * WQ;
    constexpr int QT = 32 * QB * WQ;
    constexpr int GY = MX_RT / 16;  // 1-KiB groups per Y plane
    constexpr int GQ = QT / 16;     // 1-KiB groups per Q plane
    constexpr int G = 2 * (GY + GQ);
    constexpr int GPW = G / NW;
    static_assert(G % NW == 0, "stage groups must split evenly over the waves");
    constexpr int STAGE = G * 1024;
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][STAGE];

    const int64_t b = blockIdx.x;
    int64_t ti;
    int qb;
    if (!mx_tile_of(p, b, ti, qb)) return;
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
            for (int i = t; i < MX_RT * QT; i += 64 * NW) {
                const int64_t row = r0 + (i % MX_RT);
                const int j = q0 + i / MX_RT;
                if (row < r1 && j < p.nq) emit_approx<METRIC, true>(p, j, row, -1, false, 0.f);
            }
        }
        return;
    }

    const int nb = (int)(p.dpad / MX_K);
    // LDS-DMA sources: group g = w + i NW fills 16 image rows of one plane;
    // lane -> (image row lane / 4, slot lane % 4) holds chunk swz4(row, slot)
    const unsigned char *src[GPW];
    int adv[GPW];
    bool act[GPW];
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
        const int g = w + i * NW;
        int pl, rbase;  // 0 Y hi, 1 Y fp6, 2 Q hi, 3 Q fp6
        if (g < 2 * GY) {
            pl = g / GY;
            rbase = (g % GY) * 16;
        } else {
            pl = 2 + (g - 2 * GY) / GQ;
            rbase = ((g - 2 * GY) % GQ) * 16;
        }
        const int r = rbase + (lane >> 2);
        const int c = swz4(r, lane & 3);
        int64_t u;  // plane vector
        if (pl < 2) {
            const int64_t gp = r0 + r;
            u = gp < r1 ? row_at(p, gp) : -1;
            if (u < 0) u = row_at(p, r0);  // padding: any real row, results discarded
        } else {
            int j = q0 + r;
            if (j >= p.nq) j = 0;
            u = (int64_t)variant_of(p, j, ord) * p.q_vpad + j;
        }
        if (pl == 0 || pl == 2) {
            const uint16_t *h = pl == 0 ? p.rows_hi : p.q_hi;
            src[i] = reinterpret_cast<const unsigned char *>(h) + ((u >> 4) * nb * 1024 + (u & 15) * 64 + c * 16);
            adv[i] = 1024;
            act[i] = true;
        } else {
            const uint8_t *x6 = pl == 1 ? p.rows_x6 : p.q_x6;
            src[i] = x6 + ((u >> 4) * nb * 768 + (u & 15) * MX_BLK + (c < 3 ? c : 0) * 16);
            adv[i] = 768;
            act[i] = c < 3;
        }
    }
    auto issue = [&](int s, int bf, int i0, int i1) {
        if (NO_DMA && s > 0) return;
#pragma unroll
        for (int i = 0; i < GPW; ++i)
            if (i >= i0 && i < i1 && act[i])
                __builtin_amdgcn_global_load_lds((const void *)(src[i] + (int64_t)s * adv[i]),
                                                 (lds_void *)&lds[bf][(w + i * NW) * 1024], 16, 0, 0);
    };
    auto issue_part = [&](bool more, int s, int part) {
        if (!SPLIT_ISSUE || !more) return;
        __builtin_amdgcn_sched_barrier(0);
        issue(s + 1, (s + 1) & 1, part * (GPW / 2), part == 0 ? GPW / 2 : GPW);
        __builtin_amdgcn_sched_barrier(0);
    };

    constexpr int OFF_YH = 0;
    constexpr int OFF_Y6 = GY * 1024;
    constexpr int OFF_QH = 2 * GY * 1024;
    constexpr int OFF_Q6 = OFF_QH + GQ * 1024;
    const int h = lane >> 5, l32 = lane & 31;
    auto frag = [&](const unsigned char *st, int off, int r, int c) {
        return *reinterpret_cast<const bf16x8 *>(st + off + r * 64 + swz4(r, c) * 16);
    };
    auto frag6 = [&](const unsigned char *st, int off, int r, int toff) {
        const unsigned char *rp = st + off + r * 64;
        const uint4 lo = *reinterpret_cast<const uint4 *>(rp + swz4(r, h) * 16);
        const uint2 tl = *reinterpret_cast<const uint2 *>(rp + swz4(r, 2) * 16 + toff);
        i32x8 v;
        v[0] = (int)lo.x;
        v[1] = (int)lo.y;
        v[2] = (int)lo.z;
        v[3] = (int)lo.w;
        v[4] = (int)tl.x;
        v[5] = (int)tl.y;
        v[6] = 0;
        v[7] = 0;
        return v;
    };

    const int ra0 = wr * 64 + l32;
    const int rq0 = wq * 32 * QB + l32;
    // E8M0 scales of this lane's operand halves (one per vector and half) and
    // the byte offset of its half's tail inside the tail chunk
    int ysc[2], qsc[QB], ytoff[2], qtoff[QB];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int64_t gp = r0 + ra0 + 32 * i;
        int64_t vec = gp < r1 ? row_at(p, gp) : -1;
        if (vec < 0) vec = row_at(p, r0);
        ysc[i] = p.rows_sc[vec * 2 + h];
        ytoff[i] = 8 * (h ^ (int)((vec >> 4) & 1));
    }
#pragma unroll
    for (int jb = 0; jb < QB; ++jb) {
        int j = q0 + rq0 + 32 * jb;
        if (j >= p.nq) j = 0;
        const int var = variant_of(p, j, ord);
        qsc[jb] = p.q_sc[((int64_t)j * p.maxv + var) * 2 + h];
        qtoff[jb] = 8 * (h ^ (int)((((int64_t)var * p.q_vpad + j) >> 4) & 1));
    }

    f32x16 acc[2][QB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jb = 0; jb < QB; ++jb) acc[i][jb] = f32x16{0};

    const int nst = (int)(p.dpad / MX_K);
    issue(0, 0, 0, GPW);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        const bool more = s + 1 < nst;
        if (!SPLIT_ISSUE && more) issue(s + 1, (s + 1) & 1, 0, GPW);
        const unsigned char *st = lds[s & 1];
        if (PRIO) __builtin_amdgcn_s_setprio(1);
        i32x8 ya[2], qx[QB];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int c = 2 * kk + h;
            if constexpr (NO_READ) {
                issue_part(more, s, kk);
                acc[kk][0][0] += (float)c;
                continue;
            }
            bf16x8 ah[2], bh[QB];
#pragma unroll
            for (int i = 0; i < 2; ++i) ah[i] = frag(st, OFF_YH, ra0 + 32 * i, c);
#pragma unroll
            for (int jb = 0; jb < QB; ++jb) bh[jb] = frag(st, OFF_QH, rq0 + 32 * jb, c);
            if (kk == 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i) ya[i] = frag6(st, OFF_Y6, ra0 + 32 * i, ytoff[i]);
#pragma unroll
                for (int jb = 0; jb < QB; ++jb) qx[jb] = frag6(st, OFF_Q6, rq0 + 32 * jb, qtoff[jb]);
            }
            issue_part(more, s, kk);
            if constexpr (NO_MFMA) {
                // keep the fragment reads live with one VALU op per register
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jb = 0; jb < QB; ++jb) {
                        typedef int i32x4 __attribute__((ext_vector_type(4)));
                        const i32x4 a = __builtin_bit_cast(i32x4, ah[i]) ^ __builtin_bit_cast(i32x4, bh[jb]);
                        acc[i][jb][jb] += (float)(a[0] ^ a[1] ^ a[2] ^ a[3] ^ ya[kk][jb & 3] ^ qx[jb][i]);
                    }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jb = 0; jb < QB; ++jb)
                    acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[jb], acc[i][jb], 0, 0, 0);
#pragma unroll
            for (int jb = 0; jb < QB; ++jb)
                acc[kk][jb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ya[kk], qx[jb], acc[kk][jb], 2, 2, 0,
                                                                              ysc[kk], 0, qsc[jb]);
        }
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (!NO_WAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if constexpr (NO_EMIT) {  // every accumulator stays live
        float sacc = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jb = 0; jb < QB; ++jb)
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc += acc[i][jb][r];
        if (sacc == 1.2345f && p.dbg) p.dbg[0] = 1;
        return;
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

template <int METRIC, bool PROBE, int WQ, int QB, int VAR>
static void launch_mx_shape(ScanParams p, hipStream_t s) {
    constexpr int QT = 32 * QB * WQ;
    p.num_qblocks = (p.nq + QT - 1) / QT;
    const int64_t L = p.tiles * p.num_qblocks;
    if (L < 1) return;
    int64_t grid = (L + 7) / 8 * 8;
    // XCD grouping (experimental, MQVS_MX_XCD=g with g in {2, 4, 8})
    p.xcd_mode = 0;
    if (const char *e = tune_env("MQVS_MX_XCD")) {
        const int g = std::atoi(e);
        if ((g == 2 || g == 4 || g == 8) && p.num_qblocks >= g) {
            p.xcd_mode = g;
            const int per = 8 / g;
            const int64_t nqb_max = (p.num_qblocks + g - 1) / g;
            grid = (p.tiles * nqb_max + per - 1) / per * 8;
        }
    }
    hipLaunchKernelGGL((k_scan_mx<METRIC, PROBE, WQ, QB, VAR>), dim3((unsigned)grid), dim3(256 * WQ), 0, s, p);
}

// Tuning override (tools/tune_bf16.py): MQVS_MX_TUNE="WQ,QB,VAR"
template <int METRIC, bool PROBE>
static bool launch_mx_tuned(const ScanParams &p, hipStream_t s) {
    const char *e = tune_env("MQVS_MX_TUNE");
    int wq, qb, var;
    if (!e || !*e || std::sscanf(e, "%d,%d,%d", &wq, &qb, &var) != 3) return false;
    switch ((wq * 10 + qb) * 1000 + var) {
#define MQVS_MX_CASE(WQ_, QB_, V_) \
    case (WQ_ * 10 + QB_) * 1000 + V_: launch_mx_shape<METRIC, PROBE, WQ_, QB_, V_>(p, s); return true;
        MQVS_MX_CASE(2, 4, 0) MQVS_MX_CASE(2, 4, 1) MQVS_MX_CASE(2, 4, 2) MQVS_MX_CASE(2, 4, 3)
        MQVS_MX_CASE(2, 2, 0) MQVS_MX_CASE(2, 2, 3) MQVS_MX_CASE(2, 1, 0) MQVS_MX_CASE(2, 1, 3)
        MQVS_MX_CASE(2, 4, 259) MQVS_MX_CASE(2, 4, 515) MQVS_MX_CASE(2, 4, 1027) MQVS_MX_CASE(2, 4, 1539)
        MQVS_MX_CASE(2, 4, 2051) MQVS_MX_CASE(2, 4, 2563) MQVS_MX_CASE(2, 4, 6659) MQVS_MX_CASE(2, 4, 2307)
        MQVS_MX_CASE(2, 4, 6915)
#undef MQVS_MX_CASE
        default: return false;
    }
}

template <int METRIC, bool PROBE>
static void launch_mx_t(const ScanParams &p, hipStream_t s) {
    if constexpr (METRIC == MQVS_METRIC_COSINE && !PROBE)
        if (launch_mx_tuned<METRIC, PROBE>(p, s)) return;
    if (p.nq <= 64)
        launch_mx_shape<METRIC, PROBE, 2, 1, 3>(p, s);
    else if (p.nq <= 128)
        launch_mx_shape<METRIC, PROBE, 2, 2, 3>(p, s);
    else
        launch_mx_shape<METRIC, PROBE, 2, 4, 3>(p, s);
}

void launch_scan_mx(const ScanParams &p, int metric, bool probe, hipStream_t s) {
    switch (metric) {
        case MQVS_METRIC_L2:
            probe ? launch_mx_t<MQVS_METRIC_L2, true>(p, s) : launch_mx_t<MQVS_METRIC_L2, false>(p, s);
            break;
        case MQVS_METRIC_IP:
            probe ? launch_mx_t<MQVS_METRIC_IP, true>(p, s) : launch_mx_t<MQVS_METRIC_IP, false>(p, s);
            break;
        case MQVS_METRIC_COSINE:
            probe ? launch_mx_t<MQVS_METRIC_COSINE, true>(p, s) : launch_mx_t<MQVS_METRIC_COSINE, false>(p, s);
            break;
        default:
            probe ? launch_mx_t<kMetricIpRaw, true>(p, s) : launch_mx_t<kMetricIpRaw, false>(p, s);
            break;
    }
}

}  // namespace mqvs
