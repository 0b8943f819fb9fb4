// kernels_bf16_scan.hip -- split-precision bf16 MFMA scan (the nq >= 20
// pre-filter of kernels_bf16.hip).
//
// SPLIT = 3: x = xh + xl (two bf16 roundings), x.y ~ xh.yh + (xh.yl + xl.yh),
// the hi product and the two cross products in SEPARATE fp32 accumulators,
// 3 v_mfma_f32_32x32x16_bf16 per 32x32x16 block-step (3/16 of the f32 MFMA
// cost).  Error vs the fp32 chain (kernels_bf16.hip, k_query_bound):
//   (3.1 2^-16 + 2.02 d 2^-24 + small) |x| |y|
// SPLIT = 1: hi planes only, bound (2^-7 + ...) |x| |y|.
//
// Tile: 128 rows x 128 queries per workgroup, 4 waves of 64 x 64 (2 x 2
// blocks of 32 x 32); K staged 32 bf16 deep (64 B per row per plane) by
// LDS-DMA into double-buffered planes {Y hi, Y lo, Q hi, Q lo} of 8 KiB each
// (64 KiB per workgroup, 2 workgroups per CU).  Chunk c (16 B) of image row r
// sits at slot c ^ ((r >> 2) & 3): one ds_read_b128 lane group (16 rows,
// distinct r mod 16) hits 16 distinct 16-B bank groups.
#include "mqvs_internal.h"

namespace mqvs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BS_K = 32;                       // bf16 per row per stage
constexpr int BS_ROWB = BS_K * 2;              // 64 B: 4 chunks of 16 B
constexpr int BS_PLANE = kMfmaRows * BS_ROWB;  // 8 KiB (rows == queries == 128)

__device__ inline int swz4(int r, int c) { return c ^ ((r >> 2) & 3); }

template <int METRIC, bool PROBE>
__device__ inline void emit_approx(const ScanParams &p, int j, int64_t row, bool valid, float raw) {
    if (PROBE) {
        p.probe[(int64_t)j * p.probe_ld + (row - p.row_begin)] = valid ? raw : __builtin_nanf("");
        return;
    }
    if (!valid) return;
    const float t = p.thr[j];
    const bool take = (METRIC == MQVS_METRIC_L2) ? (raw <= t) : (raw >= t);
    if (take) {
        const int pos = atomicAdd(&p.cand_count[j], 1);
        if (pos < p.cand_cap) {
            Cand c;
            c.raw = raw;
            c.row = (uint32_t)row;
            p.cand[(int64_t)j * p.cand_cap + pos] = c;
        }
    }
}

template <int METRIC, bool PROBE, int SPLIT>
__global__ __launch_bounds__(256, 2) void k_scan_bf16(ScanParams p) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][4][BS_PLANE];
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
    const int wr = w >> 1, wq = w & 1;
    const int h = lane >> 5, l32 = lane & 31;
    const int q0 = qb * kMfmaQ;

    if (ord < 0) {
        if (PROBE) {
            for (int i = t; i < kMfmaRows * kMfmaQ; i += 256) {
                const int64_t row = r0 + (i % kMfmaRows);
                const int j = q0 + i / kMfmaRows;
                if (row < r1 && j < p.nq) emit_approx<METRIC, true>(p, j, row, false, 0.f);
            }
        }
        return;
    }

    // LDS-DMA sources: wave w fills image rows [(w*2+i)*16, +16) of a plane
    // with one 1-KiB instruction per i; lane -> (row lane/4, slot lane%4)
    const uint16_t *src[4][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = (w * 2 + i) * 16 + (lane >> 2);
        const int c = swz4(r, lane & 3);
        int64_t gr = r0 + r;
        if (gr >= r1) gr = r0;  // padding rows: any valid row, results discarded
        src[0][i] = p.rows_hi + gr * p.dpad + c * 8;
        src[1][i] = (SPLIT == 3) ? p.rows_lo + gr * p.dpad + c * 8 : nullptr;
        int j = q0 + r;
        if (j >= p.nq) j = 0;
        const int64_t qo = ((int64_t)j * p.maxv + variant_of(p, j, ord)) * p.dpad + c * 8;
        src[2][i] = p.q_hi + qo;
        src[3][i] = (SPLIT == 3) ? p.q_lo + qo : nullptr;
    }
    auto issue = [&](int s, int bf) {
        const int64_t k0 = (int64_t)s * BS_K;
#pragma unroll
        for (int pl = 0; pl < 4; ++pl) {
            if (SPLIT == 1 && (pl & 1)) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                __builtin_amdgcn_global_load_lds((const void *)(src[pl][i] + k0),
                                                 (lds_void *)&lds[bf][pl][(w * 2 + i) * 16 * BS_ROWB],
                                                 16, 0, 0);
        }
    };

    f32x16 acc[2][2], cor[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            acc[i][j] = f32x16{0};
            cor[i][j] = f32x16{0};
        }
    const int nst = (int)(p.dpad / BS_K);
    int ra[2], rq[2];
    ra[0] = wr * 64 + l32;
    ra[1] = ra[0] + 32;
    rq[0] = wq * 64 + l32;
    rq[1] = rq[0] + 32;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        if (s + 1 < nst) issue(s + 1, (s + 1) & 1);
        const int bf = s & 1;
#pragma unroll
        for (int kk = 0; kk < BS_K / 16; ++kk) {
            const int c = 2 * kk + h;
            bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ah[i] = *reinterpret_cast<const bf16x8 *>(&lds[bf][0][ra[i] * BS_ROWB + swz4(ra[i], c) * 16]);
                bh[i] = *reinterpret_cast<const bf16x8 *>(&lds[bf][2][rq[i] * BS_ROWB + swz4(rq[i], c) * 16]);
                if (SPLIT == 3) {
                    al[i] = *reinterpret_cast<const bf16x8 *>(&lds[bf][1][ra[i] * BS_ROWB + swz4(ra[i], c) * 16]);
                    bl[i] = *reinterpret_cast<const bf16x8 *>(&lds[bf][3][rq[i] * BS_ROWB + swz4(rq[i], c) * 16]);
                }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    if (SPLIT == 3) {
                        cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], cor[i][j], 0, 0, 0);
                        cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], cor[i][j], 0, 0, 0);
                    }
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int qb2 = 0; qb2 < 2; ++qb2) {
            const int j = q0 + wq * 64 + qb2 * 32 + l32;
            if (j >= p.nq) continue;
            const float qn = (METRIC == MQVS_METRIC_L2) ? p.qnorms[j] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int il = wr * 64 + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int64_t row = r0 + il;
                if (row >= r1) continue;
                const float ip = (SPLIT == 3) ? acc[rb][qb2][r] + cor[rb][qb2][r] : acc[rb][qb2][r];
                float raw = ip;
                if (METRIC == MQVS_METRIC_L2) {
                    raw = (qn + p.row_norms[row]) - 2.0f * ip;
                    if (raw < 0) raw = 0;
                }
                emit_approx<METRIC, PROBE>(p, j, row, row_valid(p, row), raw);
            }
        }
}

template <int METRIC, bool PROBE>
static void launch_bf16_t(const ScanParams &p, int split, hipStream_t s) {
    const int64_t L = p.tiles * p.num_qblocks;
    if (L < 1) return;
    const int64_t grid = (L + 7) / 8 * 8;
    if (split == 3)
        hipLaunchKernelGGL((k_scan_bf16<METRIC, PROBE, 3>), dim3((unsigned)grid), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((k_scan_bf16<METRIC, PROBE, 1>), dim3((unsigned)grid), dim3(256), 0, s, p);
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
