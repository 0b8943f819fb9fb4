// kernels_bf16.hip -- bf16 MFMA pre-filter + exact fp32 re-rank (nq >= 20).
//
// The batch branch of the reference (faiss exhaustive_*_blas, nq >= 20) is a
// GEMM whose fp32 element the oracle restates as a sequential fma chain.  On
// gfx950 the f32 MFMA runs at 1/16 of the bf16 rate, so the whole part is
// first scanned with v_mfma_f32_32x32x16_bf16 on the bf16 rounding of rows and
// queries, and only rows that can still be in the top-k under a RIGOROUS bound
// on the bf16 error are re-computed exactly with the fp32 fma chain:
//
//   |ip_bf16 - ip_fp32chain| <= B = (2^-7 + 2^-16 + 2.04 d 2^-24) |x| |y|_max
//
// (element rounding 2^-8 on each side; fp32 accumulation of both sums, d
// terms each).  With a_k the k-th best approximate value among any row set,
// the true k-th exact value is within a_k +- B, so keeping every row whose
// approximate value is within 2B of a_k keeps every row of the exact top-k
// (ties included).  The final ids and distances come from the exact chain and
// are bit-identical to the fp32 path and to the oracle.
//
//   k_scan_bf16      128 rows x 128 queries per workgroup, 4 waves of 64x64;
//                    K staged 64 deep by LDS-DMA (global_load_lds_dwordx4)
//                    into an XOR-swizzled image (conflict-free ds_read_b128);
//                    PROBE / APPEND epilogues as the fp32 kernels, on the
//                    approximate value.
//   k_probe_select_wide  k-th best approximate value of the probe rows ->
//                    per-query APPEND threshold (k-th -/+ 2B) + candidates.
//   k_survivors      per query: k-th best approximate value among the
//                    candidates, keep those within 2B; their exact fp32
//                    chains are computed over the whole chip and sorted by
//                    the reference key (kernels_rerank.hip).
#include "select_common.h"

namespace mqvs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

// ---------------------------------------------------------------------------
__global__ void k_to_bf16(const float *src, int64_t rows, int d, int64_t sstride, uint16_t *hi, int64_t dpad) {
    const int64_t total = rows * dpad;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / dpad;
        const int c = (int)(e - r * dpad);
        hi[e] = c < d ? f32_to_bf16_rn(src[r * sstride + c]) : (uint16_t)0;
    }
}

void launch_to_bf16(const float *src, int64_t rows, int d, int64_t sstride, uint16_t *dst_hi, int64_t dpad,
                    hipStream_t s) {
    int64_t blocks = (rows * dpad + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) return;
    hipLaunchKernelGGL(k_to_bf16, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, d, sstride,
                       dst_hi, dpad);
}

// max_r sqrt(|y_r|^2) (non-negative floats: max of the bit patterns)
__global__ void k_max_norm(const float *norms2, int64_t n, unsigned *out) {
    unsigned m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float v = norms2[i];
        const unsigned u = (v == v) ? __builtin_bit_cast(unsigned, sqrtf(fmaxf(v, 0.f))) : 0x7F800000u;
        m = u > m ? u : m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned o = __shfl_xor(m, off);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

void launch_max_norm(const float *norms2, int64_t n, float *out_max, hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_max_norm, dim3((unsigned)blocks), dim3(256), 0, s, norms2, n,
                       (unsigned *)out_max);
}

// Per-query bound on |approx - exact| in the metric's raw value:
//   IP / cosine: B = c(d) * |x|max_over_used_variants * |y|max
//   L2 (BLAS):   raw = (xn + yn) - 2 ip -> 2 B + 2 ulp of the result
//   direct (nq < 20: the exact value is faiss's sequential product-then-add
//   formula, not the BLAS form): IP/cosine as above ((d+1) u |x||y| for the
//   sequential sum is inside the constants); L2 compares the BLAS-form
//   approximation with fl(sum (y-x)^2), so add the norms' rounding (d u each)
//   and the direct sum's own error ((d+3) u (|x|+|y|)^2 <= 2 (d+3) u top):
//   2 B + (3 d + 12) u top.
__global__ void k_query_bound(ScanParams p, int metric, int direct, const float *ynorm_max, const float *qrec,
                              const float *yrec, float *bq) {
    // one thread per query (|x| from the variants' norm records)
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= p.nq) return;
    const int nv = p.maxv <= 1 ? 1 : p.qmu[j] + p.qlam[j];
    float xmax = 0.f;
    const float ymax = *ynorm_max * (1.0f + 6e-8f * (float)p.d + 1e-6f);  // fp32 |y|^2 chain error
    const float du = (float)p.d * 5.9604645e-8f;
    float b;
    {
        // x.y - xh.yh = xh.ry + rx.yh + rx.ry (records: q[0] |xh|, q[1] |rx|,
        // q[6] |x|; Y the segment maxima); the MFMA sums d exact products, at
        // most 2 u relative per addition (2.04 d u |xh||yh|, covers
        // round-toward-zero; measured worst 95.5 u sum|p| at d = 768,
        // tools/mfma_acc_probe.hip, profiles/r02/probes/mfma_acc_probe.log); the exact
        // chain's own error 1.01 d u |x||y| + one ulp
        const float *Y = yrec;
        b = 0.f;
        for (int v = 0; v < nv; ++v) {
            const float *q = qrec + ((int64_t)j * p.maxv + v) * kMxRec;
            xmax = fmaxf(xmax, q[6]);
            const float trunc = q[0] * Y[1] + q[1] * Y[0] + q[1] * Y[1];
            const float bv = trunc + 2.04f * du * q[0] * Y[0] + 1.01f * du * q[6] * ymax + 1.2e-7f * q[6] * ymax;
            b = fmaxf(b, bv * 1.0001f);
        }
        b += 1e-30f;
    }
    if (metric == MQVS_METRIC_L2) {
        const float top = p.qnorms[j] * 1.0001f + ymax * ymax;
        const float rel = direct ? (3.0f * (float)p.d + 12.0f) * 5.9604645e-8f : 2.4e-7f;
        b = 2.0f * b + top * rel + 1e-30f;
        // the batch scan (kernels_p4.hip) starts its accumulation at -|y|^2 / 2
        // and forms fl(qn - 2 acc): the accumulation bound covers |y|^2 / 2
        // more per term, and the two final roundings
        b += 2.0f * 2.04f * du * 0.5f * ymax * ymax + 2.4e-7f * top;
    } else if (metric == MQVS_METRIC_COSINE) {
        b = b + 2.4e-7f;  // 1 - ip rounds; ties on 1-ip may differ in ip by one ulp of 1
    }
    if (!(b < 1e30f)) b = __builtin_inff();
    bq[j] = b;
}

void launch_query_bound(const ScanParams &p, int metric, const float *ynorm_max, const float *qrec,
                        const float *yrec, float *bq, hipStream_t s) {
    const int direct = !blas_formula(p);
    hipLaunchKernelGGL(k_query_bound, dim3((unsigned)((p.nq + 255) / 256)), dim3(256), 0, s, p, metric, direct, ynorm_max, qrec, yrec, bq);
}


// ---------------------------------------------------------------------------
// k-th best approximate value of each query's probe row -> its APPEND
// threshold (k-th -/+ 2B) and the probe rows that pass it (cand null: the
// threshold only -- the batch probe's per-half-tile maxima, kernels_p4.hip).  1024 threads per
// query, 16 values in flight per thread (float4 x 4) in every radix pass and
// in the append: the probe row (L2-resident) is read five times, never with
// one dependent load in flight per thread.
constexpr int kPsThreads = 1024;
constexpr int kPsKeep = 4;        // keys kept per thread for the threshold select
constexpr int kPsKeepMaxK = 256;  // k up to which the kept keys are selected (else full passes)

template <int METRIC>
__global__ __launch_bounds__(kPsThreads) void k_probe_select_wide(const float *probe, int64_t P, int64_t ld, int k,
                                                                  const float *bq, float *thr, int *cand_count,
                                                                  Cand *cand, int cap, const int32_t *row_list) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ uint32_t skeys[kPsKeep * kPsThreads];
    const int q = blockIdx.x, t = threadIdx.x;
    const float *row = probe + (int64_t)q * ld;
    // Each thread keeps its kPsKeep smallest keys in registers (one read of
    // the row), and the radix passes run over those 4096 keys in LDS: the
    // k-th smallest of a subset of the keys is an upper bound on the k-th of
    // all of them -- all a threshold needs -- and equal to it unless one
    // thread held more than kPsKeep of the k best (k 100 of 32768 values:
    // ~0.1 per thread).  Three passes over the row with an LDS atomic per
    // value took 17-27 us at nq 1.
    bool none = false;
    uint32_t prefix = 0;
    if (k <= kPsKeepMaxK) {
        uint32_t best[kPsKeep];
#pragma unroll
        for (int j = 0; j < kPsKeep; ++j) best[j] = 0xFFFFFFFFu;
        for_each_f4<kPsThreads>(row, P, [&](int64_t, float raw) {
            uint32_t key = okey<METRIC>(raw);
            if (key >= best[kPsKeep - 1]) return;
#pragma unroll
            for (int j = 0; j < kPsKeep; ++j) {  // sorted insertion; the largest falls off
                if (key < best[j]) {
                    const uint32_t o = best[j];
                    best[j] = key;
                    key = o;
                }
            }
        });
#pragma unroll
        for (int j = 0; j < kPsKeep; ++j) skeys[j * kPsThreads + t] = best[j];
        __syncthreads();
        const uint32_t sel = block_radix_select_mlp<kPsThreads, 3>([&](int64_t i) { return skeys[i]; },
                                                                  (int64_t)kPsKeep * kPsThreads, k, hist, sh);
        none = sel == 0xFFFFFFFEu;
        prefix = sel & ~0xFFu;
    } else {
        // large k: three passes over the row; the bound takes the low byte set
        // (an upper bound on the k-th key, as block_radix_select<3>)
        uint32_t mask = 0, kk = (uint32_t)k;
        for (int pass = 0; pass < 3; ++pass) {
            const int shift = 24 - 8 * pass;
            if (t < 256) hist[t] = 0;
            __syncthreads();
            RunHist rh;
            for_each_f4<kPsThreads>(row, P, [&](int64_t, float raw) {
                const uint32_t key = okey<METRIC>(raw);
                if (key != 0xFFFFFFFFu && (key & mask) == prefix) rh.add(hist, (key >> shift) & 255u);
            });
            rh.flush(hist);
            __syncthreads();
            hist_pick(hist, kk, pass == 0, sh);
            __syncthreads();
            if (sh[0]) {
                none = true;
                break;
            }
            prefix |= sh[1] << shift;
            mask |= 255u << shift;
            kk -= sh[2];
            __syncthreads();
        }
    }
    float tt;
    if (none)
        tt = (METRIC == MQVS_METRIC_L2) ? __builtin_inff() : -__builtin_inff();
    else
        tt = widen<METRIC>(okey_bound_value<METRIC>(prefix | 0xFFu), bq[q]);
    if (t == 0) thr[q] = tt;
    if (!cand) return;  // (the batch probe's maxima: threshold only)
    const int lane = t & 63;
    for_each_f4<kPsThreads>(row, P, [&](int64_t i, float raw) {
        const bool take = (METRIC == MQVS_METRIC_L2) ? (raw <= tt) : (raw >= tt);
        // one counter atomic per wave and value step (the lanes that take
        // get consecutive slots)
        const uint64_t m = __ballot(take);
        if (m == 0) return;
        const int leader = __ffsll((long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(&cand_count[q], __popcll(m));
        base = __shfl(base, leader);
        if (take) {
            const int pos = base + __popcll(m & ((1ull << lane) - 1));
            if (pos < cap) {
                Cand c;
                c.raw = raw;
                c.row = row_list ? (uint32_t)row_list[i] : (uint32_t)i;
                cand[(int64_t)q * cap + pos] = c;
            }
        }
    });
}

template <int M>
static void probe_select_approx_t(const float *probe, int64_t P, int64_t ld, int nq, int k,
                                  const float *bq, float *thr, int *cc, Cand *cand, int cap,
                                  const int32_t *row_list, hipStream_t s) {
    hipLaunchKernelGGL(k_probe_select_wide<M>, dim3(nq), dim3(kPsThreads), 0, s, probe, P, ld, k, bq, thr, cc, cand,
                       cap, row_list);
}

void launch_probe_select_approx(const float *probe, int64_t P, int64_t ld, int nq, int k,
                                int metric, const float *bq, float *thr, int *cand_count,
                                Cand *cand, int cand_cap, const int32_t *row_list, hipStream_t s) {
#define MQVS_PSA(M) probe_select_approx_t<M>(probe, P, ld, nq, k, bq, thr, cand_count, cand, cand_cap, row_list, s)
    switch (metric) {
        case MQVS_METRIC_L2: MQVS_PSA(MQVS_METRIC_L2); break;
        case MQVS_METRIC_IP: MQVS_PSA(MQVS_METRIC_IP); break;
        case MQVS_METRIC_COSINE: MQVS_PSA(MQVS_METRIC_COSINE); break;
        default: MQVS_PSA(kMetricIpRaw); break;
    }
#undef MQVS_PSA
}

// Survivors of the bound, per query (one workgroup each): the k-th best
// approximate value a_k among the candidates, then every candidate within 2B
// of it (widen) is compacted into surv[q * rs ...] (at most lcap; more sets
// overflow bit 4, fewer than the appended candidates' cap bit 1).  Stats:
// overflow[1] = max survivors, [2] = their sum, [3] = max candidates.
template <int METRIC>
__global__ __launch_bounds__(SEL_THREADS) void k_survivors(ScanParams p, const float *bq, int k, int *overflow,
                                                          uint32_t *surv, int *scnt, int lcap, int64_t rs) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh[4];
    __shared__ int s_cnt;
    const int q = blockIdx.x;
    int n = p.cand_count[q];
    if (n > p.cand_cap) {
        if (threadIdx.x == 0) atomicOr(overflow, 1);
        n = p.cand_cap;
    }
    const Cand *c = p.cand + (int64_t)q * p.cand_cap;
    // (a bound on the k-th key is enough: 3 radix passes, block_radix_select;
    // k <= 256: over the threads' 4 smallest keys, kept_kth_bound)
    __shared__ uint32_t skeys[4 * SEL_THREADS];
    auto keyof = [&](int64_t i) { return okey<METRIC>(c[i].raw); };
    const uint32_t th = k <= SEL_THREADS ? kept_kth_bound<SEL_THREADS, 4>(keyof, n, k, skeys, hist, sh)
                                         : block_radix_select_mlp<SEL_THREADS, 3>(keyof, n, k, hist, sh);
    float t;
    if (th == 0xFFFFFFFEu)
        t = (METRIC == MQVS_METRIC_L2) ? __builtin_inff() : -__builtin_inff();
    else
        t = widen<METRIC>(okey_bound_value<METRIC>(th), bq[q]);
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    uint32_t *out = surv + (int64_t)q * rs;
    for (int i = threadIdx.x; i < n; i += SEL_THREADS) {
        const Cand e = c[i];
        const bool take = (METRIC == MQVS_METRIC_L2) ? (e.raw <= t) : (e.raw >= t);
        if (take) {
            const int pos = atomicAdd(&s_cnt, 1);
            if (pos < lcap) out[pos] = e.row;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int m = s_cnt;
        atomicMax(overflow + 1, m);
        atomicAdd(overflow + 2, m);
        atomicMax(overflow + 3, n);
        if (m > lcap) atomicOr(overflow, 4);
        scnt[q] = m < lcap ? m : lcap;
    }
}

// Exact re-rank of the survivors (k_survivors -> k_exact_records over the
// whole chip -> k_sort_emit, kernels_rerank.hip).  rs: survivor / record
// slots per query (2 lcap when lcap > kSortCap: global_sort's second buffer).
void launch_rerank_select(const ScanParams &p, int metric, const float *bq, int k, int64_t id_offset,
                          int64_t *out_ids, float *out_dist, int *overflow, uint32_t *surv, int *scnt,
                          uint4 *recs, int lcap, int64_t rs, hipStream_t s, const int *fl, int *host_fl) {
    switch (metric) {
        case MQVS_METRIC_L2:
            hipLaunchKernelGGL(k_survivors<MQVS_METRIC_L2>, dim3(p.nq), dim3(SEL_THREADS), 0, s, p, bq, k, overflow,
                               surv, scnt, lcap, rs);
            break;
        case MQVS_METRIC_IP:
            hipLaunchKernelGGL(k_survivors<MQVS_METRIC_IP>, dim3(p.nq), dim3(SEL_THREADS), 0, s, p, bq, k, overflow,
                               surv, scnt, lcap, rs);
            break;
        case MQVS_METRIC_COSINE:
            hipLaunchKernelGGL(k_survivors<MQVS_METRIC_COSINE>, dim3(p.nq), dim3(SEL_THREADS), 0, s, p, bq, k,
                               overflow, surv, scnt, lcap, rs);
            break;
        default:
            hipLaunchKernelGGL(k_survivors<kMetricIpRaw>, dim3(p.nq), dim3(SEL_THREADS), 0, s, p, bq, k, overflow,
                               surv, scnt, lcap, rs);
            break;
    }
    launch_exact_rerank(p, metric, surv, scnt, rs, lcap, recs, k, id_offset, out_ids, out_dist, s, fl, host_fl);
}

}  // namespace mqvs
