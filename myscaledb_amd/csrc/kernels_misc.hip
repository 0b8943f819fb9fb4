// kernels_misc.hip -- segment preparation, query preparation and helpers.
#include "mqvs_internal.h"

namespace mqvs {

constexpr int NB_K = 32;
constexpr int NB_LD = NB_K + 4;

// Per-row squared norm, sequential fp32 with the product rounded then added
// (VectorDataset.h:105-108 for normalize; fvec_norm_L2sqr for the BLAS branch
// norms, the same order the KATs pin for fvec_*).  Rows staged through LDS so
// the HBM reads stay coalesced while each lane walks its own row in order.
__device__ void block_row_sumsq(const float *rows, int64_t r0, int64_t r1, int d,
                                float (*tile)[256 * NB_LD], float &sum) {
    const int t = threadIdx.x;
    sum = 0.0f;
    const int nst = (d + NB_K - 1) / NB_K;
    for (int s = 0; s < nst; ++s) {
        const int k0 = s * NB_K;
        for (int i = 0; i < 8; ++i) {
            const int f = t + 256 * i;
            const int lr = f >> 3, c = (f & 7) * 4;
            const int64_t gr = r0 + lr;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gr < r1) {
                const float *src = rows + gr * d + k0 + c;
                if (k0 + c + 0 < d) v.x = src[0];
                if (k0 + c + 1 < d) v.y = src[1];
                if (k0 + c + 2 < d) v.z = src[2];
                if (k0 + c + 3 < d) v.w = src[3];
            }
            *reinterpret_cast<float4 *>(&tile[0][lr * NB_LD + c]) = v;
        }
        __syncthreads();
        const float *tl = &tile[0][t * NB_LD];
        const int lim = (d - k0) < NB_K ? (d - k0) : NB_K;
        for (int kk = 0; kk < lim; ++kk) sum = sum + tl[kk] * tl[kk];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_row_norms(const float *rows, int64_t n, int d,
                                                    float *norms) {
    __shared__ __attribute__((aligned(16))) float tile[1][256 * NB_LD];
    for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < n; r0 += (int64_t)gridDim.x * 256) {
        const int64_t r1 = r0 + 256 < n ? r0 + 256 : n;
        float sum;
        block_row_sumsq(rows, r0, r1, d, tile, sum);
        if (r0 + threadIdx.x < r1) norms[r0 + threadIdx.x] = sum;
    }
}

// VectorDataset<Float>::normalize (VectorDataset.h:98-117), in place.
__global__ __launch_bounds__(256) void k_normalize_rows(float *rows, int64_t n, int d) {
    __shared__ __attribute__((aligned(16))) float tile[1][256 * NB_LD];
    __shared__ float scale[256];
    const float eps = 1.1920929e-07f;  // FLT_EPSILON
    for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < n; r0 += (int64_t)gridDim.x * 256) {
        const int64_t r1 = r0 + 256 < n ? r0 + 256 : n;
        float sum;
        block_row_sumsq(rows, r0, r1, d, tile, sum);
        // 0 marks "skip" (sum < FLT_EPSILON): the row is left untouched
        scale[threadIdx.x] = (sum < eps) ? 0.0f : sqrtf(sum);
        __syncthreads();
        const int64_t cnt = (r1 - r0) * d;
        float *base = rows + r0 * d;
        for (int64_t i = threadIdx.x; i < cnt; i += 256) {
            const float s = scale[i / d];
            if (s != 0.0f) base[i] = base[i] / s;
        }
        __syncthreads();
    }
}

void launch_row_norms(const float *rows, int64_t n, int d, float *norms, hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) return;
    hipLaunchKernelGGL(k_row_norms, dim3((unsigned)blocks), dim3(256), 0, s, rows, n, d, norms);
}

void launch_normalize_rows(float *rows, int64_t n, int d, hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) return;
    hipLaunchKernelGGL(k_normalize_rows, dim3((unsigned)blocks), dim3(256), 0, s, rows, n, d);
}

// Query preparation, one wave per query.  L2/IP: variant 0 = the query,
// qnorm = |q|^2 (BLAS branch).  Cosine: the reference normalises the SAME
// query object once per searched granule chunk (VIWithDataPart.h:358 on the
// dataset shared across chunks, MergeTreeVSManager.cpp:1279-1292,1473-1486),
// so chunk ordinal c uses normalize^(c+1)(q).  Variants are generated until a
// repeat: variants [0, mu) are the transient, [mu, mu+lam) the cycle.
//
// The sums are sequential fp32 (product rounded, then added: the order of
// VectorDataset::normalize / fvec_norm_L2sqr), a 768-long dependent chain per
// normalisation.  Lane l holds elements l + 64 j in registers (J slots); the
// chain walks them with v_readlane into the wave-uniform accumulator, so it
// costs one readlane + one add per element instead of an LDS round trip.
// J = 0: generic d (elements in LDS, lane 0 walks them).
// sum_{i<d} x_i^2, sequential fp32 (x_i held by lane i % 64, slot i / 64).
// Padding elements (i >= d) hold 0 and add +0.0f, which leaves the
// non-negative running sum bit-identical, so every slot walks all 64 lanes
// without branches; readlanes go 16 at a time ahead of their adds.
template <int J>
__device__ __forceinline__ float seq_sq_sum(const float (&x)[J], int d) {
    (void)d;
    float acc = 0.0f;
#pragma unroll
    for (int u = 0; u < J; ++u) {
        const int sq = __builtin_bit_cast(int, x[u] * x[u]);
#pragma unroll
        for (int l0 = 0; l0 < 64; l0 += 16) {
            float t[16];
#pragma unroll
            for (int l = 0; l < 16; ++l) t[l] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(sq, l0 + l));
#pragma unroll
            for (int l = 0; l < 16; ++l) acc = acc + t[l];
        }
    }
    return acc;
}

// The same sum through LDS: the rounded products are stored once, and every
// lane walks them in order from 16-B broadcast reads (4 elements per read;
// the reads run ahead of the dependent adds).  Same order, same bits.
template <int J>
__device__ __forceinline__ float seq_sq_sum_lds(const float (&x)[J], float *prod) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < J; ++u) prod[lane + 64 * u] = x[u] * x[u];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the stores landed (one wave)
    __builtin_amdgcn_wave_barrier();
    float acc = 0.0f;
    const float4 *p4 = reinterpret_cast<const float4 *>(prod);
#pragma unroll 8
    for (int i = 0; i < 16 * J; ++i) {
        const float4 v = p4[i];
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
    }
    __builtin_amdgcn_wave_barrier();  // (the next step rewrites prod)
    return acc;
}

// The same walk software-pipelined: the 16-B reads of block b + 1 are issued
// before the adds of block b, so the dependent add chain never waits on LDS
// latency (the plain loop above issues a block's reads only after the previous
// block's adds).  Same order, same bits.
template <int J>
__device__ __forceinline__ float seq_sq_sum_lds_pipe(const float (&x)[J], float *prod) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < J; ++u) prod[lane + 64 * u] = x[u] * x[u];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    constexpr int B = 4;              // float4 reads per block
    constexpr int NB = 16 * J / B;    // blocks
    const float4 *p4 = reinterpret_cast<const float4 *>(prod);
    float4 cur[B], nxt[B];
#pragma unroll
    for (int i = 0; i < B; ++i) cur[i] = p4[i];
    float acc = 0.0f;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b + 1 < NB) {
#pragma unroll
            for (int i = 0; i < B; ++i) nxt[i] = p4[(b + 1) * B + i];
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
            acc = acc + cur[i].x;
            acc = acc + cur[i].y;
            acc = acc + cur[i].z;
            acc = acc + cur[i].w;
        }
#pragma unroll
        for (int i = 0; i < B; ++i) cur[i] = nxt[i];
    }
    __builtin_amdgcn_wave_barrier();
    return acc;
}

// The same sum from registers: the rounded products go through LDS once and
// lane L < 8 loads elements [8 J L, 8 J (L + 1)) into its registers (2 J
// 16-B reads, all issued up front); then eight phases of 8 J dependent adds,
// phase L continuing the running sum of phase L - 1 (readlane broadcast) with
// lane L's elements.  The add chain never waits on LDS (the walk above
// re-reads LDS for every 4 elements); same order, same bits.
template <int J>
__device__ __forceinline__ float seq_sq_sum_lanes(const float (&x)[J], float *prod) {
    constexpr int NL = 8, PL = 8 * J;  // lanes, elements per lane (64 J = NL PL)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < J; ++u) prod[lane + 64 * u] = x[u] * x[u];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the stores landed (one wave)
    __builtin_amdgcn_wave_barrier();
    const float4 *p4 = reinterpret_cast<const float4 *>(prod + (lane < NL ? lane : 0) * PL);
    float v[PL];
#pragma unroll
    for (int j = 0; j < PL / 4; ++j) {
        const float4 t = p4[j];
        v[4 * j] = t.x;
        v[4 * j + 1] = t.y;
        v[4 * j + 2] = t.z;
        v[4 * j + 3] = t.w;
    }
    // (every read issued before the first add: left to itself the compiler
    // sinks the reads into phase 0, two at a time, each pair waited for)
    __builtin_amdgcn_sched_barrier(0);
    float acc = 0.0f;
#pragma unroll
    for (int L = 0; L < NL; ++L) {
#pragma unroll
        for (int i = 0; i < PL; ++i) acc = acc + v[i];
        acc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, acc), L));
    }
    __builtin_amdgcn_wave_barrier();  // (the next step rewrites prod)
    return acc;
}

// J > 0: d <= 64 J, the query in registers.
// phase 0: everything.  Cosine searches whose first consumers need only
// variant 0 split the work: phase 1 writes variant 0 (and |q|^2 = 0); phase 2,
// launched after it (on a side stream, concurrent with the coarse step and the
// list scan), walks the rest of the chain -- it compares against the stored
// variant 0 but does not rewrite it -- and writes mu, lambda and the status.
// SUMV: 0 = readlane walk (seq_sq_sum), 1 = LDS broadcast walk
// (seq_sq_sum_lds: 39.0 -> 35.5 us at nq 1, 72.5 -> 65.7 us at nq 1000 for
// d = 768), 2 = that walk software-pipelined (slower: 45 us), 3 = register
// phases (seq_sq_sum_lanes, the launcher's); bit-identical tables,
// tools/qprep_sum_ab.hip, profiles/r05/qprep_sum_ab.jsonl
constexpr int kLaneSigMax = 32;  // variants whose per-lane signatures fit LDS (33 x 256 B)
// qdelta (may be null; cosine): per query an upper bound on the largest
// |x_v - x_0| over the variants the chain produces (the index re-rank's bound
// pruning compares exact values of variant x_v with variant-0 approximations):
// per lane the largest fp64 partial sum of squares over the variants, summed
// over the lanes (a sum of maxima bounds the maximum of sums), rounded up.
template <int J, int SUMV = 0, bool LANESIG = false>
__global__ __launch_bounds__(64) void k_query_prep(const float *q, int nq, int d, int metric, int blas, float *qvars,
                                                   int maxv, float *qnorms, int *qmu, int *qlam, int *status,
                                                   int phase, float *qdelta) {
    __shared__ __attribute__((aligned(16))) float prod[SUMV ? 64 * J : 1];
    auto sqsum = [&](const float(&xx)[J]) -> float {
        if constexpr (SUMV == 3)
            return seq_sq_sum_lanes<J>(xx, prod);
        else if constexpr (SUMV == 2)
            return seq_sq_sum_lds_pipe<J>(xx, prod);
        else if constexpr (SUMV == 1)
            return seq_sq_sum_lds<J>(xx, prod);
        else
            return seq_sq_sum<J>(xx, 0);
    };
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t qs = (int64_t)((d + 31) / 32 * 32);
    const float *src = q + (int64_t)j * d;
    float *v0 = qvars + (int64_t)j * maxv * qs;
    float x[J];
#pragma unroll
    for (int u = 0; u < J; ++u) {
        const int i = lane + 64 * u;
        x[u] = i < d ? src[i] : 0.0f;
    }
    if (metric != MQVS_METRIC_COSINE) {
        if (phase == 2) return;
        if (qdelta && lane == 0) qdelta[j] = 0.0f;
        // (columns d .. qs: zeros; the table is not cleared beforehand and
        // the padded readers take them)
#pragma unroll
        for (int u = 0; u < J; ++u)
            if (lane + 64 * u < qs) v0[lane + 64 * u] = x[u];
        const float sum = blas ? sqsum(x) : 0.0f;
        if (lane == 0) {
            if (qnorms) qnorms[j] = sum;
            qmu[j] = 0;
            qlam[j] = 1;
        }
        return;
    }
    const float eps = 1.1920929e-07f;
    // variants 0..maxv-1 are stored; normalisation maxv is only compared, so a
    // fixed point reached at the last stored variant is still detected.  A
    // repeat is found by a signature of each variant; only a signature match
    // is confirmed element by element.  LANESIG (maxv <= kLaneSigMax): a 32-bit
    // hash per lane, kept per variant in LDS and matched with one vote (no
    // cross-lane reduction: 0.3 -> ~0.05 us per normalisation); else one 64-bit
    // hash per variant, wave-reduced.
    extern __shared__ uint64_t sig[];  // LANESIG: [maxv + 1][64] uint32; else maxv + 1 uint64
    uint32_t *lsig = reinterpret_cast<uint32_t *>(sig);
    float x0[J];
    double dl = 0.0;
    auto put_delta = [&]() {
        if (!qdelta) return;
        double t = dl;
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0) qdelta[j] = (float)(sqrt(t) * (1.0 + 1e-6)) + 1e-30f;
    };
    for (int v = 0; v <= maxv; ++v) {
        const float sum = sqsum(x);
        if (!(sum < eps)) {
            const float sr = sqrtf(sum);
#pragma unroll
            for (int u = 0; u < J; ++u) x[u] = x[u] / sr;
        }
        if (qdelta) {
            if (v == 0) {
#pragma unroll
                for (int u = 0; u < J; ++u) x0[u] = x[u];
            } else {
                double ss = 0.0;
#pragma unroll
                for (int u = 0; u < J; ++u) {
                    const double e = (double)x[u] - (double)x0[u];
                    ss += e * e;
                }
                dl = ss > dl ? ss : dl;
            }
        }
        if (v < maxv && (phase != 2 || v > 0)) {
            float *cur = v0 + (int64_t)v * qs;
            if (64 * J == qs) {
                // every slot in range: one address, immediate offsets (the
                // per-slot predicate below makes the compiler rebuild the
                // address before each store and wait for the previous store:
                // ~1 us per normalisation)
#pragma unroll
                for (int u = 0; u < J; ++u) cur[lane + 64 * u] = x[u];
            } else {
#pragma unroll
                for (int u = 0; u < J; ++u)
                    if (lane + 64 * u < qs) cur[lane + 64 * u] = x[u];  // (x = 0 past d)
            }
        }
        if (phase == 1) {
            if (lane == 0 && qnorms) qnorms[j] = 0.0f;
            return;
        }
        uint64_t h = 0;
        uint32_t hl = 0x811C9DC5u;
        if constexpr (LANESIG) {
#pragma unroll
            for (int u = 0; u < J; ++u) {
                const uint32_t b = __builtin_bit_cast(uint32_t, x[u]);
                hl = ((hl << 5) | (hl >> 27)) ^ (b + 0x9E3779B9u * (uint32_t)(u + 1));
            }
            if (v < maxv) lsig[v * 64 + lane] = hl;
            __builtin_amdgcn_wave_barrier();  // (one wave: its LDS ops complete in order)
        } else {
#pragma unroll
            for (int u = 0; u < J; ++u) {
                const uint64_t b = __builtin_bit_cast(uint32_t, x[u]);
                h += (b + 0x9E3779B97F4A7C15ull * (uint64_t)(u + 1)) * (b | 1ull) ^ (b << 29);
            }
            for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off);
            if (v < maxv && lane == 0) sig[v] = h;
            __syncthreads();
        }
        for (int u = 0; u < v; ++u) {
            if constexpr (LANESIG) {
                if (!__all(lsig[u * 64 + lane] == hl)) continue;
            } else if (sig[u] != h) {
                continue;
            }
            const float *o = v0 + (int64_t)u * qs;
            bool eq = true;
#pragma unroll
            for (int w = 0; w < J; ++w)
                if (lane + 64 * w < d)
                    eq = eq && __builtin_bit_cast(uint32_t, o[lane + 64 * w]) == __builtin_bit_cast(uint32_t, x[w]);
            if (__all(eq)) {
                if (lane == 0) {
                    qmu[j] = u;
                    qlam[j] = v - u;
                    if (qnorms) qnorms[j] = 0.0f;
                }
                // the variants past the chain are never selected, but the bf16
                // plane and the bound read every stored one: zeros (the table
                // is not cleared beforehand)
                // (16-B stores: variants are 128-B aligned, qs a multiple of 32)
                float4 *z = reinterpret_cast<float4 *>(v0 + (int64_t)v * qs);
                const int64_t n4 = (int64_t)(maxv - v) * qs / 4;
                for (int64_t i = lane; i < n4; i += 64) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
                put_delta();
                return;
            }
        }
    }
    put_delta();
    if (lane == 0) {
        // no repeat within maxv + 1 normalisations: variants 0..maxv-1 are
        // exact, later chunk ordinals are not (the host fails the search if
        // the part has that many searched chunks)
        atomicOr(status, 1);
        qmu[j] = maxv - 1;
        qlam[j] = 1;
        if (qnorms) qnorms[j] = 0.0f;
    }
}

// generic d: elements in LDS, lane 0 walks the sequential sums
// (phase 1 does everything here, phase 2 nothing)
__global__ __launch_bounds__(64) void k_query_prep_lds(const float *q, int nq, int d, int metric, int blas,
                                                       float *qvars, int maxv, float *qnorms, int *qmu, int *qlam,
                                                       int *status, int phase, float *qdelta) {
    if (phase == 2) return;
    extern __shared__ __attribute__((aligned(16))) float qbuf[];
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t qs = (int64_t)((d + 31) / 32 * 32);
    const float *src = q + (int64_t)j * d;
    float *v0 = qvars + (int64_t)j * maxv * qs;
    for (int i = lane; i < d; i += 64) qbuf[i] = src[i];
    __syncthreads();
    // qdelta as k_query_prep's, from the stored variants [1, nv)
    auto put_delta = [&](int nv) {
        if (!qdelta) return;
        double dl = 0.0;
        for (int v = 1; v < nv; ++v) {
            double ss = 0.0;
            for (int i = lane; i < d; i += 64) {
                const double e = (double)v0[(int64_t)v * qs + i] - (double)v0[i];
                ss += e * e;
            }
            dl = ss > dl ? ss : dl;
        }
        for (int off = 32; off > 0; off >>= 1) dl += __shfl_xor(dl, off);
        if (lane == 0) qdelta[j] = (float)(sqrt(dl) * (1.0 + 1e-6)) + 1e-30f;
    };
    auto seqsum = [&]() -> float {
        if (lane == 0) {
            float s = 0.0f;
#pragma unroll 8
            for (int i = 0; i < d; ++i) s = s + qbuf[i] * qbuf[i];
            qbuf[qs] = s;
        }
        __syncthreads();
        const float r = qbuf[qs];
        __syncthreads();
        return r;
    };
    if (metric != MQVS_METRIC_COSINE) {
        for (int i = lane; i < qs; i += 64) v0[i] = i < d ? qbuf[i] : 0.0f;
        const float sum = blas ? seqsum() : 0.0f;
        if (qdelta && lane == 0) qdelta[j] = 0.0f;
        if (lane == 0) {
            if (qnorms) qnorms[j] = sum;
            qmu[j] = 0;
            qlam[j] = 1;
        }
        return;
    }
    const float eps = 1.1920929e-07f;
    for (int v = 0; v <= maxv; ++v) {
        float *cur = v < maxv ? v0 + (int64_t)v * qs : nullptr;
        const float sum = seqsum();
        if (sum < eps) {
            if (cur)
                for (int i = lane; i < d; i += 64) cur[i] = qbuf[i];
        } else {
            const float s = sqrtf(sum);
            for (int i = lane; i < d; i += 64) {
                const float x = qbuf[i] / s;
                if (cur) cur[i] = x;
                qbuf[i] = x;
            }
        }
        if (cur)
            for (int i = d + lane; i < qs; i += 64) cur[i] = 0.0f;  // (padding columns)
        __syncthreads();
        for (int u = 0; u < v; ++u) {
            const float *o = v0 + (int64_t)u * qs;
            bool eq = true;
            for (int i = lane; i < d; i += 64)
                eq = eq && __builtin_bit_cast(uint32_t, o[i]) == __builtin_bit_cast(uint32_t, qbuf[i]);
            if (__all(eq)) {
                if (lane == 0) {
                    qmu[j] = u;
                    qlam[j] = v - u;
                    if (qnorms) qnorms[j] = 0.0f;
                }
                for (int w = v; w < maxv; ++w)  // (unused variants: zeros)
                    for (int i = lane; i < qs; i += 64) v0[(int64_t)w * qs + i] = 0.0f;
                put_delta(v);
                return;
            }
        }
    }
    put_delta(maxv);
    if (lane == 0) {
        atomicOr(status, 1);
        qmu[j] = maxv - 1;
        qlam[j] = 1;
        if (qnorms) qnorms[j] = 0.0f;
    }
}

void launch_query_prep(const float *q, int nq, int d, int metric, bool blas, float *qvars, int maxv,
                       float *qnorms, int *qmu, int *qlam, int *status, hipStream_t s, int phase, float *qdelta) {
    if (metric != MQVS_METRIC_COSINE) maxv = 1;
    const size_t lds = (size_t)((d + 31) / 32 * 32 + 4) * sizeof(float);
    const bool lanesig = maxv <= kLaneSigMax;
    const size_t sig = lanesig ? (size_t)(maxv + 1) * 64 * sizeof(uint32_t) : (size_t)(maxv + 1) * sizeof(uint64_t);
#define MQVS_QP(J)                                                                                                   \
    do {                                                                                                             \
        if (lanesig)                                                                                                 \
            hipLaunchKernelGGL((k_query_prep<J, 3, true>), dim3(nq), dim3(64), sig, s, q, nq, d, metric, blas ? 1 : 0, \
                               qvars, maxv, qnorms, qmu, qlam, status, phase, qdelta);                               \
        else                                                                                                         \
            hipLaunchKernelGGL((k_query_prep<J, 3, false>), dim3(nq), dim3(64), sig, s, q, nq, d, metric,             \
                               blas ? 1 : 0, qvars, maxv, qnorms, qmu, qlam, status, phase, qdelta);                 \
    } while (0)
    if (d <= 128)
        MQVS_QP(2);
    else if (d <= 256)
        MQVS_QP(4);
    else if (d <= 512)
        MQVS_QP(8);
    else if (d <= 768)
        MQVS_QP(12);
    else if (d <= 1024)
        MQVS_QP(16);
    else if (d <= 1536)
        MQVS_QP(24);
    else
        hipLaunchKernelGGL(k_query_prep_lds, dim3(nq), dim3(64), lds, s, q, nq, d, metric, blas ? 1 : 0, qvars, maxv,
                           qnorms, qmu, qlam, status, phase, qdelta);
#undef MQVS_QP
}

// Counter-based synthetic generator; bit-identical to oracle/mqvs_oracle.c
// orc_generate (integer hash, exact 16-bit fractions, one rounding).
__device__ __host__ inline uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__device__ inline float gen_gauss(uint64_t seed, uint64_t idx) {
    const uint64_t h = splitmix64(seed ^ idx);
    const float u0 = (float)(h & 0xffff) * (1.0f / 65536.0f);
    const float u1 = (float)((h >> 16) & 0xffff) * (1.0f / 65536.0f);
    const float u2 = (float)((h >> 32) & 0xffff) * (1.0f / 65536.0f);
    const float u3 = (float)((h >> 48) & 0xffff) * (1.0f / 65536.0f);
    const float s = (u0 + u1) + (u2 + u3);
    return (s - 2.0f) * 1.7320508f;
}

__global__ void k_generate(uint64_t seed, int mode, int64_t row0, int64_t n, int d, float *out) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / d;
        const int j = (int)(e - r * d);
        const uint64_t row = (uint64_t)(row0 + r);
        const uint64_t idx = row * (uint64_t)d + (uint64_t)j;
        float v;
        if (mode == 0) {
            v = (float)((int)(splitmix64(seed ^ idx) % 17ULL) - 8);
        } else if (mode == 1) {
            v = gen_gauss(seed, idx);
        } else if (mode == 2) {
            const uint64_t c =
                splitmix64(seed ^ 0xC0FFEEULL ^ (row * 0x100000001B3ULL)) % 4096ULL;
            const float center = gen_gauss(seed ^ 0xCE17E5ULL, c * (uint64_t)d + (uint64_t)j);
            v = center + 0.25f * gen_gauss(seed, idx);
        } else {
            // hard mixture: 65536 centres, noise as large as the centres
            const uint64_t c =
                splitmix64(seed ^ 0xC0FFEEULL ^ (row * 0x100000001B3ULL)) % 65536ULL;
            const float center = gen_gauss(seed ^ 0xCE17E5ULL, c * (uint64_t)d + (uint64_t)j);
            v = center + gen_gauss(seed, idx);
        }
        out[e] = v;
    }
}

void launch_generate(uint64_t seed, int mode, int64_t row0, int64_t n, int d, float *out,
                     hipStream_t s) {
    const int64_t total = n * d;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) return;
    hipLaunchKernelGGL(k_generate, dim3((unsigned)blocks), dim3(256), 0, s, seed, mode, row0, n, d,
                       out);
}

// bytes (1 = nonempty) -> LSB-first bitmap
__global__ void k_pack(const uint8_t *bytes, int64_t n, uint8_t *bits) {
    const int64_t nb = (n + 7) / 8;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb;
         b += (int64_t)gridDim.x * blockDim.x) {
        uint8_t v = 0;
        for (int i = 0; i < 8; ++i) {
            const int64_t r = b * 8 + i;
            if (r < n && bytes[r]) v |= (uint8_t)(1u << i);
        }
        bits[b] = v;
    }
}

// Up to two 32-bit fills in one launch (the small status / counter / list-tail
// fills of a search: a runtime memset is a ~4 us kernel of its own each)
__global__ void k_fill2(uint32_t *a, int64_t na, uint32_t va, uint32_t *b, int64_t nb, uint32_t vb) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += stride) {
        if (i < na)
            a[i] = va;
        else
            b[i - na] = vb;
    }
}

void launch_fill2(uint32_t *a, int64_t na, uint32_t va, uint32_t *b, int64_t nb, uint32_t vb, hipStream_t s) {
    if (!a) na = 0;
    if (!b) nb = 0;
    const int64_t n = na + nb;
    if (n <= 0) return;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill2, dim3((unsigned)blocks), dim3(256), 0, s, a, na, va, b, nb, vb);
}

void launch_pack_nonempty(const uint8_t *bytes, int64_t n, uint8_t *bits, hipStream_t s) {
    int64_t blocks = ((n + 7) / 8 + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) return;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)blocks), dim3(256), 0, s, bytes, n, bits);
}

// Bitmap words: bits [32 w, 32 w + 32) of an LSB-first byte bitmap of nbits
// bits (bits at or past nbits read 0).  The row-selection kernels below work a
// word (32 rows) per lane and a wave per granule chunk: round 3's row-per-
// thread loops with a block barrier per 256 rows took 60-90 us each on a
// 50M-row part (6104 chunks), more than a 1 %-selective scan itself.
__device__ inline uint32_t bm_word(const uint8_t *bm, int64_t nbits, int64_t w) {
    const int64_t b0 = 4 * w, nbytes = (nbits + 7) >> 3;
    uint32_t v = 0;
    if (b0 + 4 <= nbytes && (((uintptr_t)(bm + b0)) & 3) == 0) {
        v = *reinterpret_cast<const uint32_t *>(bm + b0);
    } else {
        for (int i = 0; i < 4; ++i)
            if (b0 + i < nbytes) v |= (uint32_t)bm[b0 + i] << (8 * i);
    }
    const int64_t hi = nbits - 32 * w;
    if (hi < 32) v &= hi <= 0 ? 0u : ((1u << hi) - 1u);
    return v;
}

// rows of word w inside [r0, r1)
__device__ inline uint32_t range_mask(int64_t w, int64_t r0, int64_t r1) {
    const int64_t b = 32 * w;
    uint32_t m = 0xFFFFFFFFu;
    if (r0 > b) m = r0 - b >= 32 ? 0u : m & (0xFFFFFFFFu << (r0 - b));
    if (r1 < b + 32) m = r1 <= b ? 0u : m & ((1u << (r1 - b)) - 1u);
    return m;
}

// selected rows of word w: filter (or every row when null) & non-empty & live
__device__ inline uint32_t sel_word(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists,
                                    int64_t n, int64_t w) {
    uint32_t v = filter ? bm_word(filter, n, w) : range_mask(w, 0, n);
    if (nonempty) v &= bm_word(nonempty, n, w);
    if (exists) v &= bm_word(exists, n, w);
    return v;
}

__device__ inline int64_t wave_excl_scan64(int64_t v, int64_t &total) {
    const int lane = threadIdx.x & 63;
    int64_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    total = __shfl(inc, 63);
    return inc - v;
}

// Chunk ordinals: which granule chunks the reference actually hands to
// searchWrapper, and how many such calls came before each.
//  no-filter mode (require_filter = 0): a chunk is searched iff one of its
//    arrays is non-empty (MergeTreeVSManager.cpp:1364-1368 skips src_vec.empty());
//  filter mode: a mark is searched iff it keeps >= 1 selected non-empty live
//    row (:1179-1183).
// One wave per chunk, four chunks per workgroup.
__global__ __launch_bounds__(256) void k_chunk_active(const uint8_t *filter,
                                                       const uint8_t *nonempty,
                                                       const uint8_t *exists, int64_t n,
                                                       int64_t chunk_rows, int64_t nchunks, int require_filter,
                                                       int *flag) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const int64_t r0 = c * chunk_rows;
    const int64_t r1 = r0 + chunk_rows < n ? r0 + chunk_rows : n;
    uint32_t any = 0;
    for (int64_t w = (r0 >> 5) + lane; w < ((r1 + 31) >> 5) && !any; w += 64) {
        uint32_t v = range_mask(w, r0, r1);
        if (nonempty) v &= bm_word(nonempty, n, w);
        if (require_filter) {
            v &= bm_word(filter, n, w);
            if (exists) v &= bm_word(exists, n, w);
        }
        any |= v;
    }
    const bool hit = __any(any != 0);
    if (lane == 0) flag[c] = hit ? 1 : 0;
}

// One workgroup of kScanThreads: thread t owns a contiguous run of chunks;
// the run sums are scanned by waves, then over the wave totals.
constexpr int kScanThreads = 1024;
template <int NT = kScanThreads, class Val, class Out>
__device__ void run_scan(int64_t nchunks, Val val, Out out, int64_t *sh, int64_t &grand) {
    constexpr int kScanThreads = NT;  // block size of the caller
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t per = (nchunks + kScanThreads - 1) / kScanThreads;
    const int64_t b = t * per, e = b + per < nchunks ? b + per : nchunks;
    int64_t s = 0;
    for (int64_t i = b; i < e; ++i) s += val(i);
    int64_t wt = 0;
    const int64_t ex = wave_excl_scan64(s, wt);
    if (lane == 0) sh[wv] = wt;
    __syncthreads();
    int64_t before = 0, all = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) {
        if (w < wv) before += sh[w];
        all += sh[w];
    }
    int64_t run = before + ex;
    for (int64_t i = b; i < e; ++i) {
        const int64_t v = val(i);
        out(i, run, v);
        run += v;
    }
    grand = all;
    __syncthreads();
}

__global__ __launch_bounds__(kScanThreads) void k_exclusive_ord(int *flag_ord, int64_t nchunks) {
    __shared__ int64_t sh[kScanThreads / 64];
    int64_t tot = 0;
    run_scan(
        nchunks, [&](int64_t i) -> int64_t { return flag_ord[i] ? 1 : 0; },
        [&](int64_t i, int64_t before, int64_t v) { flag_ord[i] = v ? (int)before : -1; }, sh, tot);
}

// ---------------------------------------------------------------------------
// Gather list of a selective PREWHERE scan: the rows that pass the filter,
// are non-empty and not deleted, chunk by chunk in row order, each chunk's
// run padded with -1 to a multiple of `tile` entries.
// k_chunk_count: per chunk its selected rows (one wave per chunk); the last
// workgroup to finish (an agent-scope ticket, zeroed with the search's status
// words) then scans the counts: offsets[c] = sum of padded counts before c,
// totals[0] = padded list length, totals[1] = selected rows.  host_totals
// (pinned host memory, may be null): the same two values, then host_gen in
// [2] behind a system-scope fence, so the host can act on them as soon as [2]
// shows its call's generation instead of draining the stream for a copy (a
// record left by another call's kernel never carries this call's number).
// (One launch: the separate single-workgroup scan cost ~8 us plus a launch
// gap.)
// The ticket relies on gfx9-family memory ordering (gfx950 here): stores with
// the agent-scope write-through and vmcnt counting stores, so a workgroup's
// counts have left it when its s_waitcnt vmcnt(0) (the 0x0F70 encoding: gfx9's
// field layout) retires, before its ticket; other ISA families order stores
// differently and would need release/acquire fences on the ticket.
constexpr int kCountStage = 16384;  // chunks whose counts k_chunk_count's scan stages in LDS

__global__ __launch_bounds__(kScanThreads) void k_chunk_count(const uint8_t *filter, const uint8_t *nonempty,
                                                               const uint8_t *exists, int64_t n, int64_t chunk_rows,
                                                               int64_t nchunks, int *count, int tile,
                                                               int64_t *offsets, int64_t *totals,
                                                               int64_t *host_totals, int64_t host_gen,
                                                               int *ticket) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "k_chunk_count's ticket assumes gfx94x/gfx950 store ordering (see above)"
#endif
    __shared__ int64_t sh[kScanThreads / 64];
    __shared__ int s_last;
    const int64_t c = (int64_t)blockIdx.x * (kScanThreads / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c < nchunks) {
        const int64_t r0 = c * chunk_rows;
        const int64_t r1 = r0 + chunk_rows < n ? r0 + chunk_rows : n;
        int cnt = 0;
        // (unrolled: a chunk of 8192 rows is 4 words per lane, their loads in
        // flight together)
#pragma unroll 4
        for (int64_t w = (r0 >> 5) + lane; w < ((r1 + 31) >> 5); w += 64)
            cnt += __popc(sel_word(filter, nonempty, exists, n, w) & range_mask(w, r0, r1));
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        // (write-through: the count reaches the device-coherent level
        // without an agent-scope release, which writes back the whole L2 --
        // one per workgroup cost ~50 us at 1526 workgroups)
        if (lane == 0) __hip_atomic_store(count + c, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // last workgroup in: every count stored and drained before the ticket
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    // (coherent loads of the other workgroups' counts, no acquire fence)
    // Up to kCountStage chunks: staged in LDS first, 8 independent loads in
    // flight per thread -- the two scans below read each count twice, and
    // reading them from memory there serialised ~18 coherent loads per thread
    // (k_chunk_count 21 us at 6104 chunks)
    extern __shared__ int s_cnt[];
    const bool staged = nchunks <= kCountStage;
    if (staged) {
        for (int64_t i0 = threadIdx.x; i0 < nchunks; i0 += 8 * kScanThreads) {
            int v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + (int64_t)u * kScanThreads;
                v[u] = i < nchunks ? __hip_atomic_load(count + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + (int64_t)u * kScanThreads;
                if (i < nchunks) s_cnt[i] = v[u];
            }
        }
        __syncthreads();
    }
    auto cnt_of = [&](int64_t i) -> int64_t {
        if (staged) return (int64_t)s_cnt[i];
        return (int64_t)__hip_atomic_load(count + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    int64_t padded_total = 0, selected = 0;
    run_scan(
        nchunks, [&](int64_t i) -> int64_t { return (cnt_of(i) + tile - 1) / tile * tile; },
        [&](int64_t i, int64_t before, int64_t) { offsets[i] = before; }, sh, padded_total);
    run_scan(nchunks, cnt_of, [&](int64_t, int64_t, int64_t) {}, sh, selected);
    if (threadIdx.x == 0) {
        totals[0] = padded_total;
        totals[1] = selected;
        *ticket = 0;
        if (host_totals) {
            *reinterpret_cast<volatile int64_t *>(host_totals) = padded_total;
            *reinterpret_cast<volatile int64_t *>(host_totals + 1) = selected;
            __threadfence_system();
            *reinterpret_cast<volatile int64_t *>(host_totals + 2) = host_gen;
            __threadfence_system();
        }
    }
}

// one wave per chunk: lane l takes 4 consecutive words of each 256-word round,
// a wave scan of their counts places its rows
__global__ __launch_bounds__(256) void k_compact_rows(const uint8_t *filter, const uint8_t *nonempty,
                                                       const uint8_t *exists, int64_t n, int64_t chunk_rows,
                                                       int64_t nchunks, const int *count, const int64_t *offsets,
                                                       int tile, int32_t *list, int64_t list_end,
                                                       const int64_t *dev_total, int64_t round) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const int64_t r0 = c * chunk_rows;
    const int64_t r1 = r0 + chunk_rows < n ? r0 + chunk_rows : n;
    int32_t *out = list + offsets[c];
    int64_t run = 0;
    const int64_t w0 = r0 >> 5, w1 = (r1 + 31) >> 5;
    for (int64_t base = w0; base < w1; base += 256) {
        uint32_t v[4];
        int64_t cnt = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t w = base + 4 * lane + i;
            v[i] = w < w1 ? sel_word(filter, nonempty, exists, n, w) & range_mask(w, r0, r1) : 0u;
            cnt += __popc(v[i]);
        }
        int64_t tot = 0;
        int64_t pos = run + wave_excl_scan64(cnt, tot);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t m = v[i];
            const int64_t rb = 32 * (base + 4 * lane + i);
            while (m) {
                const int bit = __ffs(m) - 1;
                m &= m - 1;
                out[pos++] = (int32_t)(rb + bit);
            }
        }
        run += tot;
    }
    const int cnt = count[c];
    const int padded = (cnt + tile - 1) / tile * tile;
    for (int i = cnt + lane; i < padded; i += 64) out[i] = -1;
    // the last chunk also pads the list's end up to list_end (whole tiles of
    // the scan; -1 entries); list_end < 0: the padded total k_chunk_count
    // left in device memory, rounded up to `round` (a list launched before
    // the host read the count)
    if (list_end < 0) list_end = (*dev_total + round - 1) / round * round;
    if (c == nchunks - 1)
        for (int64_t i = offsets[c] + padded + lane; i < list_end; i += 64) list[i] = -1;
}

void launch_gather_count(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                         int64_t chunk_rows, int tile, int *count, int64_t *offsets, int64_t *totals,
                         int64_t *host_totals, int64_t host_gen, int *ticket, hipStream_t s) {
    const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
    if (nchunks < 1) return;
    constexpr int wpb = kScanThreads / 64;  // chunks (waves) per workgroup
    const size_t lds = sizeof(int) * (size_t)(nchunks <= kCountStage ? nchunks : 0);
    hipLaunchKernelGGL(k_chunk_count, dim3((unsigned)((nchunks + wpb - 1) / wpb)), dim3(kScanThreads), lds, s, filter,
                       nonempty, exists, n, chunk_rows, nchunks, count, tile, offsets, totals, host_totals, host_gen,
                       ticket);
}

void launch_gather_list(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                        int64_t chunk_rows, int tile, const int *count, const int64_t *offsets, int32_t *list,
                        int64_t list_end, hipStream_t s, const int64_t *dev_total, int64_t round) {
    const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
    if (nchunks < 1) return;
    hipLaunchKernelGGL(k_compact_rows, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, s, filter, nonempty, exists,
                       n, chunk_rows, nchunks, count, offsets, tile, list, list_end, dev_total, round);
}

void launch_chunk_ordinals(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists,
                           int64_t n, int64_t chunk_rows, int require_filter, int *ord,
                           hipStream_t s) {
    const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
    if (nchunks < 1) return;
    hipLaunchKernelGGL(k_chunk_active, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, s, filter, nonempty,
                       exists, n, chunk_rows, nchunks, require_filter, ord);
    hipLaunchKernelGGL(k_exclusive_ord, dim3(1), dim3(kScanThreads), 0, s, ord, nchunks);
}

__global__ __launch_bounds__(256) void k_words_to_host(const int64_t *a, int na, const int *b, int nb, int64_t *ha,
                                                      int *hb, const int64_t *pq, int npq) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (pq) {
        // column sums of pq[npq][na] (na <= 4): each thread its rows' na
        // words (independent loads, 4 rows in flight), then the block sum
        __shared__ int64_t part[4][4];
        int64_t v[4] = {0, 0, 0, 0};
#pragma unroll 4
        for (int r = t; r < npq; r += 256)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < na) v[c] += pq[(int64_t)r * na + c];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            for (int off = 32; off > 0; off >>= 1) v[c] += __shfl_xor(v[c], off);
            if (lane == 0) part[wv][c] = v[c];
        }
        __syncthreads();
        if (t < na) *reinterpret_cast<volatile int64_t *>(ha + t) = part[0][t] + part[1][t] + part[2][t] + part[3][t];
    } else if (t < na) {
        *reinterpret_cast<volatile int64_t *>(ha + t) = a[t];
    }
    if (t < nb) *reinterpret_cast<volatile int *>(hb + t) = b[t];
    __threadfence_system();
}

void launch_words_to_host(const int64_t *a, int na, const int *b, int nb, int64_t *host_a, int *host_b,
                          hipStream_t s, const int64_t *pq, int npq) {
    if (pq && na > 4) fail(MQVS_ERR_LOGICAL, "words_to_host: more than 4 summed columns");
    hipLaunchKernelGGL(k_words_to_host, dim3(1), dim3(pq ? 256 : 64), 0, s, a, na, b, nb, host_a, host_b, pq, npq);
}

// ---------------------------------------------------------------------------
// ASYNC outcome of a search, OR-ed into the thread's sticky word
// (mqvs_async_check)
__global__ void k_async_flags(const int *overflow, const int *status, int status_matters, int *sticky) {
    if (threadIdx.x != 0) return;
    int w = 0;
    if (overflow && overflow[0]) w |= 1;
    if (status && status_matters && status[0]) w |= 2;
    if (w) atomicOr(sticky, w);
}

void launch_async_flags(const int *overflow, const int *status, int status_matters, int *sticky, hipStream_t s) {
    hipLaunchKernelGGL(k_async_flags, dim3(1), dim3(64), 0, s, overflow, status, status_matters, sticky);
}

// ---------------------------------------------------------------------------
// searched chunks of a row range (the cosine chunk-ordinal base of the next
// shard): k_chunk_active flags, then one block sums them
__global__ __launch_bounds__(256) void k_sum_flags(const int *flags, int64_t nchunks, int64_t *count) {
    __shared__ int64_t part[256];
    int64_t s = 0;
    for (int64_t c = threadIdx.x; c < nchunks; c += 256) s += flags[c] ? 1 : 0;
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = part[0];
}

void launch_count_active_chunks(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                                int64_t chunk_rows, int *flags_scratch, int64_t *count, hipStream_t s) {
    const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
    if (nchunks > 0)
        hipLaunchKernelGGL(k_chunk_active, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, s, filter, nonempty,
                           exists, n, chunk_rows, nchunks, filter ? 1 : 0, flags_scratch);
    hipLaunchKernelGGL(k_sum_flags, dim3(1), dim3(256), 0, s, flags_scratch, nchunks, count);
}

// ---------------------------------------------------------------------------
// Decoupled parts (a merged part whose vector index still lives in its source
// parts): VIWithColumnInPart::transferToNewRowIds (VIWithDataPart.cpp:56-67)
// and getRealBitmap (VIUtils.cpp:479-497), on the device.
__global__ void k_map_ids(int64_t *ids, int64_t count, const uint64_t *map) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = ids[i];
        if (v >= 0) ids[i] = (int64_t)map[v];
    }
}

void launch_map_ids(int64_t *ids, int64_t count, const uint64_t *map, hipStream_t s) {
    if (count <= 0) return;
    const int64_t blocks = std::min<int64_t>((count + 255) / 256, 4096);
    hipLaunchKernelGGL(k_map_ids, dim3((unsigned)blocks), dim3(256), 0, s, ids, count, map);
}

__global__ void k_copy_bits(const uint8_t *src, int64_t rows, uint32_t *words) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w * 32 >= rows) return;
    uint32_t v = 0;
    for (int b = 0; b < 4; ++b) {
        const int64_t byte = w * 4 + b;
        if (byte * 8 < rows) v |= (uint32_t)src[byte] << (8 * b);
    }
    const int64_t tail = rows - w * 32;
    if (tail < 32) v &= (1u << tail) - 1u;
    words[w] = v;
}

__global__ void k_decoupled_filter(const uint8_t *nf, int64_t new_rows, const uint64_t *inv_ids, const uint8_t *inv_src,
                                   int64_t inv_len, uint32_t own_id, uint32_t *old_words, int64_t old_rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= new_rows || i >= inv_len) return;
    if (!((nf[i >> 3] >> (i & 7)) & 1)) return;
    if ((uint32_t)inv_src[i] != own_id) return;
    const uint64_t r = inv_ids[i];
    if (r < (uint64_t)old_rows) atomicOr(&old_words[r >> 5], 1u << (r & 31));
}

void launch_decoupled_filter(const uint8_t *new_filter, int64_t new_rows, const uint64_t *inv_ids,
                             const uint8_t *inv_src, int64_t inv_len, uint32_t own_id, uint32_t *old_words,
                             int64_t old_rows, hipStream_t s) {
    const int64_t nw = (old_rows + 31) / 32;
    MQVS_HIP(hipMemsetAsync(old_words, 0, 4 * (size_t)std::max<int64_t>(nw, 1), s));
    if (!inv_ids) {  // no maps: the filter itself ("return filter")
        if (nw) hipLaunchKernelGGL(k_copy_bits, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, new_filter,
                                   std::min(new_rows, old_rows), old_words);
        return;
    }
    if (new_rows > 0)
        hipLaunchKernelGGL(k_decoupled_filter, dim3((unsigned)((new_rows + 255) / 256)), dim3(256), 0, s, new_filter,
                           new_rows, inv_ids, inv_src, inv_len, own_id, old_words, old_rows);
}

}  // namespace mqvs

namespace mqvs {

// ---------------------------------------------------------------------------
// STREAM-like HBM read sweep (bench utility: the measured denominator of the
// scan's HBM fraction).  Every lane reads 16 B per load, 4 loads in flight per
// lane per iteration, grid-stride over the whole buffer; the XOR of what it
// read keeps the loads live (written only when it equals an impossible
// pattern).
typedef unsigned rs_u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_read_sweep(const rs_u32x4 *p, int64_t n16, unsigned *sink) {
    rs_u32x4 acc = {0u, 0u, 0u, 0u};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const rs_u32x4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n16; i += stride) acc ^= p[i];
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == acc.w) sink[0] = acc.x;
}

// The same bytes, each workgroup over one contiguous slice: per round its 256
// lanes read U consecutive 4 KiB pieces (U loads in flight per lane,
// non-temporal: every byte is read once), so DRAM pages are swept in order.
template <int U>
__global__ __launch_bounds__(256) void k_read_slices(const rs_u32x4 *p, int64_t n16, unsigned *sink) {
    rs_u32x4 acc = {0u, 0u, 0u, 0u};
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t b = (int64_t)blockIdx.x * per, e = b + per < n16 ? b + per : n16;
    int64_t i = b + threadIdx.x;
    for (; i + (U - 1) * 256 < e; i += U * 256) {
        rs_u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    for (; i < e; i += 256) acc ^= p[i];
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == acc.w) sink[0] = acc.x;
}

// best time of `reps` sweeps over a fresh `bytes` buffer (filled first, so
// the sweep reads written pages) on stream s, over the sweep shapes (the
// grid-stride k_read_sweep at 8 workgroups per CU; contiguous slices at 4 and
// 8 workgroups per CU with 8 or 16 loads in flight): the best is the
// achievable read rate the bench reports beside the plane scans
double measure_read_sweep(size_t bytes, int reps, hipStream_t s, double *best_ms) {
    const int cus = device_cus();
    bytes = bytes / 16 * 16;
    void *buf = nullptr;
    MQVS_HIP(hipMalloc(&buf, bytes + 256));
    unsigned *sink = reinterpret_cast<unsigned *>(static_cast<char *>(buf) + bytes);
    MQVS_HIP(hipMemsetAsync(buf, 0x5A, bytes, s));
    hipEvent_t e0, e1;
    MQVS_HIP(hipEventCreate(&e0));
    MQVS_HIP(hipEventCreate(&e1));
    const int64_t n16 = (int64_t)(bytes / 16);
    const auto *src = static_cast<const rs_u32x4 *>(buf);
    float best = 1e30f;
    for (int shape = 0; shape < 5; ++shape) {
        for (int r = 0; r <= reps; ++r) {  // (pass 0 warms up)
            MQVS_HIP(hipEventRecord(e0, s));
            switch (shape) {
                case 0: hipLaunchKernelGGL(k_read_sweep, dim3(cus * 8), dim3(256), 0, s, src, n16, sink); break;
                case 1: hipLaunchKernelGGL(k_read_slices<8>, dim3(cus * 4), dim3(256), 0, s, src, n16, sink); break;
                case 2: hipLaunchKernelGGL(k_read_slices<8>, dim3(cus * 8), dim3(256), 0, s, src, n16, sink); break;
                case 3: hipLaunchKernelGGL(k_read_slices<16>, dim3(cus * 4), dim3(256), 0, s, src, n16, sink); break;
                default: hipLaunchKernelGGL(k_read_slices<16>, dim3(cus * 2), dim3(256), 0, s, src, n16, sink); break;
            }
            MQVS_HIP(hipEventRecord(e1, s));
            MQVS_HIP(hipEventSynchronize(e1));
            float ms = 0.f;
            MQVS_HIP(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(buf);
    if (best_ms) *best_ms = best;
    return (double)bytes / (best * 1e-3) / 1e9;
}

}  // namespace mqvs
