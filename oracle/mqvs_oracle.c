/*
 * mqvs_oracle.c -- CPU restatement of MyScaleDB's brute-force vector scan.
 *
 * TEST INFRASTRUCTURE ONLY (see mqvs_oracle.h).  Parity status: pinned by the
 * reference's SQL known-answer tests (tests/golden/kat_*.json); the reference
 * itself is unbuildable here (faiss submodule contrib/search-index is empty).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; explicit fmaf()).
 */
#include "mqvs_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <immintrin.h>
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Distance primitives: faiss fvec_L2sqr / fvec_inner_product / fvec_norm_L2sqr
 * (third-party, absent).  Sequential order, product rounded then added (no
 * fma): the reference's own KATs (00001, 00002, 00014) pin this -- an fma
 * chain misses 00001 rows 3, 4 and 6 by one ulp.  Built -ffp-contract=off. */

float orc_l2sqr(const float *x, const float *y, int64_t d) {
    float res = 0.0f;
    for (int64_t i = 0; i < d; i++) {
        const float t = x[i] - y[i];
        res = res + t * t;
    }
    return res;
}

float orc_inner_product(const float *x, const float *y, int64_t d) {
    float res = 0.0f;
    for (int64_t i = 0; i < d; i++) res = res + x[i] * y[i];
    return res;
}

float orc_norm_l2sqr(const float *x, int64_t d) {
    float res = 0.0f;
    for (int64_t i = 0; i < d; i++) res = res + x[i] * x[i];
    return res;
}

/* The sgemm of faiss's BLAS branch (nx >= 20, exhaustive_*_blas): no KAT
 * pins it; assumed to be what FMA microkernels compute for one C element, a
 * sequential fp32 fma chain over k (documented assumption). */
float orc_gemm_dot(const float *x, const float *y, int64_t d) {
    float res = 0.0f;
    for (int64_t i = 0; i < d; i++) res = fmaf(x[i], y[i], res);
    return res;
}

/* The same element under an sgemm that blocks K (kc = kb): each block is an
 * fma chain from zero, added to C in block order (C = 0 + part_0 + part_1 ...).
 * Not the assumed reference arithmetic: the parity-risk measurement of the
 * BLAS-branch assumption (tools/blas_order_risk.py). */
float orc_gemm_dot_blocked(const float *x, const float *y, int64_t d, int64_t kb) {
    float res = 0.0f;
    for (int64_t b = 0; b < d; b += kb) {
        float part = 0.0f;
        const int64_t e = b + kb < d ? b + kb : d;
        for (int64_t i = b; i < e; i++) part = fmaf(x[i], y[i], part);
        res = res + part;
    }
    return res;
}

/* VectorDataset<Float>::normalize, VectorDataset.h:98-117:
 *   sum += p[d]*p[d] (separate mul/add), skip if sum < FLT_EPSILON,
 *   sum = sqrt(sum), p[d] /= sum. */
void orc_normalize(float *data, int64_t n, int64_t d) {
    for (int64_t r = 0; r < n; r++) {
        float *p = data + r * d;
        float sum = 0.0f;
        /* built with -ffp-contract=off: separate multiply and add */
        for (int64_t i = 0; i < d; i++) sum = sum + p[i] * p[i];
        if (sum < FLT_EPSILON) continue;
        sum = sqrtf(sum);
        for (int64_t i = 0; i < d; i++) p[i] = p[i] / sum;
    }
}

/* ------------------------------------------------------------------------ */
/* faiss heap restated (faiss/utils/Heap.h, third-party, absent): 1-based
 * binary heap whose top is the current worst element; ordering by (value, id)
 * via cmp2; neutral = FLT_MAX for the L2 max-heap, -FLT_MAX (lowest) for the
 * IP min-heap.  `is_max` selects CMax (L2) or CMin (IP). */

static inline int cmp2(int is_max, float a1, float b1, int64_t a2, int64_t b2) {
    if (is_max) return (a1 > b1) || ((a1 == b1) && (a2 > b2));
    return (a1 < b1) || ((a1 == b1) && (a2 > b2));
}

static inline int cmp1(int is_max, float a, float b) {
    return is_max ? (a > b) : (a < b);
}

static void heap_heapify(int is_max, int64_t k, float *val, int64_t *ids) {
    const float neutral = is_max ? FLT_MAX : -FLT_MAX;
    for (int64_t i = 0; i < k; i++) {
        val[i] = neutral;
        ids[i] = -1;
    }
}

/* faiss heap_replace_top: replace the top with (v, id) and sift down. */
static void heap_replace_top(int is_max, int64_t k, float *bh_val,
                             int64_t *bh_ids, float v, int64_t id) {
    float *val = bh_val - 1; /* 1-based */
    int64_t *ids = bh_ids - 1;
    int64_t i = 1;
    for (;;) {
        int64_t i1 = i << 1, i2 = i1 + 1;
        if (i1 > k) break;
        if (i2 == k + 1 || cmp2(is_max, val[i1], val[i2], ids[i1], ids[i2])) {
            if (cmp2(is_max, v, val[i1], id, ids[i1])) break;
            val[i] = val[i1];
            ids[i] = ids[i1];
            i = i1;
        } else {
            if (cmp2(is_max, v, val[i2], id, ids[i2])) break;
            val[i] = val[i2];
            ids[i] = ids[i2];
            i = i2;
        }
    }
    val[i] = v;
    ids[i] = id;
}

static void heap_pop(int is_max, int64_t k, float *bh_val, int64_t *bh_ids) {
    float *val = bh_val - 1;
    int64_t *ids = bh_ids - 1;
    float v = val[k];
    int64_t id = ids[k];
    int64_t i = 1;
    k--;
    for (;;) {
        int64_t i1 = i << 1, i2 = i1 + 1;
        if (i1 > k) break;
        if (i2 == k + 1 || cmp2(is_max, val[i1], val[i2], ids[i1], ids[i2])) {
            if (cmp2(is_max, v, val[i1], id, ids[i1])) break;
            val[i] = val[i1];
            ids[i] = ids[i1];
            i = i1;
        } else {
            if (cmp2(is_max, v, val[i2], id, ids[i2])) break;
            val[i] = val[i2];
            ids[i] = ids[i2];
            i = i2;
        }
    }
    val[i] = v;
    ids[i] = id;
}

/* faiss heap_reorder: sort the heap best-first, move real entries to the
 * front and pad the tail with (neutral, -1). */
static void heap_reorder(int is_max, int64_t k, float *val, int64_t *ids) {
    int64_t i, ii;
    for (i = 0, ii = 0; i < k; i++) {
        float v = val[0];
        int64_t id = ids[0];
        heap_pop(is_max, k - i, val, ids);
        val[k - ii - 1] = v;
        ids[k - ii - 1] = id;
        if (id != -1) ii++;
    }
    memmove(val, val + k - ii, ii * sizeof(*val));
    memmove(ids, ids + k - ii, ii * sizeof(*ids));
    const float neutral = is_max ? FLT_MAX : -FLT_MAX;
    for (; ii < k; ii++) {
        val[ii] = neutral;
        ids[ii] = -1;
    }
}

/* ------------------------------------------------------------------------ */
/* knn: faiss knn_L2sqr / knn_inner_product restated.
 *   nx <  20: exhaustive_*_seq  (direct per-pair formula)
 *   nx >= 20: exhaustive_*_blas (L2 via norms: (xn + yn) - 2 ip, clamp >= 0)
 * In both, y is scanned in ascending row order and an element replaces the
 * heap top only when strictly better in value. */

int orc_knn(const float *x, const float *y, int64_t d, int64_t k, int64_t nx,
            int64_t ny, int metric, int64_t *ids, float *dist) {
    if (metric != ORC_L2 && metric != ORC_IP) return -1;
    const int is_max = (metric == ORC_L2);
    if (k <= 0) return 0;
    float *y_norms = NULL, *x_norms = NULL;
    const int blas = nx >= ORC_BLAS_THRESHOLD;
    if (blas && metric == ORC_L2) {
        y_norms = (float *)malloc(sizeof(float) * (ny > 0 ? ny : 1));
        x_norms = (float *)malloc(sizeof(float) * nx);
        for (int64_t j = 0; j < ny; j++) y_norms[j] = orc_norm_l2sqr(y + j * d, d);
        for (int64_t i = 0; i < nx; i++) x_norms[i] = orc_norm_l2sqr(x + i * d, d);
    }
    for (int64_t i = 0; i < nx; i++) {
        float *simi = dist + i * k;
        int64_t *idxi = ids + i * k;
        const float *xi = x + i * d;
        heap_heapify(is_max, k, simi, idxi);
        for (int64_t j = 0; j < ny; j++) {
            const float *yj = y + j * d;
            float dis;
            if (!blas) {
                dis = (metric == ORC_IP) ? orc_inner_product(xi, yj, d) : orc_l2sqr(xi, yj, d);
            } else if (metric == ORC_IP) {
                dis = orc_gemm_dot(xi, yj, d);
            } else {
                const float ip = orc_gemm_dot(xi, yj, d);
                dis = (x_norms[i] + y_norms[j]) - 2.0f * ip;
                if (dis < 0) dis = 0;
            }
            if (cmp1(is_max, simi[0], dis)) heap_replace_top(is_max, k, simi, idxi, dis, j);
        }
        heap_reorder(is_max, k, simi, idxi);
    }
    free(y_norms);
    free(x_norms);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Fast, bit-identical variant for CPU timing.  Distances for a block of rows
 * are computed into a buffer with the same per-pair fma chain, then offered to
 * the heap in ascending row order, exactly like orc_knn. */

#define FB_ROWS 64   /* rows per block  */
#define FB_Q 16      /* queries per block (BLAS-branch micro kernel) */

static void seq_block_dist(const float *xi, const float *y, int64_t d,
                           int64_t rows, int metric, float *out) {
    /* Transpose-free: for each k, update all rows' chains (vectorises across
     * rows via strided loads; each chain stays sequential in k). */
    float acc[FB_ROWS];
    for (int64_t r = 0; r < rows; r++) acc[r] = 0.0f;
    for (int64_t kk = 0; kk < d; kk++) {
        const float xv = xi[kk];
        if (metric == ORC_L2) {
            for (int64_t r = 0; r < rows; r++) {
                const float t = xv - y[r * d + kk];
                acc[r] = acc[r] + t * t;
            }
        } else {
            for (int64_t r = 0; r < rows; r++) acc[r] = acc[r] + xv * y[r * d + kk];
        }
    }
    for (int64_t r = 0; r < rows; r++) out[r] = acc[r];
}

/* BLAS-branch register-blocked micro-kernel (CPU-baseline timing only;
 * bench.py cpu_baseline): 6 rows x 64 queries of accumulators in 24 zmm
 * registers, one k step = 4 query loads + 24 fused multiply-adds with the
 * row element broadcast.  Each (query, row) accumulator is still ONE fp32
 * fma chain over k in ascending order -- the exact arithmetic of orc_gemm_dot
 * and of the scalar loop below -- so results stay bit-identical; only the
 * blocking changes.  xt: queries in blocks of 64, each block transposed and
 * contiguous ([nxp / 64][d][64]: the k loop streams one block sequentially). */
#define MK_R 6
#define MK_Q 64
__attribute__((target("avx512f"))) static void blas_block_avx512(const float *xt, int64_t nxp, int64_t q0,
                                                                 const float *const *yr, int64_t d,
                                                                 float out[MK_R][MK_Q]) {
    __m512 a[MK_R][4];
    for (int r = 0; r < MK_R; r++)
        for (int v = 0; v < 4; v++) a[r][v] = _mm512_setzero_ps();
    (void)nxp;
    const float *xb = xt + q0 * d;  /* block q0 / 64: [d][64] */
    for (int64_t kk = 0; kk < d; kk++) {
        const float *xk = xb + kk * MK_Q;
        const __m512 x0 = _mm512_loadu_ps(xk), x1 = _mm512_loadu_ps(xk + 16), x2 = _mm512_loadu_ps(xk + 32),
                     x3 = _mm512_loadu_ps(xk + 48);
        for (int r = 0; r < MK_R; r++) {
            const __m512 yv = _mm512_set1_ps(yr[r][kk]);
            a[r][0] = _mm512_fmadd_ps(x0, yv, a[r][0]);
            a[r][1] = _mm512_fmadd_ps(x1, yv, a[r][1]);
            a[r][2] = _mm512_fmadd_ps(x2, yv, a[r][2]);
            a[r][3] = _mm512_fmadd_ps(x3, yv, a[r][3]);
        }
    }
    for (int r = 0; r < MK_R; r++)
        for (int v = 0; v < 4; v++) _mm512_storeu_ps(out[r] + 16 * v, a[r][v]);
}

static int use_avx512(void) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("ORC_NO_AVX512");
        v = (e && e[0] == '1') ? 0 : __builtin_cpu_supports("avx512f");
    }
    return v;
}

int orc_has_avx512(void) { return use_avx512(); }

int orc_knn_fast(const float *x, const float *y, int64_t d, int64_t k,
                 int64_t nx, int64_t ny, int metric, int64_t *ids, float *dist) {
    if (metric != ORC_L2 && metric != ORC_IP) return -1;
    const int is_max = (metric == ORC_L2);
    if (k <= 0) return 0;
    const int blas = nx >= ORC_BLAS_THRESHOLD;
    for (int64_t i = 0; i < nx; i++) heap_heapify(is_max, k, dist + i * k, ids + i * k);
    float *buf = (float *)malloc(sizeof(float) * FB_ROWS * (nx > 0 ? nx : 1));
    float *x_norms = NULL, *xt = NULL;
    const int mk = blas && use_avx512();
    if (blas) {
        /* queries transposed [d][nx_pad] so a block of FB_Q (MK_Q with the
         * micro-kernel) queries is contiguous for each k */
        const int64_t qa = mk ? MK_Q : FB_Q;
        const int64_t nxp = (nx + qa - 1) / qa * qa;
        xt = (float *)calloc((size_t)d * nxp, sizeof(float));
        if (mk) {
            for (int64_t i = 0; i < nx; i++)
                for (int64_t kk = 0; kk < d; kk++) xt[((i / MK_Q) * d + kk) * MK_Q + i % MK_Q] = x[i * d + kk];
        } else {
            for (int64_t i = 0; i < nx; i++)
                for (int64_t kk = 0; kk < d; kk++) xt[kk * nxp + i] = x[i * d + kk];
        }
        if (metric == ORC_L2) {
            x_norms = (float *)malloc(sizeof(float) * nx);
            for (int64_t i = 0; i < nx; i++) x_norms[i] = orc_norm_l2sqr(x + i * d, d);
        }
    }
    const int64_t nxp = mk ? (nx + MK_Q - 1) / MK_Q * MK_Q : (nx + FB_Q - 1) / FB_Q * FB_Q;
    for (int64_t j0 = 0; j0 < ny; j0 += FB_ROWS) {
        const int64_t rows = (ny - j0) < FB_ROWS ? (ny - j0) : FB_ROWS;
        const float *yb = y + j0 * d;
        if (!blas) {
            for (int64_t i = 0; i < nx; i++)
                seq_block_dist(x + i * d, yb, d, rows, metric, buf + i * FB_ROWS);
        } else {
            float y_norms[FB_ROWS];
            if (metric == ORC_L2)
                for (int64_t r = 0; r < rows; r++) y_norms[r] = orc_norm_l2sqr(yb + r * d, d);
            if (mk) {
                float out[MK_R][MK_Q];
                for (int64_t q0 = 0; q0 < nx; q0 += MK_Q)
                    for (int64_t r0 = 0; r0 < rows; r0 += MK_R) {
                        const float *yr[MK_R];
                        for (int r = 0; r < MK_R; r++) yr[r] = yb + (r0 + r < rows ? r0 + r : r0) * d;
                        blas_block_avx512(xt, nxp, q0, yr, d, out);
                        for (int r = 0; r < MK_R && r0 + r < rows; r++)
                            for (int qq = 0; qq < MK_Q && q0 + qq < nx; qq++) {
                                float dis = out[r][qq];
                                if (metric == ORC_L2) {
                                    dis = (x_norms[q0 + qq] + y_norms[r0 + r]) - 2.0f * out[r][qq];
                                    if (dis < 0) dis = 0;
                                }
                                buf[(q0 + qq) * FB_ROWS + r0 + r] = dis;
                            }
                    }
            } else
            for (int64_t q0 = 0; q0 < nx; q0 += FB_Q) {
                for (int64_t r = 0; r < rows; r++) {
                    float acc[FB_Q];
                    for (int qq = 0; qq < FB_Q; qq++) acc[qq] = 0.0f;
                    const float *yr = yb + r * d;
                    for (int64_t kk = 0; kk < d; kk++) {
                        const float yv = yr[kk];
                        const float *xk = xt + kk * nxp + q0;
                        for (int qq = 0; qq < FB_Q; qq++) acc[qq] = fmaf(xk[qq], yv, acc[qq]);
                    }
                    for (int qq = 0; qq < FB_Q && q0 + qq < nx; qq++) {
                        float dis = acc[qq];
                        if (metric == ORC_L2) {
                            dis = (x_norms[q0 + qq] + y_norms[r]) - 2.0f * acc[qq];
                            if (dis < 0) dis = 0;
                        }
                        buf[(q0 + qq) * FB_ROWS + r] = dis;
                    }
                }
            }
        }
        for (int64_t i = 0; i < nx; i++) {
            float *simi = dist + i * k;
            int64_t *idxi = ids + i * k;
            const float *bi = buf + i * FB_ROWS;
            for (int64_t r = 0; r < rows; r++)
                if (cmp1(is_max, simi[0], bi[r]))
                    heap_replace_top(is_max, k, simi, idxi, bi[r], j0 + r);
        }
    }
    for (int64_t i = 0; i < nx; i++) heap_reorder(is_max, k, dist + i * k, ids + i * k);
    free(buf);
    free(xt);
    free(x_norms);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* VIWithColumnInPart::searchWithoutIndex, VIWithDataPart.h:341-382. */

typedef int (*knn_fn)(const float *, const float *, int64_t, int64_t, int64_t,
                      int64_t, int, int64_t *, float *);

static int search_without_index_impl(knn_fn knn, float *x, float *y, int64_t d,
                                     int64_t k, int64_t nx, int64_t ny,
                                     int metric, int64_t *ids, float *dist) {
    int m = metric;
    if (metric == ORC_COSINE) {
        m = ORC_IP;
        orc_normalize(x, nx, d);
        orc_normalize(y, ny, d);
    }
    int rc = knn(x, y, d, k, nx, ny, m, ids, dist);
    if (rc) return rc;
    if (metric == ORC_COSINE)
        for (int64_t i = 0; i < k * nx; i++) dist[i] = 1 - dist[i];
    return 0;
}

int orc_search_without_index(float *x, float *y, int64_t d, int64_t k,
                             int64_t nx, int64_t ny, int metric, int64_t *ids,
                             float *dist) {
    return search_without_index_impl(orc_knn, x, y, d, k, nx, ny, metric, ids, dist);
}

/* ------------------------------------------------------------------------ */
/* MergeTreeVSManager::searchWrapper, MergeTreeVSManager.cpp:1538-1680. */

static inline int bit_test(const uint8_t *bm, int64_t i) {
    return (bm[i >> 3] >> (i & 7)) & 1;
}

static int search_wrapper(knn_fn knn, int prewhere, float *query, int64_t nq,
                          float *base, int64_t nbase, int64_t d, int64_t k,
                          int64_t num_rows_read, int64_t *final_id,
                          float *final_dist, const int64_t *actual_id_in_range,
                          int metric, const uint8_t *row_exists_chunk,
                          int64_t delete_id_num) {
    const float init = (metric == ORC_IP) ? FLT_MIN : FLT_MAX;
    const int64_t kk = k + delete_id_num;
    float *per_dist = (float *)malloc(sizeof(float) * k * nq);
    int64_t *per_id = (int64_t *)malloc(sizeof(int64_t) * k * nq);
    float *tmp_dist = (float *)malloc(sizeof(float) * kk * nq);
    int64_t *tmp_id = (int64_t *)malloc(sizeof(int64_t) * kk * nq);
    for (int64_t i = 0; i < k * nq; i++) {
        per_dist[i] = init;
        per_id[i] = -1;
    }
    float *dd = delete_id_num > 0 ? tmp_dist : per_dist;
    int64_t *ii = delete_id_num > 0 ? tmp_id : per_id;
    int rc = search_without_index_impl(knn, query, base, d, kk, nq, nbase, metric, ii, dd);
    if (rc) goto out;
    if (delete_id_num > 0) {
        for (int64_t q = 0; q < nq; q++) {
            int64_t cur = 0, tcur = 0;
            while (cur < k && tcur < kk) {
                const int64_t tid = tmp_id[q * kk + tcur];
                if (tid >= 0 && bit_test(row_exists_chunk, tid)) {
                    per_id[q * k + cur] = tid;
                    per_dist[q * k + cur] = tmp_dist[q * kk + tcur];
                    ++cur;
                }
                ++tcur;
            }
        }
    }
    if (prewhere)
        for (int64_t i = 0; i < k * nq; i++)
            if (per_id[i] > -1) per_id[i] = actual_id_in_range[per_id[i]];
    {
        float *inter_d = (float *)malloc(sizeof(float) * k * nq);
        int64_t *inter_i = (int64_t *)malloc(sizeof(int64_t) * k * nq);
        for (int64_t q = 0; q < nq; q++) {
            int64_t j = q * k, z = q * k;
            for (int64_t i = 0; i < k; i++) {
                if ((metric != ORC_IP && final_dist[j] > per_dist[z]) ||
                    (metric == ORC_IP && final_dist[j] < per_dist[z])) {
                    inter_d[q * k + i] = per_dist[z];
                    inter_i[q * k + i] = per_id[z] + num_rows_read;
                    z++;
                } else {
                    inter_d[q * k + i] = final_dist[j];
                    inter_i[q * k + i] = final_id[j];
                    j++;
                }
            }
        }
        memcpy(final_dist, inter_d, sizeof(float) * k * nq);
        memcpy(final_id, inter_i, sizeof(int64_t) * k * nq);
        free(inter_d);
        free(inter_i);
    }
out:
    free(per_dist);
    free(per_id);
    free(tmp_dist);
    free(tmp_id);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* MergeTreeVSManager::vectorScanWithoutIndex, MergeTreeVSManager.cpp:960-1536
 * (FloatVector branch) with a single read range covering the whole part. */

static int vector_scan_impl(knn_fn knn, const float *rows, const uint8_t *nonempty,
                            int64_t n, int64_t d, const int64_t *mark_rows,
                            int64_t n_marks, const float *queries, int64_t nq,
                            int64_t k, int metric, const uint8_t *filter,
                            const uint8_t *row_exists, int64_t *out_ids,
                            float *out_dist) {
    if (metric != ORC_L2 && metric != ORC_IP && metric != ORC_COSINE) return -1;
    const float init = (metric == ORC_IP) ? FLT_MIN : FLT_MAX;
    for (int64_t i = 0; i < k * nq; i++) {
        out_dist[i] = init;
        out_ids[i] = -1;
    }
    if (n == 0 || nq == 0 || k <= 0) return 0;
    /* the query dataset object is shared across chunks (normalised in place
     * on every cosine call, VIWithDataPart.h:358) */
    float *query = (float *)malloc(sizeof(float) * nq * d);
    memcpy(query, queries, sizeof(float) * nq * d);
    int rc = 0;
    if (filter) {
        /* :1043-1331: one mark at a time; gather selected non-empty rows */
        int64_t filter_parsed = 0, row0 = 0;
        float *chunk = NULL;
        int64_t *actual = NULL;
        for (int64_t m = 0; m < n_marks && row0 < n; m++) {
            int64_t rows_m = mark_rows[m];
            if (row0 + rows_m > n) rows_m = n - row0;
            chunk = (float *)realloc(chunk, sizeof(float) * (rows_m > 0 ? rows_m : 1) * d);
            actual = (int64_t *)realloc(actual, sizeof(int64_t) * (rows_m > 0 ? rows_m : 1));
            int64_t left = 0;
            for (int64_t i = filter_parsed; i < filter_parsed + rows_m; i++) {
                if (i == n) break;
                if (bit_test(filter, i) && (!row_exists || bit_test(row_exists, i)) &&
                    (!nonempty || nonempty[i])) {
                    memcpy(chunk + left * d, rows + i * d, sizeof(float) * d);
                    actual[left] = i; /* current_rows_in_range, single range */
                    left++;
                }
            }
            filter_parsed += rows_m;
            row0 += rows_m;
            if (left == 0) continue;
            rc = search_wrapper(knn, 1, query, nq, chunk, left, d, k, 0, out_ids,
                                out_dist, actual, metric, NULL, 0);
            if (rc) break;
        }
        free(chunk);
        free(actual);
    } else {
        /* :1332-1498: uniform chunks of getMarkRows(0) rows */
        const int64_t chunk_rows = n_marks > 0 && mark_rows[0] > 0 ? mark_rows[0] : n;
        float *chunk = (float *)malloc(sizeof(float) * chunk_rows * d);
        uint8_t *exists = (uint8_t *)malloc((size_t)(chunk_rows + 7) / 8);
        for (int64_t r0 = 0; r0 < n; r0 += chunk_rows) {
            const int64_t rows_c = (n - r0) < chunk_rows ? (n - r0) : chunk_rows;
            /* src_vec.empty(): every array in the chunk is empty -> skipped */
            int any = 0;
            for (int64_t r = 0; r < rows_c && !any; r++) any = !nonempty || nonempty[r0 + r];
            if (!any) continue;
            memcpy(chunk, rows + r0 * d, sizeof(float) * rows_c * d);
            int64_t deleted = 0;
            memset(exists, 0xff, (size_t)(rows_c + 7) / 8);
            if (row_exists) {
                for (int64_t r = 0; r < rows_c; r++)
                    if (!bit_test(row_exists, r0 + r)) {
                        exists[r >> 3] &= (uint8_t)~(1u << (r & 7));
                        deleted++;
                    }
            }
            rc = search_wrapper(knn, 0, query, nq, chunk, rows_c, d, k, r0, out_ids,
                                out_dist, NULL, metric, exists, deleted);
            if (rc) break;
        }
        free(chunk);
        free(exists);
    }
    free(query);
    return rc;
}

int orc_vector_scan(const float *rows, const uint8_t *nonempty, int64_t n,
                    int64_t d, const int64_t *mark_rows, int64_t n_marks,
                    const float *queries, int64_t nq, int64_t k, int metric,
                    const uint8_t *filter, const uint8_t *row_exists,
                    int64_t *out_ids, float *out_dist) {
    return vector_scan_impl(orc_knn, rows, nonempty, n, d, mark_rows, n_marks, queries,
                            nq, k, metric, filter, row_exists, out_ids, out_dist);
}

int orc_vector_scan_fast(const float *rows, const uint8_t *nonempty, int64_t n,
                         int64_t d, const int64_t *mark_rows, int64_t n_marks,
                         const float *queries, int64_t nq, int64_t k,
                         int metric, const uint8_t *filter,
                         const uint8_t *row_exists, int64_t *out_ids,
                         float *out_dist) {
    return vector_scan_impl(orc_knn_fast, rows, nonempty, n, d, mark_rows, n_marks,
                            queries, nq, k, metric, filter, row_exists, out_ids,
                            out_dist);
}

/* ------------------------------------------------------------------------ */
/* Cross-part merge, MergeTreeBaseSearchManager.cpp:207-297: a multimap keyed
 * by score; equal scores keep insertion order (parts in order, labels in
 * their list order).  ASC takes the first k; DESC (IP) iterates in reverse,
 * so equal scores come out in reverse insertion order. */

typedef struct {
    float score;
    int64_t seq; /* insertion order */
    int64_t part, label;
} mm_entry;

static int mm_cmp(const void *a, const void *b) {
    const mm_entry *x = (const mm_entry *)a, *y = (const mm_entry *)b;
    if (x->score < y->score) return -1;
    if (x->score > y->score) return 1;
    return (x->seq < y->seq) ? -1 : (x->seq > y->seq);
}

void orc_merge_parts(int64_t nparts, int64_t k, int metric,
                     const int64_t *labels, const float *dists,
                     int64_t *out_part, int64_t *out_label, float *out_dist) {
    mm_entry *e = (mm_entry *)malloc(sizeof(mm_entry) * (nparts * k + 1));
    int64_t m = 0;
    for (int64_t p = 0; p < nparts; p++)
        for (int64_t i = 0; i < k; i++) {
            const int64_t lab = labels[p * k + i];
            if (lab < 0) continue;
            e[m].score = dists[p * k + i];
            e[m].seq = m;
            e[m].part = p;
            e[m].label = lab;
            m++;
        }
    qsort(e, (size_t)m, sizeof(mm_entry), mm_cmp);
    for (int64_t i = 0; i < k; i++) {
        out_part[i] = -1;
        out_label[i] = -1;
        out_dist[i] = (metric == ORC_IP) ? FLT_MIN : FLT_MAX;
    }
    for (int64_t i = 0; i < k && i < m; i++) {
        const mm_entry *s = (metric == ORC_IP) ? &e[m - 1 - i] : &e[i];
        out_part[i] = s->part;
        out_label[i] = s->label;
        out_dist[i] = s->score;
    }
    free(e);
}

/* ------------------------------------------------------------------------ */
/* STREAM triad a = b + s c over doubles (McCalpin's kernel and byte count:
 * 24 B per element), `threads` OpenMP threads, best of `reps`; returns GB/s.
 * Host DRAM bandwidth beside the CPU-baseline timing. */
double orc_stream_triad(int64_t n, int threads, int reps) {
    double *a = (double *)malloc(sizeof(double) * n), *b = (double *)malloc(sizeof(double) * n),
           *c = (double *)malloc(sizeof(double) * n);
    if (!a || !b || !c) {
        free(a);
        free(b);
        free(c);
        return -1.0;
    }
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < n; i++) {
        a[i] = 0.0;
        b[i] = 1.0;
        c[i] = 2.0;
    }
    double best = 0.0;
    for (int r = 0; r < reps; r++) {
        const double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int64_t i = 0; i < n; i++) a[i] = b[i] + 3.0 * c[i];
        const double t = omp_get_wtime() - t0;
        const double gbs = 24.0 * (double)n / t / 1e9;
        if (gbs > best) best = gbs;
    }
    volatile double sink = a[n / 2];
    (void)sink;
    free(a);
    free(b);
    free(c);
    return best;
}

/* ------------------------------------------------------------------------ */
/* Reference threading shape for CPU timing (see header). */

int orc_scan_parts(const float *rows, int64_t n, int64_t d, int64_t granule,
                   const float *queries, int64_t nq, int64_t k, int metric,
                   int parts, int threads, int64_t *out_ids, float *out_dist) {
    if (parts < 1) parts = 1;
    int64_t *pid = (int64_t *)malloc(sizeof(int64_t) * parts * nq * k);
    float *pdist = (float *)malloc(sizeof(float) * parts * nq * k);
    int rc = 0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : rc)
#endif
    for (int p = 0; p < parts; p++) {
        const int64_t r0 = n * p / parts, r1 = n * (p + 1) / parts;
        const int64_t g = granule;
        rc |= orc_vector_scan_fast(rows + r0 * d, NULL, r1 - r0, d, &g, 1, queries, nq, k,
                                   metric, NULL, NULL, pid + (int64_t)p * nq * k,
                                   pdist + (int64_t)p * nq * k);
        /* labels are part-local; make them global for the merged output */
        for (int64_t i = 0; i < nq * k; i++)
            if (pid[(int64_t)p * nq * k + i] >= 0) pid[(int64_t)p * nq * k + i] += r0;
    }
    (void)threads;
    int64_t *lab = (int64_t *)malloc(sizeof(int64_t) * parts * k);
    float *dd = (float *)malloc(sizeof(float) * parts * k);
    int64_t *opart = (int64_t *)malloc(sizeof(int64_t) * k);
    for (int64_t q = 0; q < nq; q++) {
        for (int p = 0; p < parts; p++) {
            memcpy(lab + p * k, pid + ((int64_t)p * nq + q) * k, sizeof(int64_t) * k);
            memcpy(dd + p * k, pdist + ((int64_t)p * nq + q) * k, sizeof(float) * k);
        }
        orc_merge_parts(parts, k, metric, lab, dd, opart, out_ids + q * k, out_dist + q * k);
    }
    free(lab);
    free(dd);
    free(opart);
    free(pid);
    free(pdist);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Counter-based synthetic generator. */

static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static inline float gen_gauss(uint64_t seed, uint64_t idx) {
    const uint64_t h = splitmix64(seed ^ idx);
    const float u0 = (float)(h & 0xffff) * (1.0f / 65536.0f);
    const float u1 = (float)((h >> 16) & 0xffff) * (1.0f / 65536.0f);
    const float u2 = (float)((h >> 32) & 0xffff) * (1.0f / 65536.0f);
    const float u3 = (float)((h >> 48) & 0xffff) * (1.0f / 65536.0f);
    const float s = (u0 + u1) + (u2 + u3);
    return (s - 2.0f) * 1.7320508f;
}

#define ORC_MIX_CENTERS 4096ULL
#define ORC_HARD_CENTERS 65536ULL /* mode 3: hard mixture, unit noise */

void orc_generate(uint64_t seed, int mode, int64_t row0, int64_t n, int64_t d,
                  float *out) {
    for (int64_t r = 0; r < n; r++) {
        const uint64_t row = (uint64_t)(row0 + r);
        const uint64_t c = splitmix64(seed ^ 0xC0FFEEULL ^ (row * 0x100000001B3ULL)) %
                           (mode == 3 ? ORC_HARD_CENTERS : ORC_MIX_CENTERS);
        for (int64_t j = 0; j < d; j++) {
            const uint64_t idx = row * (uint64_t)d + (uint64_t)j;
            float v;
            if (mode == 0) {
                v = (float)((int)(splitmix64(seed ^ idx) % 17ULL) - 8);
            } else if (mode == 1) {
                v = gen_gauss(seed, idx);
            } else if (mode == 2) {
                const float center = gen_gauss(seed ^ 0xCE17E5ULL, c * (uint64_t)d + (uint64_t)j);
                v = center + 0.25f * gen_gauss(seed, idx);
            } else {
                const float center = gen_gauss(seed ^ 0xCE17E5ULL, c * (uint64_t)d + (uint64_t)j);
                v = center + gen_gauss(seed, idx);
            }
            out[r * d + j] = v;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Binary vectors (FixedString(N) columns): tryBruteForceSearch<BinaryVector>
 * (BruteForceSearch.h:94-110).  The two callees live in the absent faiss fork
 * (contrib/search-index), so they are restated from upstream faiss
 * (utils/hamming.cpp, hammings_knn_mc; unpinned version) and from the
 * reference's own KAT 00038_mqvs_binary_vector_feature for jaccard_knn. */

static inline int popc8(uint8_t v) { return __builtin_popcount((unsigned)v); }

/* faiss::hammings_knn_mc with HCounterState: per query, counters[d] and up to
 * k ids per distance in arrival order (j ascending).  update_counter:
 *   dis <= thres:  dis < thres -> store, ++count_lt, and while count_lt == k
 *                  lower thres (count_eq = counters[thres], count_lt -= it);
 *                  dis == thres -> store only while count_eq < k.
 * Output: distances b = 0 .. nBit-1 (b < nBit: a row whose every bit differs
 * is never returned), k per query, padding -1 / INT32_MAX. */
int orc_hamming_knn(const uint8_t *x, const uint8_t *y, int64_t nbytes, int64_t k,
                    int64_t nx, int64_t ny, int64_t *ids, int32_t *dist) {
    const int nbit = (int)(nbytes * 8);
    int *counters = (int *)malloc(sizeof(int) * (nbit + 1));
    int64_t *per = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nbit + 1) * (size_t)(k > 0 ? k : 1));
    for (int64_t i = 0; i < nx; i++) {
        memset(counters, 0, sizeof(int) * (nbit + 1));
        int thres = nbit + 1, count_lt = 0, count_eq = 0;
        const uint8_t *xi = x + i * nbytes;
        for (int64_t j = 0; j < ny; j++) {
            const uint8_t *yj = y + j * nbytes;
            int dis = 0;
            for (int64_t b = 0; b < nbytes; b++) dis += popc8(xi[b] ^ yj[b]);
            if (dis > thres) continue;
            if (dis < thres) {
                per[(int64_t)dis * k + counters[dis]++] = j;
                ++count_lt;
                while (count_lt == k && thres > 0) {
                    --thres;
                    count_eq = counters[thres];
                    count_lt -= count_eq;
                }
            } else if (count_eq < k) {
                per[(int64_t)dis * k + count_eq++] = j;
                counters[dis] = count_eq;
            }
        }
        int64_t nres = 0;
        for (int b = 0; b < nbit && nres < k; b++)
            for (int l = 0; l < counters[b] && nres < k; l++) {
                ids[i * k + nres] = per[(int64_t)b * k + l];
                dist[i * k + nres] = b;
                nres++;
            }
        for (; nres < k; nres++) {
            ids[i * k + nres] = -1;
            dist[i * k + nres] = 2147483647;
        }
    }
    free(counters);
    free(per);
    return 0;
}

/* Jaccard distance of two codes.  The reference's KAT 00038 pins the fp32
 * form (den - num) / den (1 - num/den misses 0.2 and 0.22222222 by an ulp);
 * num == 0 -> 1.0 (assumed; equal to the formula unless both codes are 0). */
float orc_jaccard(const uint8_t *a, const uint8_t *b, int64_t nbytes) {
    int num = 0, den = 0;
    for (int64_t i = 0; i < nbytes; i++) {
        num += popc8(a[i] & b[i]);
        den += popc8(a[i] | b[i]);
    }
    if (num == 0) return 1.0f;
    return (float)(den - num) / (float)den;
}

/* jaccard_knn (faiss fork, absent): a max-heap of k entries that a row enters
 * only when strictly better than the current worst; output ordered by
 * (distance, row).  Equivalently: the k smallest by (distance, row). */
int orc_jaccard_knn(const uint8_t *x, const uint8_t *y, int64_t nbytes, int64_t k,
                    int64_t nx, int64_t ny, int64_t *ids, float *dist) {
    float *val = (float *)malloc(sizeof(float) * (size_t)(k > 0 ? k : 1));
    int64_t *lab = (int64_t *)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
    for (int64_t i = 0; i < nx; i++) {
        for (int64_t j = 0; j < k; j++) {
            val[j] = FLT_MAX;
            lab[j] = -1;
        }
        heap_heapify(1, k, val, lab);
        for (int64_t j = 0; j < ny; j++) {
            const float dis = orc_jaccard(x + i * nbytes, y + j * nbytes, nbytes);
            if (dis < val[0]) heap_replace_top(1, k, val, lab, dis, j);
        }
        heap_reorder(1, k, val, lab);
        memcpy(dist + i * k, val, sizeof(float) * k);
        memcpy(ids + i * k, lab, sizeof(int64_t) * k);
    }
    free(val);
    free(lab);
    return 0;
}

/* tryBruteForceSearch<BinaryVector>: d in bits.  Hamming writes int32 counts
 * into the float buffer (the reference's reinterpret_cast<int32_t*>). */
int orc_knn_binary(const uint8_t *x, const uint8_t *y, int64_t d, int64_t k, int64_t nx,
                   int64_t ny, int metric, int64_t *ids, float *dist) {
    if (metric == ORC_HAMMING) return orc_hamming_knn(x, y, d / 8, k, nx, ny, ids, (int32_t *)dist);
    if (metric == ORC_JACCARD) return orc_jaccard_knn(x, y, d / 8, k, nx, ny, ids, dist);
    return -1;
}

/* searchWrapper (MergeTreeVSManager.cpp:1538-1680) for binary chunks: per
 * chunk k + deleted results, drop deleted rows, PREWHERE id remap, strict
 * two-pointer merge (ascending).  Hamming's int32 counts are compared by the
 * reference as the float bit patterns (positive denormals, same order as the
 * integers; INT32_MAX padding is NaN and never enters); here they are
 * converted to the float values the SQL prints (KAT 00038). */
static void search_wrapper_binary(int prewhere, const uint8_t *query, int64_t nq,
                                  const uint8_t *base, int64_t nbase, int64_t nbytes, int64_t k,
                                  int64_t num_rows_read, int64_t *final_id, float *final_dist,
                                  const int64_t *actual, int metric, const uint8_t *exists_chunk,
                                  int64_t del) {
    const int64_t kk = k + del;
    int64_t *tid = (int64_t *)malloc(sizeof(int64_t) * kk * nq);
    float *tdist = (float *)malloc(sizeof(float) * kk * nq);
    int64_t *per_id = (int64_t *)malloc(sizeof(int64_t) * k * nq);
    float *per_dist = (float *)malloc(sizeof(float) * k * nq);
    for (int64_t i = 0; i < k * nq; i++) {
        per_id[i] = -1;
        per_dist[i] = FLT_MAX;
    }
    if (metric == ORC_HAMMING) {
        int32_t *hd = (int32_t *)malloc(sizeof(int32_t) * kk * nq);
        orc_hamming_knn(query, base, nbytes, kk, nq, nbase, tid, hd);
        for (int64_t i = 0; i < kk * nq; i++) tdist[i] = tid[i] >= 0 ? (float)hd[i] : FLT_MAX;
        free(hd);
    } else {
        orc_jaccard_knn(query, base, nbytes, kk, nq, nbase, tid, tdist);
    }
    for (int64_t q = 0; q < nq; q++) {
        int64_t cur = 0;
        for (int64_t t = 0; t < kk && cur < k; t++) {
            const int64_t id = tid[q * kk + t];
            if (id < 0) continue;
            if (exists_chunk && !bit_test(exists_chunk, id)) continue;
            per_id[q * k + cur] = prewhere ? actual[id] : id;
            per_dist[q * k + cur] = tdist[q * kk + t];
            cur++;
        }
    }
    float *inter_d = (float *)malloc(sizeof(float) * k * nq);
    int64_t *inter_i = (int64_t *)malloc(sizeof(int64_t) * k * nq);
    for (int64_t q = 0; q < nq; q++) {
        int64_t j = q * k, z = q * k;
        for (int64_t i = 0; i < k; i++) {
            if (final_dist[j] > per_dist[z]) {
                inter_d[q * k + i] = per_dist[z];
                inter_i[q * k + i] = per_id[z] + num_rows_read;
                z++;
            } else {
                inter_d[q * k + i] = final_dist[j];
                inter_i[q * k + i] = final_id[j];
                j++;
            }
        }
    }
    memcpy(final_dist, inter_d, sizeof(float) * k * nq);
    memcpy(final_id, inter_i, sizeof(int64_t) * k * nq);
    free(inter_d);
    free(inter_i);
    free(tid);
    free(tdist);
    free(per_id);
    free(per_dist);
}

/* vectorScanWithoutIndex<BinaryVector> (MergeTreeVSManager.cpp:1188-1273
 * filtered gather of FixedString rows, :1395-1425 whole-chunk copy): codes
 * n x nbytes; same chunking, filter and delete handling as the float path. */
int orc_vector_scan_binary(const uint8_t *rows, int64_t n, int64_t nbytes,
                           const int64_t *mark_rows, int64_t n_marks, const uint8_t *queries,
                           int64_t nq, int64_t k, int metric, const uint8_t *filter,
                           const uint8_t *row_exists, int64_t *out_ids, float *out_dist) {
    if (metric != ORC_HAMMING && metric != ORC_JACCARD) return -1;
    for (int64_t i = 0; i < k * nq; i++) {
        out_dist[i] = FLT_MAX;
        out_ids[i] = -1;
    }
    if (n == 0 || nq == 0 || k <= 0) return 0;
    if (filter) {
        int64_t parsed = 0;
        uint8_t *chunk = NULL;
        int64_t *actual = NULL;
        for (int64_t m = 0; m < n_marks && parsed < n; m++) {
            int64_t rows_m = mark_rows[m];
            if (parsed + rows_m > n) rows_m = n - parsed;
            chunk = (uint8_t *)realloc(chunk, (size_t)(rows_m > 0 ? rows_m : 1) * nbytes);
            actual = (int64_t *)realloc(actual, sizeof(int64_t) * (rows_m > 0 ? rows_m : 1));
            int64_t left = 0;
            for (int64_t i = parsed; i < parsed + rows_m; i++)
                if (bit_test(filter, i) && (!row_exists || bit_test(row_exists, i))) {
                    memcpy(chunk + left * nbytes, rows + i * nbytes, nbytes);
                    actual[left++] = i;
                }
            parsed += rows_m;
            if (left == 0) continue;
            search_wrapper_binary(1, queries, nq, chunk, left, nbytes, k, 0, out_ids, out_dist, actual,
                                  metric, NULL, 0);
        }
        free(chunk);
        free(actual);
    } else {
        const int64_t chunk_rows = n_marks > 0 && mark_rows[0] > 0 ? mark_rows[0] : n;
        uint8_t *exists = (uint8_t *)malloc((size_t)(chunk_rows + 7) / 8);
        for (int64_t r0 = 0; r0 < n; r0 += chunk_rows) {
            const int64_t rows_c = (n - r0) < chunk_rows ? (n - r0) : chunk_rows;
            int64_t del = 0;
            memset(exists, 0xff, (size_t)(rows_c + 7) / 8);
            if (row_exists)
                for (int64_t r = 0; r < rows_c; r++)
                    if (!bit_test(row_exists, r0 + r)) {
                        exists[r >> 3] &= (uint8_t)~(1u << (r & 7));
                        del++;
                    }
            search_wrapper_binary(0, queries, nq, rows + r0 * nbytes, rows_c, nbytes, k, r0, out_ids,
                                  out_dist, NULL, metric, del ? exists : NULL, del);
        }
        free(exists);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Column ingest: a MergeTree Array(Float32) column as its
 * compressed files -- the nested Float32 stream (`<col>.bin`) and the array
 * sizes stream (`<col>.size0.bin`, UInt64 per row) -- decoded into the rows
 * matrix of MergeTreeVSManager.cpp:1381-1393.
 *
 * Framing (CompressedReadBufferBase.cpp:115-160, CompressionInfo.h:22-49):
 * per block 16-B CityHash128 checksum, then a 9-B header: method byte
 * (0x82 LZ4, 0x02 NONE), UInt32 compressed size (header + payload), UInt32
 * decompressed size; then the payload.
 *
 * LZ4 block format as LZ4_decompress_faster.cpp:480-640 decodes it: token
 * (literal length high nibble, match length - 4 low nibble, 15 = extended by
 * 255-continued bytes), literals, 2-B little-endian offset, match copy (may
 * overlap); the block ends when a literal run reaches the decompressed size. */

static inline uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Block checksum: CityHash128 v1.0.2 (the pre-1.0.3 variant ClickHouse keeps,
 * contrib/cityhash102/src/city.cc:256-358, Hash128to64 city.h:91-100) over
 * the 9-B header + payload, validated before decompression
 * (CompressedReadBufferBase.cpp:37-45, 192-196; written by
 * CompressedWriteBuffer.cpp:44).  Restated on 64-bit little-endian words;
 * h[0] = low half (uint128.first), h[1] = high half; the stored 16 checksum
 * bytes are h[0] then h[1], little-endian. */
static const uint64_t CH_K0 = 0xc3a5c85c97cb3127ULL, CH_K1 = 0xb492b66fbe98f273ULL,
                      CH_K2 = 0x9ae16a3b2f90404fULL, CH_K3 = 0xc949d7c7509e6557ULL;

static inline uint64_t ch_ld64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
static inline uint64_t ch_ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t ch_ror(uint64_t v, int s) { return s ? (v >> s) | (v << (64 - s)) : v; }
static inline uint64_t ch_mix47(uint64_t v) { return v ^ (v >> 47); }
/* Hash128to64(uint128(lo, hi)) */
static inline uint64_t ch_pair(uint64_t lo, uint64_t hi) {
    const uint64_t m = 0x9ddfea08eb382d69ULL;
    uint64_t a = ch_mix47((lo ^ hi) * m);
    uint64_t b = ch_mix47((hi ^ a) * m);
    return b * m;
}
static uint64_t ch_short(const uint8_t *s, uint64_t len) { /* HashLen0to16, city.cc:125-144 */
    if (len > 8) {
        const uint64_t a = ch_ld64(s), b = ch_ld64(s + len - 8);
        return ch_pair(a, ch_ror(b + len, (int)len)) ^ b;
    }
    if (len >= 4) return ch_pair(len + (ch_ld32(s) << 3), ch_ld32(s + len - 4));
    if (len > 0) {
        const uint32_t y = (uint32_t)s[0] + ((uint32_t)s[len >> 1] << 8);
        const uint32_t z = (uint32_t)len + ((uint32_t)s[len - 1] << 2);
        return ch_mix47(y * CH_K2 ^ z * CH_K3) * CH_K2;
    }
    return CH_K2;
}
/* WeakHashLen32WithSeeds over s[0, 32) (city.cc:159-179) */
static inline void ch_weak32(const uint8_t *s, uint64_t a, uint64_t b, uint64_t *o1, uint64_t *o2) {
    const uint64_t w = ch_ld64(s), x = ch_ld64(s + 8), y = ch_ld64(s + 16), z = ch_ld64(s + 24);
    a += w;
    b = ch_ror(b + a + z, 21);
    const uint64_t c = a;
    a += x + y;
    b += ch_ror(a, 44);
    *o1 = a + z;
    *o2 = b + c;
}
/* CityMurmur (city.cc:256-284): len < 128 */
static void ch_murmur(const uint8_t *s, uint64_t len, uint64_t a, uint64_t b, uint64_t h[2]) {
    uint64_t c, d;
    if (len <= 16) {
        a = ch_mix47(a * CH_K1) * CH_K1;
        c = b * CH_K1 + ch_short(s, len);
        d = ch_mix47(a + (len >= 8 ? ch_ld64(s) : c));
    } else {
        c = ch_pair(ch_ld64(s + len - 8) + CH_K1, a);
        d = ch_pair(b + len, c + ch_ld64(s + len - 16));
        a += d;
        for (int64_t l = (int64_t)len - 16; l > 0; l -= 16, s += 16) {
            a ^= ch_mix47(ch_ld64(s) * CH_K1) * CH_K1;
            a *= CH_K1;
            b ^= a;
            c ^= ch_mix47(ch_ld64(s + 8) * CH_K1) * CH_K1;
            c *= CH_K1;
            d ^= c;
        }
    }
    a = ch_pair(a, c);
    b = ch_pair(d, b);
    h[0] = a ^ b;
    h[1] = ch_pair(b, a);
}
/* CityHash128WithSeed (city.cc:286-342), seed = (lo, hi) */
static void ch_seeded(const uint8_t *s, uint64_t len, uint64_t lo, uint64_t hi, uint64_t h[2]) {
    if (len < 128) {
        ch_murmur(s, len, lo, hi, h);
        return;
    }
    uint64_t x = lo, y = hi, z = len * CH_K1;
    uint64_t v1 = ch_ror(y ^ CH_K1, 49) * CH_K1 + ch_ld64(s);
    uint64_t v2 = ch_ror(v1, 42) * CH_K1 + ch_ld64(s + 8);
    uint64_t w1 = ch_ror(y + z, 35) * CH_K1 + x;
    uint64_t w2 = ch_ror(x + ch_ld64(s + 88), 53) * CH_K1;
    do { /* two 64-byte rounds per 128 bytes */
        for (int r = 0; r < 2; r++) {
            x = ch_ror(x + y + v1 + ch_ld64(s + 16), 37) * CH_K1;
            y = ch_ror(y + v2 + ch_ld64(s + 48), 42) * CH_K1;
            x ^= w2;
            y ^= v1;
            z = ch_ror(z ^ w1, 33);
            ch_weak32(s, v2 * CH_K1, x + w1, &v1, &v2);
            ch_weak32(s + 32, z + w2, y, &w1, &w2);
            const uint64_t t = z;
            z = x;
            x = t;
            s += 64;
        }
        len -= 128;
    } while (len >= 128);
    y += ch_ror(w1, 37) * CH_K0 + z;
    x += ch_ror(v1 + z, 49) * CH_K0;
    for (uint64_t done = 0; done < len;) { /* up to four 32-byte tail pieces, from the end */
        done += 32;
        y = ch_ror(y - x, 42) * CH_K0 + v2;
        w1 += ch_ld64(s + len - done + 16);
        x = ch_ror(x, 49) * CH_K0 + w1;
        w1 += v1;
        ch_weak32(s + len - done, v1, v2, &v1, &v2);
    }
    x = ch_pair(x, v1);
    y = ch_pair(y, w1);
    h[0] = ch_pair(x + v2, w2) + y;
    h[1] = ch_pair(x + w2, y + v2);
}
/* CityHash128 (city.cc:344-358) */
void orc_cityhash128(const uint8_t *s, int64_t len, uint64_t h[2]) {
    const uint64_t n = (uint64_t)len;
    if (n >= 16)
        ch_seeded(s + 16, n - 16, ch_ld64(s) ^ CH_K3, ch_ld64(s + 8), h);
    else if (n >= 8)
        ch_seeded(NULL, 0, ch_ld64(s) ^ (n * CH_K0), ch_ld64(s + n - 8) ^ CH_K1, h);
    else
        ch_seeded(s, n, CH_K0, CH_K1, h);
}

/* Returns 0, or -1 on malformed input (ClickHouse: CANNOT_DECOMPRESS). */
int orc_lz4_decompress(const uint8_t *src, int64_t src_size, uint8_t *dst, int64_t dst_size) {
    const uint8_t *ip = src, *iend = src + src_size;
    uint8_t *op = dst, *oend = dst + dst_size;
    for (;;) {
        if (ip >= iend) return -1;
        const unsigned token = *ip++;
        size_t length = token >> 4;
        if (length == 15) {
            unsigned s;
            do {
                if (ip >= iend) return -1;
                s = *ip++;
                length += s;
            } while (s == 255);
        }
        if ((int64_t)length > oend - op || (int64_t)length > iend - ip) return -1;
        memcpy(op, ip, length);
        op += length;
        ip += length;
        if (op == oend) return 0;
        if (iend - ip < 2) return -1;
        const size_t offset = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        if (offset == 0 || (int64_t)offset > op - dst) return -1;
        length = token & 15;
        if (length == 15) {
            unsigned s;
            do {
                if (ip >= iend) return -1;
                s = *ip++;
                length += s;
            } while (s == 255);
        }
        length += 4;
        if ((int64_t)length > oend - op) return -1;
        const uint8_t *match = op - offset;
        for (size_t i = 0; i < length; i++) op[i] = match[i]; /* byte order: overlap replicates */
        op += length;
    }
}

/* Test-data LZ4 compressor (greedy, 4-byte hash, 64 KiB window) producing the
 * standard block format (last 5 bytes literal, no match starting in the last
 * 12 bytes).  Returns the compressed size, or -1 if cap is too small. */
int64_t orc_lz4_compress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
    enum { HBITS = 16 };
    int64_t *table = (int64_t *)malloc(sizeof(int64_t) << HBITS);
    for (int64_t i = 0; i < ((int64_t)1 << HBITS); i++) table[i] = -1;
    int64_t ip = 0, anchor = 0, o = 0;
    const int64_t mflimit = n - 12;
#define EMIT_LEN(v)                                       \
    do {                                                  \
        int64_t v_ = (v);                                 \
        while (v_ >= 255) {                               \
            if (o >= cap) goto fail;                      \
            dst[o++] = 255;                               \
            v_ -= 255;                                    \
        }                                                 \
        if (o >= cap) goto fail;                          \
        dst[o++] = (uint8_t)v_;                           \
    } while (0)
    while (ip < mflimit) {
        const uint32_t seq = rd32(src + ip);
        const uint32_t h = (seq * 2654435761u) >> (32 - HBITS);
        const int64_t ref = table[h];
        table[h] = ip;
        if (ref < 0 || ip - ref > 65535 || rd32(src + ref) != seq) {
            ip++;
            continue;
        }
        int64_t mlen = 4;
        while (ip + mlen < n - 5 && src[ref + mlen] == src[ip + mlen]) mlen++;
        const int64_t lit = ip - anchor;
        if (o >= cap) goto fail;
        const int64_t tok = o++;
        dst[tok] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mlen - 4 >= 15 ? 15 : mlen - 4));
        if (lit >= 15) EMIT_LEN(lit - 15);
        if (o + lit + 2 > cap) goto fail;
        memcpy(dst + o, src + anchor, lit);
        o += lit;
        dst[o++] = (uint8_t)((ip - ref) & 255);
        dst[o++] = (uint8_t)((ip - ref) >> 8);
        if (mlen - 4 >= 15) EMIT_LEN(mlen - 4 - 15);
        ip += mlen;
        anchor = ip;
    }
    {
        const int64_t lit = n - anchor;
        if (o >= cap) goto fail;
        dst[o++] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
        if (lit >= 15) EMIT_LEN(lit - 15);
        if (o + lit > cap) goto fail;
        memcpy(dst + o, src + anchor, lit);
        o += lit;
    }
#undef EMIT_LEN
    free(table);
    return o;
fail:
    free(table);
    return -1;
}

/* CompressedWriteBuffer framing of `n` bytes in blocks of at most block_size
 * (method 0x82 LZ4 or 0x02 NONE), each with its CityHash128 checksum. */
int64_t orc_compress_stream(const uint8_t *src, int64_t n, int64_t block_size, int method, uint8_t *dst,
                            int64_t cap) {
    int64_t o = 0;
    for (int64_t b = 0; b < n; b += block_size) {
        const int64_t len = (n - b) < block_size ? (n - b) : block_size;
        if (o + 25 > cap) return -1;
        memset(dst + o, 0, 16);
        uint8_t *hdr = dst + o + 16;
        int64_t payload;
        if (method == 0x02) {
            if (o + 25 + len > cap) return -1;
            memcpy(hdr + 9, src + b, len);
            payload = len;
        } else {
            payload = orc_lz4_compress(src + b, len, hdr + 9, cap - (o + 25));
            if (payload < 0) return -1;
        }
        hdr[0] = (uint8_t)method;
        const uint32_t csize = (uint32_t)(9 + payload), usize = (uint32_t)len;
        memcpy(hdr + 1, &csize, 4);
        memcpy(hdr + 5, &usize, 4);
        uint64_t h[2];
        orc_cityhash128(hdr, csize, h);
        memcpy(dst + o, h, 16);
        o += 25 + payload;
    }
    return o;
}

/* CompressedReadBuffer over a whole stream: returns the decompressed size,
 * -1 (malformed framing / payload, or more than cap bytes) or -2 (a block
 * checksum does not match; checked first, when verify != 0). */
int64_t orc_decompress_stream(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int verify) {
    int64_t pos = 0, o = 0;
    while (pos < n) {
        if (n - pos < 25) return -1;
        const uint8_t method = src[pos + 16];
        const int64_t csize = rd32(src + pos + 17), usize = rd32(src + pos + 21);
        if (csize < 9 || pos + 16 + csize > n || o + usize > cap) return -1;
        if (verify) {
            uint64_t h[2];
            orc_cityhash128(src + pos + 16, csize, h);
            if (memcmp(h, src + pos, 16)) return -2; /* CHECKSUM_DOESNT_MATCH */
        }
        const uint8_t *payload = src + pos + 25;
        if (method == 0x82) {
            if (orc_lz4_decompress(payload, csize - 9, dst + o, usize)) return -1;
        } else if (method == 0x02) {
            if (csize - 9 != usize) return -1;
            memcpy(dst + o, payload, usize);
        } else {
            return -1;
        }
        o += usize;
        pos += 16 + csize;
    }
    return o;
}

/* MergeTreeVSManager.cpp:1381-1393: rows pre-filled with FLT_MAX; a non-empty
 * array copies its first min(size, d) elements (a shorter one keeps FLT_MAX
 * in the rest); nonempty[r] = size > 0.  Returns -1 if the sizes need more
 * elements than `nelem`. */
int orc_array_rows(const float *data, int64_t nelem, const uint64_t *sizes, int64_t n, int64_t d, float *rows,
                   uint8_t *nonempty) {
    int64_t off = 0;
    for (int64_t r = 0; r < n; r++) {
        const int64_t sz = (int64_t)sizes[r];
        if (off + sz > nelem) return -1;
        for (int64_t j = 0; j < d; j++) rows[r * d + j] = (j < sz) ? data[off + j] : FLT_MAX;
        nonempty[r] = sz > 0;
        off += sz;
    }
    return off == nelem ? 0 : -1;
}
