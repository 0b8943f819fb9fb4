/*
 * mqvs_oracle.h -- CPU restatement of MyScaleDB's brute-force vector-scan path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libmqvs.so, myscaledb_amd/)
 * may link, load or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, as the checker / the timed CPU baseline.
 *
 * Pinning: the reference cannot be built here (contrib/search-index, the faiss
 * fork that holds knn_L2sqr/knn_inner_product, is an empty submodule), so this
 * restatement is pinned by the reference's own SQL known-answer tests
 * (tests/queries/2_vector_search/NNNNN_*.reference), re-stated as fixtures under
 * tests/golden/ and checked by tests/test_oracle_kat.py.
 *
 * Numeric conventions (documented assumptions; faiss is unpinned):
 *   - fvec_* (direct distances, norms; the nx < 20 branch): sequential fp32
 *     over k = 0..d-1 from 0, product rounded then added (pinned by KATs);
 *   - the sgemm of the nx >= 20 branch: sequential fp32 fma chain (assumed);
 *   - VectorDataset::normalize uses separate multiply and add (the ClickHouse
 *     build has no FMA for that loop), sqrtf and a true division;
 *   - nx < 20 uses the direct formula, nx >= 20 the faiss BLAS formula
 *     (|x|^2 + |y|^2) - 2<x,y> clamped at 0;
 *   - heap semantics: an element enters only when strictly better than the
 *     current worst; results ordered by (distance, row id).
 */
#ifndef MQVS_ORACLE_H
#define MQVS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_L2 = 0, ORC_IP = 1, ORC_COSINE = 2, ORC_HAMMING = 4, ORC_JACCARD = 5 };

/* faiss distance_compute_blas_threshold */
#define ORC_BLAS_THRESHOLD 20

float orc_l2sqr(const float *x, const float *y, int64_t d);
float orc_inner_product(const float *x, const float *y, int64_t d);
float orc_norm_l2sqr(const float *x, int64_t d);
float orc_gemm_dot(const float *x, const float *y, int64_t d);
float orc_gemm_dot_blocked(const float *x, const float *y, int64_t d, int64_t kb);

/* VectorDataset<Float>::normalize (VectorDataset.h:98-117), in place. */
void orc_normalize(float *data, int64_t n, int64_t d);

/* tryBruteForceSearch<FloatVector> (BruteForceSearch.h:62-111) -> faiss
 * knn_L2sqr / knn_inner_product. metric is ORC_L2 or ORC_IP; anything else
 * returns -1 (NOT_IMPLEMENTED).  ids/dist are caller-owned nx*k. */
int orc_knn(const float *x, const float *y, int64_t d, int64_t k, int64_t nx,
            int64_t ny, int metric, int64_t *ids, float *dist);

/* Same contract and bit-identical output as orc_knn, written for speed
 * (blocked, vectorisable across rows/queries; each (query,row) pair is still
 * one sequential fma chain).  Used as the timed CPU baseline. */
int orc_knn_fast(const float *x, const float *y, int64_t d, int64_t k,
                 int64_t nx, int64_t ny, int metric, int64_t *ids, float *dist);

/* VIWithColumnInPart::searchWithoutIndex (VIWithDataPart.h:341-382).
 * For cosine, normalises x and y IN PLACE, runs IP, then dist = 1 - dist. */
int orc_search_without_index(float *x, float *y, int64_t d, int64_t k,
                             int64_t nx, int64_t ny, int metric, int64_t *ids,
                             float *dist);

/* MergeTreeVSManager::vectorScanWithoutIndex + searchWrapper
 * (MergeTreeVSManager.cpp:960-1680) over one data part.
 *   rows      n*d, dense; rows whose Array was empty are FLT_MAX-filled
 *             (the no-filter copy loop, :1381-1393)
 *   nonempty  n bytes (1 = array non-empty) or NULL for all non-empty
 *   mark_rows rows per mark (index_granularity), n_marks entries
 *   filter    PREWHERE bitmap, LSB-first, n bits, or NULL
 *   row_exists lightweight-delete mask, LSB-first, n bits (1 = live), or NULL
 *   out_ids/out_dist nq*k, -1 ids where fewer than k results.
 * Returns 0, or -1 for an unsupported metric. */
int orc_vector_scan(const float *rows, const uint8_t *nonempty, int64_t n,
                    int64_t d, const int64_t *mark_rows, int64_t n_marks,
                    const float *queries, int64_t nq, int64_t k, int metric,
                    const uint8_t *filter, const uint8_t *row_exists,
                    int64_t *out_ids, float *out_dist);

/* Same as orc_vector_scan but every per-chunk knn goes through orc_knn_fast;
 * `threads` > 1 runs independent parts in parallel is NOT done here (one part
 * = one thread, VIWithDataPart.h:350); see orc_scan_parts. */
int orc_vector_scan_fast(const float *rows, const uint8_t *nonempty, int64_t n,
                         int64_t d, const int64_t *mark_rows, int64_t n_marks,
                         const float *queries, int64_t nq, int64_t k,
                         int metric, const uint8_t *filter,
                         const uint8_t *row_exists, int64_t *out_ids,
                         float *out_dist);

/* The reference's threading shape for CPU timing: `parts` equal row-range
 * parts, each scanned single-threaded (VIWithDataPart.h:350), up to `threads`
 * parts at a time (MergeTreeSelectWithHybridSearchProcessor.cpp:1212-1241),
 * then the cross-part top-k merge (MergeTreeBaseSearchManager.cpp:207-297).
 * Uniform granularity `granule` rows.  Returns 0. */
/* CPU-baseline helpers: AVX-512 micro-kernel in use by orc_knn_fast (runtime
 * CPU check; ORC_NO_AVX512=1 disables it), STREAM triad GB/s. */
int orc_has_avx512(void);
double orc_stream_triad(int64_t n, int threads, int reps);
int orc_scan_parts(const float *rows, int64_t n, int64_t d, int64_t granule,
                   const float *queries, int64_t nq, int64_t k, int metric,
                   int parts, int threads, int64_t *out_ids, float *out_dist);

/* Cross-part top-k merge (MergeTreeBaseSearchManager::getTotalTopSearchResultImpl,
 * MergeTreeBaseSearchManager.cpp:207-297) for one query: nparts lists of up
 * to k (label, dist), label -1 = empty.  Output (part, label, dist), k entries,
 * part = -1 where fewer than k. */
void orc_merge_parts(int64_t nparts, int64_t k, int metric,
                     const int64_t *labels, const float *dists,
                     int64_t *out_part, int64_t *out_label, float *out_dist);

/* Counter-based synthetic generator; must match the device
 * generator in libmqvs bit for bit.  mode 0 = exact integers in [-8, 8],
 * mode 1 = approx N(0,1) (Irwin-Hall of 4), mode 2 = Gaussian mixture. */
void orc_generate(uint64_t seed, int mode, int64_t row0, int64_t n, int64_t d,
                  float *out);

/* ---- binary vectors (FixedString(N)), BruteForceSearch.h:94-110 ----------
 * faiss::hammings_knn_mc restated (upstream faiss utils/hamming.cpp, version
 * unpinned): k nearest by (distance, row), distances < d bits only, int32
 * counts, padding -1 / INT32_MAX. */
int orc_hamming_knn(const uint8_t *x, const uint8_t *y, int64_t nbytes, int64_t k,
                    int64_t nx, int64_t ny, int64_t *ids, int32_t *dist);
/* Jaccard distance, fp32 (den - num) / den, 1.0 when the codes share no bit
 * (pinned by KAT 00038). */
float orc_jaccard(const uint8_t *a, const uint8_t *b, int64_t nbytes);
/* jaccard_knn (absent faiss fork): k smallest by (distance, row); -1/FLT_MAX pad. */
int orc_jaccard_knn(const uint8_t *x, const uint8_t *y, int64_t nbytes, int64_t k,
                    int64_t nx, int64_t ny, int64_t *ids, float *dist);
/* tryBruteForceSearch<BinaryVector>: d in bits; Hamming distances are int32
 * stored in the float buffer; other metrics -> -1 (NOT_IMPLEMENTED). */
int orc_knn_binary(const uint8_t *x, const uint8_t *y, int64_t d, int64_t k, int64_t nx,
                   int64_t ny, int metric, int64_t *ids, float *dist);
/* vectorScanWithoutIndex<BinaryVector> over one part (codes n x nbytes);
 * Hamming distances as float values, ascending; -1 / FLT_MAX padding. */
int orc_vector_scan_binary(const uint8_t *rows, int64_t n, int64_t nbytes,
                           const int64_t *mark_rows, int64_t n_marks, const uint8_t *queries,
                           int64_t nq, int64_t k, int metric, const uint8_t *filter,
                           const uint8_t *row_exists, int64_t *out_ids, float *out_dist);

/* ---- column ingest: MergeTree Array(Float32) files -> rows -------------
 * LZ4 block format as src/Compression/LZ4_decompress_faster.cpp:480-640
 * decodes it; 0 or -1 (CANNOT_DECOMPRESS). */
int orc_lz4_decompress(const uint8_t *src, int64_t src_size, uint8_t *dst, int64_t dst_size);
/* test-data compressor (standard LZ4 block format); size or -1 */
int64_t orc_lz4_compress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);
/* CompressedWriteBuffer / CompressedReadBuffer framing (CityHash128 block checksums) */
int64_t orc_compress_stream(const uint8_t *src, int64_t n, int64_t block_size, int method, uint8_t *dst,
                            int64_t cap);
int64_t orc_decompress_stream(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int verify);
/* CityHash128 v1.0.2 (contrib/cityhash102/src/city.cc:344-358): h[0] low, h[1] high */
void orc_cityhash128(const uint8_t *s, int64_t len, uint64_t h[2]);
/* MergeTreeVSManager.cpp:1381-1393 copy loop: FLT_MAX fill, truncation at d */
int orc_array_rows(const float *data, int64_t nelem, const uint64_t *sizes, int64_t n, int64_t d, float *rows,
                   uint8_t *nonempty);

#ifdef __cplusplus
}
#endif
#endif
