/*
 * mqvs.h -- C-ABI of libmqvs.so, the MI355X (gfx950) vector-scan engine that
 * sits behind MyScaleDB's brute-force distance() path.
 *
 * Every entry point is plain C (pointers, sizes, ints); no HIP, torch or C++
 * types cross this boundary.  The reference-side C++ binding that a MyScaleDB
 * maintainer drops in is include/mqvs_vector_index.hpp.
 *
 * Reference interfaces replaced (paths relative to the MyScaleDB tree):
 *   mqvs_knn_raw        VectorIndex::tryBruteForceSearch<FloatVector>
 *                       src/VectorIndex/Common/BruteForceSearch.h:62-111
 *   mqvs_segment_*      the per-granule copy of the Array(Float32) column into
 *                       `vector_raw_data` + VectorDataset construction,
 *                       src/VectorIndex/Storages/MergeTreeVSManager.cpp:1366-1393,
 *                       src/VectorIndex/Common/VectorDataset.h:31-60
 *                       (a whole data part is registered once and stays in HBM)
 *   mqvs_search         MergeTreeVSManager::vectorScanWithoutIndex<Float> +
 *                       searchWrapper + VIWithColumnInPart::searchWithoutIndex,
 *                       MergeTreeVSManager.cpp:960-1680, VIWithDataPart.h:341-382
 *   mqvs_rerank         VIWithColumnInPart::computeTopDistanceSubset,
 *                       src/VectorIndex/Common/VIWithDataPart.cpp:838-856
 *   mqvs_merge_shards   MergeTreeBaseSearchManager::getTotalTopSearchResultImpl,
 *                       src/VectorIndex/Storages/MergeTreeBaseSearchManager.cpp:207-297
 *                       (and the Distributed engine's shard merge)
 *   mqvs_last_error /   DB::Exception(code, message) thrown by the above
 *   status codes        (ErrorCodes NOT_IMPLEMENTED, LOGICAL_ERROR, ...)
 *
 * Threading: re-entrant.  Each calling thread gets its own HIP stream and
 * scratch workspace; segments are read-only after creation and may be searched
 * from any number of threads (the reference admits 2 x physical cores
 * concurrent scans, MergeTreeVSManager.cpp:974-975).
 */
#ifndef MQVS_H
#define MQVS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQVS_ABI_VERSION 4

/* Metric ids (VICommon.h VIMetric).  L2 / IP / Cosine: Float32 vectors;
 * Hamming / Jaccard: binary vectors (FixedString(N) columns, mqvs_*_binary). */
enum {
    MQVS_METRIC_L2 = 0,      /* squared L2, ascending */
    MQVS_METRIC_IP = 1,      /* inner product, descending */
    MQVS_METRIC_COSINE = 2,  /* 1 - <q/|q|, y/|y|>, ascending */
    MQVS_METRIC_HAMMING = 4, /* popcount(q ^ y), ascending (value 3 is internal) */
    MQVS_METRIC_JACCARD = 5  /* (|q|y| - |q&y|) / |q|y| in fp32, ascending */
};

/* Status codes; each maps 1:1 onto the DB::ErrorCodes the reference throws. */
enum {
    MQVS_OK = 0,
    MQVS_ERR_NOT_IMPLEMENTED = 1,   /* unsupported metric (BruteForceSearch.h:89) */
    MQVS_ERR_LOGICAL = 2,           /* dim mismatch, wrong segment metric (LOGICAL_ERROR) */
    MQVS_ERR_ILLEGAL_COLUMN = 3,    /* malformed column data */
    MQVS_ERR_BAD_ARGUMENTS = 4,     /* null pointers, k <= 0, ... */
    MQVS_ERR_MEMORY_LIMIT = 5,      /* HBM allocation failed (MEMORY_LIMIT_EXCEEDED) */
    MQVS_ERR_DEVICE = 6,            /* HIP runtime / kernel failure */
    MQVS_ERR_CHECKSUM = 7           /* compressed block checksum mismatch (CHECKSUM_DOESNT_MATCH) */
};

/* mqvs_search / mqvs_rerank flags */
#define MQVS_F_DEVICE_PTRS 0x1u /* queries, bitmaps, candidates and outputs are
                                   device pointers on the segment's GPU */
#define MQVS_F_ASYNC 0x2u       /* with DEVICE_PTRS: do not synchronise the
                                   stream before returning.  The results are
                                   valid once the stream drains AND
                                   mqvs_async_check returns MQVS_OK: a search
                                   that would have needed a host-driven
                                   fallback (candidate overflow, cosine variant
                                   check) is reported there as
                                   MQVS_ERR_LOGICAL and must be repeated
                                   without ASYNC */
/* Per-call path selection (override the process-wide mqvs_set_* defaults for
 * this call only; all paths return the same bits): */
#define MQVS_F_EXACT 0x20u         /* exact fp32 scan of every row (no bf16 pre-filter) */
#define MQVS_F_GATHER_NEVER 0x40u  /* PREWHERE: scan every row and mask */
#define MQVS_F_GATHER_ALWAYS 0x80u /* PREWHERE: always walk a gather list of the selected rows */
#define MQVS_F_TIMING 0x100u       /* per-launch HIP-event timing in mqvs_last_search_stats */

typedef struct mqvs_segment *mqvs_segment_t;
typedef void *mqvs_stream_t; /* a hipStream_t, or NULL for the caller thread's stream */

/* ---- lifecycle ---------------------------------------------------------- */
int mqvs_abi_version(void);
/* Bind the calling thread to `device` (a HIP ordinal). */
int mqvs_init(int device);
int mqvs_device_count(int *count);
/* Thread-local message of the last failing call on this thread. */
const char *mqvs_last_error(void);
/* Outcome of this thread's MQVS_F_ASYNC calls on the current device since the
 * last check: synchronises `stream` (NULL: the thread's own stream), then
 * returns MQVS_OK, or MQVS_ERR_LOGICAL when one of them needed a host-driven
 * fallback (its results are then invalid: repeat it synchronously).  Clears
 * the record.  Callers that used several streams synchronise them first. */
int mqvs_async_check(mqvs_stream_t stream);
/* Release this thread's streams and workspaces -- the FLAT search workspace
 * and the index search workspace (its scratch, events and the side stream of
 * the cosine variant chain) -- after their last searches' kernels finish
 * (optional; a pool thread that retires should call it). */
int mqvs_thread_release(void);
/* Library shutdown for the calling thread (SURVEY 8(b) lifecycle): waits for
 * the thread's streams and releases its workspaces, as mqvs_thread_release.
 * Segments, indexes, caches and communicators stay owned by the caller and
 * are freed with their own *_free calls. */
int mqvs_shutdown(void);

/* ---- segments: one data part's Array(Float32) column resident in HBM ---- */
/* host_rows: n*d row-major fp32; rows whose Array is empty must be FLT_MAX
 *   filled (MergeTreeVSManager.cpp:1381) and flagged 0 in `nonempty`.
 * nonempty: n bytes (1 = non-empty array) or NULL (all non-empty).
 * metric: the column's metric; COSINE segments are normalised in HBM once
 *   (VectorDataset.h:98-117 per row) and serve only cosine searches; L2/IP
 *   segments serve both L2 and IP.
 * granule_rows: index_granularity (rows per mark; reads are chunked by it).
 * row_offset: id of row 0 (0 for a whole part; shard start for a row-range
 *   shard of a part -- must be a multiple of granule_rows). */
int mqvs_segment_create(const float *host_rows, int64_t n, int32_t d, int32_t metric,
                        int64_t granule_rows, const uint8_t *nonempty, int64_t row_offset,
                        mqvs_segment_t *out);
/* Same from a device buffer on the current device (copied). */
int mqvs_segment_create_device(const float *dev_rows, int64_t n, int32_t d, int32_t metric,
                               int64_t granule_rows, const uint8_t *dev_nonempty,
                               int64_t row_offset, mqvs_segment_t *out);
/* Synthetic segment generated in HBM by the counter-based generator
 * (mode 0 exact ints in [-8,8], 1 ~N(0,1), 2 Gaussian mixture of 4096 centres
 * with noise 0.25, 3 "hard" mixture of 65536 centres with noise 1.0); row r of the
 * segment is generator row row_offset + r. */
int mqvs_segment_generate(uint64_t seed, int32_t mode, int64_t n, int32_t d, int32_t metric,
                          int64_t granule_rows, int64_t row_offset, mqvs_segment_t *out);
int mqvs_segment_free(mqvs_segment_t seg);
int mqvs_segment_info(mqvs_segment_t seg, int64_t *n, int32_t *d, int32_t *metric,
                      int64_t *granule_rows, int64_t *row_offset, size_t *hbm_bytes);
/* The segment's pre-filter planes: *split = 2 (the bf16 plane, see
 * mqvs_set_prefilter) or 0 when the planes were off or did not fit in HBM --
 * batches then run the exact fp32 MFMA path over every row (same bits, about
 * 1/16 of the bf16 MFMA rate); *plane_bytes = their HBM bytes (included in
 * mqvs_segment_info's hbm_bytes); *approx_ok = 1 when the pre-filter serves
 * searches (planes present and the rows' norms finite and moderate). */
int mqvs_segment_prefilter(mqvs_segment_t seg, int32_t *split, size_t *plane_bytes, int32_t *approx_ok);
/* Where the segment's Float32 rows live.  host = 1 moves them to pinned host
 * memory mapped into the device's address space: HBM then holds the bf16
 * pre-filter plane, the norms and the maps (2 B per element instead of 6), so
 * a part about 3x larger fits.  Searches keep the same pipeline and return the
 * same bits; the exact re-rank reads its survivors' rows over PCIe (a few
 * hundred rows per query), while paths that read every row (no plane, no
 * pre-filter, mqvs_set_batch_mode(1), index build) stream the whole part over
 * PCIe: correct, slow.  host = 0 moves the rows back into HBM.  The caller
 * keeps searches on the segment from running meanwhile, and changes the
 * residency before handing the segment to the part cache (its weight is
 * taken at put).  *host (mqvs_segment_rows_host) = 1 when the rows are in host
 * memory.  (No reference counterpart: MyScaleDB re-reads the column from disk
 * per search, MergeTreeVSManager.cpp:1348-1393.) */
int mqvs_segment_set_rows_host(mqvs_segment_t seg, int32_t host);
int mqvs_segment_rows_host(mqvs_segment_t seg, int32_t *host);
/* Device pointer of the resident rows (normalised rows for cosine). */
int mqvs_segment_rows(mqvs_segment_t seg, const float **dev_rows);

/* ---- search --------------------------------------------------------------
 * Brute-force top-k over the whole segment, with the reference operator's
 * exact output: k (id, distance) per query, ascending for L2/Cosine,
 * descending for IP, ties by row order; ids are row_offset + row; slots past
 * the last result hold id -1 and distance FLT_MAX (L2, Cosine) or FLT_MIN (IP).
 * queries: nq*d fp32 (original, un-normalised).
 * filter: PREWHERE bitmap, LSB-first, n bits, or NULL (no PREWHERE).
 * row_exists: lightweight-delete mask, LSB-first, n bits (1 = live), or NULL.
 * out_ids: nq*k int64; out_dist: nq*k fp32 (caller-owned).
 * k: 1 .. 16384 (the reference's max_search_result_window is 10000,
 * Settings.h:923); above 4096 the final sort runs through a device scratch
 * and large batches are searched in query sub-batches. */
int mqvs_search(mqvs_segment_t seg, const float *queries, int32_t nq, int32_t k,
                int32_t metric, const uint8_t *filter, const uint8_t *row_exists,
                int64_t *out_ids, float *out_dist, uint32_t flags, mqvs_stream_t stream);

/* mqvs_search for a row-range shard of a part, with the cosine chunk-ordinal
 * base given: the number of granule chunks BEFORE the shard's first row that
 * the reference searches for this query (MergeTreeVSManager.cpp:960-1536:
 * a chunk is searched iff it holds a non-empty row that, with a PREWHERE
 * filter, also passes the filter and is not deleted).  The query is
 * re-normalised once per searched chunk, so this base picks the variant.
 * chunk_ord_base < 0: row_offset / granule_rows (every earlier chunk
 * searched).  Only cosine results depend on it. */
int mqvs_search_ex(mqvs_segment_t seg, const float *queries, int32_t nq, int32_t k, int32_t metric,
                   const uint8_t *filter, const uint8_t *row_exists, int64_t chunk_ord_base,
                   int64_t *out_ids, float *out_dist, uint32_t flags, mqvs_stream_t stream);

/* tryBruteForceSearch contract (BruteForceSearch.h:62-111): x nx*d queries,
 * y ny*d base (host pointers), one pass with no granule chunking, metric L2 or
 * IP only (anything else -> MQVS_ERR_NOT_IMPLEMENTED); result_id / distance
 * nx*k, faiss layout (-1 / FLT_MAX or -FLT_MAX padding). */
int mqvs_knn_raw(const float *x, const float *y, int64_t d, int64_t k, int64_t nx, int64_t ny,
                 int32_t metric, int64_t *result_id, float *distance);

/* Exact re-rank of candidate rows (computeTopDistanceSubset contract,
 * VIWithDataPart.cpp:838-856): cand is nq*ncand segment-local row ids (-1 or
 * out-of-range = none; distinct rows per query), ncand <= 32768, k <= 16384
 * (above 4096 candidates the records are sorted through global scratch).  Each
 * candidate gets the distance mqvs_search computes for the same batch size
 * (nq < 20 sequential formula, else BLAS form; cosine with the row's chunk
 * query variant); rows cleared in row_exists (LSB-first, n bits, or NULL)
 * are skipped.  Output: top-k as mqvs_search (same order key and padding). */
int mqvs_rerank(mqvs_segment_t seg, const float *queries, int32_t nq, const int64_t *cand,
                int32_t ncand, int32_t k, int32_t metric, const uint8_t *row_exists,
                int64_t *out_ids, float *out_dist, uint32_t flags, mqvs_stream_t stream);

/* Merge per-list top-k results: in_ids/in_dist [nshards][nq][k] as returned
 * by mqvs_search; out nq*k (nshards * k <= 2^20; above 4096 the records are
 * sorted through a device scratch of 32 B per record and query).
 * Default (row-range shards of ONE part, shard s holding lower ids than shard
 * s+1): order distance (desc for IP), then shard, then position -- the result
 * equals the unsharded part's search.
 * MQVS_F_PART_MERGE (lists = different data parts): the reference's cross-part
 * merge MergeTreeBaseSearchManager::getTotalTopSearchResultImpl
 * (MergeTreeBaseSearchManager.cpp:207-297), an insertion-ordered multimap read
 * backwards for IP -- equal IP scores come out last-inserted first. */
#define MQVS_F_PART_MERGE 0x4u
int mqvs_merge_shards(int32_t nshards, int32_t nq, int32_t k, int32_t metric,
                      const int64_t *in_ids, const float *in_dist, int64_t *out_ids,
                      float *out_dist, uint32_t flags, mqvs_stream_t stream);

/* ---- column ingest: a part's Array(Float32) column from its compressed files
 * Replaces the per-granule host read + copy of vectorScanWithoutIndex
 * (MergeTreeVSManager.cpp:1348-1393): data_bin = the bytes of the nested
 * Float32 stream (`<column>.bin`), sizes_bin = the array sizes stream
 * (`<column>.size0.bin`, UInt64 per row), both as ClickHouse writes them
 * (CompressedWriteBuffer blocks: 16-B checksum, method 0x82 LZ4 or 0x02 NONE,
 * UInt32 compressed size, UInt32 decompressed size, payload).  Every block's
 * checksum -- CityHash128 v1.0.2 of header + payload -- is verified on the GPU
 * first (CompressedReadBufferBase.cpp:37-45, 192-196) unless flags has
 * MQVS_F_NO_CHECKSUM (the reference's disable_checksum).  Decoded on the GPU into the rows of :1381-1393 (FLT_MAX fill;
 * empty arrays flagged empty; arrays longer than d truncated, shorter ones
 * FLT_MAX-padded) and prepared as mqvs_segment_create.  flags:
 * MQVS_F_DEVICE_PTRS when the streams are already in HBM.  Errors:
 * MQVS_ERR_CHECKSUM (a block checksum does not match: CHECKSUM_DOESNT_MATCH),
 * MQVS_ERR_ILLEGAL_COLUMN (malformed blocks, sizes that do not match the data
 * stream or n), MQVS_ERR_NOT_IMPLEMENTED (other codecs). */
#define MQVS_F_NO_CHECKSUM 0x10u
int mqvs_segment_create_from_column(const uint8_t *data_bin, int64_t data_bytes, const uint8_t *sizes_bin,
                                    int64_t sizes_bytes, int64_t n, int32_t d, int32_t metric, int64_t granule_rows,
                                    int64_t row_offset, uint32_t flags, mqvs_segment_t *out);

/* ---- binary vectors: FixedString(N) columns, Hamming / Jaccard ----------
 * tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110) over
 * vectorScanWithoutIndex<BinaryVector> (MergeTreeVSManager.cpp:1188-1273,
 * 1395-1425).  Codes are n rows x dim_bits/8 bytes (the FixedString bytes).
 *
 * mqvs_segment_create_binary: register a part's binary column (host codes, or
 * device codes with MQVS_F_DEVICE_PTRS in flags); metric is the column's
 * default (Hamming or Jaccard; a search may use either).
 * mqvs_search_binary: mqvs_search for binary segments -- queries nq x N bytes;
 * output ascending by (distance, row), Hamming distances as float values
 * (KAT 00038 prints 4, 8, ...), -1 / FLT_MAX padding.  Rows at Hamming
 * distance == dim_bits are never returned (hammings_knn_mc emits b < nBit).
 * mqvs_knn_binary_raw: the tryBruteForceSearch<BinaryVector> contract itself
 * (host pointers, one pass): Hamming writes int32 counts into `distance`
 * (reinterpret as int32_t*, padding -1 / INT32_MAX, faiss::hammings_knn_mc);
 * Jaccard writes floats (padding -1 / FLT_MAX).  Float metrics ->
 * MQVS_ERR_NOT_IMPLEMENTED ("Metric not implemented in brute force search
 * for Binary Vector"), as BruteForceSearch.h:107. */
int mqvs_segment_create_binary(const uint8_t *codes, int64_t n, int32_t dim_bits, int32_t metric,
                               int64_t granule_rows, int64_t row_offset, uint32_t flags,
                               mqvs_segment_t *out);
int mqvs_search_binary(mqvs_segment_t seg, const uint8_t *queries, int32_t nq, int32_t k, int32_t metric,
                       const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids, float *out_dist,
                       uint32_t flags, mqvs_stream_t stream);
int mqvs_knn_binary_raw(const uint8_t *x, const uint8_t *y, int64_t d, int64_t k, int64_t nx, int64_t ny,
                        int32_t metric, int64_t *result_id, float *distance);

/* ---- multi-GPU: one part sharded by row range over the GPUs of a node ----
 * One rank per GPU (process or thread); rank r holds the granule-aligned row
 * range [r0, r1) of the part as a segment created with row_offset = r0 (ids
 * stay part-global).  The communicator is an RCCL one over xGMI:
 *   mqvs_comm_unique_id  on ONE rank; ship the 128 bytes to the others out of
 *                        band (the Distributed engine's channel, MPI, a file)
 *   mqvs_comm_init       on every rank, with its device current (mqvs_init);
 *                        blocks until all nranks have joined
 *   mqvs_sharded_search  on every rank, same queries / k / metric: the local
 *                        top-k of the rank's shard, ONE all-gather of the
 *                        per-rank (id, distance) lists (nq*k*12 B per rank),
 *                        and the device merge by (distance, rank, position);
 *                        every rank gets the merged result, bit-identical to
 *                        mqvs_search over the whole part.  filter / row_exists
 *                        are the shard's bitmaps (its n bits).  Cosine: the
 *                        ranks also all-gather how many granule chunks of
 *                        their range the reference searches, which fixes each
 *                        shard's query re-normalisation count (chunk-ordinal
 *                        base) exactly, filters and deletes included.
 * Replaces the cross-part / cross-shard merges of the reference
 * (MergeTreeBaseSearchManager.cpp:207-297 getTotalTopSearchResultImpl; the
 * Distributed engine's per-shard LIMIT + initiator merge,
 * StorageDistributed.cpp:1057-1060) for one part spread over GPUs.  A
 * communicator serves one search at a time.  Before any search work the
 * ranks exchange a header (shard rows, granule, dimension, nq / k / metric,
 * argument errors): shards out of row order, disagreeing calls or a failing
 * rank make EVERY rank return the error instead of leaving the others in a
 * collective; a rank whose local search fails still joins the exchange, and
 * all ranks then fail together.
 * Host syncs: a call equal to the last call every rank completed together
 * (same shard, nq, k, metric and bitmap presence) synchronises the host ONCE
 * (header, local search, exchange and merge enqueued back to back; the
 * exchanged table is read at the end).  The first call, a changed call, or a
 * call whose local search needs a host-driven fallback or whose cosine
 * chunk-ordinal bases changed (filters that empty whole chunks) runs the
 * validated path: header exchange and sync, local search, exchange and sync.
 * MQVS_F_ASYNC is ignored (the call always ends with the merged result). */
#define MQVS_COMM_ID_BYTES 128
typedef struct mqvs_comm *mqvs_comm_t;
int mqvs_comm_unique_id(uint8_t *id /* MQVS_COMM_ID_BYTES */);
int mqvs_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, mqvs_comm_t *out);
int mqvs_comm_free(mqvs_comm_t comm);
/* A loopback communicator group: nranks (<= 64) virtual ranks of ONE process
 * on the current device, out[0 .. nranks-1] one handle per rank.  Each rank's
 * mqvs_sharded_search runs on its own thread (the exchanges are device copies
 * between host barriers); everything else is the RCCL communicator's code.
 * For tests and single-GPU rehearsal of a multi-GPU layout; free every handle. */
int mqvs_comm_init_loopback(int32_t nranks, mqvs_comm_t *out);
int mqvs_sharded_search(mqvs_comm_t comm, mqvs_segment_t shard, const float *queries, int32_t nq, int32_t k,
                        int32_t metric, const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids,
                        float *out_dist, uint32_t flags, mqvs_stream_t stream);
/* Calls of this communicator that took the one-sync fast path, and how many
 * of those were re-run on the validated path. */
int mqvs_comm_stats(mqvs_comm_t comm, int64_t *fast_calls, int64_t *redo_calls);

/* Fill a device buffer with generator rows [row0, row0+n) (for queries). */
int mqvs_generate_device(uint64_t seed, int32_t mode, int64_t row0, int64_t n, int32_t d,
                         float *dev_out, mqvs_stream_t stream);

/* ---- index path: MSTG-type vector index over a resident segment ----------
 * The reference's index seam for one data part and vector column:
 *   mqvs_index_build   Search::createVectorIndex<IStream, OStream, DenseBitmap,
 *                      FloatVector>(name, IndexType::MSTG, metric, dim, total_vec,
 *                      params, ...) + VectorIndex::build(...)
 *                      (src/VectorIndex/Common/VIWithDataPart.cpp:416-447,
 *                      VIWithDataPart.h:295-339)
 *   mqvs_index_search  VectorIndex::search(queries, k, params, first_stage_only,
 *                      filter) as VIWithColumnInPart::search calls it
 *                      (VIWithDataPart.cpp:858-957, the call at :926)
 *   computeTopDistanceSubset (stage 2 of a two-stage search,
 *                      VIWithDataPart.cpp:838-856) is mqvs_rerank on the
 *                      index's segment.
 * The MSTG library is absent from the reference snapshot; this
 * is a GPU-native index with its parameter surface: a k-means partition of the
 * part into lists stored as one bf16 plane in list order, an MFMA scan of the
 * lists each query probes, and an exact fp32 re-rank of the best num_reorder
 * candidates (distances bit-identical to mqvs_search / mqvs_rerank for the
 * same rows).
 * The segment must outlive the index.  index_type: "MSTG" (also accepted:
 * "IVFFLAT").  params: comma-separated key=value (Search::Parameters):
 *   metric_type  L2 | IP | Cosine (must match the segment's metric family;
 *                default: the segment's metric)
 *   alpha        default search alpha (MSTG's accuracy knob, [1, 4], default 3)
 *   nlist        lists (default about n / 256, at most 65536)
 *   kmeans_iters k-means iterations (default 8)
 *   sample       k-means training rows (default min(n, max(16 nlist, min(64 nlist, 2^20))))
 * Unknown keys fail with MQVS_ERR_BAD_ARGUMENTS. */
typedef struct mqvs_index *mqvs_index_t;
int mqvs_index_build(mqvs_segment_t seg, const char *index_type, const char *params, mqvs_index_t *out);
int mqvs_index_free(mqvs_index_t idx);
typedef struct {
    int64_t nlist;        /* lists */
    int64_t npos;         /* positions of the list-ordered plane (with padding) */
    int64_t max_list;     /* longest list */
    int64_t rows_indexed; /* rows in some list (empty arrays are not indexed) */
    int32_t metric;
    int32_t dim;
    size_t hbm_bytes;     /* index-owned HBM (the segment's rows not counted) */
    double build_ms;
} mqvs_index_info_t;
int mqvs_index_info(mqvs_index_t idx, mqvs_index_info_t *out);
/* Search params (comma-separated key=value, may be NULL or ""):
 *   alpha        [1, 4]: probes nprobe(alpha) lists (more = higher recall; alpha 3:
 *                max(4, nlist / 256, lists of 4096 rows), doubling per unit)
 *   nprobe       lists probed per query (overrides alpha; <= min(nlist, 4096))
 *   num_reorder  candidates re-ranked exactly (default max(2k, 64), capped at
 *                4096 for k <= 2048; k .. 32768; above 4096 the select and the
 *                re-rank sort through device scratch, 2 num_reorder records of
 *                16 B per query each, in query sub-batches of <= 1 GB)
 * k: 1 .. 16384, as mqvs_search (max_search_result_window, Settings.h:923).
 * filter / row_exists: LSB-first bitmaps over the segment's rows, or NULL.
 * Output as mqvs_search (k per query, reference order, -1 padding).  With
 * MQVS_F_FIRST_STAGE the call returns the first stage only: the k best rows
 * by the approximate bf16 distance (approximate distances), to be re-ranked
 * by mqvs_rerank (the reference's two-stage search). */
#define MQVS_F_FIRST_STAGE 0x8u
/* Re-rank every one of the num_reorder candidates.  By default a candidate
 * whose approximate value is more than twice the query's bf16 bound past the
 * k-th best approximate value is not re-ranked: its exact value cannot reach
 * the top k, so the results are the same either way (the flag is for tests
 * and measurements). */
#define MQVS_F_RERANK_ALL 0x200u
int mqvs_index_search(mqvs_index_t idx, const float *queries, int32_t nq, int32_t k, const char *params,
                      const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids, float *out_dist,
                      uint32_t flags, mqvs_stream_t stream);
/* Introspection of the coarse step (no reference counterpart: the MSTG
 * library's quantizer is not exposed through VectorIndex; these let a caller
 * or a test check the probes against its own exact top-nprobe):
 * mqvs_index_centroids: the nlist x dim fp32 centroid table (normalised for
 *   cosine indexes) into host memory; cap = floats out holds.
 * mqvs_index_probes: for each of nq host queries the list ids the search with
 *   `params` (alpha / nprobe as mqvs_index_search) would probe, in no
 *   guaranteed order, into out_probes[nq][nprobe] (host; nprobe as
 *   mqvs_index_last_stats then reports it; nq x nlist always suffices).
 *   For nprobe <= 64 (the coarse pick) and for indexes of more than 16384
 *   lists (a FLAT search of the centroids) the lists are the exact top nprobe
 *   by the coarse metric (L2; the raw inner product for IP and cosine parts),
 *   up to fp32 rounding of near ties; otherwise they are ranked by the bf16
 *   approximate value (the centroid list pass). */
int mqvs_index_centroids(mqvs_index_t idx, float *out, int64_t cap);
int mqvs_index_probes(mqvs_index_t idx, const float *queries, int32_t nq, const char *params, int64_t *out_probes);
/* Decoupled parts: a part merged from several source parts whose index still
 * serves the source part's rows (the reference's VIWithMeta row_ids_map /
 * inverted maps, VICacheObject.h:50-64).
 * mqvs_index_set_row_ids_map: register the source part's row -> decoupled
 *   part row map (UInt64 per source row, len >= the indexed rows); every later
 *   mqvs_index_search on this index returns decoupled-part row ids
 *   (VIWithColumnInPart::transferToNewRowIds, VIWithDataPart.cpp:56-67, applied
 *   at :938-943).  NULL / len 0 clears it.  The map lives in HBM with the index.
 * mqvs_decoupled_filter: getRealBitmap (VIUtils.cpp:479-497) -- a PREWHERE
 *   bitmap over the decoupled part's new_rows rows -> the bitmap over this
 *   source part's old_rows rows: old bit inverted_row_ids_map[i] is set for
 *   every set bit i whose inverted_row_sources_map[i] == own_id.  With no
 *   inverted map (len 0) the filter is returned as it is.  MQVS_F_DEVICE_PTRS:
 *   all pointers on the device. */
int mqvs_index_set_row_ids_map(mqvs_index_t idx, const uint64_t *row_ids_map, int64_t len, uint32_t flags);
int mqvs_decoupled_filter(const uint8_t *new_filter, int64_t new_rows, const uint64_t *inverted_row_ids_map,
                          const uint8_t *inverted_row_sources_map, int64_t inverted_len, uint32_t own_id,
                          uint8_t *old_filter, int64_t old_rows, uint32_t flags, mqvs_stream_t stream);

/* Stats of the calling thread's last mqvs_index_search (times only with
 * mqvs_set_timing(1)). */
typedef struct {
    double coarse_ms;     /* nearest lists per query (FLAT search over the centroids) */
    double plan_ms;       /* grouping (query, list) pairs into work items */
    double scan_ms;       /* bf16 MFMA scan of the probed lists */
    double select_ms;     /* num_reorder best approximate values per query */
    double rerank_ms;     /* exact fp32 re-rank + top-k */
    double total_ms;
    int64_t values;       /* approximate values computed (query x probed position) */
    int64_t items;        /* scan work items (list x 16-query group) */
    int64_t plane_bytes;  /* bf16 plane bytes streamed by the scan */
    int64_t pairs;        /* (query, list) pairs */
    int32_t nq, k, nprobe, num_reorder;
    int64_t reranked;     /* candidates re-ranked exactly (sum over queries, <= nq x num_reorder): the bf16
                             bound prunes those that cannot reach the top k (MQVS_F_RERANK_ALL: none) */
    int32_t pick_overflow;/* queries whose coarse pick found more near-tie centroid groups than its
                             working set holds and scored them in batches (the probes stay exact) */
    int32_t reserved;
} mqvs_index_search_stats;
int mqvs_index_last_stats(mqvs_index_search_stats *out);

/* ---- device-resident cache of parts (VICacheManager, VICacheManager.h:82-114)
 * An LRU of segments (+ an optional index over each) keyed by the caller's
 * CacheKey string, weighed by HBM bytes against max_bytes.
 *   put      takes ownership of seg / idx (the index must be over seg); evicts
 *            least-recently-used unheld entries to make room; a key already
 *            present is replaced (putting the same pair under its own key
 *            again only refreshes it).  MQVS_ERR_MEMORY_LIMIT when the budget
 *            cannot hold it, MQVS_ERR_BAD_ARGUMENTS for an index over another
 *            segment or a handle already cached under another key (ownership
 *            then stays with the caller).
 *   acquire  *seg = NULL on a miss; on a hit the entry is held (never evicted)
 *            and becomes most recently used; the handles stay owned by the
 *            cache.  Every hit is paired with release(key, seg).
 *   remove   forceExpire: freed now, or at the last release if held.
 * Thread-safe (one mutex; searches on acquired handles run lock-free). */
typedef struct mqvs_cache *mqvs_cache_t;
typedef struct {
    int64_t items;        /* entries in the LRU */
    size_t bytes;         /* their HBM bytes */
    size_t max_bytes;
    int64_t hits, misses, evictions;
    int64_t pinned;       /* entries held now */
    int64_t expired_held; /* removed / replaced entries still held */
} mqvs_cache_stats_t;
int mqvs_cache_create(size_t max_bytes, mqvs_cache_t *out);
int mqvs_cache_free(mqvs_cache_t cache);
int mqvs_cache_put(mqvs_cache_t cache, const char *key, mqvs_segment_t seg, mqvs_index_t idx);
int mqvs_cache_acquire(mqvs_cache_t cache, const char *key, mqvs_segment_t *seg, mqvs_index_t *idx);
int mqvs_cache_release(mqvs_cache_t cache, const char *key, mqvs_segment_t seg);
int mqvs_cache_remove(mqvs_cache_t cache, const char *key);
int mqvs_cache_stats(mqvs_cache_t cache, mqvs_cache_stats_t *out);

/* ---- observability -------------------------------------------------------
 * Stats of the calling thread's last mqvs_search: per-launch kernel times
 * (ms, HIP events on the search stream; only with mqvs_set_timing(1)), rows
 * scanned by each launch and which path ran. */
typedef struct {
    double probe_ms;        /* probe scan kernel */
    double probe_select_ms; /* radix select over the probe */
    double main_ms;         /* main scan kernels (rows [probe_rows, n), all segments) */
    double refine_ms;       /* threshold refinements between main-scan segments */
    double final_ms;        /* final select (or exact re-rank + select) kernel */
    double total_ms;        /* first to last event of the search */
    int64_t rows_scanned;
    int64_t probe_rows;
    int64_t main_rows;
    int32_t nq;
    int32_t k;
    int32_t path;           /* 0 = VALU direct formula (nq < 20), 1 = fp32 MFMA,
                               2 = bf16 MFMA pre-filter + exact fp32 re-rank */
    int32_t rescans;        /* candidate-overflow re-scans / fallbacks */
    int32_t segments;       /* main-scan segments (threshold refinements + 1) */
    int32_t gather;         /* 1: selective PREWHERE, the scan walked the gather list
                               of selected rows (rows_scanned = list entries) */
    int32_t prefilter;      /* path 2: pre-filter split (2 = bf16 hi) */
    int32_t batch_kernel;   /* path 2: 1 when the main scan ran the one-wave-per-SIMD batch
                               kernel (nq > 128, contiguous rows), else 0 */
    int64_t survivors_total;/* path 2: rows re-ranked exactly (sum over queries) */
    int32_t survivors_max;  /* path 2: most rows re-ranked for one query */
    int32_t candidates_max; /* path 2: longest candidate list before the final bound */
} mqvs_search_stats;
int mqvs_last_search_stats(mqvs_search_stats *out);
/* Enable per-search HIP-event timing (off by default: one extra event pair). */
int mqvs_set_timing(int enabled);
/* Batch (nq >= 20) scan: 0 = bf16 MFMA pre-filter with a rigorous error bound
 * and exact fp32 re-rank of the survivors (default; falls back to 1 when the
 * bound admits too many rows), 1 = fp32 MFMA over every row.  Both return the
 * same bits. */
int mqvs_set_batch_mode(int mode);
/* Selective PREWHERE scans: 0 = always scan every row and mask, 1 = scan only
 * the selected rows (a device-built gather list) when few enough pass the
 * filter (default: <= 60% when the bf16 pre-filter serves the batch, <= 30%
 * for the exact small-batch kernel), 2 = always gather.  All return the same
 * bits. */
int mqvs_set_gather_mode(int mode);
/* Pre-filter planes built by segments created AFTER the call: 2 = bf16 hi
 * plane, one bf16 MFMA product bounded by measured residual norms (default;
 * 2 B per element), 0 = no planes (batches run the exact fp32 MFMA path over
 * every row).  Other values (rounds 1-2 also had 3 and 6) are
 * MQVS_ERR_BAD_ARGUMENTS.  Both return the same bits. */
int mqvs_set_prefilter(int split);
/* Device scratch that one call may allocate for large-k sorts and candidate
 * lists (default 1 GiB per buffer, at least 1 MiB): calls whose buffers would
 * exceed it run in query sub-batches, which keep the whole call's distance
 * formula (faiss's nx >= 20 branch) and return the same bits.  Returns the
 * previous value; 0 leaves it unchanged. */
size_t mqvs_set_scratch_budget(size_t bytes);
/* Process-wide cap on the device memory of all threads' search workspaces
 * (each calling thread keeps one per device: query variants, candidate lists,
 * sort scratch -- about 1 GB at nq 1000).  The reference admits 2 x physical
 * cores concurrent scans (MergeTreeVSManager.cpp:972-975); here a workspace
 * growth that would pass the cap first frees idle threads' workspaces, then
 * waits until running searches finish and give theirs back (a search that
 * ends while others wait frees its workspace).  Only when every running
 * search is waiting does one go over the cap (counted in over_budget) instead
 * of deadlocking.  Default: a quarter of the device memory.  Returns the
 * previous value; 0 leaves it unchanged.  Index searches (mqvs_index_search,
 * mqvs_decoupled_filter) pass the same gate: their scratch is counted in, and
 * trimmed with, the calling thread's workspace.  (Segments, indexes and
 * communicators are not counted.) */
size_t mqvs_set_workspace_budget(size_t bytes);
typedef struct {
    size_t budget;       /* the cap */
    size_t held;         /* device bytes of all workspaces now */
    size_t peak;         /* most held at once (since the last reset) */
    int64_t waits;       /* growths that waited for memory */
    int64_t trims;       /* workspaces freed for others */
    int64_t over_budget; /* growths let over the cap (every running search waiting) */
    int32_t active;      /* threads inside a search now */
    int32_t workspaces;  /* workspaces registered (threads x devices) */
} mqvs_workspace_stats_t;
/* reset_peak: restart peak (at held) and the counters after reading */
int mqvs_workspace_stats(mqvs_workspace_stats_t *out, int32_t reset_peak);
/* Achievable HBM read rate of this device (a bench utility: the measured
 * denominator of the scan's HBM fraction).  A STREAM-like read
 * sweep -- every lane loads 16 B, 4 loads in flight, grid-stride, 8
 * workgroups of 256 per CU -- over a fresh device buffer of `bytes` (>= 1 MiB;
 * >= 4 GiB defeats the 256 MiB Infinity Cache), best of `reps` timed passes
 * after one warm-up: *gbs = bytes / best time (1e9 B/s), *best_ms (optional). */
int mqvs_measure_read_bandwidth(size_t bytes, int32_t reps, double *gbs, double *best_ms);
/* How a calling thread waits for its GPU work (every synchronous call ends
 * with a wait; a selective PREWHERE search also waits for its selected-row
 * count).  The reference runs up to 2 x physical cores scans at once
 * (ScanThreadLimiter.h:25-58, MergeTreeVSManager.cpp:974-975): a thread that
 * spins for the length of its search holds a host core meanwhile.
 *   MQVS_WAIT_RUNTIME  hipStreamSynchronize (the HIP runtime's own policy;
 *                      on ROCm it spins, also with BlockingSync events)
 *   MQVS_WAIT_HYBRID   poll for up to spin_us, then sleep: most of the time
 *                      this thread's recent waits took, then short
 *                      sleep-polls (default, 50 us)
 *   MQVS_WAIT_BLOCK    the same without the first poll
 * Results are identical in every mode.  Returns the previous mode;
 * spin_us < 0 leaves the poll budget unchanged; other modes are
 * MQVS_ERR_BAD_ARGUMENTS (returned as a negative value: -4). */
#define MQVS_WAIT_RUNTIME 0
#define MQVS_WAIT_HYBRID 1
#define MQVS_WAIT_BLOCK 2
int mqvs_set_wait_mode(int mode, int spin_us);
/* Fault drill for a caller's host fallback (on a device error the
 * host runs its CPU path; include/mqvs_vector_index.hpp takes the fallback as
 * a callable): the next `calls` search entry points made by THIS thread --
 * mqvs_search, mqvs_search_ex, mqvs_knn_raw, mqvs_search_binary,
 * mqvs_knn_binary_raw, mqvs_index_search -- return `status` (MQVS_ERR_DEVICE
 * or MQVS_ERR_MEMORY_LIMIT) without touching the device or the outputs.
 * calls = 0 disarms.  Other statuses are MQVS_ERR_BAD_ARGUMENTS.
 * status | MQVS_FAULT_MID_CALL: the fault fires inside a filtered mqvs_search
 * instead, right after its selected-row count kernel is queued (a device
 * failure after launches; the next call must not see that call's work). */
#define MQVS_FAULT_MID_CALL 0x100
int mqvs_inject_fault(int32_t status, int32_t calls);

#ifdef __cplusplus
}
#endif
#endif /* MQVS_H */
