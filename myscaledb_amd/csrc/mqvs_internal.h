// mqvs_internal.h -- shared definitions of libmqvs (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <initializer_list>
#include <string>
#include <stdexcept>
#include <algorithm>

#include "../../include/mqvs.h"
#include "tuning.h"

struct mqvs_segment {
    int device = 0;
    int64_t n = 0;
    int d = 0;
    int metric = 0;
    int64_t granule = 0;
    int64_t row_offset = 0;
    float *rows = nullptr;           // device address (HBM, or mapped pinned host memory)
    void *rows_host = nullptr;       // the pinned host allocation when the rows live in host memory
    float *norms = nullptr;          // |y|^2 per row (fvec_norm_L2sqr order)
    uint16_t *rows_hi = nullptr;     // bf16 rounding of the rows, [n][dpad]
    float *ynorm_max = nullptr;      // device scalar: max_r |y_r|; splits 2, 6: + [kMxRec] norm maxima at +16 B
    int split = 0;                   // pre-filter planes built: 2 (bf16 hi), 0 = none
    int64_t dpad = 0;
    bool approx_ok = false;          // bf16 pre-filter usable for this segment
    size_t plane_bytes = 0;          // HBM of the pre-filter planes (0: none built)
    uint8_t *nonempty_bits = nullptr;// null when every array is non-empty
    int *chunk_ord = nullptr;        // no-filter chunk ordinals (null = identity)
    // binary segments (FixedString(N) codes; rows == nullptr)
    bool binary = false;
    uint32_t *codes = nullptr;       // [n][code_words], 16-B aligned rows, zero padded
    int code_bytes = 0;              // N = d / 8
    int code_words = 0;              // row stride in 32-bit words (multiple of 4)
    size_t bytes = 0;
};

namespace mqvs {

// ---------------------------------------------------------------------------
// Tunables
constexpr int kBlasThreshold = 20;   // faiss distance_compute_blas_threshold
constexpr int kMaxVariants = 32;     // cosine query re-normalisation variants kept (default table)
constexpr int kMaxVariantsCap = 16384;  // one variant per chunk ordinal when a chain does not repeat
constexpr int kSortCap = 4096;       // candidates sorted in LDS per query
constexpr int kMaxK = 16384;         // largest k (max_search_result_window is 10000, Settings.h:923)
constexpr int kLargeCap = 32768;     // records per query sorted through global scratch (k > kSortCap)
constexpr int64_t kCandBudget = 1 << 25;  // candidate slots per search (x 8 B)
constexpr int64_t kCandMax = 1 << 20;     // candidate slots per query
constexpr int kSmallRows = 256;      // rows per tile, VALU scan
constexpr int kMfmaRows = 128;       // rows per tile, MFMA scan
constexpr int kMfmaQ = 128;          // queries per tile, MFMA scan
constexpr int kBfRows = 256;         // rows per tile, bf16 pre-filter scans (kernels_hi.hip)
constexpr int kBfRowsSmall = 64;     // short tiles of k_scan_hi_reg (scan_hi_small_tiles_ok)
// Internal metric id: raw faiss inner product (knn_inner_product: every
// ip > -FLT_MAX enters the heap), used by mqvs_knn_raw only.  The operator
// path (mqvs_search) applies searchWrapper's FLT_MIN cut instead.
constexpr int kMetricIpRaw = 3;

// Candidate record: raw metric value (d for L2, ip for IP/cosine) + local row.
struct __attribute__((aligned(8))) Cand {
    float raw;
    uint32_t row;
};

// ---------------------------------------------------------------------------
// Ordering keys.  key32(raw) is a monotone encoding of the primary sort key
// (smaller = better) and 0xFFFFFFFF for rows the reference never returns:
//   L2:     d < FLT_MAX (faiss neutral FLT_MAX is strict, NaN never enters)
//   IP:     ip > FLT_MIN (searchWrapper's FLT_MIN init, MergeTreeVSManager.cpp:1033,1661)
//   Cosine: ip > -FLT_MAX and 1 - ip < FLT_MAX; primary key 1 - ip
__host__ __device__ inline uint32_t ord_asc(float f) {
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__host__ __device__ inline float cos_dist(float ip) {
    // 1 - ip exactly as VIWithDataPart.h:376 computes it (one fp32 subtraction)
    return 1.0f - ip;
}

template <int METRIC>
__host__ __device__ inline uint32_t key32(float raw) {
    const float FLTMAX = 3.40282347e+38f;
    const float FLTMIN = 1.17549435e-38f;
    if (METRIC == MQVS_METRIC_L2) {
        if (!(raw < FLTMAX)) return 0xFFFFFFFFu;
        return ord_asc(raw);
    } else if (METRIC == MQVS_METRIC_IP) {
        if (!(raw > FLTMIN)) return 0xFFFFFFFFu;
        return ~ord_asc(raw);  // descending ip
    } else if (METRIC == kMetricIpRaw) {
        if (!(raw > -FLTMAX)) return 0xFFFFFFFFu;
        return ~ord_asc(raw);
    } else {
        if (!(raw > -FLTMAX)) return 0xFFFFFFFFu;
        const float d = cos_dist(raw);
        if (!(d < FLTMAX)) return 0xFFFFFFFFu;
        return ord_asc(d);
    }
}

__host__ __device__ inline uint32_t key32_rt(int metric, float raw) {
    return metric == MQVS_METRIC_L2       ? key32<MQVS_METRIC_L2>(raw)
           : metric == MQVS_METRIC_IP     ? key32<MQVS_METRIC_IP>(raw)
           : metric == MQVS_METRIC_COSINE ? key32<MQVS_METRIC_COSINE>(raw)
                                          : key32<kMetricIpRaw>(raw);
}

// bf16 bits of x, round to nearest even (NaN stays NaN)
__host__ __device__ inline uint16_t f32_to_bf16_rn(float x) {
    uint32_t u = __builtin_bit_cast(uint32_t, x);
    if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)((u >> 16) | ((u & 0xFFFF) ? 0x40 : 0));
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

__device__ inline bool bit_test(const uint8_t *bm, int64_t i) {
    return (bm[i >> 3] >> (i & 7)) & 1;
}

// ---------------------------------------------------------------------------
// Scan parameters shared by the VALU and MFMA scan kernels.
struct ScanParams {
    const float *rows;      // segment rows (normalised for cosine)
    const float *row_norms; // |y|^2 per row (L2 BLAS branch), may be null
    int64_t n;              // segment rows
    int d;
    int nq;
    const float *qvars;     // [nq][maxv][d] query variants
    const float *qnorms;    // [nq] |q|^2 (L2 BLAS branch)
    const int *qmu;         // [nq] cosine variant cycle start
    const int *qlam;        // [nq] cosine variant cycle length
    int maxv;
    int64_t chunk_rows;     // granule rows (chunking for cosine variants)
    const int *chunk_ord;   // [nchunks] ordinal, -1 = chunk never searched; null = identity
    int ord_base;           // ordinal of the segment's first chunk (row-range shards)
    const uint8_t *filter;  // PREWHERE bitmap or null
    const uint8_t *exists;  // LWD bitmap or null
    const uint8_t *nonempty;// nonempty bitmap or null (only consulted with a filter)
    int64_t row_begin, row_end;  // scan range [row_begin, row_end)
    int64_t tiles;          // number of row tiles in the range
    int64_t tiles_per_chunk;// tiles per chunk (chunk-aligned tiling) or 0 = contiguous
    int64_t tile_rows;
    // PROBE output: dense raw values [nq][probe_ld], column = row - row_begin
    float *probe;
    int64_t probe_ld;
    // APPEND output
    const uint32_t *tau;    // [nq] key threshold (inclusive)
    int *cand_count;        // [nq]
    Cand *cand;             // [nq][cand_cap]
    int cand_cap;
    int num_qblocks;        // MFMA: query blocks
    // bf16 pre-filter path (nq >= 20): hi bf16 planes, row stride dpad
    const uint16_t *rows_hi;  // row-blocked [n/16][dpad/32][16][32] (launch_to_hi)
    const uint16_t *q_hi;     // query variants, same layout, vector v q_vpad + j
    int64_t dpad;
    int64_t q_vpad;           // nq rounded up to 16 (query planes)
    // cosine ordinal planes (kernels_p4.hip): plane pl holds every query's
    // variant for chunk ordinals of class pl; desc = {m0, lam, ok}
    const uint16_t *q_ord;
    const int *q_ord_desc;
    int split;                // pre-filter planes of the scan: kHiSplit
    const float *thr;         // [nq] APPEND threshold on the approximate raw value
    // gather mode (selective PREWHERE): the scan walks positions of this list
    // of selected rows instead of rows; each chunk's rows are padded with -1 to
    // whole 256-entry tiles, so a tile never spans two chunks.  Probe columns
    // are list positions; candidates store rows.
    const int32_t *row_list;  // null = contiguous rows
    // binary scan (kernels_binary.hip)
    const uint32_t *codes;    // [n][code_words]
    const uint32_t *qcodes;   // [nq][code_words]
    int code_words;
    int nbits;                // d: Hamming distances == nbits are never returned
    int tau_strict;           // APPEND takes key < tau (segments after the probe) instead of <=
    unsigned long long *dbg;  // diagnostic builds only (stage timing stamps)
    void *p4_queue;           // batch scan (kernels_p4.hip): per-wave candidate queues, p4_queue_bytes()
    float *p4_gmax;           // batch PROBE (kernels_p4.hip): [nq][p4_gld] best approximate value per
                              // (query, 128-row half tile), as a raw metric value; NaN = no row
    int64_t p4_gld;
    int blas_nq;              // batch size that selects faiss's distance formula (0: nq); a query
                              // sub-batch of a larger call keeps the call's formula
};

// faiss's formula branch (distance_compute_blas_threshold) for this scan's call
__host__ __device__ inline bool blas_formula(const ScanParams &p) {
    return (p.blas_nq > 0 ? p.blas_nq : p.nq) >= kBlasThreshold;
}

// Row at scan position pos (-1 = padding entry of the gather list).
__device__ inline int64_t row_at(const ScanParams &p, int64_t pos) {
    return p.row_list ? (int64_t)p.row_list[pos] : pos;
}

// Tile -> [r0, r1) and chunk index ([r0, r1) are scan positions: rows, or
// gather-list positions).
__device__ inline void tile_range(const ScanParams &p, int64_t t, int64_t &r0, int64_t &r1,
                                  int64_t &chunk) {
    if (p.row_list) {
        // the first entry of a tile is a real row (padding only ends a chunk)
        r0 = p.row_begin + t * p.tile_rows;
        r1 = r0 + p.tile_rows;
        if (r1 > p.row_end) r1 = p.row_end;
        chunk = r0 < r1 ? (int64_t)p.row_list[r0] / p.chunk_rows : 0;
        return;
    }
    if (p.tiles_per_chunk > 0) {
        const int64_t c0 = p.row_begin / p.chunk_rows;  // row_begin is chunk-aligned
        chunk = c0 + t / p.tiles_per_chunk;
        r0 = chunk * p.chunk_rows + (t % p.tiles_per_chunk) * p.tile_rows;
        int64_t ce = (chunk + 1) * p.chunk_rows;
        r1 = r0 + p.tile_rows;
        if (r1 > ce) r1 = ce;
    } else {
        r0 = p.row_begin + t * p.tile_rows;
        r1 = r0 + p.tile_rows;
        chunk = p.chunk_rows > 0 ? r0 / p.chunk_rows : 0;
    }
    if (r1 > p.row_end) r1 = p.row_end;
}

// Ordinal of a granule chunk: how many searchWrapper calls the reference made
// on this part before it (cosine re-normalises the query on each call);
// -1 = the reference never searches this chunk.
__device__ inline int chunk_ordinal(const ScanParams &p, int64_t chunk) {
    if (!p.chunk_ord) return (int)chunk + p.ord_base;
    const int o = p.chunk_ord[chunk];
    return o < 0 ? o : o + p.ord_base;
}

__device__ inline int variant_of(const ScanParams &p, int q, int ord) {
    if (p.maxv <= 1) return 0;
    const int mu = p.qmu[q], lam = p.qlam[q];
    return ord < mu ? ord : mu + (ord - mu) % lam;
}

__device__ inline bool row_valid(const ScanParams &p, int64_t r) {
    if (p.filter) {
        if (!bit_test(p.filter, r)) return false;
        if (p.nonempty && !bit_test(p.nonempty, r)) return false;
    }
    if (p.exists && !bit_test(p.exists, r)) return false;
    return true;
}

// ---------------------------------------------------------------------------
// Launchers (kernels_*.hip)
void launch_scan_small(const ScanParams &p, int metric, bool probe, hipStream_t s);
void launch_gather_count(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                         int64_t chunk_rows, int tile, int *count, int64_t *offsets, int64_t *totals,
                         int64_t *host_totals, int64_t host_gen, int *ticket, hipStream_t s);
void launch_gather_list(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                        int64_t chunk_rows, int tile, const int *count, const int64_t *offsets, int32_t *list, int64_t list_end,
                        hipStream_t s, const int64_t *dev_total = nullptr, int64_t round = 1);
// Bound pruning of an index re-rank (kernels_rerank.hip): the candidates come
// sorted by their approximate value; those more than 2 B past the k-th
// approximate value cannot reach the exact top k and are not re-ranked (same
// output).  raw = null: every candidate is re-ranked.
struct RerankPrune {
    const float *raw = nullptr;           // [nq][ncand] approximate raw values in candidate order (NaN: none)
    const float *bq = nullptr;            // [nq] bound on |approx - exact| for query variant 0 (k_query_bound)
    const float *ymax = nullptr;          // device scalar: max |y| over the rows (cosine variant term)
    const float *qdelta = nullptr;        // [nq] cosine: >= max_v |x_v - x_0| (k_query_prep); null: computed here
    unsigned long long *count = nullptr;  // += candidates re-ranked (may be null)
};
void launch_rerank_ids(const ScanParams &p, int metric, const int64_t *cand, int ncand, int k,
                       int64_t id_offset, int64_t *out_ids, float *out_dist, uint4 *scratch, hipStream_t s,
                       const RerankPrune &prune = RerankPrune{});
// the same re-rank over waves (k_rerank_plan + k_exact_records_w +
// k_sort_emit; ncand <= kSortCap, d % 4 == 0, else false and nothing runs):
// scratch surv [nq][ncand] u32, cnt [nq], recs [nq][ncand]
bool launch_rerank_ids_wide(const ScanParams &p, int metric, const int64_t *cand, int ncand, int k,
                            int64_t id_offset, int64_t *out_ids, float *out_dist, const RerankPrune &pr,
                            uint32_t *surv, int *cnt, uint4 *recs, hipStream_t s);
void launch_scan_mfma(const ScanParams &p, int metric, bool probe, hipStream_t s);
void launch_probe_select(const float *probe, int64_t P, int64_t ld, int nq, int k, int metric,
                         uint32_t *tau, int *cand_count, Cand *cand, int cand_cap,
                         int64_t row_base, const int32_t *row_list, hipStream_t s);
void launch_cand_tau(const Cand *cand, const int *cand_count, int cand_cap, int nq, int k,
                     int metric, uint32_t *tau, const int *overflow_q, hipStream_t s);
// decoupled parts (index.hip): ids[i] = map[ids[i]] for ids >= 0
// (transferToNewRowIds); new-part filter -> old-part filter (getRealBitmap):
// old bit inv_ids[i] for every set new bit i < inv_len with inv_src[i] ==
// own_id (inv_ids null: the filter passes through unchanged); old_words is
// zeroed first, (old_rows + 31) / 32 words.
void launch_map_ids(int64_t *ids, int64_t count, const uint64_t *map, hipStream_t s);
void launch_decoupled_filter(const uint8_t *new_filter, int64_t new_rows, const uint64_t *inv_ids,
                             const uint8_t *inv_src, int64_t inv_len, uint32_t own_id, uint32_t *old_words,
                             int64_t old_rows, hipStream_t s);

// mqvs_search with device pointers on `stream` (sharded.hip)
void search_segment(mqvs_segment *seg, const float *queries, int nq, int k, int metric, const uint8_t *filter,
                    const uint8_t *exists, int64_t *out_ids, float *out_dist, uint32_t flags, hipStream_t stream,
                    int64_t ord_base);
// the same, asynchronous: no host sync; the fallback flags (bit 0 candidate
// overflow, bit 1 cosine variant table too short) are OR-ed into *flag_word,
// and search_collect_stats(device) fills the thread's stats after the
// caller's stream sync
void search_segment_async(mqvs_segment *seg, const float *queries, int nq, int k, int metric, const uint8_t *filter,
                          const uint8_t *exists, int64_t *out_ids, float *out_dist, uint32_t flags,
                          hipStream_t stream, int64_t ord_base, int *flag_word);
void search_collect_stats(int device);
// number of granule chunks of [0, n) the reference searches (a non-empty row
// that, under a PREWHERE filter, passes it and is not deleted) -> *count
void launch_count_active_chunks(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists, int64_t n,
                                int64_t chunk_rows, int *flags_scratch, int64_t *count, hipStream_t s);

// ASYNC calls: OR a search's device flags into the calling thread's sticky
// word (read and cleared by mqvs_async_check): bit 0 = candidate overflow
// (overflow[0] != 0), bit 1 = cosine variant chain did not repeat (status[0]
// != 0 and status_matters).  overflow / status may be null.
void launch_async_flags(const int *overflow, const int *status, int status_matters, int *sticky, hipStream_t s);
int *async_sticky(int device, hipStream_t s);

// scratch: null, or 2 kLargeCap uint4 records per query (k > kSortCap)
void launch_final_select(const Cand *cand, const int *cand_count, int cand_cap, int nq, int k,
                         int metric, int64_t chunk_rows, int64_t id_offset, int64_t *out_ids,
                         float *out_dist, int *overflow, uint4 *scratch, hipStream_t s);
// scratch: 2 nshards k uint4 records per query when nshards k > kSortCap
void launch_merge_shards(int nshards, int nq, int k, int metric, const int64_t *in_ids,
                         const float *in_dist, int64_t *out_ids, float *out_dist, bool part_merge,
                         uint4 *scratch, hipStream_t s);
void launch_normalize_rows(float *rows, int64_t n, int d, hipStream_t s);
void launch_row_norms(const float *rows, int64_t n, int d, float *norms, hipStream_t s);
// maxv: variants stored per query (1 unless cosine)
// phase: 0 everything; 1 variant 0 only; 2 the rest of the chain (after 1)
void launch_query_prep(const float *q, int nq, int d, int metric, bool blas, float *qvars, int maxv,
                       float *qnorms, int *qmu, int *qlam, int *status, hipStream_t s, int phase = 0,
                       float *qdelta = nullptr);
void launch_generate(uint64_t seed, int mode, int64_t row0, int64_t n, int d, float *out,
                     hipStream_t s);
void launch_pack_nonempty(const uint8_t *bytes, int64_t n, uint8_t *bits, hipStream_t s);
// up to two 32-bit fills (a: na words of va, b: nb words of vb) in one launch
void launch_fill2(uint32_t *a, int64_t na, uint32_t va, uint32_t *b, int64_t nb, uint32_t vb, hipStream_t s);
void launch_chunk_ordinals(const uint8_t *filter, const uint8_t *nonempty, const uint8_t *exists,
                           int64_t n, int64_t chunk_rows, int require_filter, int *ord,
                           hipStream_t s);

// column ingest (kernels_ingest.hip): compressed MergeTree column files -> rows
struct IngestBlock {
    int64_t src;      // payload offset in the compressed stream
    int64_t dst;      // offset in the decompressed stream
    uint32_t csize;   // payload bytes
    uint32_t usize;   // decompressed bytes
    uint32_t method;  // 0x82 LZ4, 0x02 NONE
    uint32_t pad;
};
void launch_block_table(const uint8_t *src, int64_t n, IngestBlock *tab, int64_t max_blocks, int64_t *out,
                        hipStream_t s);
void launch_decode_blocks(const uint8_t *src, int64_t src_bytes, const IngestBlock *tab, int64_t nblocks, uint8_t *dst,
                          int *status, hipStream_t s);
// CityHash128 of block i's header + payload != its stored checksum -> *status |= flag;
// hash_out (optional) receives [nblocks][2] (low, high)
void launch_block_checksum(const uint8_t *src, const IngestBlock *tab, int64_t nblocks, int flag, int *status,
                           uint64_t *hash_out, hipStream_t s);
void launch_sizes_scan(const uint64_t *sizes, int64_t n, int d, int64_t *offsets, int64_t *scratch, int64_t *stats,
                       hipStream_t s);
void launch_array_rows(const float *data, const int64_t *offsets, const uint64_t *sizes, int64_t n, int d,
                       float *rows, uint8_t *nonempty, hipStream_t s);

// binary vectors (kernels_binary.hip)
void launch_scan_binary(const ScanParams &p, int metric, bool probe, hipStream_t s);
void launch_hamming_to_int(const int64_t *ids, float *dist, int64_t m, hipStream_t s);

// bf16 pre-filter path (kernels_bf16.hip)
constexpr int kBfK = 64;    // bf16 planes padded to a multiple of this
// bf16 plane layout (rows_hi, q_hi, q_ord; written by launch_to_hi): vectors
// in groups of 16; a group is dpad / kPlaneSlab column slabs back to back, each
// [16 vectors][kPlaneSlab columns] with one vector's slab columns contiguous.
// Readers address k-step s (32 columns) of vector v16 of a group at
// plane_step_off(s) + plane_vec_off(v16).  kPlaneSlab = 32: a stage's piece
// of 16 vectors is 1 KiB contiguous (8 whole 128-B lines per wave
// instruction).  64 would give each vector one whole 128-B line per slab, so
// a gathered row (selective PREWHERE) would fetch none of its neighbour's
// bytes -- measured in round 4 (profiles/r04/layout/bench_slab64.json, every
// GPU test green): the 10 % configs[4] main scan 2.29 -> 1.88 ms, but the
// streaming scans read 16 half lines per instruction and slowed: nq 1 full
// scan 10.9 -> 13.9 ms (50M x 768), nq 1000 batch 12.6 -> 13.6 ms.
constexpr int kPlaneSlab = 32;
static_assert(kBfK % kPlaneSlab == 0, "dpad is a whole number of slabs");
__host__ __device__ constexpr uint32_t plane_vec_off(uint32_t v16) { return v16 * (uint32_t)(kPlaneSlab * 2); }
__host__ __device__ constexpr uint32_t plane_step_off(uint32_t s) {
    return (s / (uint32_t)(kPlaneSlab / 32)) * (16u * kPlaneSlab * 2) + (s % (uint32_t)(kPlaneSlab / 32)) * 64u;
}
constexpr int kHiSplit = 2; // bf16 hi*hi, bound from measured residual norms (kernels_hi.hip)
constexpr int kMxRec = 8;   // floats per vector in the norm records (launch_to_hi)
// dst_hi = bf16_rn(x), row-major [rows][dpad] (the index's list planes)
void launch_to_bf16(const float *src, int64_t rows, int d, int64_t src_stride, uint16_t *dst_hi, int64_t dpad,
                    hipStream_t s);
void launch_max_norm(const float *norms2, int64_t n, float *out_max, hipStream_t s);
// qrec [nq][maxv][kMxRec] query-variant norm records, yrec [kMxRec] segment maxima
void launch_query_bound(const ScanParams &p, int metric, const float *ynorm_max, const float *qrec,
                        const float *yrec, float *bq, hipStream_t s);
// split 2 (kernels_hi.hip): row-blocked bf16 hi plane (16 vectors x 32
// columns contiguous; source vector v goes to plane vector
// (v % vgroup) vpad + v / vgroup) + records [|h|, |r|, -, -, -, -, |x|] per
// vector (rec) / maxima (maxrec, atomic)
void launch_to_hi(const float *src, int64_t rows, int d, int64_t src_stride, int64_t dpad, int64_t vgroup,
                  int64_t vpad, uint16_t *hi, float *rec, float *maxrec, hipStream_t s);
void launch_scan_hi(const ScanParams &p, int metric, bool probe, hipStream_t s);
bool scan_hi_small_tiles_ok(int nq, int64_t dpad);
// batch APPEND scan at one wave per SIMD (kernels_p4.hip): false when the
// scan's shape is not served (gather lists, chunk-ordinal tables, no queue)
bool launch_scan_p4(const ScanParams &p, int metric, hipStream_t s);
// the batch probe (p.p4_gmax, p.p4_gld >= 2 p.tiles): false when the rows
// cannot take the batch kernel
bool launch_scan_p4_probe(const ScanParams &p, int metric, hipStream_t s);
// cosine ordinal planes for the batch kernel: at most pcap planes, built on
// the device from q_hi / qmu / qlam (desc[2] = 0 when the chains need more)
constexpr int kP4OrdPlanesMax = 32;
void launch_ord_planes(const uint16_t *q_hi, uint16_t *q_ord, int *desc, const int *qmu, const int *qlam, int nq,
                       int64_t vpad, int64_t dpad, int pcap, hipStream_t s);
size_t p4_queue_bytes();  // p4_queue workspace for the current device
int take_batch_kernel_flag();  // 1 when a main scan since the last call ran kernels_p4 (then cleared)
void launch_probe_select_approx(const float *probe, int64_t P, int64_t ld, int nq, int k,
                                int metric, const float *bq, float *thr, int *cand_count,
                                Cand *cand, int cand_cap, const int32_t *row_list, hipStream_t s);
void launch_refine(const Cand *cin, const int *cnt_in, int cap, int nq, int k, int metric,
                   bool approx, const float *bq, uint32_t *tau, float *thr, Cand *cout, int *cnt_out,
                   hipStream_t s);
// the segment an index was built over (cache.hip validates put pairs)
mqvs_segment *index_segment(mqvs_index *idx);
// fl / host_fl (optional): the final select's first workgroup also stores the
// 8 words fl (written by earlier kernels of the stream) into pinned host_fl --
// the search's status copy without a kernel of its own
void launch_rerank_select(const ScanParams &p, int metric, const float *bq, int k, int64_t id_offset,
                          int64_t *out_ids, float *out_dist, int *overflow, uint32_t *surv, int *scnt,
                          uint4 *recs, int lcap, int64_t rs, hipStream_t s, const int *fl = nullptr,
                          int *host_fl = nullptr);
void launch_exact_rerank(const ScanParams &p, int metric, const uint32_t *surv, const int *cnt, int64_t rs,
                         int cap, uint4 *recs, int k, int64_t id_offset, int64_t *out_ids, float *out_dist,
                         hipStream_t s, const int *fl = nullptr, int *host_fl = nullptr);

// ---------------------------------------------------------------------------
// Index path (kernels_ivf.hip, index.hip)
constexpr int kIvfPad = 16;  // list lengths padded to this many positions

constexpr int kIvfChunk = 512;  // default list positions per scan work item (balances long and short lists)

struct IvfParams {
    const uint16_t *plane;    // [npos][dpad] bf16 rows in list order
    const int32_t *perm;      // [npos] segment row of each position, -1 = padding
    const float *pnorm;       // [npos] |y|^2 per position
    const int64_t *list_off;  // [nlist+1] list start positions (multiples of kIvfPad)
    int nlist;
    int64_t dpad;
    int nq, nprobe;
    int qg;                   // queries per scan work item: 16 or 32 (MFMA B blocks x 16)
    int chunk;                // list positions per scan work item (multiple of 64)
    const int64_t *probes;    // [nq][nprobe] list ids (-1 = none)
    const uint16_t *q_hi;     // [nq][dpad] bf16 query (cosine: normalised)
    const float *qnorm;       // [nq] |q|^2 (L2)
    const uint8_t *filter;    // PREWHERE bitmap (rows) or null
    const uint8_t *exists;    // LWD bitmap (rows) or null
    int *lcount;              // [nlist] queries probing each list
    int *lfill;               // [nlist] scatter cursors
    int64_t *lstart;          // [nlist] first pair of each list in lq
    int *lq;                  // [nq*nprobe] pairs (q*nprobe + probe) grouped by list
    int *item_list;           // [nq*nprobe] work item -> list
    int *item_grp;            // work item -> query group within the list
    int *item_chk;            // work item -> slice of the list
    int *nitems;              // number of work items
    int64_t *qbase;           // [nq*nprobe] start of each pair's region in cand
    int64_t *qstart;          // [nq+1] start of each query's region
    Cand *cand;               // approximate values, one per (pair, list position)
    int64_t *stats;           // [4] values written, items, plane bytes, pairs
    int64_t *bsum;            // [3 * plan workgroups] per-workgroup list totals (k_plan_lists_reg)
    // pair mode (pair_stride > 0; few pairs per list): no plan -- work item
    // it is (pair it / pair_nch, slice it % pair_nch) of one query, query q's
    // region starts at q * pair_stride and holds its probes' lists back to back
    int64_t pair_stride;
    int pair_nch;
};

// The per-query candidate regions of a list pass, as the select reads them:
// the plan's qstart[nq + 1], or pair mode's fixed strides (regions filled by
// the probed lists' lengths; the select then also sums the stats).
struct IvfRegions {
    const int64_t *qstart = nullptr;
    int64_t stride = 0;
    int nprobe = 0, nlist = 0, chunk = 0;
    int64_t dpad = 0;
    const int64_t *probes = nullptr;
    const int64_t *list_off = nullptr;
    int64_t *stats = nullptr;  // pair mode: [nq][4] values, items, plane bytes, pairs per query
};

void launch_ivf_plan(const IvfParams &p, hipStream_t s);
void launch_iota_probes(int64_t *probes, int nq, int np, hipStream_t s);
void launch_ivf_plan_dense(const IvfParams &p, int64_t npos, hipStream_t s);
void launch_ivf_scan(const IvfParams &p, int metric, int grid, hipStream_t s);
// expect_len: typical per-query region length (sizes the LDS key cache)
void launch_ivf_select(const Cand *cand, const IvfRegions &rg, int nq, int R, int metric, int64_t *out_rows,
                       int64_t id_offset, float *out_approx, int64_t expect_len, hipStream_t s, uint4 *gscr = nullptr,
                       float *out_raw = nullptr);
void launch_ivf_pack(const float *rows, const float *norms, int d, const int32_t *perm, int64_t npos, int64_t dpad,
                     uint16_t *plane, float *pnorm, hipStream_t s);
void launch_gather_rows(const float *src, int64_t src_ld, int d, const int64_t *idx, int64_t m, float *dst,
                        hipStream_t s);
constexpr int kCoarsePickMaxT = 64;  // core groups (and nprobe) of a coarse pick
constexpr int kCoarsePickCap = 128;  // groups a pick's working set holds (more: its batched overflow path)
// the coarse step's pick from the batch probe's 16-centroid group maxima
// (kernels_ivf.hip): per query the T best groups (T <= 64) and every group
// within 2 bq[q] of the T-th (bq: the query's bf16 bound, k_query_bound;
// null = none), the exact values of their centroids (coarse metric: L2 or
// kMetricIpRaw), the nprobe best -> probes[q][0, nprobe) (-1 when fewer)
void index_thread_release();  // index.hip: the calling thread's index workspaces
void launch_coarse_pick(const float *gmax, int64_t gld, int64_t ngroups, int T, int nprobe, int metric,
                        const float *q, int64_t qld, const float *cent, const float *cnorm, int64_t ncent, int d,
                        const float *bq, const float *qnorms, int gs_log2, int nq, int64_t *probes,
                        unsigned long long *ovf, hipStream_t s);
// the batch probe by 16-row groups (kernels_p4.hip): p.p4_gmax[q][16 t + r]
// = the best value of rows [16 r, 16 r + 16) of tile t (p.p4_gld >= 16
// p.tiles); false when the rows cannot take the batch kernel
// the call's per-kernel timing events (MQVS_F_TIMING or mqvs_set_timing)
bool timing_on(uint32_t flags);
// a[0, na) and b[0, nb) into pinned host memory (system-scope stores; one
// launch instead of two copy kernels before the caller's stream sync)
// (pq: a's words are the sums over npq rows of pq[npq][na] instead)
void launch_words_to_host(const int64_t *a, int na, const int *b, int nb, int64_t *host_a, int *host_b,
                          hipStream_t s, const int64_t *pq = nullptr, int npq = 0);
bool launch_scan_p4_groups(const ScanParams &p, int metric, int grp, hipStream_t s);
void launch_centroid_mean(const float *rows, int d, const int32_t *order, const int64_t *off, int nlist, float *cent,
                          hipStream_t s);

// ---------------------------------------------------------------------------
// Error plumbing
void set_error(const std::string &msg);

struct Error {
    int code;
    std::string msg;
};

#define MQVS_HIP(call)                                                                 \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            throw ::mqvs::Error{e_ == hipErrorOutOfMemory ? MQVS_ERR_MEMORY_LIMIT         \
                                                          : MQVS_ERR_DEVICE,             \
                                std::string(#call) + ": " + hipGetErrorString(e_)};    \
    } while (0)

// ---------------------------------------------------------------------------
// Host-side plumbing shared by mqvs.hip (segments, FLAT search) and
// index.hip (the index path)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (bytes > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            MQVS_HIP(hipMalloc(&p, bytes));
            cap = bytes;
        }
        return p;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Pinned host staging of a synchronous call's host inputs and outputs: the
// caller's (pageable) arrays are copied by the CPU into it and DMA'd from it,
// so the HIP runtime never stages a pageable copy itself (it waits for those
// by spinning: with 16 threads searching 10M x 768 at nq 1000 from host
// arrays, 18 % of each thread's wall time was CPU time, profiles/r06).
// Reused across calls (each synchronous call ends after its copies).
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes == 0) bytes = 16;
        if (bytes > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            MQVS_HIP(hipHostMalloc(&p, bytes, hipHostMallocDefault));
            cap = bytes;
        }
        return p;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};
// host -> device through `pin` (the CPU copy now, the DMA queued on s)
inline void stage_in(HostBuf &pin, void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    void *h = pin.get(bytes);
    std::memcpy(h, src, bytes);
    MQVS_HIP(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s));
}

// Per-thread scratch of another path (the index's, index.hip) counted in, and
// trimmed with, the calling thread's FLAT workspace under the process-wide
// HBM budget (mqvs_set_workspace_budget): the reference runs index searches
// from as many part threads as FLAT scans (VIWithDataPart.cpp:900-901 under
// ScanThreadLimiter.h:25-58), so both share one admission gate.
struct WsExt {
    // every gated buffer freed once the owner's work on it has drained (the
    // caller holds the owner's workspace); returns the bytes freed
    virtual size_t free_scratch() = 0;

   protected:
    ~WsExt() = default;
};
// a DevBuf whose growth passes the gate of the calling thread's current
// WsScope (fails outside one: no ungated scratch)
struct GBuf : DevBuf {
    void *get(size_t bytes);
};
// one call on the calling thread's workspace of `device` (admission, nests
// with FLAT calls), with `ext` attached to it
class WsScope {
   public:
    WsScope(int device, WsExt *ext);
    ~WsScope();
    void set_stream(hipStream_t s);  // the stream whose completion ends the call's use of its buffers
    WsScope(const WsScope &) = delete;
    WsScope &operator=(const WsScope &) = delete;

   private:
    void *impl_ = nullptr;
    void *prev_ = nullptr;
};
// index_thread_release: `ext`'s scratch freed and detached from the thread's workspace
void ws_detach_ext(int device, WsExt *ext);
// the search entry points' fault drill (mqvs_inject_fault): throws the armed
// status while this thread's count lasts
void fault_point();

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        MQVS_HIP(hipGetDevice(&prev));
        if (prev != dev) MQVS_HIP(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename F>
static int guarded(F &&f) {
    try {
        f();
        return MQVS_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MQVS_ERR_MEMORY_LIMIT;
    } catch (...) {
        set_error("unknown error");
        return MQVS_ERR_DEVICE;
    }
}

[[noreturn]] inline void fail(int code, const std::string &msg) { throw Error{code, msg}; }

// mqvs.hip services used by the index path
hipStream_t thread_stream(int device);
// compute units of the current device (cached per device: launchers size
// their persistent grids from it on every call)
int device_cus();
// The host's wait for the work queued on `s` (every synchronous call ends with
// one): the policy of mqvs_set_wait_mode -- the runtime's own
// hipStreamSynchronize, or a short poll of a blocking-sync event's completion
// followed by a blocking wait on it (the calling thread sleeps instead of
// holding a core for the length of the search).  The current device must be
// s's.
void host_wait(hipStream_t s);
// The wait history's key for the host_waits of one API call: set by the
// entry points from the call's shape (function, segment, nq, k, filter,
// flags); each wait position within the call keeps its own history, so a
// thread alternating nq 1000 and nq 1 searches sleeps each for its own length.
struct WaitScope {
    uint64_t prev_key;
    int prev_ord;
    explicit WaitScope(std::initializer_list<uint64_t> parts);
    ~WaitScope();
    WaitScope(const WaitScope &) = delete;
    WaitScope &operator=(const WaitScope &) = delete;
};
inline uint64_t wait_str_hash(const char *p) {  // (a parameter string's part of a wait key)
    uint64_t h = 1469598103934665603ull;
    for (; p && *p; ++p) h = (h ^ (unsigned char)*p) * 1099511628211ull;
    return h;
}
// the ids and distances of a synchronous host-pointer call: device ->
// pinned `pin` -> the caller's arrays (m results each), after the work queued
// on s (one host_wait)
void stage_out_results(HostBuf &pin, int64_t *ids, float *dist, const int64_t *dids, const float *ddist, size_t m,
                       hipStream_t s);
// the same in two halves, so the call's last host_wait covers the copies:
// begin queues the device -> pinned copies on s, end (after that wait)
// copies pinned -> the caller's arrays
void stage_out_begin(HostBuf &pin, const int64_t *dids, const float *ddist, size_t m, hipStream_t s);
void stage_out_end(const HostBuf &pin, int64_t *ids, float *dist, size_t m);
// poll budget of the hybrid wait (microseconds; 0 in MQVS_WAIT_BLOCK, -1 in
// MQVS_WAIT_RUNTIME): also bounds the spin on a pinned-memory word
int wait_spin_us();
// one pause of a host spin loop (x86 PAUSE: the core yields to its sibling
// hyper-thread and saves power while polling)
void cpu_relax();
double measure_read_sweep(size_t bytes, int reps, hipStream_t s, double *best_ms);
size_t scratch_budget();  // bytes per scratch buffer of one call (mqvs_set_scratch_budget)
// FLAT search of a segment (MergeTreeVSManager::vectorScanWithoutIndex);
// metric may be kMetricIpRaw (faiss knn_inner_product contract)
void search_internal(mqvs_segment *seg, const float *queries, int nq, int k, int metric,
                     const uint8_t *filter, const uint8_t *exists, int64_t *out_ids, float *out_dist,
                     uint32_t flags, hipStream_t stream);
// segment from rows already on the current device (copied); granule = n
mqvs_segment *segment_from_device(const float *dev_rows, int64_t n, int d, int metric, hipStream_t st);
void segment_release(mqvs_segment *s);

}  // namespace mqvs
