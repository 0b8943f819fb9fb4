/*
 * mqvs_vector_index.hpp -- header-only C++ binding of libmqvs.so (include/mqvs.h)
 * for the MyScaleDB tree: the drop-in for the brute-force vector-scan seams.
 *
 * What it replaces (paths relative to the MyScaleDB source tree):
 *   VectorIndex::MI355X::tryBruteForceSearch
 *       VectorIndex::tryBruteForceSearch<Search::DataType::FloatVector>
 *       (src/VectorIndex/Common/BruteForceSearch.h:62-92): faiss knn_L2sqr /
 *       knn_inner_product over host buffers, NOT_IMPLEMENTED for other metrics.
 *   VectorIndex::MI355X::PartScan
 *       the per-part body of MergeTreeVSManager::vectorScanWithoutIndex<Float>
 *       + searchWrapper + VIWithColumnInPart::searchWithoutIndex
 *       (src/VectorIndex/Storages/MergeTreeVSManager.cpp:960-1680,
 *       src/VectorIndex/Common/VIWithDataPart.h:341-382): the part's
 *       Array(Float32) column is registered once in HBM (instead of being
 *       copied granule by granule into vector_raw_data) and every query batch
 *       is one call; scan() assembles the label / vector_id / distance columns
 *       exactly as MergeTreeVSManager.cpp:1502-1532 does (-1 ids dropped).
 *   VectorIndex::MI355X::PartScan::rerank
 *       VIWithColumnInPart::computeTopDistanceSubset (VIWithDataPart.cpp:838-856)
 *   VectorIndex::MI355X::mergeShardResults
 *       MergeTreeBaseSearchManager::getTotalTopSearchResultImpl
 *       (MergeTreeBaseSearchManager.cpp:207-297) for row-range shards.
 *   VectorIndex::MI355X::ShardComm
 *       one part spread over the GPUs of a node as row-range shards, searched
 *       with RCCL inside libmqvs (one all-gather of (id, distance), device
 *       merge) instead of per-shard LIMIT + the initiator's merge
 *       (StorageDistributed.cpp:1057-1060).
 *   VectorIndex::MI355X::GpuIndex
 *       the Search::VectorIndex object VIWithColumnInPart holds
 *       (VIWithDataPart.h:295-339): build (VIWithDataPart.cpp:416-447), search
 *       (:926, with the decoupled-part row_ids_map remap of :938-943 /
 *       transferToNewRowIds :56-67) and computeTopDistanceSubset (:838-856).
 *   VectorIndex::MI355X::getRealBitmap
 *       VIUtils.cpp:479-497 (decoupled part filter -> source part filter).
 *   VectorIndex::MI355X::PartCache
 *       VICacheManager (src/VectorIndex/Cache/VICacheManager.h:82-114): an LRU
 *       of parts (+ index) resident in HBM under a byte budget; load() is
 *       LRUResourceCache::getOrSet, the returned holder pins the entry.
 *
 * Errors: every non-zero mqvs status is rethrown as DB::Exception with the
 * ErrorCodes value the reference throws for the same condition.  Threading:
 * a PartScan is immutable after construction and may be searched from any
 * number of threads at once (the library keeps one HIP stream and workspace
 * per calling thread; no global lock).
 *
 * Define MQVS_SHIM_STANDALONE to build without the ClickHouse headers (the
 * repository's own tests do); DB::Exception / DB::ErrorCodes are then minimal
 * stand-ins with the same codes.
 */
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "mqvs.h"

#if defined(MQVS_SHIM_STANDALONE)
#include <stdexcept>
namespace DB
{
namespace ErrorCodes
{
    constexpr int BAD_ARGUMENTS = 36;
    constexpr int CHECKSUM_DOESNT_MATCH = 40;
    constexpr int ILLEGAL_COLUMN = 44;
    constexpr int NOT_IMPLEMENTED = 48;
    constexpr int LOGICAL_ERROR = 49;
    constexpr int MEMORY_LIMIT_EXCEEDED = 241;
}
class Exception : public std::runtime_error
{
public:
    Exception(int code_, const char * /*fmt "{}"*/, const std::string & message)
        : std::runtime_error(message), error_code(code_) {}
    int code() const { return error_code; }

private:
    int error_code;
};
}
#else
#include <Common/Exception.h>
namespace DB
{
namespace ErrorCodes
{
    extern const int BAD_ARGUMENTS;
    extern const int CHECKSUM_DOESNT_MATCH;
    extern const int ILLEGAL_COLUMN;
    extern const int NOT_IMPLEMENTED;
    extern const int LOGICAL_ERROR;
    extern const int MEMORY_LIMIT_EXCEEDED;
}
}
#endif

namespace VectorIndex::MI355X
{

/// DB::ErrorCodes value for a libmqvs status (include/mqvs.h).
inline int dbErrorCode(int status)
{
    switch (status)
    {
        case MQVS_ERR_NOT_IMPLEMENTED: return DB::ErrorCodes::NOT_IMPLEMENTED;
        case MQVS_ERR_ILLEGAL_COLUMN: return DB::ErrorCodes::ILLEGAL_COLUMN;
        case MQVS_ERR_BAD_ARGUMENTS: return DB::ErrorCodes::BAD_ARGUMENTS;
        case MQVS_ERR_MEMORY_LIMIT: return DB::ErrorCodes::MEMORY_LIMIT_EXCEEDED;
        case MQVS_ERR_CHECKSUM: return DB::ErrorCodes::CHECKSUM_DOESNT_MATCH;
        default: return DB::ErrorCodes::LOGICAL_ERROR;  /// LOGICAL / DEVICE
    }
}

inline void check(int status)
{
    if (status == MQVS_OK)
        return;
    const char * msg = mqvs_last_error();
    throw DB::Exception(dbErrorCode(status), "{}", std::string("MI355X vector scan: ") + (msg ? msg : ""));
}

/// VIMetric (Search::Metric) -> mqvs metric id; -1 for metrics this path does
/// not serve (the callers then throw NOT_IMPLEMENTED like the reference).
template <typename MetricEnum>
int toMqvsMetric(const MetricEnum & metric)
{
    if (metric == MetricEnum::L2)
        return MQVS_METRIC_L2;
    if (metric == MetricEnum::IP)
        return MQVS_METRIC_IP;
    if (metric == MetricEnum::Cosine)
        return MQVS_METRIC_COSINE;
    if (metric == MetricEnum::Hamming)
        return MQVS_METRIC_HAMMING;
    if (metric == MetricEnum::Jaccard)
        return MQVS_METRIC_JACCARD;
    return -1;
}

/// Host fallback on a device failure ("on device error the host
/// falls back to the CPU path").  The seams below take an optional callable
/// that runs the reference's own CPU code in place of the GPU call when
/// libmqvs returns MQVS_ERR_DEVICE or MQVS_ERR_MEMORY_LIMIT (a lost or
/// exhausted device); every other status still throws.  In the ClickHouse
/// tree the callable is the call the seam replaced, e.g. faiss::knn_L2sqr /
/// knn_inner_product for tryBruteForceSearch (BruteForceSearch.h:80-87), the
/// per-part CPU vectorScanWithoutIndex for PartScan, the CPU index for
/// GpuIndex.  fallbackCount() counts the calls it served (a metric to export).
inline bool isFallbackStatus(int status)
{
    return status == MQVS_ERR_DEVICE || status == MQVS_ERR_MEMORY_LIMIT;
}

inline std::atomic<uint64_t> & fallbackCount()
{
    static std::atomic<uint64_t> n{0};
    return n;
}

/// status -> done (OK), `run` (a device failure and the caller gave a
/// fallback), or DB::Exception
template <typename F>
void checkOrFallback(int status, bool have_fallback, const F & run)
{
    if (status != MQVS_OK && isFallbackStatus(status) && have_fallback)
    {
        run();
        fallbackCount().fetch_add(1, std::memory_order_relaxed);
        return;
    }
    check(status);
}

/// The CPU search tryBruteForceSearch replaces (faiss knn_L2sqr /
/// knn_inner_product, BruteForceSearch.h:80-87), same arguments.
using BruteForceFallback = std::function<void(const float * x, const float * y, size_t d, size_t k, size_t nx,
                                              size_t ny, int64_t * result_id, float * distance, int mqvs_metric)>;

/// tryBruteForceSearch<FloatVector> (BruteForceSearch.h:62-92): x nx*d
/// queries, y ny*d base, result_id / distance nx*k in faiss layout.
/// fallback: runs instead when the device fails (see isFallbackStatus).
inline void tryBruteForceSearch(
    const float * x, const float * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, int mqvs_metric, const BruteForceFallback & fallback = nullptr)
{
    if (mqvs_metric != MQVS_METRIC_L2 && mqvs_metric != MQVS_METRIC_IP)
        throw DB::Exception(DB::ErrorCodes::NOT_IMPLEMENTED, "{}",
                            std::string("Metric not implemented in brute force search for Float32 Vector"));
    const int st = mqvs_knn_raw(x, y, static_cast<int64_t>(d), static_cast<int64_t>(k), static_cast<int64_t>(nx),
                                static_cast<int64_t>(ny), mqvs_metric, result_id, distance);
    checkOrFallback(st, static_cast<bool>(fallback),
                    [&] { fallback(x, y, d, k, nx, ny, result_id, distance, mqvs_metric); });
}

template <typename MetricEnum>
void tryBruteForceSearch(
    const float * x, const float * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, const MetricEnum & metric_type,
    const BruteForceFallback & fallback = nullptr)
{
    tryBruteForceSearch(x, y, d, k, nx, ny, result_id, distance, toMqvsMetric(metric_type), fallback);
}

/// tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110): x nx*(d/8)
/// query codes, y ny*(d/8) base codes (FixedString bytes), d in bits.
/// Hamming fills `distance` with int32 counts as faiss::hammings_knn_mc does
/// through reinterpret_cast<int32_t*>(distance); Jaccard with floats.
inline void tryBruteForceSearchBinary(
    const uint8_t * x, const uint8_t * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, int mqvs_metric)
{
    if (mqvs_metric != MQVS_METRIC_HAMMING && mqvs_metric != MQVS_METRIC_JACCARD)
        throw DB::Exception(DB::ErrorCodes::NOT_IMPLEMENTED, "{}",
                            std::string("Metric not implemented in brute force search for Binary Vector"));
    check(mqvs_knn_binary_raw(x, y, static_cast<int64_t>(d), static_cast<int64_t>(k), static_cast<int64_t>(nx),
                              static_cast<int64_t>(ny), mqvs_metric, result_id, distance));
}

template <typename MetricEnum>
void tryBruteForceSearchBinary(
    const uint8_t * x, const uint8_t * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, const MetricEnum & metric_type)
{
    tryBruteForceSearchBinary(x, y, d, k, nx, ny, result_id, distance, toMqvsMetric(metric_type));
}

/// Columns emitted by vectorScanWithoutIndex (MergeTreeVSManager.cpp:1502-1532).
struct ScanColumns
{
    std::vector<uint32_t> label;      /// part-local row (result_columns[0])
    std::vector<uint32_t> vector_id;  /// query index, batch only
    std::vector<float> distance;
};

/// Owner of a libmqvs handle: frees it unless ownership was handed on (to a
/// PartCache) or the handle is borrowed (from a PartCache holder).
template <typename H, int (*Free)(H)>
struct Handle
{
    H h = nullptr;
    bool owned = true;
    Handle(H h_, bool owned_) : h(h_), owned(owned_) {}
    Handle(const Handle &) = delete;
    Handle & operator=(const Handle &) = delete;
    ~Handle()
    {
        if (owned && h)
            (void)Free(h);
    }
};
using SegmentHandle = Handle<mqvs_segment_t, mqvs_segment_free>;
using IndexHandle = Handle<mqvs_index_t, mqvs_index_free>;

/// One data part (or a granule-aligned row-range shard of it) resident on a GPU.
class PartScan
{
public:
    /// rows: n*d fp32, row-major; rows whose Array is empty FLT_MAX-filled and
    /// flagged 0 in `nonempty` (n bytes, or nullptr when none is empty).
    PartScan(const float * rows, int64_t n, int32_t d, int mqvs_metric, int64_t granule_rows,
             const uint8_t * nonempty = nullptr, int64_t row_offset = 0, int device = 0)
    {
        check(mqvs_init(device));
        mqvs_segment_t s = nullptr;
        check(mqvs_segment_create(rows, n, d, mqvs_metric, granule_rows, nonempty, row_offset, &s));
        adopt(s, true);
    }

    /// A view of a segment owned elsewhere (a PartCache entry).
    static PartScan borrow(mqvs_segment_t s) { return PartScan(s, false); }

    int32_t dimension() const { return dim; }
    int64_t rows() const { return n; }
    int64_t rowOffset() const { return row_offset; }
    int metricId() const { return metric; }
    mqvs_segment_t handle() const { return seg->h; }

    /// Hand the segment to a new owner (PartCache::put); this object and its
    /// copies stay usable until that owner frees it.
    mqvs_segment_t release() const
    {
        seg->owned = false;
        return seg->h;
    }

    /// HBM bytes held (rows, norms, pre-filter planes).
    size_t hbmBytes() const
    {
        size_t b = 0;
        check(mqvs_segment_info(seg->h, nullptr, nullptr, nullptr, nullptr, nullptr, &b));
        return b;
    }

    /// false when the pre-filter planes did not fit in HBM at creation (or the
    /// rows' norms are not finite): batches then run the exact fp32 MFMA path.
    bool prefilterActive() const
    {
        int32_t ok = 0;
        check(mqvs_segment_prefilter(seg->h, nullptr, nullptr, &ok));
        return ok != 0;
    }

    /// Float32 rows to pinned host memory (HBM keeps the bf16 plane: a part
    /// ~3x larger fits; same results) or back (mqvs_segment_set_rows_host).
    void setRowsHost(bool host) { check(mqvs_segment_set_rows_host(seg->h, host ? 1 : 0)); }

    /// The CPU part scan PartScan replaces (vectorScanWithoutIndex over this
    /// part, MergeTreeVSManager.cpp:960-1536), same arguments and outputs.
    using ScanFallback = std::function<void(const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                                            const uint8_t * row_exists, int64_t * ids, float * dist)>;

    /// Raw top-k: ids / dist nq*k (caller-owned), -1 / FLT_MAX (FLT_MIN for IP)
    /// padded.  filter: PREWHERE bitmap, row_exists: lightweight-delete mask
    /// (LSB-first, n bits, or nullptr).  flags: MQVS_F_* (per call).
    /// fallback: runs instead when the device fails (isFallbackStatus).
    void search(const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                const uint8_t * row_exists, int64_t * ids, float * dist, uint32_t flags = 0,
                const ScanFallback & fallback = nullptr) const
    {
        const int st = mqvs_search(seg->h, queries, nq, k, metric, filter, row_exists, ids, dist, flags, nullptr);
        checkOrFallback(st, static_cast<bool>(fallback),
                        [&] { fallback(queries, nq, k, filter, row_exists, ids, dist); });
    }

    /// Raw top-k of a row-range shard of a larger part: chunk_ord_base = chunks
    /// before the shard that the reference searches (cosine query variant).
    void searchShard(const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                     const uint8_t * row_exists, int64_t chunk_ord_base, int64_t * ids, float * dist) const
    {
        check(mqvs_search_ex(seg->h, queries, nq, k, metric, filter, row_exists, chunk_ord_base, ids, dist, 0,
                             nullptr));
    }

    /// The operator's output for this part, -1 ids dropped; vector_id filled
    /// for batch searches (is_batch) as in MergeTreeVSManager.cpp:1502-1517.
    ScanColumns scan(const float * queries, int32_t nq, int32_t k, bool is_batch,
                     const uint8_t * filter = nullptr, const uint8_t * row_exists = nullptr) const
    {
        std::vector<int64_t> ids(static_cast<size_t>(nq) * k);
        std::vector<float> dist(ids.size());
        search(queries, nq, k, filter, row_exists, ids.data(), dist.data());
        return toColumns(ids, dist, k, is_batch);
    }

    /// As above, after the reference's dimension check (generateVectorDataset,
    /// MergeTreeVSManager.cpp:135-182 throws on a mismatch).
    ScanColumns scan(const float * queries, int32_t nq, int32_t query_dim, int32_t k, bool is_batch,
                     const uint8_t * filter, const uint8_t * row_exists, const ScanFallback & fallback = nullptr) const
    {
        checkDimension(query_dim);
        std::vector<int64_t> ids(static_cast<size_t>(nq) * k);
        std::vector<float> dist(ids.size());
        search(queries, nq, k, filter, row_exists, ids.data(), dist.data(), 0, fallback);
        return toColumns(ids, dist, k, is_batch);
    }

    /// computeTopDistanceSubset: exact distances to nq*ncand candidate rows.
    void rerank(const float * queries, int32_t nq, const int64_t * cand, int32_t ncand, int32_t k,
                const uint8_t * row_exists, int64_t * ids, float * dist) const
    {
        check(mqvs_rerank(seg->h, queries, nq, cand, ncand, k, metric, row_exists, ids, dist, 0, nullptr));
    }

    void checkDimension(int32_t query_dim) const
    {
        if (query_dim != dim)
            throw DB::Exception(DB::ErrorCodes::LOGICAL_ERROR, "{}",
                                "The dimension of searched vector (" + std::to_string(query_dim)
                                    + ") doesn't match the dimension of the vector column (" + std::to_string(dim) + ")");
    }

    /// (ids, dist) nq*k -> the operator's columns, -1 ids dropped.
    static ScanColumns toColumns(const std::vector<int64_t> & ids, const std::vector<float> & dist, int32_t k,
                                 bool is_batch)
    {
        ScanColumns out;
        for (size_t i = 0; i < ids.size(); ++i)
        {
            if (ids[i] <= -1)
                continue;
            out.label.push_back(static_cast<uint32_t>(ids[i]));
            if (is_batch)
                out.vector_id.push_back(static_cast<uint32_t>(i / static_cast<size_t>(k)));
            out.distance.push_back(dist[i]);
        }
        return out;
    }

private:
    PartScan(mqvs_segment_t s, bool owned) { adopt(s, owned); }

    void adopt(mqvs_segment_t s, bool owned)
    {
        seg = std::make_shared<SegmentHandle>(s, owned);
        int32_t d = 0, m = 0;
        check(mqvs_segment_info(s, &n, &d, &m, nullptr, &row_offset, nullptr));
        dim = d;
        metric = m;
    }

    std::shared_ptr<SegmentHandle> seg;
    int64_t n = 0;
    int64_t row_offset = 0;
    int32_t dim = 0;
    int metric = 0;
};

/// The Search::VectorIndex of one part's vector column (VIWithDataPart.h:295-339)
/// as VIWithColumnInPart drives it, over a resident PartScan (which must
/// outlive it).
class GpuIndex
{
public:
    /// createVectorIndex(name, IndexType::MSTG, metric, dim, total_vec, params)
    /// + build (VIWithDataPart.cpp:416-447).  params: "key=value,..." as
    /// include/mqvs.h documents (metric_type, alpha, nlist, kmeans_iters, sample).
    GpuIndex(const PartScan & part_, const std::string & index_type = "MSTG", const std::string & params = "")
        : part(part_)
    {
        mqvs_index_t h = nullptr;
        check(mqvs_index_build(part.handle(), index_type.c_str(), params.c_str(), &h));
        idx = std::make_shared<IndexHandle>(h, true);
    }

    /// A view of an index owned elsewhere (a PartCache entry).
    static GpuIndex borrow(const PartScan & part, mqvs_index_t h) { return GpuIndex(part, h); }

    mqvs_index_t handle() const { return idx->h; }
    const PartScan & segment() const { return part; }
    mqvs_index_t release() const
    {
        idx->owned = false;
        return idx->h;
    }

    /// VectorIndex::search(queries, k, params, first_stage_only, filter)
    /// (VIWithDataPart.cpp:926): nq*k ids / distances, reference order, -1
    /// padded; filter = the PREWHERE bitmap ANDed with the lightweight-delete
    /// bitmap by the library (row_exists).  With a row_ids_map registered, the
    /// ids are decoupled-part rows.  params: alpha / nprobe / num_reorder.
    /// The CPU index search GpuIndex replaces (the part's Search::VectorIndex
    /// search, VIWithDataPart.cpp:926), same arguments and outputs.
    using SearchFallback = std::function<void(const float * queries, int32_t nq, int32_t k, const std::string & params,
                                              const uint8_t * filter, const uint8_t * row_exists,
                                              bool first_stage_only, int64_t * ids, float * dist)>;

    /// fallback: runs instead when the device fails (isFallbackStatus).
    void search(const float * queries, int32_t nq, int32_t query_dim, int32_t k, const std::string & params,
                const uint8_t * filter, const uint8_t * row_exists, bool first_stage_only, int64_t * ids,
                float * dist, const SearchFallback & fallback = nullptr) const
    {
        part.checkDimension(query_dim);
        const int st = mqvs_index_search(idx->h, queries, nq, k, params.c_str(), filter, row_exists, ids, dist,
                                         first_stage_only ? MQVS_F_FIRST_STAGE : 0u, nullptr);
        checkOrFallback(st, static_cast<bool>(fallback), [&] {
            fallback(queries, nq, k, params, filter, row_exists, first_stage_only, ids, dist);
        });
    }

    /// computeTopDistanceSubset (VIWithDataPart.cpp:838-856): exact distances of
    /// the first stage's candidates (part rows, -1 = none), top_k per query.
    void computeTopDistanceSubset(const float * queries, int32_t nq, const int64_t * first_stage_ids,
                                  int32_t ncand, int32_t top_k, const uint8_t * row_exists, int64_t * ids,
                                  float * dist) const
    {
        std::vector<int64_t> local(static_cast<size_t>(nq) * ncand);
        const int64_t off = part.rowOffset();
        for (size_t i = 0; i < local.size(); ++i)
            local[i] = first_stage_ids[i] >= 0 ? first_stage_ids[i] - off : -1;
        part.rerank(queries, nq, local.data(), ncand, top_k, row_exists, ids, dist);
    }

    /// VIWithMeta::row_ids_map of a decoupled part (source row -> new row);
    /// an empty map clears it.
    void setRowIdsMap(const std::vector<uint64_t> & row_ids_map) const
    {
        check(mqvs_index_set_row_ids_map(idx->h, row_ids_map.empty() ? nullptr : row_ids_map.data(),
                                         static_cast<int64_t>(row_ids_map.size()), 0));
    }

private:
    GpuIndex(const PartScan & part_, mqvs_index_t h) : part(part_), idx(std::make_shared<IndexHandle>(h, false)) {}

    PartScan part;
    std::shared_ptr<IndexHandle> idx;
};

/// getRealBitmap (VIUtils.cpp:479-497): a filter over the decoupled part's
/// new_rows rows -> the filter over source part own_id's old_rows rows.
inline std::vector<uint8_t> getRealBitmap(const std::vector<uint8_t> & new_filter, int64_t new_rows,
                                          const std::vector<uint64_t> & inverted_row_ids_map,
                                          const std::vector<uint8_t> & inverted_row_sources_map, uint32_t own_id,
                                          int64_t old_rows)
{
    std::vector<uint8_t> out(static_cast<size_t>((old_rows + 7) / 8));
    check(mqvs_decoupled_filter(new_filter.data(), new_rows,
                                inverted_row_ids_map.empty() ? nullptr : inverted_row_ids_map.data(),
                                inverted_row_sources_map.empty() ? nullptr : inverted_row_sources_map.data(),
                                static_cast<int64_t>(inverted_row_ids_map.size()), own_id, out.data(), old_rows, 0,
                                nullptr));
    return out;
}

/// One part as granule-aligned row-range shards over the GPUs of a node, one
/// rank (thread or process) per GPU, searched through RCCL inside libmqvs.
class ShardComm
{
public:
    /// Rank 0 creates the id and hands it to every rank (any side channel).
    static std::vector<uint8_t> uniqueId()
    {
        std::vector<uint8_t> id(MQVS_COMM_ID_BYTES);
        check(mqvs_comm_unique_id(id.data()));
        return id;
    }

    /// Collective: every rank constructs its communicator together.
    ShardComm(int32_t nranks, int32_t rank, const std::vector<uint8_t> & id, int device)
    {
        if (id.size() != MQVS_COMM_ID_BYTES)
            throw DB::Exception(DB::ErrorCodes::BAD_ARGUMENTS, "{}", std::string("bad communicator id size"));
        check(mqvs_init(device));
        check(mqvs_comm_init(nranks, rank, id.data(), &comm));
    }
    ShardComm(const ShardComm &) = delete;
    ShardComm & operator=(const ShardComm &) = delete;
    ~ShardComm() { (void)mqvs_comm_free(comm); }

    /// Collective: every rank passes its shard; each rank receives the global
    /// top-k (nq*k), == one search over the whole part.
    void search(const PartScan & shard, const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                const uint8_t * row_exists, int64_t * ids, float * dist) const
    {
        check(mqvs_sharded_search(comm, shard.handle(), queries, nq, k, shard.metricId(), filter, row_exists, ids,
                                  dist, 0, nullptr));
    }

    /// Searches that synchronised the host once (a repeat of the last call
    /// every rank completed), and how many of them re-ran on the validated path.
    std::pair<int64_t, int64_t> stats() const
    {
        int64_t fast = 0, redo = 0;
        check(mqvs_comm_stats(comm, &fast, &redo));
        return {fast, redo};
    }

private:
    mqvs_comm_t comm = nullptr;
};

/// Cap on the device memory of all threads' search workspaces (the
/// ScanThreadLimiter's 2 x cores concurrent scans, MergeTreeVSManager.cpp:972-975):
/// searches wait for memory instead of failing.  Returns the previous cap.
inline size_t setWorkspaceBudget(size_t bytes)
{
    return mqvs_set_workspace_budget(bytes);
}

/// VICacheManager (VICacheManager.h:82-114) on the device: parts (+ index)
/// resident in HBM, LRU under max_bytes, pinned while a Holder lives.
class PartCache
{
public:
    struct Entry
    {
        PartScan part;
        std::shared_ptr<GpuIndex> index;  /// null when the entry has no index
    };
    using Holder = std::shared_ptr<const Entry>;

    explicit PartCache(size_t max_bytes) { check(mqvs_cache_create(max_bytes, &cache)); }
    PartCache(const PartCache &) = delete;
    PartCache & operator=(const PartCache &) = delete;
    ~PartCache() { (void)mqvs_cache_free(cache); }

    /// Hand a part (and its index) to the cache.
    void put(const std::string & key, const PartScan & part, const GpuIndex * index = nullptr)
    {
        check(mqvs_cache_put(cache, key.c_str(), part.handle(), index ? index->handle() : nullptr));
        part.release();
        if (index)
            index->release();
    }

    /// The entry, pinned while the holder lives; nullptr on a miss.
    Holder get(const std::string & key)
    {
        mqvs_segment_t s = nullptr;
        mqvs_index_t i = nullptr;
        check(mqvs_cache_acquire(cache, key.c_str(), &s, &i));
        if (!s)
            return nullptr;
        mqvs_cache_t c = cache;
        auto * e = new Entry{PartScan::borrow(s), nullptr};
        if (i)
            e->index = std::make_shared<GpuIndex>(GpuIndex::borrow(e->part, i));
        return Holder(e, [c, key, s](const Entry * p) {
            (void)mqvs_cache_release(c, key.c_str(), s);
            delete p;
        });
    }

    /// LRUResourceCache::getOrSet: load_func builds the part (and index) on a
    /// miss; they are put and returned pinned.
    Holder load(const std::string & key, const std::function<std::pair<PartScan, std::shared_ptr<GpuIndex>>()> & load_func)
    {
        if (auto h = get(key))
            return h;
        auto loaded = load_func();
        put(key, loaded.first, loaded.second.get());
        return get(key);
    }

    /// forceExpire: freed now, or when its last holder goes.
    void forceExpire(const std::string & key) { check(mqvs_cache_remove(cache, key.c_str())); }

    mqvs_cache_stats_t stats() const
    {
        mqvs_cache_stats_t st{};
        check(mqvs_cache_stats(cache, &st));
        return st;
    }

private:
    mqvs_cache_t cache = nullptr;
};

/// Merge per-shard results [nshards][nq][k] of row-range shards of ONE part
/// (shard s holds lower row ids than s+1) into nq*k == the unsharded search.
inline void mergeShardResults(int32_t nshards, int32_t nq, int32_t k, int mqvs_metric, const int64_t * in_ids,
                              const float * in_dist, int64_t * out_ids, float * out_dist)
{
    check(mqvs_merge_shards(nshards, nq, k, mqvs_metric, in_ids, in_dist, out_ids, out_dist, 0, nullptr));
}

/// Cross-part top-k (getTotalTopSearchResultImpl, MergeTreeBaseSearchManager.cpp:207-297):
/// per-part lists [nparts][nq][k] merged with the insertion-ordered multimap
/// (read backwards for IP).
inline void mergePartResults(int32_t nparts, int32_t nq, int32_t k, int mqvs_metric, const int64_t * in_ids,
                             const float * in_dist, int64_t * out_ids, float * out_dist)
{
    check(mqvs_merge_shards(nparts, nq, k, mqvs_metric, in_ids, in_dist, out_ids, out_dist, MQVS_F_PART_MERGE,
                            nullptr));
}

}
