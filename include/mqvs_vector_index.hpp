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

#include <cstddef>
#include <cstdint>
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

/// tryBruteForceSearch<FloatVector> (BruteForceSearch.h:62-92): x nx*d
/// queries, y ny*d base, result_id / distance nx*k in faiss layout.
inline void tryBruteForceSearch(
    const float * x, const float * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, int mqvs_metric)
{
    if (mqvs_metric != MQVS_METRIC_L2 && mqvs_metric != MQVS_METRIC_IP)
        throw DB::Exception(DB::ErrorCodes::NOT_IMPLEMENTED, "{}",
                            std::string("Metric not implemented in brute force search for Float32 Vector"));
    check(mqvs_knn_raw(x, y, static_cast<int64_t>(d), static_cast<int64_t>(k), static_cast<int64_t>(nx),
                       static_cast<int64_t>(ny), mqvs_metric, result_id, distance));
}

template <typename MetricEnum>
void tryBruteForceSearch(
    const float * x, const float * y, size_t d, size_t k, size_t nx, size_t ny,
    int64_t * result_id, float * distance, const MetricEnum & metric_type)
{
    tryBruteForceSearch(x, y, d, k, nx, ny, result_id, distance, toMqvsMetric(metric_type));
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

/// One data part (or a granule-aligned row-range shard of it) resident on a GPU.
class PartScan
{
public:
    /// rows: n*d fp32, row-major; rows whose Array is empty FLT_MAX-filled and
    /// flagged 0 in `nonempty` (n bytes, or nullptr when none is empty).
    PartScan(const float * rows, int64_t n, int32_t d, int mqvs_metric, int64_t granule_rows,
             const uint8_t * nonempty = nullptr, int64_t row_offset = 0, int device = 0)
        : dim(d), metric(mqvs_metric)
    {
        check(mqvs_init(device));
        mqvs_segment_t s = nullptr;
        check(mqvs_segment_create(rows, n, d, mqvs_metric, granule_rows, nonempty, row_offset, &s));
        seg = std::shared_ptr<mqvs_segment>(s, [](mqvs_segment_t p) { mqvs_segment_free(p); });
    }

    int32_t dimension() const { return dim; }

    /// Raw top-k: ids / dist nq*k (caller-owned), -1 / FLT_MAX (FLT_MIN for IP)
    /// padded.  filter: PREWHERE bitmap, row_exists: lightweight-delete mask
    /// (LSB-first, n bits, or nullptr).
    void search(const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                const uint8_t * row_exists, int64_t * ids, float * dist) const
    {
        check(mqvs_search(seg.get(), queries, nq, k, metric, filter, row_exists, ids, dist, 0, nullptr));
    }

    /// Raw top-k of a row-range shard of a larger part: chunk_ord_base = chunks
    /// before the shard that the reference searches (cosine query variant).
    void searchShard(const float * queries, int32_t nq, int32_t k, const uint8_t * filter,
                     const uint8_t * row_exists, int64_t chunk_ord_base, int64_t * ids, float * dist) const
    {
        check(mqvs_search_ex(seg.get(), queries, nq, k, metric, filter, row_exists, chunk_ord_base, ids, dist, 0,
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

    /// As above, after the reference's dimension check (generateVectorDataset,
    /// MergeTreeVSManager.cpp:135-182 throws on a mismatch).
    ScanColumns scan(const float * queries, int32_t nq, int32_t query_dim, int32_t k, bool is_batch,
                     const uint8_t * filter, const uint8_t * row_exists) const
    {
        if (query_dim != dim)
            throw DB::Exception(DB::ErrorCodes::LOGICAL_ERROR, "{}",
                                "The dimension of searched vector (" + std::to_string(query_dim)
                                    + ") doesn't match the dimension of the vector column (" + std::to_string(dim) + ")");
        return scan(queries, nq, k, is_batch, filter, row_exists);
    }

    /// computeTopDistanceSubset: exact distances to nq*ncand candidate rows.
    void rerank(const float * queries, int32_t nq, const int64_t * cand, int32_t ncand, int32_t k,
                const uint8_t * row_exists, int64_t * ids, float * dist) const
    {
        check(mqvs_rerank(seg.get(), queries, nq, cand, ncand, k, metric, row_exists, ids, dist, 0, nullptr));
    }

private:
    std::shared_ptr<mqvs_segment> seg;
    int32_t dim;
    int metric;
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
