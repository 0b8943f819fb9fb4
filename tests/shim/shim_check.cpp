// shim_check.cpp -- exercises include/mqvs_vector_index.hpp (the reference-side
// C++ binding) against libmqvs.so; driven by tests/test_shim.py.
//
//   shim_check errors          no GPU needed: status -> DB::Exception codes
//   shim_check gpu <outdir>    tryBruteForceSearch + PartScan::scan / rerank on
//                              deterministic integer data; raw outputs written
//                              to <outdir> for comparison with the oracle
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mqvs_vector_index.hpp"

namespace MI = VectorIndex::MI355X;

// The metric enum the reference passes (Search::Metric, absent library):
// only the member names matter to the shim.
enum class Metric { L2, IP, Cosine, Hamming, Jaccard };

static float val(int i, int j) { return float((i * 31 + j * 17) % 23 - 11); }

static void write(const std::string &path, const void *p, size_t bytes) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fwrite(p, 1, bytes, f);
    std::fclose(f);
}

static int errors() {
    // unsupported metric: NOT_IMPLEMENTED before any device work
    float x[4] = {0}, y[8] = {0};
    int64_t id[2];
    float dist[2];
    try {
        MI::tryBruteForceSearch(x, y, 4, 1, 1, 2, id, dist, Metric::Cosine);
        std::printf("no exception\n");
        return 1;
    } catch (const DB::Exception &e) {
        std::printf("cosine code=%d\n", e.code());
        if (e.code() != DB::ErrorCodes::NOT_IMPLEMENTED) return 1;
    }
    try {
        MI::tryBruteForceSearch(x, y, 4, 1, 1, 2, id, dist, Metric::Hamming);
        return 1;
    } catch (const DB::Exception &e) {
        std::printf("hamming code=%d\n", e.code());
        if (e.code() != DB::ErrorCodes::NOT_IMPLEMENTED) return 1;
    }
    // binary seam: float metrics are NOT_IMPLEMENTED (BruteForceSearch.h:107)
    try {
        const uint8_t bx[4] = {0}, by[8] = {0};
        MI::tryBruteForceSearchBinary(bx, by, 32, 1, 1, 2, id, dist, Metric::L2);
        return 1;
    } catch (const DB::Exception &e) {
        std::printf("binary l2 code=%d\n", e.code());
        if (e.code() != DB::ErrorCodes::NOT_IMPLEMENTED) return 1;
    }
    // direct C-ABI status mapping
    const int st[] = {MQVS_ERR_NOT_IMPLEMENTED, MQVS_ERR_LOGICAL, MQVS_ERR_ILLEGAL_COLUMN,
                      MQVS_ERR_BAD_ARGUMENTS, MQVS_ERR_MEMORY_LIMIT, MQVS_ERR_DEVICE, MQVS_ERR_CHECKSUM};
    const int want[] = {48, 49, 44, 36, 241, 49, 40};
    for (int i = 0; i < 7; ++i) {
        try {
            MI::check(st[i]);
            return 1;
        } catch (const DB::Exception &e) {
            if (e.code() != want[i]) {
                std::printf("status %d -> %d, want %d\n", st[i], e.code(), want[i]);
                return 1;
            }
        }
    }
    std::printf("errors ok\n");
    return 0;
}

static int gpu(const std::string &dir) {
    const int n = 3000, d = 24, nq = 5, k = 12, gran = 512;
    std::vector<float> rows((size_t)n * d), q((size_t)nq * d);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < d; ++j) rows[(size_t)i * d + j] = val(i, j);
    for (int i = 0; i < nq; ++i)
        for (int j = 0; j < d; ++j) q[(size_t)i * d + j] = val(i + 7777, j) * 0.5f;
    // tryBruteForceSearch, L2 and IP
    std::vector<int64_t> ids((size_t)nq * k);
    std::vector<float> dist(ids.size());
    MI::tryBruteForceSearch(q.data(), rows.data(), d, k, nq, n, ids.data(), dist.data(), Metric::L2);
    write(dir + "/knn_l2_ids.bin", ids.data(), ids.size() * 8);
    write(dir + "/knn_l2_dist.bin", dist.data(), dist.size() * 4);
    MI::tryBruteForceSearch(q.data(), rows.data(), d, k, nq, n, ids.data(), dist.data(), Metric::IP);
    write(dir + "/knn_ip_ids.bin", ids.data(), ids.size() * 8);
    write(dir + "/knn_ip_dist.bin", dist.data(), dist.size() * 4);
    // PartScan: cosine part, batch scan columns
    MI::PartScan part(rows.data(), n, d, MI::toMqvsMetric(Metric::Cosine), gran);
    MI::ScanColumns cols = part.scan(q.data(), nq, k, /*is_batch=*/true);
    write(dir + "/scan_label.bin", cols.label.data(), cols.label.size() * 4);
    write(dir + "/scan_vid.bin", cols.vector_id.data(), cols.vector_id.size() * 4);
    write(dir + "/scan_dist.bin", cols.distance.data(), cols.distance.size() * 4);
    // rerank every row == search
    std::vector<int64_t> cand((size_t)nq * n);
    for (int i = 0; i < nq; ++i)
        for (int r = 0; r < n; ++r) cand[(size_t)i * n + r] = (r < 4096) ? r : -1;
    std::vector<int64_t> ids2(ids.size());
    std::vector<float> dist2(ids.size());
    part.search(q.data(), nq, k, nullptr, nullptr, ids.data(), dist.data());
    part.rerank(q.data(), nq, cand.data(), n, k, nullptr, ids2.data(), dist2.data());
    const bool same = std::memcmp(ids.data(), ids2.data(), ids.size() * 8) == 0 &&
                      std::memcmp(dist.data(), dist2.data(), dist.size() * 4) == 0;
    std::printf("rerank==search %d\n", same ? 1 : 0);
    // a bad-arguments error through the shim: null segment
    try {
        std::vector<int64_t> i3(ids.size());
        std::vector<float> d3(ids.size());
        MI::check(mqvs_search(nullptr, q.data(), nq, k, MQVS_METRIC_L2, nullptr, nullptr, i3.data(), d3.data(), 0,
                          nullptr));
        return 1;
    } catch (const DB::Exception &e) {
        std::printf("null segment code=%d\n", e.code());
        if (e.code() != DB::ErrorCodes::BAD_ARGUMENTS) return 1;
    }
    return same ? 0 : 1;
}

int main(int argc, char **argv) {
    if (argc >= 2 && std::string(argv[1]) == "errors") return errors();
    if (argc >= 3 && std::string(argv[1]) == "gpu") {
        try {
            return gpu(argv[2]);
        } catch (const std::exception &e) {
            std::printf("exception: %s\n", e.what());
            return 1;
        }
    }
    std::fprintf(stderr, "usage: shim_check errors | gpu <outdir>\n");
    return 2;
}
