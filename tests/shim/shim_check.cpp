// shim_check.cpp -- exercises include/mqvs_vector_index.hpp (the reference-side
// C++ binding) against libmqvs.so; driven by tests/test_shim.py.
//
//   shim_check errors          no GPU needed: status -> DB::Exception codes
//   shim_check gpu <outdir>    tryBruteForceSearch + PartScan::scan / rerank on
//                              deterministic integer data; raw outputs written
//                              to <outdir> for comparison with the oracle
//   shim_check fallback        no GPU needed: an injected device failure
//                              (mqvs_inject_fault) runs the caller's fallback
#include <algorithm>
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

// The CPU path a maintainer passes as the fallback (in the ClickHouse tree:
// faiss::knn_L2sqr / knn_inner_product, BruteForceSearch.h:80-87).  Here a
// plain scan: on integer data every order of the sums gives the same floats,
// so its distances equal the GPU's bit for bit (ties may order differently).
static void cpu_knn(const float *x, const float *y, size_t d, size_t k, size_t nx, size_t ny, int64_t *ids,
                    float *dist, int metric) {
    std::vector<std::pair<float, int64_t>> all(ny);
    for (size_t i = 0; i < nx; ++i) {
        for (size_t r = 0; r < ny; ++r) {
            float acc = 0.f;
            for (size_t j = 0; j < d; ++j) {
                const float a = x[i * d + j], b = y[r * d + j];
                acc += metric == MQVS_METRIC_L2 ? (a - b) * (a - b) : a * b;
            }
            all[r] = {metric == MQVS_METRIC_L2 ? acc : -acc, (int64_t)r};
        }
        std::sort(all.begin(), all.end());
        for (size_t j = 0; j < k; ++j) {
            ids[i * k + j] = j < ny ? all[j].second : -1;
            dist[i * k + j] = j < ny ? (metric == MQVS_METRIC_L2 ? all[j].first : -all[j].first) : 0.f;
        }
    }
}

static int fallback() {
    float x[2 * 4] = {1, 2, 3, 4, 0, 0, 1, 1}, y[3 * 4] = {1, 2, 3, 5, 0, 0, 0, 0, 4, 4, 4, 4};
    int64_t id[2 * 2];
    float dist[2 * 2];
    int served = 0;
    MI::BruteForceFallback fb = [&](const float *a, const float *b, size_t d, size_t k, size_t nx, size_t ny,
                                    int64_t *i, float *o, int m) {
        ++served;
        cpu_knn(a, b, d, k, nx, ny, i, o, m);
    };
    // a device failure (and an HBM shortage) runs the fallback ...
    for (int status : {MQVS_ERR_DEVICE, MQVS_ERR_MEMORY_LIMIT}) {
        if (mqvs_inject_fault(status, 1) != MQVS_OK) return 1;
        MI::tryBruteForceSearch(x, y, 4, 2, 2, 3, id, dist, Metric::L2, fb);
    }
    const bool ok = served == 2 && id[0] == 0 && dist[0] == 1.f && id[1] == 2 && dist[1] == 14.f && id[2] == 1 &&
                    dist[2] == 2.f && MI::fallbackCount().load() == 2;
    std::printf("fallback served %d ids %lld %lld dist %g %g\n", served, (long long)id[0], (long long)id[1],
                (double)dist[0], (double)dist[1]);
    if (!ok) return 1;
    // ... without one the failure is rethrown with its code
    if (mqvs_inject_fault(MQVS_ERR_DEVICE, 1) != MQVS_OK) return 1;
    try {
        MI::tryBruteForceSearch(x, y, 4, 2, 2, 3, id, dist, Metric::IP);
        return 1;
    } catch (const DB::Exception &e) {
        if (e.code() != DB::ErrorCodes::LOGICAL_ERROR) return 1;
    }
    if (mqvs_inject_fault(MQVS_ERR_MEMORY_LIMIT, 1) != MQVS_OK) return 1;
    try {
        MI::tryBruteForceSearch(x, y, 4, 2, 2, 3, id, dist, Metric::IP);
        return 1;
    } catch (const DB::Exception &e) {
        if (e.code() != DB::ErrorCodes::MEMORY_LIMIT_EXCEEDED) return 1;
    }
    // other statuses never fall back: an unsupported metric stays NOT_IMPLEMENTED
    try {
        MI::tryBruteForceSearch(x, y, 4, 2, 2, 3, id, dist, Metric::Cosine, fb);
        return 1;
    } catch (const DB::Exception &e) {
        if (e.code() != DB::ErrorCodes::NOT_IMPLEMENTED || served != 2) return 1;
    }
    // the drill accepts only the two fallback statuses
    if (mqvs_inject_fault(MQVS_ERR_LOGICAL, 1) != MQVS_ERR_BAD_ARGUMENTS) return 1;
    if (mqvs_inject_fault(MQVS_ERR_DEVICE, 0) != MQVS_OK) return 1;
    std::printf("fallback ok\n");
    return 0;
}

// k = 8000 (above the old 4096 cap; the reference's max_search_result_window
// is 10000), the 1-rank RCCL sharded search, the index seam, getRealBitmap and
// the part cache.
static int gpu_more(const std::string &dir, const std::vector<float> &rows, const std::vector<float> &q, int n,
                    int d, int nq, int gran, const MI::PartScan &cos_part) {
    // large k over a 12000-row L2 part
    const int nl = 12000, kl = 8000;
    std::vector<float> lrows((size_t)nl * d);
    for (int i = 0; i < nl; ++i)
        for (int j = 0; j < d; ++j) lrows[(size_t)i * d + j] = val(i + 3, j);
    MI::PartScan lpart(lrows.data(), nl, d, MI::toMqvsMetric(Metric::L2), gran);
    std::vector<int64_t> lid((size_t)nq * kl);
    std::vector<float> ldist(lid.size());
    lpart.search(q.data(), nq, kl, nullptr, nullptr, lid.data(), ldist.data());
    write(dir + "/bigk_ids.bin", lid.data(), lid.size() * 8);
    write(dir + "/bigk_dist.bin", ldist.data(), ldist.size() * 4);
    std::printf("prefilter active %d\n", lpart.prefilterActive() ? 1 : 0);

    // 1-rank communicator: the sharded search == the plain search
    const int k = 12;
    {
        MI::ShardComm comm(1, 0, MI::ShardComm::uniqueId(), 0);
        std::vector<int64_t> a((size_t)nq * k), b(a.size());
        std::vector<float> da(a.size()), db(a.size());
        cos_part.search(q.data(), nq, k, nullptr, nullptr, a.data(), da.data());
        comm.search(cos_part, q.data(), nq, k, nullptr, nullptr, b.data(), db.data());
        const bool same = std::memcmp(a.data(), b.data(), a.size() * 8) == 0 &&
                          std::memcmp(da.data(), db.data(), da.size() * 4) == 0;
        std::printf("sharded==search %d\n", same ? 1 : 0);
        if (!same) return 1;
    }

    // device-failure fallbacks at the part and index seams: the injected
    // failure runs the caller's CPU path (here: the GPU answer computed
    // before, standing in for the CPU scan); the next call runs on the GPU
    {
        std::vector<int64_t> a((size_t)nq * k), b(a.size());
        std::vector<float> da(a.size()), db(a.size());
        cos_part.search(q.data(), nq, k, nullptr, nullptr, a.data(), da.data());
        int served = 0;
        MI::PartScan::ScanFallback sfb = [&](const float *, int32_t, int32_t, const uint8_t *, const uint8_t *,
                                             int64_t *i, float *o) {
            ++served;
            std::memcpy(i, a.data(), a.size() * 8);
            std::memcpy(o, da.data(), da.size() * 4);
        };
        mqvs_inject_fault(MQVS_ERR_DEVICE, 1);
        cos_part.search(q.data(), nq, k, nullptr, nullptr, b.data(), db.data(), 0, sfb);
        bool ok = served == 1 && std::memcmp(a.data(), b.data(), a.size() * 8) == 0;
        std::fill(b.begin(), b.end(), -7);
        cos_part.search(q.data(), nq, k, nullptr, nullptr, b.data(), db.data(), 0, sfb);  // GPU again
        ok = ok && served == 1 && std::memcmp(a.data(), b.data(), a.size() * 8) == 0;
        MI::GpuIndex index(lpart, "MSTG", "nlist=16");
        std::vector<int64_t> ia(a.size()), ib(a.size());
        std::vector<float> ida(a.size()), idb(a.size());
        index.search(q.data(), nq, d, k, "nprobe=16", nullptr, nullptr, false, ia.data(), ida.data());
        MI::GpuIndex::SearchFallback ifb = [&](const float *, int32_t, int32_t, const std::string &, const uint8_t *,
                                               const uint8_t *, bool, int64_t *i, float *o) {
            ++served;
            std::memcpy(i, ia.data(), ia.size() * 8);
            std::memcpy(o, ida.data(), ida.size() * 4);
        };
        mqvs_inject_fault(MQVS_ERR_MEMORY_LIMIT, 1);
        index.search(q.data(), nq, d, k, "nprobe=16", nullptr, nullptr, false, ib.data(), idb.data(), ifb);
        ok = ok && served == 2 && std::memcmp(ia.data(), ib.data(), ia.size() * 8) == 0;
        std::printf("gpu fallback %d\n", ok ? 1 : 0);
        if (!ok) return 1;
    }

    // index seam: build, search, computeTopDistanceSubset, row_ids_map remap
    {
        MI::GpuIndex index(lpart, "MSTG", "nlist=16");
        std::vector<int64_t> a((size_t)nq * k), b(a.size()), c(a.size());
        std::vector<float> da(a.size()), db(a.size()), dc(a.size());
        index.search(q.data(), nq, d, k, "nprobe=16", nullptr, nullptr, false, a.data(), da.data());
        write(dir + "/index_ids.bin", a.data(), a.size() * 8);
        // two-stage: first stage 64 candidates, exact re-rank
        const int nc = 64;
        std::vector<int64_t> fs((size_t)nq * nc);
        std::vector<float> fd(fs.size());
        index.search(q.data(), nq, d, nc, "nprobe=16", nullptr, nullptr, true, fs.data(), fd.data());
        index.computeTopDistanceSubset(q.data(), nq, fs.data(), nc, k, nullptr, c.data(), dc.data());
        write(dir + "/index_fs_ids.bin", fs.data(), fs.size() * 8);
        write(dir + "/index_rerank_ids.bin", c.data(), c.size() * 8);
        write(dir + "/index_rerank_dist.bin", dc.data(), dc.size() * 4);
        std::vector<uint64_t> map((size_t)nl);
        for (int i = 0; i < nl; ++i) map[(size_t)i] = (uint64_t)(nl - 1 - i) * 2 + 5;
        index.setRowIdsMap(map);
        index.search(q.data(), nq, d, k, "nprobe=16", nullptr, nullptr, false, b.data(), db.data());
        bool ok = std::memcmp(da.data(), db.data(), da.size() * 4) == 0;
        for (size_t i = 0; i < a.size(); ++i) ok = ok && b[i] == (a[i] < 0 ? -1 : (int64_t)map[(size_t)a[i]]);
        std::printf("row_ids_map %d\n", ok ? 1 : 0);
        if (!ok) return 1;
        try {
            index.search(q.data(), nq, d + 1, k, "", nullptr, nullptr, false, b.data(), db.data());
            return 1;
        } catch (const DB::Exception &e) {
            if (e.code() != DB::ErrorCodes::LOGICAL_ERROR) return 1;
        }
    }

    // getRealBitmap: decoupled rows 0..9 from sources (0,1,0,1,...), row i -> i/2
    {
        std::vector<uint8_t> nf = {0xFF, 0x03};  // rows 0..9 set
        std::vector<uint64_t> inv(10);
        std::vector<uint8_t> src(10);
        for (int i = 0; i < 10; ++i) {
            inv[(size_t)i] = (uint64_t)(i / 2);
            src[(size_t)i] = (uint8_t)(i % 2);
        }
        nf[0] = 0xAD;  // rows 0,2,3,5,7 set (+8,9 from nf[1])
        auto old0 = MI::getRealBitmap(nf, 10, inv, src, 0, 5);  // even rows 0,2,8 -> 0,1,4
        auto old1 = MI::getRealBitmap(nf, 10, inv, src, 1, 5);  // odd rows 3,5,7,9 -> 1,2,3,4
        const bool ok = old0.size() == 1 && old0[0] == 0x13 && old1.size() == 1 && old1[0] == 0x1E;
        std::printf("getRealBitmap %d (%02x %02x)\n", ok ? 1 : 0, old0.empty() ? 0 : old0[0],
                    old1.empty() ? 0 : old1[0]);
        if (!ok) return 1;
    }

    // part cache: load = getOrSet, holders pin, LRU eviction under the budget
    {
        auto make = [&](int seed) {
            std::vector<float> r((size_t)n * d);
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < d; ++j) r[(size_t)i * d + j] = val(i + seed, j);
            return MI::PartScan(r.data(), n, d, MI::toMqvsMetric(Metric::L2), gran);
        };
        const size_t one = make(1).hbmBytes();
        MI::PartCache cache(2 * one + one / 2);
        int loads = 0;
        auto loader = [&](int seed) {
            return [&, seed] {
                ++loads;
                return std::make_pair(make(seed), std::shared_ptr<MI::GpuIndex>());
            };
        };
        {
            auto h0 = cache.load("db.t/all_1_1_0/v", loader(1));
            auto h0b = cache.load("db.t/all_1_1_0/v", loader(1));  // hit: no second load
            std::vector<int64_t> a((size_t)nq * k);
            std::vector<float> da(a.size());
            h0->part.search(q.data(), nq, k, nullptr, nullptr, a.data(), da.data());
        }
        cache.load("db.t/all_2_2_0/v", loader(2));
        cache.get("db.t/all_1_1_0/v");               // part 1 most recently used
        cache.load("db.t/all_3_3_0/v", loader(3));  // evicts part 2
        const bool evicted = cache.get("db.t/all_2_2_0/v") == nullptr;
        auto st = cache.stats();
        auto held = cache.get("db.t/all_3_3_0/v");
        cache.forceExpire("db.t/all_3_3_0/v");
        auto st2 = cache.stats();
        held.reset();
        auto st3 = cache.stats();
        const bool ok = loads == 3 && evicted && st.items == 2 && st.evictions == 1 && st2.expired_held == 1 &&
                        st3.expired_held == 0 && st3.items == 1;
        std::printf("cache %d (loads %d items %lld evictions %lld)\n", ok ? 1 : 0, loads, (long long)st.items,
                    (long long)st.evictions);
        if (!ok) return 1;
    }
    (void)rows;
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
    if (!same) return 1;
    return gpu_more(dir, rows, q, n, d, nq, gran, part);
}

int main(int argc, char **argv) {
    if (argc >= 2 && std::string(argv[1]) == "errors") return errors();
    if (argc >= 2 && std::string(argv[1]) == "fallback") {
        try {
            return fallback();
        } catch (const std::exception &e) {
            std::printf("exception: %s\n", e.what());
            return 1;
        }
    }
    if (argc >= 3 && std::string(argv[1]) == "gpu") {
        try {
            return gpu(argv[2]);
        } catch (const std::exception &e) {
            std::printf("exception: %s\n", e.what());
            return 1;
        }
    }
    std::fprintf(stderr, "usage: shim_check errors | fallback | gpu <outdir>\n");
    return 2;
}
