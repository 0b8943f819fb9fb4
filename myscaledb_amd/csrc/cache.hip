// cache.hip -- device-resident LRU of parts' segments (and their indexes),
// the GPU counterpart of the reference's VICacheManager
// (src/VectorIndex/Cache/VICacheManager.h:82-114, over DB::LRUResourceCache):
// entries are keyed by the caller's CacheKey string (table / part / column /
// index), weighed by their HBM bytes, pinned while a search holds them
// (acquire ... release, the MappedHolderPtr of LRUResourceCache), and evicted
// least-recently-used first when a put would exceed the byte budget.  Pinned
// entries are never evicted; forceExpire (remove) of a pinned entry frees it
// when its last holder releases it.  Control plane only: no kernel runs here.
#include <hip/hip_runtime.h>

#include <list>
#include <mutex>
#include <string>
#include <unordered_map>

#include "mqvs_internal.h"

namespace {

struct Entry {
    std::string key;
    mqvs_segment_t seg = nullptr;
    mqvs_index_t idx = nullptr;
    size_t bytes = 0;
    int pins = 0;
    bool expired = false;  // removed from the map; freed at the last release
};

void destroy(Entry &e) {
    if (e.idx) (void)mqvs_index_free(e.idx);
    if (e.seg) (void)mqvs_segment_free(e.seg);
    e.idx = nullptr;
    e.seg = nullptr;
}

size_t weight(mqvs_segment_t seg, mqvs_index_t idx) {
    size_t b = 0;
    if (seg) (void)mqvs_segment_info(seg, nullptr, nullptr, nullptr, nullptr, nullptr, &b);
    if (idx) {
        mqvs_index_info_t ii{};
        if (mqvs_index_info(idx, &ii) == MQVS_OK) b += ii.hbm_bytes;
    }
    return b;
}

}  // namespace

struct mqvs_cache {
    size_t max_bytes = 0;
    size_t bytes = 0;
    std::list<Entry> lru;  // front = most recently used
    std::unordered_map<std::string, std::list<Entry>::iterator> map;
    std::list<Entry> expired;  // pinned entries removed from the map
    int64_t hits = 0, misses = 0, evictions = 0;
    std::mutex mu;

    // evict unpinned entries from the LRU end until `need` more bytes fit
    bool make_room(size_t need) {
        auto it = lru.end();
        while (bytes + need > max_bytes && it != lru.begin()) {
            --it;
            if (it->pins > 0) continue;
            bytes -= it->bytes;
            map.erase(it->key);
            destroy(*it);
            it = lru.erase(it);
            ++evictions;
        }
        return bytes + need <= max_bytes;
    }
};

using namespace mqvs;

extern "C" {

int mqvs_cache_create(size_t max_bytes, mqvs_cache_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        auto *c = new mqvs_cache();
        c->max_bytes = max_bytes;
        *out = c;
    });
}

int mqvs_cache_free(mqvs_cache_t c) {
    return guarded([&] {
        if (!c) return;
        {
            std::lock_guard<std::mutex> lock(c->mu);
            for (auto &e : c->lru)
                if (e.pins > 0) fail(MQVS_ERR_LOGICAL, "cache entry '" + e.key + "' is still held");
            for (auto &e : c->expired)
                if (e.pins > 0) fail(MQVS_ERR_LOGICAL, "cache entry '" + e.key + "' is still held");
            for (auto &e : c->lru) destroy(e);
        }
        delete c;
    });
}

int mqvs_cache_put(mqvs_cache_t c, const char *key, mqvs_segment_t seg, mqvs_index_t idx) {
    return guarded([&] {
        if (!c || !key || !seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null cache, key or segment");
        if (idx && index_segment(idx) != seg) fail(MQVS_ERR_BAD_ARGUMENTS, "the index was not built over this segment");
        const size_t w = weight(seg, idx);
        std::lock_guard<std::mutex> lock(c->mu);
        auto found = c->map.find(key);
        if (found != c->map.end() && found->second->seg == seg && found->second->idx == idx) {
            c->lru.splice(c->lru.begin(), c->lru, found->second);  // the same entry again: most recently used
            return;
        }
        // a handle has one owner: never two entries over the same segment / index
        for (const std::list<Entry> *l : {&c->lru, &c->expired})
            for (const Entry &e : *l)
                if (e.seg == seg || (idx && e.idx == idx))
                    fail(MQVS_ERR_BAD_ARGUMENTS, "segment or index already cached (key '" + e.key + "')");
        if (found != c->map.end()) {  // replace: the old entry leaves the map
            auto it = found->second;
            c->bytes -= it->bytes;
            c->map.erase(found);
            if (it->pins > 0) {
                it->expired = true;
                c->expired.splice(c->expired.end(), c->lru, it);
            } else {
                destroy(*it);
                c->lru.erase(it);
            }
        }
        if (!c->make_room(w))
            fail(MQVS_ERR_MEMORY_LIMIT, "cache budget of " + std::to_string(c->max_bytes) + " bytes cannot hold '" +
                                            key + "' (" + std::to_string(w) + " bytes; the rest is held)");
        Entry e;
        e.key = key;
        e.seg = seg;
        e.idx = idx;
        e.bytes = w;
        c->lru.push_front(std::move(e));
        c->map[key] = c->lru.begin();
        c->bytes += w;
    });
}

int mqvs_cache_acquire(mqvs_cache_t c, const char *key, mqvs_segment_t *seg, mqvs_index_t *idx) {
    return guarded([&] {
        if (!c || !key || !seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        *seg = nullptr;
        if (idx) *idx = nullptr;
        std::lock_guard<std::mutex> lock(c->mu);
        auto found = c->map.find(key);
        if (found == c->map.end()) {
            ++c->misses;
            return;
        }
        ++c->hits;
        auto it = found->second;
        it->pins += 1;
        c->lru.splice(c->lru.begin(), c->lru, it);  // most recently used
        *seg = it->seg;
        if (idx) *idx = it->idx;
    });
}

int mqvs_cache_release(mqvs_cache_t c, const char *key, mqvs_segment_t seg) {
    return guarded([&] {
        if (!c || !key || !seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        std::lock_guard<std::mutex> lock(c->mu);
        auto found = c->map.find(key);
        if (found != c->map.end() && found->second->seg == seg) {
            if (found->second->pins <= 0) fail(MQVS_ERR_LOGICAL, "release without acquire of '" + std::string(key) + "'");
            found->second->pins -= 1;
            return;
        }
        for (auto it = c->expired.begin(); it != c->expired.end(); ++it) {
            if (it->key == key && it->seg == seg) {
                if (--it->pins == 0) {
                    destroy(*it);
                    c->expired.erase(it);
                }
                return;
            }
        }
        fail(MQVS_ERR_LOGICAL, "release of an entry the cache does not hold: '" + std::string(key) + "'");
    });
}

int mqvs_cache_remove(mqvs_cache_t c, const char *key) {
    return guarded([&] {
        if (!c || !key) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        std::lock_guard<std::mutex> lock(c->mu);
        auto found = c->map.find(key);
        if (found == c->map.end()) return;
        auto it = found->second;
        c->bytes -= it->bytes;
        c->map.erase(found);
        if (it->pins > 0) {
            it->expired = true;
            c->expired.splice(c->expired.end(), c->lru, it);
        } else {
            destroy(*it);
            c->lru.erase(it);
        }
    });
}

int mqvs_cache_stats(mqvs_cache_t c, mqvs_cache_stats_t *out) {
    return guarded([&] {
        if (!c || !out) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        std::lock_guard<std::mutex> lock(c->mu);
        out->items = (int64_t)c->lru.size();
        out->bytes = c->bytes;
        out->max_bytes = c->max_bytes;
        out->hits = c->hits;
        out->misses = c->misses;
        out->evictions = c->evictions;
        int64_t pinned = 0;
        for (auto &e : c->lru) pinned += e.pins > 0;
        out->pinned = pinned;
        out->expired_held = (int64_t)c->expired.size();
    });
}

}  // extern "C"
