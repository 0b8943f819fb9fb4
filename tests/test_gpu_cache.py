"""Index-path object on the GPU: the device LRU of parts
(VICacheManager.h:82-114), decoupled-part row-id maps (transferToNewRowIds,
VIWithDataPart.cpp:56-67) and the decoupled filter (getRealBitmap,
VIUtils.cpp:479-497)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def _seg(mq, seed, n=20000, d=32, metric="L2"):
    return mq.VectorScanSegment.from_rows(O.generate(seed, 1, 0, n, d), metric=metric, granule=1024)


def test_lru_evicts_least_recently_used(mq):
    from myscaledb_amd.cache import PartCache
    s0 = _seg(mq, 1)
    one = s0.info()["hbm_bytes"]
    cache = PartCache(2 * one + one // 2)  # room for two parts
    q = O.generate(9, 1, 0, 3, 32)
    want0 = s0.search(q, 10)
    cache.put("db.t/p0/v", s0)
    cache.put("db.t/p1/v", _seg(mq, 2))
    hit = cache.acquire("db.t/p0/v")  # p0 becomes most recently used
    seg0, idx = hit
    assert idx is None
    got = seg0.search(q, 10)
    assert np.array_equal(got[0], want0[0]) and np.array_equal(got[1].view(np.uint32), want0[1].view(np.uint32))
    cache.release("db.t/p0/v", seg0)
    cache.put("db.t/p2/v", _seg(mq, 3))  # evicts p1, the least recently used
    assert cache.acquire("db.t/p1/v") is None
    st = cache.stats()
    assert st["items"] == 2 and st["evictions"] == 1 and st["hits"] == 1 and st["misses"] == 1
    for key in ("db.t/p0/v", "db.t/p2/v"):
        s, _ = cache.acquire(key)
        cache.release(key, s)
    cache.free()


def test_held_entries_are_never_evicted(mq):
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.cache import PartCache
    s0 = _seg(mq, 4)
    one = s0.info()["hbm_bytes"]
    cache = PartCache(one + one // 2)
    cache.put("a", s0)
    sa, _ = cache.acquire("a")
    s1 = _seg(mq, 5)
    with pytest.raises(MqvsError) as e:
        cache.put("b", s1)  # "a" is held: no room
    assert e.value.code == 241
    s1.free()  # ownership stayed with the caller
    cache.remove("a")  # forceExpire while held: freed at the release
    assert cache.stats()["expired_held"] == 1
    q = O.generate(6, 1, 0, 2, 32)
    sa.search(q, 5)  # still valid while held
    cache.release("a", sa)
    st = cache.stats()
    assert st["expired_held"] == 0 and st["items"] == 0 and st["bytes"] == 0
    cache.free()


def test_cache_holds_index_with_its_part(mq):
    from myscaledb_amd.cache import PartCache
    seg = mq.VectorScanSegment.from_rows(O.generate(7, 2, 0, 30000, 64), metric="Cosine", granule=2048)
    idx = mq.VectorIndex.build(seg, "MSTG", "nlist=64")
    q = O.generate(8, 2, 0, 5, 64)
    want = idx.search(q, 10, "nprobe=64")
    cache = PartCache(1 << 34)
    cache.put("p/idx", seg, idx)
    s2, i2 = cache.acquire("p/idx")
    got = i2.search(q, 10, "nprobe=64")
    assert np.array_equal(got[0], want[0])
    cache.release("p/idx", s2)
    cache.free()


def test_decoupled_part_row_ids_and_filter(mq):
    """A decoupled part made of two source parts (own ids 0 and 1), rows
    interleaved: source 0's index returns decoupled-part ids, and a filter over
    the decoupled part maps to the right source rows."""
    from myscaledb_amd.vector_index import decoupled_filter
    n0, n1, d = 6000, 5000, 32
    rng = np.random.default_rng(12)
    order = rng.permutation(n0 + n1)  # decoupled row -> (source, row)
    src = (order >= n0).astype(np.uint8)
    inv = np.where(order >= n0, order - n0, order).astype(np.uint64)
    row_ids_map0 = np.empty(n0, np.uint64)
    row_ids_map0[inv[src == 0]] = np.nonzero(src == 0)[0].astype(np.uint64)
    rows0 = O.generate(21, 1, 0, n0, d)
    seg = mq.VectorScanSegment.from_rows(rows0, metric="L2", granule=1024)
    idx = mq.VectorIndex.build(seg, "MSTG", "nlist=16")
    q = O.generate(22, 1, 0, 4, d)
    plain = idx.search(q, 20, "nprobe=16")
    idx.set_row_ids_map(row_ids_map0)
    mapped = idx.search(q, 20, "nprobe=16")
    want = np.where(plain[0] >= 0, row_ids_map0[np.maximum(plain[0], 0)].astype(np.int64), -1)
    assert np.array_equal(mapped[0], want)
    assert np.array_equal(mapped[1].view(np.uint32), plain[1].view(np.uint32))
    idx.set_row_ids_map(None)
    assert np.array_equal(idx.search(q, 20, "nprobe=16")[0], plain[0])
    # getRealBitmap: decoupled-part filter -> source-part filter
    keep_new = rng.random(n0 + n1) < 0.3
    newf = mq.pack_bitmap(keep_new)
    for own in (0, 1):
        n_old = n0 if own == 0 else n1
        want_old = np.zeros(n_old, bool)
        sel = keep_new & (src == own)
        want_old[inv[sel].astype(np.int64)] = True
        got = decoupled_filter(newf, n0 + n1, inv, src, own, n_old)
        assert np.array_equal(got, mq.pack_bitmap(want_old)), own
    # no inverted map: the filter passes unchanged
    assert np.array_equal(decoupled_filter(newf, n0 + n1, None, None, 0, n0 + n1), newf)
    idx.free()
    seg.free()


def test_cache_rejects_double_ownership(mq):
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.cache import PartCache
    cache = PartCache(1 << 34)
    s0 = _seg(mq, 31)
    h = s0._h
    cache.put("a", s0)
    s0._h = h  # a stale Python handle to the cached segment
    with pytest.raises(MqvsError) as e:
        cache.put("b", s0)  # the same segment under a second key
    assert e.value.name == "BAD_ARGUMENTS"
    cache.put("a", s0)  # the same pair again: a refresh, not a double free
    s0._h = None
    other = _seg(mq, 32)
    idx = mq.VectorIndex.build(other, "MSTG", "nlist=8")
    s1 = _seg(mq, 33)
    with pytest.raises(MqvsError) as e:
        cache.put("c", s1, idx)  # index over another segment
    assert e.value.name == "BAD_ARGUMENTS"
    idx.free()
    other.free()
    s1.free()
    assert cache.stats()["items"] == 1
    cache.free()
