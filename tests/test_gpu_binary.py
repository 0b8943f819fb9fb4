"""Binary vectors (FixedString(N) columns, Hamming / Jaccard) through the HIP
path vs the CPU oracle: bit-identical ids and distances.

Reference: tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110) ->
faiss::hammings_knn_mc / jaccard_knn under vectorScanWithoutIndex<BinaryVector>
(MergeTreeVSManager.cpp:1188-1273, 1395-1425) and searchWrapper.  Pinned by
the reference's KAT 00038 (tests/golden/binary_kats.json); beyond it the
oracle restatement (oracle/mqvs_oracle.c) is the checker.
"""
import numpy as np
import pytest

from kat_harness import check_binary_case, load_binary_cases
from oracle import oracle as O

pytestmark = pytest.mark.gpu

BCASES = load_binary_cases()


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def gpu_binary_scan(m):
    def fn(codes, gran, queries, k, metric, flt, rex):
        seg = m.BinaryVectorScanSegment.from_codes(codes, metric=metric, granule=gran)
        try:
            return seg.search(queries, k, metric, flt, rex)
        finally:
            seg.free()
    return fn


@pytest.mark.parametrize("case", BCASES, ids=[c["name"] for c in BCASES])
def test_gpu_binary_kat(mq, case):
    """KAT 00038 through mqvs_search_binary."""
    check_binary_case(case, gpu_binary_scan(mq))


def assert_same(ids_g, dist_g, ids_o, dist_o, ctx):
    ids_g, ids_o = np.asarray(ids_g), np.asarray(ids_o)
    dg, do = np.asarray(dist_g, np.float32).view(np.uint32), np.asarray(dist_o, np.float32).view(np.uint32)
    if not (np.array_equal(ids_g, ids_o) and np.array_equal(dg, do)):
        bad = np.argwhere((ids_g != ids_o) | (dg != do))
        q, j = bad[0]
        raise AssertionError(f"{ctx}: {len(bad)} mismatches; first q{q} slot {j}: gpu ({ids_g[q, j]}, "
                             f"{dist_g[q, j]!r}) oracle ({ids_o[q, j]}, {dist_o[q, j]!r})")


def codes_of(rng, n, nbytes, density=0.5):
    bits = rng.random((n, nbytes * 8)) < density
    return np.packbits(bits, axis=1, bitorder="little")


# (n, bytes per code, nq, k, metric, granule, filter, deletes, density)
CASES = [
    (20000, 32, 1, 10, "Hamming", 8192, False, False, 0.5),
    (70000, 32, 4, 100, "Hamming", 8192, False, False, 0.5),      # probe + main segments
    (70000, 4, 2, 100, "Hamming", 8192, False, False, 0.5),       # 32-bit codes: heavy ties
    (60000, 64, 33, 50, "Jaccard", 8192, False, False, 0.3),
    (50000, 136, 3, 20, "Jaccard", 1000, False, False, 0.5),      # > 1024 bits, odd length
    (50000, 136, 9, 20, "Hamming", 1000, True, True, 0.5),
    (80000, 16, 2, 64, "Hamming", 8192, True, False, 0.5),
    (80000, 16, 1, 64, "Jaccard", 4096, False, True, 0.1),
    (3000, 8, 3, 200, "Hamming", 512, True, True, 0.5),
    (30000, 128, 5, 30, "Jaccard", 8192, True, False, 0.5),     # 1024-bit codes, coalesced kernel
    (40000, 128, 2, 40, "Hamming", 2048, False, True, 0.5),
    (40000, 64, 12, 40, "Hamming", 8192, False, False, 0.5),    # nq > 8: row-per-lane kernel
]


@pytest.mark.parametrize("n,nb,nq,k,metric,gran,use_f,use_d,dens", CASES)
def test_gpu_binary_vs_oracle(mq, n, nb, nq, k, metric, gran, use_f, use_d, dens):
    rng = np.random.default_rng(n + nb + nq + k)
    codes = codes_of(rng, n, nb, dens)
    queries = codes_of(rng, nq, nb, dens)
    queries[0] = codes[n // 3]  # an exact match
    flt = np.packbits(rng.random(n) < 0.4, bitorder="little") if use_f else None
    rex = np.packbits(rng.random(n) > 0.1, bitorder="little") if use_d else None
    seg = mq.BinaryVectorScanSegment.from_codes(codes, metric=metric, granule=gran)
    try:
        ids, dist = seg.search(queries, k, metric, flt, rex)
    finally:
        seg.free()
    ids_o, dist_o = O.vector_scan_binary(codes, queries, k, O.METRICS[metric], gran, filter_bits=flt,
                                         row_exists_bits=rex)
    assert_same(ids, dist, ids_o, dist_o, f"{metric} n={n} N={nb} nq={nq} k={k}")


def test_gpu_binary_all_ties(mq):
    """Every row at the same distance: the (distance, row) rule keeps the
    first k rows, also when more than 4096 rows reach the k-th distance."""
    n = 100000
    codes = np.zeros((n, 32), np.uint8)
    q = np.full((1, 32), 0x0F, np.uint8)
    seg = mq.BinaryVectorScanSegment.from_codes(codes, metric="Hamming")
    try:
        for k in (10, 600, 4096):
            ids, dist = seg.search(q, k)
            assert ids[0].tolist() == list(range(k))
            assert np.all(dist == 128.0)
    finally:
        seg.free()


def test_gpu_float_l2_all_ties_over_sort_capacity(mq):
    """Float path, same tie rule: > 4096 candidates at the k-th key."""
    n = 60000
    rows = np.ones((n, 16), np.float32)
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2")
    try:
        ids, dist = seg.search(np.zeros((1, 16), np.float32), 600)
    finally:
        seg.free()
    assert ids[0].tolist() == list(range(600))
    assert np.all(dist == 16.0)


def test_gpu_hamming_max_distance_never_returned(mq):
    """hammings_knn_mc emits distances b < nBit: a row whose every bit differs
    from the query is not a result (padding instead)."""
    codes = np.array([[0xFF, 0xFF], [0x01, 0x00], [0x00, 0x00]], np.uint8)
    seg = mq.BinaryVectorScanSegment.from_codes(codes, metric="Hamming")
    try:
        ids, dist = seg.search(np.zeros((1, 2), np.uint8), 4)
    finally:
        seg.free()
    assert ids[0].tolist() == [2, 1, -1, -1]
    assert dist[0, :2].tolist() == [0.0, 1.0]
    assert dist[0, 2] == np.float32(3.4028235e38)


@pytest.mark.parametrize("metric", ["Hamming", "Jaccard"])
def test_gpu_knn_binary_raw_contract(mq, metric):
    """mqvs_knn_binary_raw == tryBruteForceSearch<BinaryVector>: Hamming int32
    counts in the distance buffer, INT32_MAX padding; Jaccard floats."""
    rng = np.random.default_rng(7)
    x = codes_of(rng, 5, 16)
    y = codes_of(rng, 3000, 16)
    y[5] = ~x[1]  # every bit differs: never returned by hammings_knn_mc
    for k, ny in ((10, 3000), (8, 5)):
        ids, dist = mq.try_brute_force_search_binary(x, y[:ny], 128, k, 5, ny, metric)
        ids_o, dist_o = O.knn_binary(x, y[:ny], k, O.METRICS[metric])
        assert np.array_equal(ids.reshape(5, k), ids_o)
        assert np.array_equal(dist.reshape(5, k).view(np.uint32), dist_o.view(np.uint32))


def test_gpu_binary_device_pointers_and_shards(mq):
    """torch uint8 codes on the GPU; two row-range shards merged equal the
    whole part."""
    import torch
    rng = np.random.default_rng(3)
    n, nb, nq, k = 40960, 32, 6, 50
    codes = codes_of(rng, n, nb)
    q = codes_of(rng, nq, nb)
    tc = torch.from_numpy(codes).cuda()
    tq = torch.from_numpy(q).cuda()
    whole = mq.BinaryVectorScanSegment.from_codes(tc, metric="Hamming")
    ids, dist = whole.search(tq, k)
    ids_o, dist_o = O.vector_scan_binary(codes, q, k, O.HAMMING, 8192)
    assert_same(ids.cpu().numpy(), dist.cpu().numpy(), ids_o, dist_o, "device pointers")
    half = 8192 * 2
    s0 = mq.BinaryVectorScanSegment.from_codes(codes[:half], metric="Hamming", row_offset=0)
    s1 = mq.BinaryVectorScanSegment.from_codes(codes[half:], metric="Hamming", granule=8192, row_offset=half)
    r0 = s0.search(q, k)
    r1 = s1.search(q, k)
    mi, md = mq.merge_shards(np.stack([r0[0], r1[0]]), np.stack([r0[1], r1[1]]), "Hamming")
    assert_same(mi, md, ids_o, dist_o, "merged shards")
    for s in (whole, s0, s1):
        s.free()


def test_gpu_binary_errors(mq):
    from myscaledb_amd import _lib
    codes = np.zeros((10, 4), np.uint8)
    seg = mq.BinaryVectorScanSegment.from_codes(codes, metric="Jaccard")
    try:
        with pytest.raises(_lib.MqvsError) as e:
            seg.search(np.zeros((1, 4), np.uint8), 3, metric="L2")
        assert e.value.status == _lib.ERR_NOT_IMPLEMENTED
        with pytest.raises(_lib.MqvsError) as e:
            seg.search(np.zeros((1, 5), np.uint8), 3)
        assert e.value.status == _lib.ERR_LOGICAL
        with pytest.raises(_lib.MqvsError) as e:
            _lib.check(_lib.lib.mqvs_search(seg._h, None, 1, 3, 0, None, None, None, None, 0, None))
        assert e.value.status == _lib.ERR_LOGICAL
    finally:
        seg.free()
    with pytest.raises(_lib.MqvsError) as e:
        mq.try_brute_force_search_binary(codes, codes, 32, 3, 10, 10, "L2")
    assert e.value.status == _lib.ERR_NOT_IMPLEMENTED
