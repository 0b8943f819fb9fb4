"""Boundary contract items of the C-ABI (include/mqvs.h), through the HIP path:

* k up to 16384 -- the reference answers LIMIT up to max_search_result_window
  = 10000 (Settings.h:923, VSUtils.cpp:258) and plain LIMIT without a cap; above
  the 4096-record LDS sort the final select sorts through a device scratch;
* mqvs_merge_shards with nshards * k above 4096;
* per-call path flags (MQVS_F_EXACT / GATHER_*), which replace racing the
  process-wide mqvs_set_* knobs between threads;
* MQVS_F_ASYNC: a search that needs a host-driven fallback is reported by
  mqvs_async_check instead of returning a silently wrong top-k.
"""
import threading
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def _eq(a_ids, a_dist, b_ids, b_dist, ctx):
    a_ids, b_ids = np.asarray(a_ids), np.asarray(b_ids)
    a_dist, b_dist = np.asarray(a_dist, np.float32), np.asarray(b_dist, np.float32)
    bad = np.argwhere((a_ids != b_ids) | (a_dist.view(np.uint32) != b_dist.view(np.uint32)))
    assert len(bad) == 0, (f"{ctx}: {len(bad)} slots differ, first {tuple(bad[0])}: "
                           f"({a_ids[tuple(bad[0])]}, {a_dist[tuple(bad[0])]!r}) vs "
                           f"({b_ids[tuple(bad[0])]}, {b_dist[tuple(bad[0])]!r})")


LARGE_K = [
    # name,           n,      d,  nq, k,     metric,  mode, gran
    ("l2_k5000_nq1",   60000,  32, 1,  5000,  "L2",    1, 8192),
    ("ip_k8000_nq3",   50000,  24, 3,  8000,  "IP",    1, 4096),
    ("cos_k10000_nq2", 40000,  16, 2,  10000, "Cosine", 1, 2048),
    ("l2_k16384_nq24", 30000,  16, 24, 16384, "L2",    1, 8192),
    ("cos_k6000_nq40", 30000,  32, 40, 6000,  "Cosine", 2, 1024),
    ("l2_ties_k7000",  40000,  4,  5,  7000,  "L2",    0, 2048),
    ("l2_k9000_short", 5000,   8,  3,  9000,  "L2",    1, 1024),  # fewer rows than k: -1 padding
]


@pytest.mark.parametrize("cfg", LARGE_K, ids=[c[0] for c in LARGE_K])
def test_large_k_matches_oracle(mq, cfg):
    name, n, d, nq, k, metric, mode, gran = cfg
    seed = zlib.crc32(name.encode())
    rows = O.generate(0x5EED0001 ^ seed, mode, 0, n, d)
    q = O.generate(0x5EED0002 ^ seed, mode, 0, nq, d)
    io, do = O.vector_scan(rows, q, k, O.METRICS[metric], gran, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        ig, dg = seg.search(q, k)
        _eq(ig, dg, io, do, name)
        ie, de = seg.search(q, k, exact=True)
        _eq(ie, de, io, do, name + " exact")
    finally:
        seg.free()


def test_large_k_with_filter_and_deletes(mq):
    n, d, nq, k = 50000, 32, 4, 6000
    rows = O.generate(91, 1, 0, n, d)
    q = O.generate(92, 1, 0, nq, d)
    rng = np.random.default_rng(3)
    flt = mq.pack_bitmap(rng.random(n) < 0.5)
    rex = mq.pack_bitmap(rng.random(n) >= 0.1)
    io, do = O.vector_scan(rows, q, k, O.L2, 4096, filter_bits=flt, row_exists_bits=rex, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=4096)
    try:
        for gather in (None, False, True):
            ig, dg = seg.search(q, k, filter_bitmap=flt, row_exists=rex, gather=gather)
            _eq(ig, dg, io, do, f"filtered k {k} gather {gather}")
    finally:
        seg.free()


def test_k_above_max_rejected(mq):
    from myscaledb_amd._lib import MqvsError
    seg = mq.VectorScanSegment.from_rows(O.generate(1, 1, 0, 100, 8), metric="L2")
    try:
        with pytest.raises(MqvsError) as e:
            seg.search(O.generate(2, 1, 0, 1, 8), 16385)
        assert e.value.code == 36  # BAD_ARGUMENTS
    finally:
        seg.free()


def test_large_k_binary_matches_oracle(mq):
    rng = np.random.default_rng(11)
    n, nb, nq, k = 40000, 16, 3, 7000
    codes = rng.integers(0, 256, size=(n, nb), dtype=np.uint8)
    q = rng.integers(0, 256, size=(nq, nb), dtype=np.uint8)
    for metric in ("Hamming", "Jaccard"):
        io, do = O.vector_scan_binary(codes, q, k, O.METRICS[metric], 8192)
        seg = mq.BinaryVectorScanSegment.from_codes(codes, metric=metric)
        try:
            ig, dg = seg.search(q, k)
        finally:
            seg.free()
        _eq(ig, dg, io, do, f"binary {metric} k {k}")


@pytest.mark.parametrize("metric,part", [("L2", False), ("IP", False), ("IP", True), ("L2", True), ("Cosine", False)])
def test_merge_shards_large(mq, metric, part):
    """nshards * k above the 4096-record LDS sort: the device-scratch merge ==
    the oracle's merge (shards of one part, or the cross-part multimap)."""
    n, d, nq, k, gran = 24576, 16, 5, 3000, 2048
    rows = O.generate(33, 1, 0, n, d)
    q = O.generate(34, 1, 0, nq, d)
    bounds = [0, 8192, 16384, 24576]
    ids_s, dist_s = [], []
    for s in range(3):
        seg = mq.VectorScanSegment.from_rows(rows[bounds[s]:bounds[s + 1]], metric=metric, granule=gran,
                                             row_offset=0 if part else bounds[s])
        i, dd = seg.search(q, k)
        seg.free()
        ids_s.append(i)
        dist_s.append(dd)
    mi, md = mq.merge_shards(np.stack(ids_s), np.stack(dist_s), metric, part_merge=part)
    if part:
        ids, dists = np.stack(ids_s), np.stack(dist_s)
        oi, od = np.empty_like(mi), np.empty_like(md)
        m = O.IP if metric == "IP" else O.L2
        for j in range(nq):
            _, oi[j], od[j] = O.merge_parts(ids[:, j, :], dists[:, j, :], m)
    else:
        full = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
        oi, od = full.search(q, k)
        full.free()
    _eq(mi, md, oi, od, f"merge {metric} part={part}")


def test_per_call_flags_match_global_modes(mq):
    from myscaledb_amd.vector_scan import set_batch_mode, set_gather_mode
    n, d, nq, k = 30000, 64, 24, 50
    rows = O.generate(51, 2, 0, n, d)
    q = O.generate(52, 2, 0, nq, d)
    flt = mq.pack_bitmap(np.random.default_rng(5).random(n) < 0.2)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=2048)
    try:
        base = seg.search(q, k, filter_bitmap=flt)
        set_batch_mode(1)
        try:
            glob = seg.search(q, k, filter_bitmap=flt)
        finally:
            set_batch_mode(0)
        from myscaledb_amd import _lib
        call = seg.search(q, k, filter_bitmap=flt, exact=True)
        assert _lib.last_search_stats()["path"] == 1
        _eq(*call, *glob, "exact flag")
        _eq(*call, *base, "exact vs default")
        for g in (False, True):
            r = seg.search(q, k, filter_bitmap=flt, gather=g)
            assert _lib.last_search_stats()["gather"] == (1 if g else 0)
            _eq(*r, *base, f"gather={g}")
        set_gather_mode(2)
        try:
            r = seg.search(q, k, filter_bitmap=flt, gather=False)  # the call's flag wins
            assert _lib.last_search_stats()["gather"] == 0
        finally:
            set_gather_mode(1)
    finally:
        seg.free()


def test_concurrent_threads_with_per_call_flags(mq):
    """Threads searching one segment with different per-call paths while a
    third flips the process-wide default: every result stays bit-identical."""
    from myscaledb_amd.vector_scan import set_batch_mode
    n, d, nq, k = 40000, 48, 30, 64
    rows = O.generate(61, 1, 0, n, d)
    q = O.generate(62, 1, 0, nq, d)
    seg = mq.VectorScanSegment.from_rows(rows, metric="IP", granule=4096)
    want = seg.search(q, k)
    errors = []
    stop = threading.Event()

    def worker(exact):
        try:
            mq.init(0)
            for _ in range(6):
                got = seg.search(q, k, exact=exact)
                _eq(*got, *want, f"thread exact={exact}")
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def flipper():
        i = 0
        while not stop.is_set():
            set_batch_mode(i & 1)
            i += 1
    th = [threading.Thread(target=worker, args=(e,)) for e in (False, True, False)]
    fl = threading.Thread(target=flipper)
    fl.start()
    for t in th:
        t.start()
    for t in th:
        t.join()
    stop.set()
    fl.join()
    set_batch_mode(0)
    seg.free()
    assert not errors, errors[0]


def test_async_overflow_is_reported(mq):
    """ASYNC search whose candidate lists overflow (every row ties): the call
    returns at once, mqvs_async_check then reports LOGICAL_ERROR; a clean
    ASYNC search afterwards checks OK and equals the synchronous result."""
    import torch
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.vector_scan import async_check
    n, d, nq, k = 600_000, 8, 64, 10
    rows = torch.ones((n, d), dtype=torch.float32, device="cuda")
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=8192)
    q = torch.zeros((nq, d), dtype=torch.float32, device="cuda")
    try:
        seg.search(q, k, async_=True)
        with pytest.raises(MqvsError) as e:
            async_check()
        assert e.value.code == 49
        async_check()  # cleared
    finally:
        seg.free()
    rows2 = torch.from_numpy(O.generate(71, 1, 0, 20000, d)).cuda()
    seg2 = mq.VectorScanSegment.from_rows(rows2, metric="L2", granule=8192)
    try:
        q2 = torch.from_numpy(O.generate(72, 1, 0, nq, d)).cuda()
        ia, da = seg2.search(q2, k, async_=True)
        async_check()
        isy, dsy = seg2.search(q2, k)
        _eq(ia.cpu().numpy(), da.cpu().numpy(), isy.cpu().numpy(), dsy.cpu().numpy(), "async vs sync")
    finally:
        seg2.free()


@pytest.mark.parametrize("nq,budget", [(5, None), (24, None), (24, 1 << 20)])
def test_cosine_long_normalisation_chains(mq, nq, budget):
    """Small-integer queries whose fp32 re-normalisation chain does not repeat
    within the default 32 variants (a third of them at d = 768) on a part of
    60 granule chunks: the variant table grows to one per chunk ordinal and
    the result equals the oracle's per-chunk re-normalisation bit for bit.
    Under a 1 MiB scratch budget the grown table (60 x 4.5 KiB per query) is
    built in query sub-batches of 3 that keep the 24-query call's BLAS
    formula."""
    from myscaledb_amd.vector_scan import set_scratch_budget
    n, d, k, gran = 60 * 64, 768, 40, 64
    rows = O.generate(0x5EED0001, 0, 0, n, d)
    q = O.generate(0x5EED0002, 0, 0, nq, d)
    io, do = O.vector_scan(rows, q, k, O.COSINE, gran, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=gran)
    old = set_scratch_budget(budget) if budget else None
    try:
        ig, dg = seg.search(q, k)
        _eq(ig, dg, io, do, f"cosine long chains nq {nq}")
        ie, de = seg.search(q, k, exact=True)
        _eq(ie, de, io, do, f"cosine long chains nq {nq} exact")
        # computeTopDistanceSubset over every row == the search
        cand = np.tile(np.arange(n, dtype=np.int64)[None, :], (nq, 1))
        ri, rd = seg.rerank(q, cand, k)
        _eq(ri, rd, io, do, f"cosine long chains nq {nq} rerank")
    finally:
        if old:
            set_scratch_budget(old)
        seg.free()


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
def test_sub_batches_keep_the_calls_formula(mq, metric):
    """A call split into query sub-batches (large k under a small scratch
    budget) keeps the distance formula of the WHOLE call: faiss picks the
    BLAS branch from nx >= 20 (BruteForceSearch.h:80-87), so a 25-query call
    whose sub-batches hold 6, 6, 6, 6 and 1 queries still ranks with the BLAS
    form -- the oracle's bits.  Same for computeTopDistanceSubset (31 queries
    in sub-batches of 21 and 10)."""
    from myscaledb_amd.vector_scan import set_scratch_budget
    seed = zlib.crc32(("subbatch_" + metric).encode())
    n, d, nq, k, gran = 50000, 24, 25, 5000, 4096
    rows = O.generate(seed, 1, 0, n, d)
    q = O.generate(seed + 1, 1, 0, nq, d)
    io, do = O.vector_scan(rows, q, k, O.METRICS[metric], gran, fast=True)
    rows2 = O.generate(seed + 2, 1, 0, 6000, d)
    q2 = O.generate(seed + 3, 1, 0, 31, d)
    io2, do2 = O.vector_scan(rows2, q2, 100, O.METRICS[metric], gran, fast=True)
    prev = set_scratch_budget(4 << 20)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    seg2 = mq.VectorScanSegment.from_rows(rows2, metric=metric, granule=gran)
    try:
        ig, dg = seg.search(q, k)
        _eq(ig, dg, io, do, f"{metric} k={k} nq={nq} in sub-batches")
        cand = np.tile(np.arange(6000, dtype=np.int64)[None, :], (31, 1))
        ri, rd = seg2.rerank(q2, cand, 100)
        _eq(ri, rd, io2, do2, f"{metric} rerank 31 queries in sub-batches")
    finally:
        set_scratch_budget(prev)
        seg.free()
        seg2.free()
