"""mqvs_sharded_search -- libmqvs's own multi-GPU path -- on the GPU box's
one GPU.

* A 1-rank RCCL communicator: the local search plus the (id, distance)
  exchange and the device merge through RCCL must equal mqvs_search bit for
  bit.  (One rank runs no chunk-count exchange: its ordinal base is 0.)
* A LOOPBACK communicator group (mqvs_comm_init_loopback) of N = 2, 4 and 8
  virtual ranks, one thread each: every rank holds a granule-aligned row
  range of the part as its own segment, and the whole multi-rank code of
  mqvs_sharded_search runs -- the header exchange (shard order, cosine
  active-chunk counts from k_count_active_chunks and the ordinal-base sum),
  the local searches, the (id, distance, status) exchange and the merge by
  (distance, rank, position), including nranks * k above the 4096-record LDS
  sort.  Only the transport differs from RCCL (device copies between host
  barriers).  The merged result must equal the ORACLE's scan of the whole
  part (MergeTreeVSManager.cpp:960-1680, per-chunk cosine re-normalisation,
  VIWithDataPart.h:358) bit for bit, with PREWHERE filters that empty whole
  chunks, deletes and empty arrays.
* Error paths: shards out of row order, and a rank whose arguments are bad,
  fail on EVERY rank instead of leaving the others in a collective.
"""
import threading
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FLT_MAX = np.float32(3.4028235e38)


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


@pytest.fixture(scope="module")
def comm(mq):
    from myscaledb_amd.sharded import RcclComm
    c = RcclComm(1, 0, RcclComm.unique_id())
    yield c
    c.free()


@pytest.mark.parametrize("metric,nq,k,filt", [("Cosine", 24, 50, None), ("L2", 3, 20, 0.3), ("IP", 40, 100, None),
                                              ("Cosine", 2, 30, 0.2), ("L2", 20, 5000, None)])
def test_one_rank_sharded_search_equals_search(mq, comm, metric, nq, k, filt):
    n, d, gran = 30000, 48, 1024
    rows = O.generate(101, 1, 0, n, d)
    q = O.generate(102, 1, 0, nq, d)
    rng = np.random.default_rng(4)
    flt = mq.pack_bitmap(rng.random(n) < filt) if filt else None
    rex = mq.pack_bitmap(rng.random(n) >= 0.1)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        a = seg.search(q, k, filter_bitmap=flt, row_exists=rex)
        b = comm.sharded_search(seg, q, k, filter_bitmap=flt, row_exists=rex)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
        import torch
        tq = torch.from_numpy(q).cuda()
        ti, td = comm.sharded_search(seg, tq, k, filter_bitmap=None if flt is None else torch.from_numpy(flt).cuda(),
                                     row_exists=torch.from_numpy(rex).cuda())
        assert np.array_equal(ti.cpu().numpy(), a[0])
        assert np.array_equal(td.cpu().numpy().view(np.uint32), a[1].view(np.uint32))
    finally:
        seg.free()


def _run_ranks(ranks, fn):
    """fn(rank_index) on one thread per rank; returns results or raises the
    first error (all threads joined)."""
    out, errs = [None] * len(ranks), [None] * len(ranks)

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(len(ranks))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
        assert not t.is_alive(), "a rank did not finish (exchange deadlock)"
    return out, errs


LOOP = [
    # name,              world, n,     d,  nq, k,    metric,  mode, gran, filt, lwd, empty
    ("cos_w2_filter",    2,     24576, 32, 7,  30,   "Cosine", 1,   1024, 0.7,  0.1, 0.0),
    ("cos_w4_empty",     4,     20000, 24, 5,  40,   "Cosine", 1,   1024, None, 0.1, 0.2),
    ("cos_w8_nofilter",  8,     33000, 16, 22, 25,   "Cosine", 2,   512,  None, None, 0.0),
    ("l2_w4_filter",     4,     30000, 32, 30, 100,  "L2",     1,   2048, 0.5,  0.2, 0.0),
    ("ip_w8_exact",      8,     40960, 8,  3,  50,   "IP",     0,   1024, None, 0.1, 0.0),
    ("l2_w2_bigk",       2,     16384, 16, 4,  3000, "L2",     1,   4096, None, None, 0.0),
    ("cos_w4_batch",     4,     40000, 32, 150, 20,  "Cosine", 1,   1024, 0.9,  None, 0.0),
    # cosine batch with no filter and no empty chunks: the one-wave-per-SIMD
    # batch kernel with the ordinal planes and a non-zero ordinal base per rank
    ("cos_w4_batch_plain", 4,   262144, 64, 200, 20, "Cosine", 1,   2048, None, None, 0.0),
]


def _chunk_filter(rng, n, gran, filt):
    keep = rng.random(n) < filt
    # whole chunks filtered out, in the first and a middle shard: the chunk
    # ordinals of the later shards must skip them (cosine)
    keep[0:gran] = False
    mid = (n // gran // 2) * gran
    keep[mid:mid + gran] = False
    return keep


@pytest.mark.parametrize("cfg", LOOP, ids=[c[0] for c in LOOP])
def test_loopback_ranks_equal_oracle(mq, cfg):
    from myscaledb_amd.sharded import LoopbackComm, shard_rows, slice_bitmap
    name, world, n, d, nq, k, metric, mode, gran, filt, lwd, empty = cfg
    seed = zlib.crc32(name.encode())
    rows = O.generate(0x5EED0001 ^ seed, mode, 0, n, d)
    q = O.generate(0x5EED0002 ^ seed, mode, 0, nq, d)
    rng = np.random.default_rng(seed)
    ne = None
    if empty:
        ne = (rng.random(n) >= empty).astype(np.uint8)
        ne[gran:2 * gran] = 0  # an all-empty chunk
        rows[ne == 0] = FLT_MAX
    flt = mq.pack_bitmap(_chunk_filter(rng, n, gran, filt)) if filt is not None else None
    rex = mq.pack_bitmap(rng.random(n) >= lwd) if lwd is not None else None
    io, do = O.vector_scan(rows, q, k, O.METRICS[metric], gran, nonempty=ne, filter_bits=flt,
                           row_exists_bits=rex, fast=True)
    ranks = LoopbackComm.group(world)
    segs = []
    try:
        for r in range(world):
            r0, r1 = shard_rows(n, gran, r, world)
            segs.append((r0, r1, mq.VectorScanSegment.from_rows(
                rows[r0:r1], metric=metric, granule=gran, nonempty=None if ne is None else ne[r0:r1],
                row_offset=r0)))

        def one(r):
            # the same call three times: the first runs the validated path
            # (header exchange + sync), the repeats the one-sync fast path
            from myscaledb_amd import _lib
            r0, r1, seg = segs[r]
            res = []
            for _ in range(3):
                res.append(ranks[r].sharded_search(seg, q, k, filter_bitmap=slice_bitmap(flt, n, r0, r1),
                                                   row_exists=slice_bitmap(rex, n, r0, r1)))
            return res, ranks[r].stats(), _lib.last_search_stats()

        out, errs = _run_ranks(ranks, one)
        for e in errs:
            if e is not None:
                raise e
        for r in range(world):
            res, cst, sst = out[r]
            for i, (ig, dg) in enumerate(res):
                bad = np.argwhere((ig != io) | (dg.view(np.uint32) != do.view(np.uint32)))
                assert len(bad) == 0, f"{name} rank {r} call {i}: {len(bad)} slots differ, first {tuple(bad[0])}"
            assert cst["fast_calls"] == 2, cst
            if metric != "Cosine" or filt is None:
                # (cosine with chunk-emptying filters re-runs: the guessed
                # ordinal bases are wrong; every other case stays on one sync)
                assert cst["redo_calls"] == 0, cst
            if name == "cos_w4_batch_plain":
                assert sst["batch_kernel"] == 1, sst
    finally:
        for _, _, s in segs:
            s.free()
        for c in ranks:
            c.free()


def test_loopback_out_of_order_shards_fail_everywhere(mq):
    """Rank 0 holding the UPPER half: every rank returns the error."""
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import LoopbackComm
    n, d, gran = 8192, 16, 1024
    rows = O.generate(5, 1, 0, n, d)
    q = O.generate(6, 1, 0, 3, d)
    ranks = LoopbackComm.group(2)
    segs = [mq.VectorScanSegment.from_rows(rows[4096:], metric="L2", granule=gran, row_offset=4096),
            mq.VectorScanSegment.from_rows(rows[:4096], metric="L2", granule=gran, row_offset=0)]
    try:
        _, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(segs[r], q, 10))
        assert all(isinstance(e, MqvsError) for e in errs), errs
        assert all("row order" in str(e) for e in errs), errs
    finally:
        for s in segs:
            s.free()
        for c in ranks:
            c.free()


def test_loopback_bad_rank_fails_everywhere(mq):
    """One rank asks for k above the maximum: both ranks fail (the other rank
    would otherwise wait in the exchange forever)."""
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import LoopbackComm
    n, d, gran = 8192, 16, 1024
    rows = O.generate(7, 1, 0, n, d)
    q = O.generate(8, 1, 0, 3, d)
    ranks = LoopbackComm.group(2)
    segs = [mq.VectorScanSegment.from_rows(rows[:4096], metric="IP", granule=gran, row_offset=0),
            mq.VectorScanSegment.from_rows(rows[4096:], metric="IP", granule=gran, row_offset=4096)]
    try:
        _, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(segs[r], q, 10 if r == 0 else 100000))
        assert all(isinstance(e, MqvsError) for e in errs), errs
    finally:
        for s in segs:
            s.free()
        for c in ranks:
            c.free()


def test_comm_errors(comm):
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import RcclComm
    with pytest.raises(MqvsError):
        RcclComm(2, 5, bytes(128))


def test_loopback_rank_failing_after_header_fails_everywhere(mq):
    """a rank whose LOCAL SEARCH fails (after the header exchange
    validated the call: here its shard was prepared for cosine, the call asks
    for L2) still joins the list exchange; every rank returns an error, none
    hangs, and the next valid call works."""
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import LoopbackComm
    n, d, gran = 8192, 16, 1024
    rows = O.generate(9, 1, 0, n, d)
    q = O.generate(10, 1, 0, 5, d)
    ranks = LoopbackComm.group(2)
    good = [mq.VectorScanSegment.from_rows(rows[:4096], metric="L2", granule=gran, row_offset=0),
            mq.VectorScanSegment.from_rows(rows[4096:], metric="L2", granule=gran, row_offset=4096)]
    bad = mq.VectorScanSegment.from_rows(rows[4096:], metric="Cosine", granule=gran, row_offset=4096)
    try:
        _, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(good[0] if r == 0 else bad, q, 10,
                                                                      metric="L2"))
        assert all(isinstance(e, MqvsError) for e in errs), errs
        assert "rank 1" in str(errs[0]) and "different metric" in str(errs[1]), errs
        io, do = O.vector_scan(rows, q, 10, O.METRICS["L2"], gran, fast=True)
        out, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(good[r], q, 10))
        assert errs == [None, None], errs
        for ig, dg in out:
            assert np.array_equal(ig, io) and np.array_equal(dg.view(np.uint32), do.view(np.uint32))
    finally:
        for s_ in good + [bad]:
            s_.free()
        for c in ranks:
            c.free()


def test_loopback_ranks_on_different_paths_fail_then_recover(mq):
    """Rank 0 repeats the last validated call (fast path: header, search and
    list exchange enqueued without a sync) while rank 1 changes k (validated
    path: header exchange + sync).  Rank 1 sees rank 0's fast flag, joins the
    pending list exchange, and both fail; the next agreeing call succeeds."""
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import LoopbackComm
    n, d, gran = 8192, 16, 1024
    rows = O.generate(11, 1, 0, n, d)
    q = O.generate(12, 1, 0, 4, d)
    ranks = LoopbackComm.group(2)
    segs = [mq.VectorScanSegment.from_rows(rows[:4096], metric="IP", granule=gran, row_offset=0),
            mq.VectorScanSegment.from_rows(rows[4096:], metric="IP", granule=gran, row_offset=4096)]
    try:
        _, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(segs[r], q, 10))
        assert errs == [None, None], errs
        _, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(segs[r], q, 10 if r == 0 else 12))
        assert all(isinstance(e, MqvsError) for e in errs), errs
        assert all("disagree" in str(e) for e in errs), errs
        io, do = O.vector_scan(rows, q, 12, O.METRICS["IP"], gran, fast=True)
        for _ in range(2):
            out, errs = _run_ranks(ranks, lambda r: ranks[r].sharded_search(segs[r], q, 12))
            assert errs == [None, None], errs
            for ig, dg in out:
                assert np.array_equal(ig, io) and np.array_equal(dg.view(np.uint32), do.view(np.uint32))
        assert ranks[0].stats()["fast_calls"] == 2  # the failed repeat and the last call
    finally:
        for s_ in segs:
            s_.free()
        for c in ranks:
            c.free()
