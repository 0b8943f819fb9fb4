"""mqvs_segment_set_rows_host: a segment whose Float32 rows live in pinned
host memory (HBM keeps the bf16 plane, norms and maps) returns the same bits
as the resident segment -- the pre-filter scans run unchanged and the exact
re-rank reads its survivors' rows over PCIe -- on every path: small and batch
searches, L2 / IP / cosine, PREWHERE filters and deletes, mqvs_rerank, the
exact paths that read every row, and an index built over it.  The rows come
back into HBM bit-identical."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
def test_host_rows_same_bits(mq, metric):
    rng = np.random.default_rng(31)
    n, d, gran = 120000, 96, 8192
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric=metric, granule=gran)
    try:
        flt = np.packbits(rng.random(n) < 0.6, bitorder="little")
        ex = np.packbits(rng.random(n) < 0.95, bitorder="little")
        cases = []
        for nq, k in ((1, 10), (16, 50), (300, 100)):
            q = O.generate(0x5EED0002, 2, 0, nq, d)
            for f, e in ((None, None), (flt, ex)):
                cases.append((q, k, f, e))
        want = [seg.search(q, k, filter_bitmap=f, row_exists=e) for q, k, f, e in cases]
        q0 = cases[2][0]
        cand = want[2][0][:, :40].copy()
        want_rr = seg.rerank(q0, cand, 20)
        info0 = seg.info()
        assert not info0["rows_host"]
        seg.set_rows_host(True)
        info1 = seg.info()
        assert info1["rows_host"] and info1["approx_ok"]
        assert info0["hbm_bytes"] - info1["hbm_bytes"] == 4 * n * d
        for (q, k, f, e), (wi, wd) in zip(cases, want):
            ids, dist = seg.search(q, k, filter_bitmap=f, row_exists=e)
            assert np.array_equal(ids, wi)
            assert np.array_equal(dist.view(np.uint32), wd.view(np.uint32))
        ids, dist = seg.rerank(q0, cand, 20)
        assert np.array_equal(ids, want_rr[0]) and np.array_equal(dist.view(np.uint32), want_rr[1].view(np.uint32))
        # the exact path reads every row over PCIe: same bits
        q, k = cases[2][0], cases[2][1]
        ids, dist = seg.search(q, k, exact=True)
        assert np.array_equal(ids, want[2][0]) and np.array_equal(dist.view(np.uint32), want[2][1].view(np.uint32))
        seg.set_rows_host(False)
        assert not seg.info()["rows_host"] and seg.info()["hbm_bytes"] == info0["hbm_bytes"]
        ids, dist = seg.search(*cases[5][:2], filter_bitmap=cases[5][2], row_exists=cases[5][3])
        assert np.array_equal(ids, want[5][0]) and np.array_equal(dist.view(np.uint32), want[5][1].view(np.uint32))
    finally:
        seg.free()


def test_host_rows_oracle_and_index(mq):
    """Cosine part with rows in host memory: the batch result equals the
    oracle's whole-part scan, and an index built over the segment equals the
    index built while the rows were resident."""
    n, d, nq, k = 40000, 64, 40, 20
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric="Cosine", granule=4096)
    try:
        q = O.generate(0x5EED0003, 2, 0, nq, d)
        idx0 = mq.VectorIndex.build(seg, "MSTG", "nlist=64")
        try:
            want_i = idx0.search(q, k, "nprobe=8")
        finally:
            idx0.free()
        seg.set_rows_host(True)
        base = O.generate(0x5EED0001, 2, 0, n, d)
        ids_o, dist_o = O.vector_scan(base, q, k, O.COSINE, 4096)
        ids, dist = seg.search(q, k)
        assert np.array_equal(ids, ids_o) and np.array_equal(dist.view(np.uint32), dist_o.view(np.uint32))
        idx1 = mq.VectorIndex.build(seg, "MSTG", "nlist=64")
        try:
            got_i = idx1.search(q, k, "nprobe=8")
        finally:
            idx1.free()
        assert np.array_equal(got_i[0], want_i[0])
        assert np.array_equal(got_i[1].view(np.uint32), want_i[1].view(np.uint32))
    finally:
        seg.free()


def test_host_rows_errors(mq):
    from myscaledb_amd import _lib
    with pytest.raises(_lib.MqvsError):
        _lib.check(_lib.lib.mqvs_segment_set_rows_host(None, 1))
