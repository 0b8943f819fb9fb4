"""Index path (mqvs_index_*, through the C-ABI) on the GPU.

The MSTG library is absent from the reference snapshot, so the index is pinned
three ways ("Index-path and MSTG goldens"):

* the reference's own MSTG known-answer tests (00028, 00029; fixtures in
  tests/golden/index_kats.json): ids exact, distances within the tolerance
  the survey states (2 ulp relative; 2.4e-7 absolute for cosine, one ulp of
  the inner product near 1), since the absent library's reduction order is
  unknown;
* exhaustive probing (nprobe = nlist) equals the FLAT search bit for bit --
  ids, distances, order, padding -- because the re-rank computes the exact
  distance mqvs_search computes for the same rows;
* recall@10 against the FLAT ground truth at the default search parameters.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "index_kats.json")))["cases"]


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def kat_table(c):
    n, d = c["n"], c["d"]
    if c["table"] == "mstg768":
        nn = np.arange(n, dtype=np.float64)[:, None]
        x = np.arange(d, dtype=np.float64)[None, :]
        sign = np.where(np.arange(d) % 2 == 0, -1.0, 1.0)[None, :]
        return ((0.00001 * (nn * 768 + x + 1)) * sign).astype(np.float32)
    nn = np.arange(n)[:, None]
    return (nn + np.array([0, 7, 6, 5, 4, 3, 2, 1])[None, :]).astype(np.float32)


def bitmap_without(n, ids):
    m = np.ones(n, np.uint8)
    m[list(ids)] = 0
    return np.packbits(m, bitorder="little")


@pytest.mark.parametrize("case", KATS, ids=[c["name"] for c in KATS])
def test_index_kat(mq, case):
    rows = kat_table(case)
    q = np.array(case["query"], np.float64).astype(np.float32)[None, :]
    seg = mq.VectorScanSegment.from_rows(rows, metric=case["metric"], granule=case["granularity"])
    idx = mq.VectorIndex.build(seg, "MSTG", f"metric_type={case['metric']}")
    try:
        flt = bitmap_without(case["n"], case["where_not"]) if case["where_not"] else None
        ex = bitmap_without(case["n"], case["deleted"]) if case["deleted"] else None
        ids, dist = idx.search(q, case["k"], case["params"], filter_bitmap=flt, row_exists=ex)
    finally:
        idx.free()
        seg.free()
    exp_ids = [e[0] for e in case["expect"]]
    exp_d = np.array([np.float32(e[1]) for e in case["expect"]], np.float32)
    assert list(ids[0]) == exp_ids
    if case["metric"] == "Cosine":
        assert np.all(np.abs(dist[0] - exp_d) <= 2.4e-7), (dist[0], exp_d)
    else:
        ulp = np.abs(dist[0].view(np.int32).astype(np.int64) - exp_d.view(np.int32).astype(np.int64))
        assert np.all(ulp <= 2), (dist[0], exp_d, ulp)


EXHAUSTIVE = [
    # name,           n,     d,   nq, k,   metric,  mode, gran, nlist, filter, lwd
    ("l2_nq1",        6000,  64,  1,  10,  "L2",     2, 1024, 8,  None, None),
    ("l2_nq32",       9000,  128, 32, 50,  "L2",     2, 2048, 16, None, None),
    ("ip_nq5",        7000,  96,  5,  20,  "IP",     1, 1024, 8,  None, None),
    ("ip_nq40",       7000,  96,  40, 100, "IP",     2, 1024, 12, None, None),
    ("cos_nq3",       8000,  128, 3,  30,  "Cosine", 2, 512,  10, None, None),
    ("cos_nq64_768",  6000,  768, 64, 100, "Cosine", 2, 1024, 16, None, None),
    ("l2_filter",     8000,  64,  24, 40,  "L2",     2, 1024, 8,  0.3,  None),
    ("cos_filter_lwd", 8000, 64,  7,  40,  "Cosine", 2, 512,  8,  0.5,  0.2),
    ("ip_lwd",        8000,  48,  21, 30,  "IP",     1, 1024, 8,  None, 0.3),
    ("l2_d3_small",   300,   3,   20, 100, "L2",     0, 64,   4,  None, None),
]


@pytest.mark.parametrize("cfg", EXHAUSTIVE, ids=[c[0] for c in EXHAUSTIVE])
def test_index_exhaustive_equals_flat(mq, cfg):
    name, n, d, nq, k, metric, mode, gran, nlist, fsel, lwd = cfg
    rows = O.generate(0x5EED0001, mode, 0, n, d)
    q = O.generate(0x5EED0002, mode, 0, nq, d)
    rng = np.random.default_rng(n + nq)
    flt = np.packbits((rng.random(n) < fsel).astype(np.uint8), bitorder="little") if fsel else None
    ex = np.packbits((rng.random(n) >= lwd).astype(np.uint8), bitorder="little") if lwd else None
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": nlist})
    try:
        info = idx.info()
        assert info["nlist"] == nlist and info["rows_indexed"] == n
        ids_i, dist_i = idx.search(q, k, {"nprobe": nlist, "num_reorder": 4096}, filter_bitmap=flt, row_exists=ex)
        ids_f, dist_f = seg.search(q, k, filter_bitmap=flt, row_exists=ex)
        st = mq.vector_index.last_index_stats()
    finally:
        idx.free()
        seg.free()
    assert st["nprobe"] == nlist and st["num_reorder"] == 4096
    assert np.array_equal(ids_i, ids_f), name
    assert np.array_equal(dist_i.view(np.uint32), dist_f.view(np.uint32)), name


@pytest.mark.parametrize("nq", [5, 24])
def test_index_cosine_long_normalisation_chains(mq, nq):
    """Small-integer queries whose fp32 cosine re-normalisation chain does not
    repeat within the default variant table, on a part of 60 granule chunks:
    the index search queues no host round trip for it (the chain's tail runs
    on a side stream), finds it from the status word at its final sync and
    re-runs with one variant per chunk ordinal.  The exhaustive setting then
    equals the oracle's per-chunk re-normalisation bit for bit (the FLAT
    counterpart: test_gpu_boundary.py::test_cosine_long_normalisation_chains)."""
    n, d, k, gran = 60 * 64, 768, 40, 64
    rows = O.generate(0x5EED0001, 0, 0, n, d)
    q = O.generate(0x5EED0002, 0, 0, nq, d)
    io, do = O.vector_scan(rows, q, k, O.COSINE, gran, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=gran)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": 16})
    try:
        ids, dist = idx.search(q, k, {"nprobe": 16, "num_reorder": 4096})
        ids2, dist2 = idx.search(q, k, {"nprobe": 16, "num_reorder": 4096})  # warm workspace: same bits
    finally:
        idx.free()
        seg.free()
    for a, b in ((ids, dist), (ids2, dist2)):
        assert np.array_equal(a, io)
        assert np.array_equal(b.view(np.uint32), do.view(np.uint32))


def test_index_search_after_thread_release(mq):
    """mqvs_thread_release also frees the calling thread's index workspace
    (scratch, events, the variant chain's side stream): searches before and
    after it, from this thread and from a fresh one, return the same bits."""
    import threading
    from myscaledb_amd import _lib
    n, d, nq, k = 20000, 96, 40, 30
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric="Cosine")
    q = O.generate(0x5EED0001, 2, n, nq, d)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": 64})
    out = {}
    try:
        out["a"] = idx.search(q, k, {"nprobe": 4})
        _lib.check(_lib.lib.mqvs_thread_release())
        out["b"] = idx.search(q, k, {"nprobe": 4})

        def worker():
            out["c"] = idx.search(q, k, {"nprobe": 4})
            _lib.check(_lib.lib.mqvs_thread_release())

        t = threading.Thread(target=worker)
        t.start()
        t.join()
    finally:
        idx.free()
        seg.free()
    for key in ("b", "c"):
        assert np.array_equal(out[key][0], out["a"][0]), key
        assert np.array_equal(out[key][1].view(np.uint32), out["a"][1].view(np.uint32)), key


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
def test_index_recall_default_params(mq, metric):
    """Gaussian-mixture part, default nlist / alpha: recall@10 >= 0.95 against
    the FLAT search, and every returned distance is the exact one.  Queries
    are held-out draws of the same mixture (generator rows past the part)."""
    n, d, nq, k = 60000, 128, 200, 100
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric=metric)
    q = O.generate(0x5EED0001, 2, n, nq, d)
    idx = mq.VectorIndex.build(seg, "MSTG")
    try:
        ids_i, dist_i = idx.search(q, k)
        ids_f, _ = seg.search(q, k)
        # returned rows carry their exact distances (mqvs_rerank of the same ids)
        ids_r, dist_r = seg.rerank(q, ids_i, k)
    finally:
        idx.free()
        seg.free()
    hit = [len(set(ids_i[i, :10]) & set(ids_f[i, :10])) for i in range(nq)]
    recall = np.mean(hit) / 10
    assert recall >= 0.95, recall
    assert np.array_equal(ids_r, ids_i)
    assert np.array_equal(dist_r.view(np.uint32), dist_i.view(np.uint32))


def test_index_two_stage(mq):
    """first_stage_only + compute_top_distance_subset == one-call search."""
    n, d, nq, k, R = 20000, 64, 30, 20, 200
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric="Cosine", granule=2048)
    q = O.generate(0x5EED0002, 2, 0, nq, d)
    idx = mq.VectorIndex.build(seg, "MSTG", "nlist=20")
    try:
        c_ids, c_dist = idx.search(q, R, "nprobe=4", first_stage_only=True)
        ids2, dist2 = idx.compute_top_distance_subset(q, c_ids, k)
        ids1, dist1 = idx.search(q, k, f"nprobe=4,num_reorder={R}")
    finally:
        idx.free()
        seg.free()
    # stage 1 is sorted by the approximate distance, ascending for cosine
    valid = c_ids >= 0
    assert valid[:, :k].all()
    assert np.all(np.diff(np.where(valid, c_dist, np.inf), axis=1) >= 0)
    assert np.array_equal(ids1, ids2)
    assert np.array_equal(dist1.view(np.uint32), dist2.view(np.uint32))


@pytest.mark.parametrize("metric,k,R,lwd", [("L2", 5000, None, None), ("Cosine", 8000, 16000, None),
                                             ("IP", 4000, 12000, 0.3)])
def test_index_large_k_equals_flat(mq, metric, k, R, lwd):
    """k above 4096 (LIMIT up to max_search_result_window, Settings.h:923;
    the reference searches k + deleted rows, MergeTreeVSManager.cpp:1565):
    num_reorder above 4096 takes the global-scratch select and re-rank; with
    every list probed the result equals FLAT bit for bit."""
    n, d, nq, nlist = 30000, 64, 6, 16
    rows = O.generate(0x5EED0001, 1, 0, n, d)
    q = O.generate(0x5EED0002, 1, 0, nq, d)
    ex = None
    if lwd:
        rng = np.random.default_rng(7)
        ex = np.packbits((rng.random(n) >= lwd).astype(np.uint8), bitorder="little")
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=8192)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": nlist})
    try:
        params = {"nprobe": nlist}
        if R:
            params["num_reorder"] = R
        ids_i, dist_i = idx.search(q, k, params, row_exists=ex)
        st = mq.vector_index.last_index_stats()
        ids_f, dist_f = seg.search(q, k, row_exists=ex)
    finally:
        idx.free()
        seg.free()
    assert st["num_reorder"] == (R or min(32768, 2 * k))
    assert (ids_i[:, k - 1] >= 0).all()
    assert np.array_equal(ids_i, ids_f)
    assert np.array_equal(dist_i.view(np.uint32), dist_f.view(np.uint32))


def test_index_params_errors(mq):
    from myscaledb_amd import _lib
    seg = mq.VectorScanSegment.generate(1, 1, 2000, 16, metric="L2")
    try:
        with pytest.raises(_lib.MqvsError, match="MSTG doesn't support index parameter: `disk_mode`"):
            mq.VectorIndex.build(seg, "MSTG", "disk_mode=1")
        with pytest.raises(_lib.MqvsError, match="LOGICAL_ERROR"):
            mq.VectorIndex.build(seg, "MSTG", "metric_type=Cosine")
        with pytest.raises(_lib.NotImplementedMetric):
            mq.VectorIndex.build(seg, "HNSWSQ")
        idx = mq.VectorIndex.build(seg, "MSTG", "nlist=4")
        q = np.ones((2, 16), np.float32)
        with pytest.raises(_lib.MqvsError, match="search parameter: `ef_s`"):
            idx.search(q, 5, "ef_s=100")
        with pytest.raises(_lib.MqvsError, match="alpha"):
            idx.search(q, 5, "alpha=9")
        with pytest.raises(_lib.MqvsError, match="dimension"):
            idx.search(np.ones((2, 8), np.float32), 5)
        ids, dist = idx.search(q, 5, "alpha=1")
        assert ids.shape == (2, 5) and (ids >= 0).all()
        idx.free()
    finally:
        seg.free()


def test_index_torch_device_pointers(mq):
    import torch
    n, d, nq, k = 30000, 96, 100, 10
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric="L2")
    idx = mq.VectorIndex.build(seg, "MSTG")
    try:
        qh = O.generate(0x5EED0002, 2, 0, nq, d)
        qd = torch.from_numpy(qh).cuda()
        ids_d, dist_d = idx.search(qd, k)
        ids_h, dist_h = idx.search(qh, k)
    finally:
        idx.free()
        seg.free()
    assert np.array_equal(ids_d.cpu().numpy(), ids_h)
    assert np.array_equal(dist_d.cpu().numpy().view(np.uint32), dist_h.view(np.uint32))


def test_index_many_lists(mq):
    """More than 16384 lists (the strided plan kernel, k_plan_lists, and the
    FLAT coarse step): the returned rows carry their exact distances and the
    recall against FLAT is high when many lists are probed."""
    n, d, nq, k, nlist = 60000, 32, 50, 10, 20000
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric="L2")
    q = O.generate(0x5EED0001, 2, n, nq, d)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": nlist})
    try:
        assert idx.info()["nlist"] == nlist
        ids_i, dist_i = idx.search(q, k, {"nprobe": 4096, "num_reorder": 400})
        ids_f, _ = seg.search(q, k)
        ids_r, dist_r = seg.rerank(q, ids_i, k)
    finally:
        idx.free()
        seg.free()
    recall = np.mean([len(set(ids_i[i]) & set(ids_f[i])) for i in range(nq)]) / k
    assert recall >= 0.9, recall
    assert np.array_equal(ids_r, ids_i)
    assert np.array_equal(dist_r.view(np.uint32), dist_i.view(np.uint32))


@pytest.mark.parametrize("metric,d,nlist", [("L2", 128, 96), ("IP", 64, 64), ("Cosine", 768, 48)])
def test_index_coarse_probes_are_exact_top_nprobe(mq, metric, d, nlist):
    """The coarse pick (nprobe <= 62: bf16 group maxima of the centroid scan,
    then exact fp32 values for every group the bf16 bound cannot rule out)
    returns the exact top-nprobe centroids.  Queries sit between two centroids
    at a relative offset of 1e-2 .. 1e-4 -- near ties the bf16 values cannot
    order -- and at random points.  Checked against float64 scores of the
    index's own centroid table: no unpicked centroid is better than a picked
    one by more than fp32 rounding of the score (parity unpinned: the MSTG
    quantizer is absent from the reference snapshot)."""
    n = 40000
    rows = O.generate(0x5EED0011, 2, 0, n, d)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=1024)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": nlist})
    try:
        C = idx.centroids().astype(np.float64)
        assert C.shape == (nlist, d) and np.all(np.isfinite(C))
        rng = np.random.default_rng(d)
        a = rng.integers(0, nlist, 96)
        b = (a + 1 + rng.integers(0, nlist - 1, 96)) % nlist
        eps = 10.0 ** -rng.integers(2, 5, 96)[:, None]
        m, v = (C[a] + C[b]) / 2, C[a] - C[b]
        if metric == "IP":  # equal inner products with a and b (centroid norms differ)
            m = m - np.sum(m * v, axis=1, keepdims=True) / np.sum(v * v, axis=1, keepdims=True) * v
        q = np.concatenate([m + eps * v,
                            O.generate(0x5EED0012, 2, 0, 32, d).astype(np.float64)]).astype(np.float32)
        got = {}
        for nprobe in (1, 2, 5, 17, min(60, nlist - 2)):
            got[nprobe] = idx.probes(q, {"nprobe": nprobe})
    finally:
        idx.free()
        seg.free()
    q64 = q.astype(np.float64)
    if metric == "Cosine":
        q64 /= np.linalg.norm(q64, axis=1, keepdims=True)
    qn = np.sum(q64 * q64, axis=1)[:, None]
    cn = np.sum(C * C, axis=1)[None, :]
    if metric == "L2":
        score = qn + cn - 2 * q64 @ C.T          # smaller is better
        tol = 4e-6 * (qn + cn).max(axis=1)
    else:
        score = -(q64 @ C.T)                      # raw inner product, larger is better
        tol = 4e-6 * np.sqrt(qn[:, 0] * cn.max())
    near_ties = 0
    for nprobe, pr in got.items():
        assert pr.shape == (len(q), nprobe)
        for i in range(len(q)):
            s = set(pr[i].tolist())
            assert len(s) == nprobe and min(s) >= 0 and max(s) < nlist, (nprobe, i, pr[i])
            picked = score[i, pr[i]]
            rest = np.delete(score[i], pr[i])
            if rest.size:
                assert picked.max() <= rest.min() + tol[i], (metric, nprobe, i, picked.max() - rest.min(), tol[i])
                srt = np.sort(score[i])
                near_ties += int(srt[nprobe] - srt[nprobe - 1] < 1e3 * tol[i])
    assert near_ties > 0  # the set holds boundaries bf16 alone cannot order


@pytest.mark.parametrize("n,nprobe", [(2048, 8), (4096, 60), (4096, 64)])
def test_index_coarse_pick_overflow_is_exact(mq, n, nprobe):
    """More near-tie centroid groups than the coarse pick's working set holds
    (groups past Tcap were cut silently).  With nlist = n and no
    k-means iteration the centroids are the rows themselves (evenly spaced
    initial centroids = every row), so they are built to tie: every row holds
    two ones (inner product 2 with the all-ones query, exactly, in bf16 too),
    and four rows at the end of the table hold 1 + 2^-12 in place of one of
    them -- an exact fp32 inner product of 2 + 2^-12 that the bf16 values
    (both 2) cannot see.  Every one of the n / 8 groups is then within the
    bound of the nprobe-th value; the pick must score them all (its batched
    overflow path, counted in the stats) and return the four rows plus the
    lowest-numbered ties (the (value, centroid) order)."""
    d = 128
    rows = np.zeros((n, d), np.float32)
    i = np.arange(n)
    rows[i, i % d] = 1.0
    rows[i, (i // d + 1 + i) % d] = 1.0   # a second column, never the first one
    special = np.arange(n - 4, n)
    rows[special, (special // d + 1 + special) % d] = np.float32(1 + 2.0 ** -12)
    seg = mq.VectorScanSegment.from_rows(rows, metric="IP", granule=1024)
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": n, "kmeans_iters": 0})
    try:
        C = idx.centroids()
        assert np.array_equal(C, rows)   # the construction the test relies on
        q = np.ones((3, d), np.float32)
        pr = idx.probes(q, {"nprobe": nprobe})
        st = mq.vector_index.last_index_stats()
    finally:
        idx.free()
        seg.free()
    expect = set(special.tolist()) | set(range(nprobe - 4))
    for r in range(len(q)):
        assert set(pr[r].tolist()) == expect, (nprobe, sorted(set(pr[r].tolist()) ^ expect)[:8])
    assert st["pick_overflow"] == len(q), st


@pytest.mark.parametrize("metric,nq,fsel,lwd", [("L2", 200, None, None), ("IP", 64, 0.4, None),
                                                 ("Cosine", 300, 0.5, 0.2), ("L2", 7, None, 0.3),
                                                 ("Cosine", 12, None, None)])
def test_index_pruned_rerank_equals_full(mq, metric, nq, fsel, lwd):
    """The re-rank's bound pruning (candidates more than 2 B past
    the k-th approximate value cannot reach the exact top k) returns the same
    ids and distance bits as re-ranking all num_reorder candidates, on both
    distance formulas (nq < 20: faiss's sequential one), with a PREWHERE
    filter and deletes, and re-ranks fewer candidates."""
    n, d, k, R = 40000, 768 if metric == "Cosine" else 128, 50, 400
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric=metric, granule=1024)
    q = O.generate(0x5EED0001, 2, n, nq, d)
    rng = np.random.default_rng(nq)
    flt = np.packbits((rng.random(n) < fsel).astype(np.uint8), bitorder="little") if fsel else None
    ex = np.packbits((rng.random(n) >= lwd).astype(np.uint8), bitorder="little") if lwd else None
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": 64})
    try:
        params = {"nprobe": 6, "num_reorder": R}
        ids_a, dist_a = idx.search(q, k, params, filter_bitmap=flt, row_exists=ex, rerank_all=True)
        st_a = mq.vector_index.last_index_stats()
        ids_p, dist_p = idx.search(q, k, params, filter_bitmap=flt, row_exists=ex)
        st_p = mq.vector_index.last_index_stats()
    finally:
        idx.free()
        seg.free()
    assert np.array_equal(ids_p, ids_a)
    assert np.array_equal(dist_p.view(np.uint32), dist_a.view(np.uint32))
    assert st_a["reranked"] == nq * R
    assert 0 < st_p["reranked"] < nq * R, st_p


@pytest.mark.parametrize("metric,fsel,lwd", [("L2", None, None), ("IP", 0.5, None), ("Cosine", 0.4, 0.2)])
def test_index_pair_mode_equals_grouped_plan(mq, metric, fsel, lwd):
    """Few (query, list) pairs per list (16 nq nprobe <= nlist) take pair
    mode: no plan, one work item per (pair, list slice), fixed per-query
    regions.  The same 40 queries searched alone (pair mode) and inside a
    batch of 400 (the same queries ten times: the grouped plan) return the
    same ids and distance bits (queries are independent; both batches use the
    nq >= 20 formula), with a PREWHERE filter and deletes, and the stats count
    the pairs and values of the pass."""
    n, d, nq, k, nlist, nprobe = 120000, 64, 40, 50, 1600, 2
    seg = mq.VectorScanSegment.generate(0x5EED0001, 2, n, d, metric=metric, granule=4096)
    q = O.generate(0x5EED0001, 2, n, nq, d)
    rng = np.random.default_rng(5)
    flt = np.packbits((rng.random(n) < fsel).astype(np.uint8), bitorder="little") if fsel else None
    ex = np.packbits((rng.random(n) >= lwd).astype(np.uint8), bitorder="little") if lwd else None
    idx = mq.VectorIndex.build(seg, "MSTG", {"nlist": nlist})
    try:
        params = {"nprobe": nprobe}
        ids_p, dist_p = idx.search(q, k, params, filter_bitmap=flt, row_exists=ex)
        st = mq.vector_index.last_index_stats()
        ids_g, dist_g = idx.search(np.concatenate([q] * 10), k, params, filter_bitmap=flt, row_exists=ex)
    finally:
        idx.free()
        seg.free()
    assert np.array_equal(ids_p, ids_g[:nq])
    assert np.array_equal(dist_p.view(np.uint32), dist_g[:nq].view(np.uint32))
    assert st["pairs"] == nq * nprobe and st["values"] > 0 and st["plane_bytes"] == st["values"] * 2 * 64, st
