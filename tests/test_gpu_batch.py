"""The batch pre-filter scan (kernels_p4.hip: nq > 128, one wave per SIMD,
256 x 256 work items) against the CPU oracle, bit for bit.

These parts are large enough (n > 32768) that the search runs a probe and a
segmented main scan, so the batch kernel's appends -- not the dense probe --
decide the candidates.  The cases cover every metric (L2 through its
-|y|^2/2 accumulator start, IP, cosine with per-granule query variants),
partial last tiles and granules, several query blocks (nq up to 600), padded
queries (nq not a multiple of 256), dpad 64 .. 768, and integer data with
heavy ties.  `batch_kernel` in the search stats proves the kernel ran; a
granule that is not a multiple of 16 must fall back to the 8-wave kernels
with the same bits.  The oracle restates MergeTreeVSManager.cpp:960-1680 and
faiss's BLAS branch (oracle/mqvs_oracle.c).
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from test_gpu_parity import assert_bitwise, make_part

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


BATCH_P4 = [
    # name,                  n,      d,   nq,  k,   metric,  mode, gran, uses_p4
    ("p4_cos_nq300_mix",     60000,  128, 300, 100, "Cosine", 2, 8192, True),
    ("p4_cos_nq129_d768",    50000,  768, 129, 50,  "Cosine", 1, 4096, True),
    ("p4_cos_nq600_d64",     45056,  64,  600, 20,  "Cosine", 2, 2048, True),
    ("p4_l2_nq256_gauss",    70000,  256, 256, 100, "L2",     1, 8192, True),
    ("p4_l2_nq300_exact",    60000,  64,  300, 100, "L2",     0, 1024, True),
    ("p4_l2_nq257_d768",     40000,  768, 257, 100, "L2",     2, 8192, True),
    ("p4_ip_nq400_gauss",    50000,  96,  400, 64,  "IP",     1, 2048, True),
    ("p4_ip_nq140_exact",    48000,  40,  140, 100, "IP",     0, 8192, True),
    ("p4_cos_partial_tail",  40123,  128, 200, 30,  "Cosine", 1, 8192, True),
    ("p4_l2_partial_tail",   45001,  32,  150, 10,  "L2",     2, 512,  True),
    ("p4_ip_granule_1000",   50000,  64,  200, 20,  "IP",     1, 1000, True),
    # cosine tiles are granule aligned: a granule that is not a multiple of 16
    # rows is served by the 8-wave kernels
    ("p4_cos_granule_1000",  50000,  64,  200, 20,  "Cosine", 1, 1000, False),
]


@pytest.mark.parametrize("cfg", BATCH_P4, ids=[c[0] for c in BATCH_P4])
def test_batch_kernel_vs_oracle(mq, cfg):
    from myscaledb_amd import _lib
    name, n, d, nq, k, metric, mode, gran, uses = cfg
    seed = zlib.crc32(name.encode())
    rows, _ = make_part(0x5EED0001 ^ seed, n, d, mode)
    q = O.generate(0x5EED0002 ^ seed, mode, 0, nq, d)
    ids_o, dist_o = O.vector_scan(rows, q, k, O.METRICS[metric], gran, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        ids_g, dist_g = seg.search(q, k, metric)
        st = _lib.last_search_stats()
    finally:
        seg.free()
    assert st["path"] == 2 and st["main_rows"] > 0, st
    assert st["batch_kernel"] == (1 if uses else 0), st
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, name)


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
def test_batch_kernel_filters_and_deletes(mq, metric):
    """A PREWHERE bitmap that selects most rows (masked scan, not the gather
    list) and lightweight deletes: the batch kernel's candidates pass through
    the same row_valid test as every other scan's."""
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_gather_mode
    n, d, nq, k, gran = 50000, 64, 200, 40, 8192
    seed = zlib.crc32(("p4_filter_" + metric).encode())
    rows, _ = make_part(seed, n, d, 1)
    q = O.generate(seed + 1, 1, 0, nq, d)
    rng = np.random.default_rng(seed)
    flt = mq.pack_bitmap(rng.random(n) < 0.9)
    rex = mq.pack_bitmap(rng.random(n) >= 0.1)
    ids_o, dist_o = O.vector_scan(rows, q, k, O.METRICS[metric], gran, filter_bits=flt,
                                  row_exists_bits=rex, fast=True)
    set_gather_mode(0)  # masked scan at any selectivity
    try:
        seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
        ids_g, dist_g = seg.search(q, k, metric, flt, rex)
        st = _lib.last_search_stats()
        seg.free()
    finally:
        set_gather_mode(1)
    # (cosine with a filter keeps a chunk-ordinal table: 8-wave kernels)
    assert st["batch_kernel"] == (0 if metric == "Cosine" else 1), st
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, f"filter+lwd {metric}")


@pytest.mark.parametrize("metric,how", [("L2", "lwd"), ("IP", "lwd"), ("Cosine", "lwd"),
                                        ("L2", "filter"), ("IP", "filter")])
def test_batch_probe_ignores_invalid_best_rows(mq, metric, how):
    """The batch probe (nq > 128) turns per-(query, 128-row group) maxima into
    the append threshold.  Here each probe group's best row for EVERY query is
    a planted near-copy of the queries' common centre that is deleted (LWD) or
    rejected by the PREWHERE bitmap: were those rows to count, the k-th group
    maximum would sit far above every valid row and the main scan would append
    nothing valid.  Results must equal the oracle's (which never sees those
    rows), at k = 2 (two probe groups of L2 / IP parts) and k = 20."""
    from myscaledb_amd.vector_scan import set_gather_mode
    n, d, nq, gran = 40000, 64, 200, 8192
    seed = zlib.crc32(f"probe_invalid_{metric}_{how}".encode())
    rng = np.random.default_rng(seed)
    rows = rng.standard_normal((n, d)).astype(np.float32)
    c = rng.standard_normal(d).astype(np.float32)
    hot = np.arange(3, n, 61)  # several rows in every 128-row group
    rows[hot] = (5.0 * c if metric == "IP" else c)[None, :]
    q = (c[None, :] + 0.05 * rng.standard_normal((nq, d))).astype(np.float32)
    keep = np.ones(n, bool)
    keep[hot] = False
    keep &= rng.random(n) >= 0.05
    bits = mq.pack_bitmap(keep)
    flt, rex = (bits, None) if how == "filter" else (None, bits)
    set_gather_mode(0)  # masked scan: the probe sees the rejected rows
    try:
        seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
        try:
            for k in (2, 20):
                ids_o, dist_o = O.vector_scan(rows, q, k, O.METRICS[metric], gran, filter_bits=flt,
                                              row_exists_bits=rex, fast=True)
                ids_g, dist_g = seg.search(q, k, metric, flt, rex)
                assert_bitwise(ids_g, dist_g, ids_o, dist_o, f"{metric} {how} k={k}")
        finally:
            seg.free()
    finally:
        set_gather_mode(1)


def test_batch_kernel_many_candidates(mq):
    """Every row ties with the query (identical rows): each wave's candidate
    queue overflows into the direct appends, then the candidate lists
    overflow and the search falls back to the exact path -- still the
    oracle's bits (ties ordered by row)."""
    n, d, nq, k = 40000, 64, 200, 10
    rows = np.ones((n, d), np.float32)
    rows[::7] = 2.0
    q = np.ones((nq, d), np.float32)
    ids_o, dist_o = O.vector_scan(rows, q, k, O.L2, 8192, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=8192)
    ids_g, dist_g = seg.search(q, k, "L2")
    seg.free()
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, "all ties")


@pytest.mark.parametrize("slow,budget", [(False, None), (True, None), (True, 1 << 20)])
def test_batch_kernel_cosine_ordinal_planes(mq, slow, budget):
    """Cosine batches read a chunk's query variants as one contiguous ordinal
    plane when every query's re-normalisation chain fits the planes (max mu +
    lcm of the cycle lengths, at most 32 within the scratch budget).  A query
    whose chain first repeats at step 16 (generator mode 2, seed 12, d 256,
    query 259) needs 16 planes; under a 1 MiB budget only 9 fit and the scan
    keeps per-query variant reads.  Every case must equal the oracle's
    per-chunk re-normalisation (VIWithDataPart.h:358) bit for bit on 40
    chunks."""
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_scratch_budget
    q = O.generate(12, 2, 0, 300, 256)
    queries = np.concatenate([q[259:260], q[:199]]) if slow else q[:200]
    rows = O.generate(77, 2, 0, 40960, 256)
    ids_o, dist_o = O.vector_scan(rows, queries, 20, O.COSINE, 1024, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=1024)
    old = set_scratch_budget(budget) if budget else None
    try:
        ids_g, dist_g = seg.search(queries, 20, "Cosine")
        st = _lib.last_search_stats()
    finally:
        if old:
            set_scratch_budget(old)
        seg.free()
    assert st["batch_kernel"] == 1, st
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, f"ordinal planes slow={slow}")
