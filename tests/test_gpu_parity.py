"""HIP path (through the C-ABI, libmqvs.so) vs the CPU oracle: bit-identical
ids and distances on the same seeded inputs.

The oracle restates MergeTreeVSManager::vectorScanWithoutIndex
(MergeTreeVSManager.cpp:960-1680) chunk by chunk; the GPU path scans the whole
part at once and selects -- the outputs must still agree bit for bit: ids,
distances, order, -1 padding.  Cases cover both faiss formula branches
(nq < 20 direct, nq >= 20 BLAS / MFMA), L2 / IP / Cosine, PREWHERE bitmaps,
lightweight deletes, empty arrays, many-way ties (integer data) and cosine's
per-granule query re-normalisation.
"""
import zlib

import numpy as np
import pytest

from kat_harness import check_case, load_cases
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FLT_MAX = np.float32(3.4028235e38)
CASES = load_cases()


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def gpu_scan(m):
    def fn(rows, nonempty, gran, queries, k, metric, flt, rex):
        seg = m.VectorScanSegment.from_rows(rows, metric=metric, granule=gran, nonempty=nonempty)
        try:
            return seg.search(queries, k, metric, flt, rex)
        finally:
            seg.free()
    return fn


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_kat(mq, case):
    """The reference's own SQL known-answer tests, through the HIP path."""
    check_case(case, gpu_scan(mq))


def assert_bitwise(ids_g, dist_g, ids_o, dist_o, ctx=""):
    ids_g, ids_o = np.asarray(ids_g), np.asarray(ids_o)
    dist_g, dist_o = np.asarray(dist_g, np.float32), np.asarray(dist_o, np.float32)
    if not np.array_equal(ids_g, ids_o) or not np.array_equal(dist_g.view(np.uint32),
                                                              dist_o.view(np.uint32)):
        bad = np.argwhere((ids_g != ids_o) | (dist_g.view(np.uint32) != dist_o.view(np.uint32)))
        q, j = bad[0]
        raise AssertionError(
            f"{ctx}: {len(bad)} mismatches; first at query {q} slot {j}: gpu ({ids_g[q, j]}, "
            f"{dist_g[q, j]!r}) oracle ({ids_o[q, j]}, {dist_o[q, j]!r})\n"
            f"gpu ids {ids_g[q, :12]}\norc ids {ids_o[q, :12]}")


def make_part(seed, n, d, mode, empty_frac=0.0):
    rows = O.generate(seed, mode, 0, n, d)
    nonempty = None
    if empty_frac > 0:
        rng = np.random.default_rng(seed)
        ne = (rng.random(n) >= empty_frac).astype(np.uint8)
        rows[ne == 0] = FLT_MAX
        nonempty = ne
    return rows, nonempty


PARITY = [
    # name,            n,     d,   nq,  k,  metric, mode, gran, filt, lwd,  empty
    ("l2_nq1_exact",    5000,  128, 1,   10, "L2",  0, 8192, None, None, 0.0),
    ("l2_nq3_gauss",    7000,  96,  3,   50, "L2",  1, 1024, None, None, 0.0),
    ("l2_nq19_exact",   3000,  64,  19,  100, "L2", 0, 512,  None, None, 0.0),
    ("l2_nq20_exact",   3000,  64,  20,  100, "L2", 0, 512,  None, None, 0.0),
    ("l2_nq64_gauss",   9000,  128, 64,  100, "L2", 1, 8192, None, None, 0.0),
    ("l2_nq200_mix",    6000,  256, 200, 30,  "L2", 2, 8192, None, None, 0.0),
    ("ip_nq1_gauss",    5000,  128, 1,   10, "IP",  1, 8192, None, None, 0.0),
    ("ip_nq8_exact",    4000,  37,  8,   64, "IP",  0, 128,  None, None, 0.0),
    ("ip_nq40_gauss",   4000,  128, 40,  100, "IP", 1, 8192, None, None, 0.0),
    ("cos_nq1_gauss",   5000,  128, 1,   10, "Cosine", 1, 256, None, None, 0.0),
    ("cos_nq5_exact",   3000,  48,  5,   50, "Cosine", 0, 64,  None, None, 0.0),
    ("cos_nq32_gauss",  6000,  128, 32,  100, "Cosine", 1, 512, None, None, 0.0),
    ("cos_nq150_mix",   5000,  768, 150, 100, "Cosine", 2, 1024, None, None, 0.0),
    ("l2_filter_nq2",   8000,  64,  2,   100, "L2", 0, 256, 0.3, None, 0.0),
    ("l2_filter_nq30",  8000,  64,  30,  100, "L2", 1, 256, 0.05, None, 0.0),
    ("cos_filter_nq4",  6000,  64,  4,   40, "Cosine", 1, 128, 0.2, None, 0.0),
    ("cos_filter_nq24", 6000,  64,  24,  40, "Cosine", 1, 128, 0.02, None, 0.0),
    ("ip_filter_nq3",   6000,  32,  3,   20, "IP", 1, 128, 0.5, None, 0.0),
    ("l2_lwd_nq1",      6000,  64,  1,   50, "L2", 0, 1024, None, 0.2, 0.0),
    ("ip_lwd_nq25",     6000,  64,  25,  50, "IP", 1, 1024, None, 0.3, 0.0),
    ("l2_empty_nq2",    4000,  16,  2,   30, "L2", 0, 128, None, None, 0.3),
    ("ip_empty_nq2",    4000,  16,  2,   30, "IP", 1, 128, None, None, 0.3),
    ("cos_empty_nq3",   4000,  16,  3,   30, "Cosine", 1, 128, None, None, 0.3),
    ("cos_empty_filter_lwd", 4000, 16, 21, 30, "Cosine", 1, 128, 0.4, 0.1, 0.3),
    ("l2_d3_nq21",      200,   3,   21,  100, "L2", 0, 64,  None, None, 0.0),
    ("l2_k_gt_n",       50,    8,   4,   100, "L2", 1, 16,  None, None, 0.0),
    ("l2_big_probe",    100000, 32, 2,   100, "L2", 1, 8192, None, None, 0.0),
    ("cos_big_probe",   80000, 32, 24,  100, "Cosine", 1, 8192, None, None, 0.0),
    # long candidate lists: two-stage final select (radix k-th, then LDS sort)
    ("l2_k1000_twostage", 200000, 16, 2, 1000, "L2", 1, 8192, None, None, 0.0),
    ("cos_k512_twostage", 120000, 32, 20, 512, "Cosine", 1, 8192, None, None, 0.0),
    ("ip_exact_ties_k700", 150000, 8, 3, 700, "IP", 0, 4096, None, None, 0.0),
    # granule-aligned tiling with a short last granule (tiles past the end)
    ("cos_partial_last_granule", 8292, 64, 24, 50, "Cosine", 1, 8192, None, None, 0.0),
    ("cos_partial_last_granule_nq3", 8292, 64, 3, 50, "Cosine", 1, 8192, None, None, 0.0),
    # nq 8..19: bf16 pre-filter + re-rank with faiss's sequential (direct) formula
    ("l2_nq8_gauss",    9000,  96,  8,   50, "L2", 1, 1024, None, None, 0.0),
    ("l2_nq12_mix",     9000,  256, 12,  100, "L2", 2, 2048, None, None, 0.0),
    ("ip_nq10_gauss",   7000,  64,  10,  40, "IP", 1, 512, None, None, 0.0),
    ("ip_nq17_exact",   5000,  40,  17,  64, "IP", 0, 256, None, None, 0.0),
    ("cos_nq9_mix",     8000,  768, 9,   100, "Cosine", 2, 1024, None, None, 0.0),
    ("cos_nq16_gauss",  8000,  128, 16,  100, "Cosine", 1, 512, None, None, 0.0),
    ("l2_filter_lwd_nq14", 8000, 64, 14, 60, "L2", 1, 256, 0.1, 0.2, 0.0),
    ("cos_empty_filter_nq11", 5000, 32, 11, 30, "Cosine", 1, 128, 0.3, None, 0.2),
    ("cos_big_probe_nq15", 90000, 32, 15, 100, "Cosine", 1, 8192, None, None, 0.0),
    ("l2_partial_granule_nq18", 8292, 64, 18, 50, "L2", 1, 8192, None, None, 0.0),
]


BATCH = [c for c in PARITY if c[3] >= 8]

# selective PREWHERE: gather list (default when <= 50% pass) vs masked full scan
FILTERED = [c for c in PARITY if c[8] is not None] + [
    ("l2_filter_none_nq2", 6000, 32, 2, 20, "L2", 1, 512, 0.0, None, 0.0),
    ("cos_filter_all_nq9", 6000, 32, 9, 20, "Cosine", 1, 512, 1.0, None, 0.0),
    ("cos_filter_sparse_nq3", 50000, 64, 3, 50, "Cosine", 2, 2048, 0.003, 0.2, 0.1),
    ("ip_filter_sparse_nq30", 50000, 64, 30, 50, "IP", 1, 1000, 0.01, None, 0.0),
    ("l2_filter_mid_nq12", 40000, 96, 12, 100, "L2", 2, 4096, 0.08, 0.1, 0.05),
    # gathered scans long enough for a probe and several segments: 64-row
    # tiles for the probe and the short L2 segments, and (cosine) short tiles
    # that hold chunk padding only
    ("l2_filter_segments_nq1", 400000, 32, 1, 100, "L2", 1, 8192, 0.3, None, 0.0),
    ("ip_filter_segments_nq16", 300000, 32, 16, 50, "IP", 1, 4096, 0.2, 0.1, 0.0),
    ("cos_filter_pad_tiles_nq2", 400000, 32, 2, 50, "Cosine", 1, 8192, 0.1, None, 0.0),
]


@pytest.mark.parametrize("gmode", [0, 2])
@pytest.mark.parametrize("cfg", FILTERED, ids=[c[0] for c in FILTERED])
def test_gpu_vs_oracle_gather_modes(mq, cfg, gmode):
    """Selective PREWHERE through the gather list (mode 2: always) and the
    masked full scan (mode 0: never): same bits as the oracle either way."""
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_gather_mode
    set_gather_mode(gmode)
    try:
        run_parity(mq, cfg)
        st = _lib.last_search_stats()
        # (the exact fp32 MFMA path, path 1, always scans every row)
        assert st["gather"] == (1 if gmode == 2 and st["path"] != 1 else 0), st
    finally:
        set_gather_mode(1)


@pytest.mark.parametrize("cfg", PARITY, ids=[c[0] for c in PARITY])
def test_gpu_vs_oracle(mq, cfg):
    run_parity(mq, cfg)


@pytest.mark.parametrize("cfg", BATCH, ids=[c[0] for c in BATCH])
def test_gpu_vs_oracle_fp32_batch_mode(mq, cfg):
    """nq >= 8 through the exact-kernels-only mode (VALU below 20, fp32 MFMA
    from 20; the default is the bf16 pre-filter + exact re-rank): same bits."""
    from myscaledb_amd.vector_scan import set_batch_mode
    set_batch_mode(1)
    try:
        run_parity(mq, cfg)
    finally:
        set_batch_mode(0)


@pytest.mark.parametrize("cfg", BATCH, ids=[c[0] for c in BATCH])
def test_gpu_vs_oracle_without_planes(mq, cfg):
    """Segments built without the bf16 plane (mqvs_set_prefilter(0), as when
    the plane does not fit in HBM): nq < 20 on the VALU kernel, nq >= 20 on the
    fp32 MFMA kernel over every row; the default (split 2) is the bf16
    pre-filter + exact re-rank.  Same bits."""
    from myscaledb_amd.vector_scan import set_prefilter
    set_prefilter(0)
    try:
        run_parity(mq, cfg)
    finally:
        set_prefilter(2)


def _wide_range_part(seed, n, d, nq, near):
    """Rows whose elements span ~8 decades inside one vector (the per-vector
    fp6 scales leave the small elements almost nothing), plus `near` rows that
    are tiny perturbations of one row (many approximate values inside the
    bound's window)."""
    rng = np.random.default_rng(seed)
    mag = 10.0 ** rng.uniform(-4, 4, size=(n, d))
    rows = (rng.standard_normal((n, d)) * mag).astype(np.float32)
    base = rows[0].copy()
    for i in range(1, near + 1):
        rows[i] = base * (1 + 1e-6 * rng.standard_normal(d)).astype(np.float32)
    q = (rng.standard_normal((nq, d)) * 10.0 ** rng.uniform(-4, 4, size=(nq, d))).astype(np.float32)
    q[: nq // 2] = base * (1 + 1e-3 * rng.standard_normal(d)).astype(np.float32)
    return rows, q


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
@pytest.mark.parametrize("nq", [12, 40, 200])
def test_prefilter_wide_dynamic_range(mq, metric, nq):
    """The pre-filter bound holds on adversarial magnitudes: bit-identical to
    the oracle (the bound is computed from measured quantisation norms, so
    poorly represented data only widens the candidate window)."""
    rows, q = _wide_range_part(1000 + nq, 6000, 96, nq, near=300)
    m = O.METRICS[metric]
    ids_o, dist_o = O.vector_scan(rows, q, 50, m, 1024, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=1024)
    try:
        ids_g, dist_g = seg.search(q, 50, metric)
    finally:
        seg.free()
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, f"wide {metric} nq={nq}")


def run_parity(mq, cfg):
    name, n, d, nq, k, metric, mode, gran, filt, lwd, empty = cfg
    seed = zlib.crc32(name.encode())
    rows, nonempty = make_part(0x5EED0001 ^ seed, n, d, mode, empty)
    queries = O.generate(0x5EED0002 ^ seed, mode, 0, nq, d)
    rng = np.random.default_rng(seed)
    flt = rex = None
    if filt is not None:
        flt = mq.pack_bitmap(rng.random(n) < filt)
    if lwd is not None:
        rex = mq.pack_bitmap(rng.random(n) >= lwd)
    m = O.METRICS[metric]
    ids_o, dist_o = O.vector_scan(rows, queries, k, m, gran, nonempty=nonempty, filter_bits=flt,
                                  row_exists_bits=rex, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran, nonempty=nonempty)
    ids_g, dist_g = seg.search(queries, k, metric, flt, rex)
    seg.free()
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, name)


@pytest.mark.parametrize("metric", ["L2", "IP", "Cosine"])
@pytest.mark.parametrize("sel", [0.01, 0.1])
def test_gather_unaligned_device_bitmaps(mq, metric, sel):
    """Device filter and delete bitmaps at byte offsets 1 and 3 (the
    word-per-lane selection kernels fall back to byte loads), a granule of 1000
    rows (chunks not on 32-row words) and a part whose length is not a whole
    word: the gather list (dense for L2/IP, per-chunk padded for cosine), the
    masked scan and the oracle agree bit for bit."""
    import torch
    from myscaledb_amd.vector_scan import set_gather_mode
    n, d, nq, k, gran = 50021, 64, 3, 40, 1000
    rows = O.generate(0x5EED0001, 1, 0, n, d)
    queries = O.generate(0x5EED0002, 1, 0, nq, d)
    rng = np.random.default_rng(int(sel * 1000) + len(metric))
    flt = mq.pack_bitmap(rng.random(n) < sel)
    rex = mq.pack_bitmap(rng.random(n) >= 0.1)
    io, do = O.vector_scan(rows, queries, k, O.METRICS[metric], gran, filter_bits=flt, row_exists_bits=rex,
                           fast=True)

    def at_offset(bits, off):
        buf = torch.zeros(len(bits) + 8, dtype=torch.uint8, device="cuda")
        buf[off:off + len(bits)] = torch.from_numpy(np.ascontiguousarray(bits)).cuda()
        return buf[off:off + len(bits)]

    fdev, edev = at_offset(flt, 1), at_offset(rex, 3)
    assert fdev.data_ptr() % 4 == 1 and edev.data_ptr() % 4 == 3
    q = torch.from_numpy(queries).cuda()
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        for gmode in (2, 0):
            set_gather_mode(gmode)
            ids, dist = seg.search(q, k, metric, fdev, edev)
            torch.cuda.synchronize()
            assert_bitwise(ids.cpu().numpy(), dist.cpu().numpy(), io, do, f"{metric} sel {sel} gather {gmode}")
    finally:
        set_gather_mode(1)
        seg.free()


def test_knn_raw_matches_oracle(mq):
    """tryBruteForceSearch contract: faiss layout, raw IP (negatives kept)."""
    rng = np.random.default_rng(7)
    for nx, metric in ((1, O.L2), (5, O.IP), (25, O.L2), (33, O.IP)):
        x = rng.standard_normal((nx, 24)).astype(np.float32)
        y = rng.standard_normal((700, 24)).astype(np.float32)
        ids, dist = mq.try_brute_force_search(x, y, 24, 16, nx, 700, "L2" if metric == O.L2 else "IP")
        io, do = O.knn(x, y, 16, metric)
        assert_bitwise(ids.reshape(nx, 16), dist.reshape(nx, 16), io, do, f"knn nx={nx}")
    # fewer rows than k: faiss padding
    ids, dist = mq.try_brute_force_search(x[:2], y[:3], 24, 8, 2, 3, "IP")
    io, do = O.knn(x[:2], y[:3], 8, O.IP)
    assert_bitwise(ids.reshape(2, 8), dist.reshape(2, 8), io, do, "knn pad")


def test_knn_raw_rejects_cosine(mq):
    from myscaledb_amd._lib import NotImplementedMetric
    with pytest.raises(NotImplementedMetric):
        mq.try_brute_force_search(np.zeros(4, np.float32), np.zeros(8, np.float32), 4, 1, 1, 2,
                                  "Cosine")


def test_device_generator_matches_oracle(mq):
    import torch
    for mode in (0, 1, 2, 3):
        t = torch.empty((300, 77), dtype=torch.float32, device="cuda")
        from myscaledb_amd.vector_scan import generate_device
        generate_device(0x1234 + mode, mode, 12345, 300, 77, t)
        torch.cuda.synchronize()
        ref = O.generate(0x1234 + mode, mode, 12345, 300, 77)
        assert np.array_equal(t.cpu().numpy().view(np.uint32), ref.view(np.uint32)), mode


def test_generated_segment_matches_host_segment(mq):
    n, d = 5000, 64
    seg = mq.VectorScanSegment.generate(99, 1, n, d, "L2", granule=1024)
    rows = O.generate(99, 1, 0, n, d)
    q = O.generate(5, 1, 0, 3, d)
    ids_g, dist_g = seg.search(q, 20)
    ids_o, dist_o = O.vector_scan(rows, q, 20, O.L2, 1024)
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, "generated")


def test_device_pointer_search(mq):
    import torch
    n, d, nq, k = 20000, 128, 50, 64
    rows = O.generate(11, 1, 0, n, d)
    q = O.generate(12, 1, 0, nq, d)
    seg = mq.VectorScanSegment.from_rows(torch.from_numpy(rows).cuda(), metric="Cosine",
                                         granule=4096)
    ids, dist = seg.search(torch.from_numpy(q).cuda(), k)
    torch.cuda.synchronize()
    ids_o, dist_o = O.vector_scan(rows, q, k, O.COSINE, 4096, fast=True)
    assert_bitwise(ids.cpu().numpy(), dist.cpu().numpy(), ids_o, dist_o, "device ptrs")


def test_merge_shards_matches_single_part(mq):
    """Row-range shards (granule aligned) + merge == the unsharded part."""
    n, d, nq, k, gran = 12288, 32, 22, 50, 1024
    for metric, mode in (("L2", 0), ("IP", 1), ("Cosine", 1)):
        rows = O.generate(21, mode, 0, n, d)
        q = O.generate(22, mode, 0, nq, d)
        full = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
        ids_f, dist_f = full.search(q, k)
        full.free()
        bounds = [0, 4096, 8192, 12288]
        ids_s, dist_s = [], []
        for s in range(3):
            seg = mq.VectorScanSegment.from_rows(rows[bounds[s]:bounds[s + 1]], metric=metric,
                                                 granule=gran, row_offset=bounds[s])
            i, dd = seg.search(q, k)
            seg.free()
            ids_s.append(i)
            dist_s.append(dd)
        mi, md = mq.merge_shards(np.stack(ids_s), np.stack(dist_s), metric)
        assert_bitwise(mi, md, ids_f, dist_f, f"merge {metric}")


def test_errors(mq):
    from myscaledb_amd._lib import MqvsError
    seg = mq.VectorScanSegment.from_rows(np.zeros((10, 4), np.float32), metric="Cosine", granule=8)
    with pytest.raises(MqvsError) as e:
        seg.search(np.zeros((1, 4), np.float32), 3, "L2")
    assert e.value.name == "LOGICAL_ERROR"
    with pytest.raises(MqvsError):
        seg.search(np.zeros((1, 5), np.float32), 3)
    seg.free()


@pytest.mark.parametrize("metric,nq,mode", [("L2", 3, 1), ("IP", 5, 1), ("Cosine", 4, 1),
                                            ("L2", 25, 2), ("IP", 21, 0), ("Cosine", 30, 2)])
def test_rerank_all_rows_equals_search(mq, metric, nq, mode):
    """mqvs_rerank over every row of the segment reproduces mqvs_search bit
    for bit (same formula branch, cosine variant per chunk, order key, padding),
    with and without a lightweight-delete mask."""
    n, d, k, gran = 3000, 48, 40, 512
    rows = O.generate(31, mode, 0, n, d)
    q = O.generate(32, mode, 0, nq, d)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        cand = np.tile(np.arange(n, dtype=np.int64), (nq, 1))
        ids_s, dist_s = seg.search(q, k)
        ids_r, dist_r = seg.rerank(q, cand, k)
        assert_bitwise(ids_r, dist_r, ids_s, dist_s, f"rerank all {metric} nq={nq}")
        rng = np.random.default_rng(3)
        rex = np.packbits(rng.random(n) > 0.3, bitorder="little")
        ids_s, dist_s = seg.search(q, k, row_exists=rex)
        ids_r, dist_r = seg.rerank(q, cand, k, row_exists=rex)
        assert_bitwise(ids_r, dist_r, ids_s, dist_s, f"rerank lwd {metric} nq={nq}")
    finally:
        seg.free()


def test_rerank_subset_matches_oracle_knn(mq):
    """Per-query candidate subsets (with -1 and out-of-range entries) against
    the oracle's faiss knn over exactly those rows (nq < 20: direct formula)."""
    n, d, nq, k, ncand = 5000, 40, 6, 16, 700
    rows = O.generate(41, 1, 0, n, d)
    q = O.generate(42, 1, 0, nq, d)
    rng = np.random.default_rng(5)
    cand = np.stack([rng.choice(n, ncand, replace=False) for _ in range(nq)]).astype(np.int64)
    cand[:, :5] = -1
    cand[:, 5:8] = n + 10
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=1024)
    try:
        ids_r, dist_r = seg.rerank(q, cand, k)
    finally:
        seg.free()
    ids_o = np.empty((nq, k), np.int64)
    dist_o = np.empty((nq, k), np.float32)
    for i in range(nq):
        valid = np.sort(cand[i][(cand[i] >= 0) & (cand[i] < n)])
        io, do = O.knn(q[i:i + 1], rows[valid], k, O.L2)
        ids_o[i] = np.where(io[0] >= 0, valid[np.maximum(io[0], 0)], -1)
        dist_o[i] = do[0]
    assert_bitwise(ids_r, dist_r, ids_o, dist_o, "rerank subset")


def test_rerank_errors(mq):
    from myscaledb_amd._lib import MqvsError
    seg = mq.VectorScanSegment.from_rows(np.ones((10, 4), np.float32), metric="L2", granule=8)
    try:
        with pytest.raises(MqvsError) as e:
            seg.rerank(np.ones((1, 4), np.float32), np.zeros((1, 40000), np.int64), 3)
        assert e.value.name == "BAD_ARGUMENTS"
        with pytest.raises(MqvsError) as e:
            seg.rerank(np.ones((1, 4), np.float32), np.zeros((1, 5), np.int64), 3, "Cosine")
        assert e.value.name == "LOGICAL_ERROR"
        ids, dist = seg.rerank(np.ones((2, 4), np.float32), np.full((2, 3), -1, np.int64), 4)
        assert (ids == -1).all() and (dist == FLT_MAX).all()
    finally:
        seg.free()


@pytest.mark.parametrize("metric", ["IP", "L2"])
def test_merge_parts_mode_matches_oracle(mq, metric):
    """MQVS_F_PART_MERGE = getTotalTopSearchResultImpl (MergeTreeBaseSearchManager.cpp:207-297):
    three data parts of small-integer rows (many exact ties), per-part lists
    merged with the insertion-ordered multimap (IP read backwards)."""
    nq, k, d = 9, 25, 8
    parts = [O.generate(80 + p, 0, 0, 700, d) for p in range(3)]
    q = O.generate(90, 0, 0, nq, d)
    ids, dists = [], []
    for rows in parts:
        seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=256)
        i, dd = seg.search(q, k)
        seg.free()
        ids.append(i)
        dists.append(dd)
    ids, dists = np.stack(ids), np.stack(dists)
    mi, md = mq.merge_shards(ids, dists, metric, part_merge=True)
    m = O.IP if metric == "IP" else O.L2
    for j in range(nq):
        _, lab, dd = O.merge_parts(ids[:, j, :], dists[:, j, :], m)
        assert np.array_equal(mi[j], lab), (metric, j, mi[j][:10], lab[:10])
        assert np.array_equal(md[j].view(np.uint32), dd.view(np.uint32)), (metric, j)


def test_path_selection(mq):
    """Default (bf16-hi planes, split 2): the bf16 pre-filter serves every
    batch size (path 2; it streams half the bytes of the fp32 rows).  A
    segment without planes (mqvs_set_prefilter(0)): VALU direct formula below
    nq 20 (path 0), fp32 MFMA from 20 (path 1).  Batch mode 1: exact kernels
    only, the same split."""
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_batch_mode, set_prefilter
    rows = O.generate(3, 1, 0, 4000, 64)
    seg = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=512)
    set_prefilter(0)
    try:
        seg6 = mq.VectorScanSegment.from_rows(rows, metric="L2", granule=512)
    finally:
        set_prefilter(2)
    try:
        assert seg6.info()["prefilter"] == 0 and seg.info()["prefilter"] == 2
        for nq in (1, 7, 8, 20):
            seg.search(O.generate(4, 1, 0, nq, 64), 10)
            st = _lib.last_search_stats()
            assert st["path"] == 2 and st["prefilter"] == 2, nq
        for nq, want in ((7, 0), (8, 0), (19, 0), (20, 1)):
            seg6.search(O.generate(4, 1, 0, nq, 64), 10)
            assert _lib.last_search_stats()["path"] == want, nq
        set_batch_mode(1)
        for nq, want in ((8, 0), (19, 0), (20, 1)):
            seg.search(O.generate(4, 1, 0, nq, 64), 10)
            assert _lib.last_search_stats()["path"] == want, nq
    finally:
        set_batch_mode(0)
        seg.free()
        seg6.free()


@pytest.mark.parametrize("nq", [1, 9, 24])
def test_cosine_slow_normalisation_cycle(mq, nq):
    """A query whose repeated fp32 re-normalisation first repeats at step 16
    (mu 15, lam 1: generator mode 2, seed 12, d 256, query 259) on a part of
    24 chunks, so chunk ordinals 15 and up use the late variants."""
    q = O.generate(12, 2, 0, 300, 256)
    queries = np.concatenate([q[259:260], q[:nq - 1]])
    rows = O.generate(77, 2, 0, 24 * 128, 256)
    ids_o, dist_o = O.vector_scan(rows, queries, 20, O.COSINE, 128, fast=True)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=128)
    try:
        ids_g, dist_g = seg.search(queries, 20, "Cosine")
    finally:
        seg.free()
    assert_bitwise(ids_g, dist_g, ids_o, dist_o, f"slow cycle nq={nq}")


def test_prefilter_no_exact_fallback(mq):
    """The pre-filter keeps the survivors within the re-rank's capacity on
    ordinary data (no silent fallback to the exact fp32 path: rescans 0)."""
    from myscaledb_amd import _lib
    for metric, mode in (("L2", 1), ("IP", 1), ("Cosine", 1)):
        rows = O.generate(11, mode, 0, 30000, 256)
        seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=8192)
        try:
            for nq in (1, 8, 64, 300):
                seg.search(O.generate(12, mode, 0, nq, 256), 100)
                st = _lib.last_search_stats()
                assert st["path"] == 2 and st["rescans"] == 0, (metric, nq, st)
        finally:
            seg.free()


@pytest.mark.parametrize("nq", [3, 12, 40])
def test_cosine_shards_with_skipped_chunks(mq, nq):
    """Row-range shards of a cosine part whose earlier chunks the reference
    never searches (fully filtered out / all empty): mqvs_search_ex with the
    chunk-ordinal base from sharded.chunk_ordinal_base + merge == one part."""
    from myscaledb_amd.sharded import chunk_ordinal_base, shard_rows, slice_bitmap
    n, d, k, gran, world = 12000, 48, 30, 3000, 3
    rows = O.generate(61, 2, 0, n, d)
    q = O.generate(62, 2, 0, nq, d)
    rng = np.random.default_rng(4)
    keep = rng.random(n) > 0.3
    keep[0:gran] = False                     # chunk 0: filtered out entirely
    ne = (rng.random(n) > 0.1).astype(np.uint8)
    ne[gran:2 * gran] = 0                    # chunk 1: all arrays empty
    rows[ne == 0] = FLT_MAX
    flt = np.packbits(keep, bitorder="little")
    for f in (flt, None):
        ids_o, dist_o = O.vector_scan(rows, q, k, O.COSINE, gran, nonempty=ne, filter_bits=f, fast=True)
        got_i, got_d = [], []
        for r in range(world):
            r0, r1 = shard_rows(n, gran, r, world)
            seg = mq.VectorScanSegment.from_rows(rows[r0:r1], metric="Cosine", granule=gran,
                                                 nonempty=ne[r0:r1], row_offset=r0)
            base = chunk_ordinal_base(r0, gran, n, ne, f)
            i, dd = seg.search(q, k, filter_bitmap=slice_bitmap(f, n, r0, r1), ord_base=base)
            seg.free()
            got_i.append(i)
            got_d.append(dd)
        mi, md = mq.merge_shards(np.stack(got_i), np.stack(got_d), "Cosine")
        assert_bitwise(mi, md, ids_o, dist_o, f"cosine shards nq={nq} filter={f is not None}")


@pytest.mark.parametrize("d,metric,nq,k,ncand", [(40, "L2", 6, 6000, 10000), (37, "IP", 25, 64, 9000),
                                                 (40, "L2", 21, 16384, 20000)])
def test_rerank_large_candidate_lists(mq, d, metric, nq, k, ncand):
    """More candidates than the LDS sort (> 4096, through global scratch) and
    k up to 16384: == the oracle's knn over exactly those rows; -1 padding when
    fewer valid candidates than k."""
    n = 40000
    m = O.L2 if metric == "L2" else O.IP
    rows = O.generate(43, 1, 0, n, d)
    q = O.generate(44, 1, 0, nq, d)
    rng = np.random.default_rng(6)
    cand = np.stack([rng.choice(n, ncand, replace=False) for _ in range(nq)]).astype(np.int64)
    cand[:, 100:110] = -1
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=1024)
    try:
        ids_r, dist_r = seg.rerank(q, cand, k)
    finally:
        seg.free()
    ids_o = np.empty((nq, k), np.int64)
    dist_o = np.empty((nq, k), np.float32)
    for i in range(nq):
        valid = np.sort(cand[i][cand[i] >= 0])
        io, do = O.knn(q[i:i + 1], rows[valid], k, m) if nq < 20 else O.knn(q, rows[valid], k, m)
        j = 0 if nq < 20 else i
        ids_o[i] = np.where(io[j] >= 0, valid[np.maximum(io[j], 0)], -1)
        dist_o[i] = do[j]
    assert_bitwise(ids_r, dist_r, ids_o, dist_o, f"rerank {ncand} candidates k {k}")


def test_rerank_every_row_equals_search_cosine(mq):
    """Cosine part of 30000 rows: re-ranking every row (shuffled, > 4096
    candidates) == mqvs_search, query variant per chunk included."""
    n, d, k = 30000, 64, 500
    rows = O.generate(45, 2, 0, n, d)
    seg = mq.VectorScanSegment.from_rows(rows, metric="Cosine", granule=2048)
    try:
        for nq in (3, 24):
            q = O.generate(46, 2, 0, nq, d)
            rng = np.random.default_rng(nq)
            cand = np.stack([rng.permutation(n) for _ in range(nq)]).astype(np.int64)
            ids_r, dist_r = seg.rerank(q, cand, k)
            ids_s, dist_s = seg.search(q, k)
            assert_bitwise(ids_r, dist_r, ids_s, dist_s, f"cosine rerank all rows nq {nq}")
    finally:
        seg.free()
