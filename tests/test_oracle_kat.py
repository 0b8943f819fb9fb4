"""The CPU oracle against the reference's own SQL known-answer tests.

Pins oracle/mqvs_oracle.c (restatement of MergeTreeVSManager.cpp:960-1680,
VIWithDataPart.h:341-382, BruteForceSearch.h:62-111, VectorDataset.h:98-117).
"""
import pytest

from kat_harness import check_case, load_cases
from oracle import oracle as O

CASES = load_cases()


def _oracle_scan(fast):
    def fn(rows, nonempty, gran, queries, k, metric, flt, rex):
        return O.vector_scan(rows, queries, k, metric, gran, nonempty=nonempty,
                             filter_bits=flt, row_exists_bits=rex, fast=fast)
    return fn


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_kat(case):
    check_case(case, _oracle_scan(False))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_fast_kat(case):
    check_case(case, _oracle_scan(True))


# ---- binary vectors: KAT 00038 (tryBruteForceSearch<BinaryVector>) ---------
from kat_harness import check_binary_case, load_binary_cases  # noqa: E402

BCASES = load_binary_cases()


@pytest.mark.parametrize("case", BCASES, ids=[c["name"] for c in BCASES])
def test_oracle_binary_kat(case):
    def fn(codes, gran, queries, k, metric, flt, rex):
        return O.vector_scan_binary(codes, queries, k, O.METRICS[metric], gran, filter_bits=flt,
                                    row_exists_bits=rex)
    check_binary_case(case, fn)


def test_oracle_hamming_knn_contract():
    """faiss::hammings_knn_mc: int32 distances, (distance, row) order, a row
    at distance == d bits never returned, -1 / INT32_MAX padding."""
    import numpy as np
    x = np.array([[0x00, 0x00]], np.uint8)
    y = np.array([[0xFF, 0xFF], [0x01, 0x00], [0x00, 0x00], [0x03, 0x00], [0x01, 0x00]], np.uint8)
    ids, dist = O.knn_binary(x, y, 6, O.HAMMING)
    assert ids.tolist() == [[2, 1, 4, 3, -1, -1]]
    assert dist.tolist() == [[0, 1, 1, 2, 2147483647, 2147483647]]
    ids, dist = O.knn_binary(x, y, 6, O.JACCARD)
    assert ids.tolist() == [[0, 1, 2, 3, 4, -1]]  # num == 0 -> 1.0 for every row
    assert dist[0, :5].tolist() == [1.0] * 5


def test_fast_blas_microkernel_bit_identical():
    """The CPU baseline's register-blocked AVX-512 micro-kernel (orc_knn_fast,
    BLAS branch, nq >= 20) returns the scalar orc_knn's bits: every element is
    still one ascending fp32 fma chain."""
    import numpy as np
    from oracle import oracle as O
    rng = np.random.default_rng(17)
    for nx, ny, d in ((20, 700, 7), (33, 513, 64), (64, 300, 96), (130, 257, 768)):
        x = rng.standard_normal((nx, d)).astype(np.float32)
        y = rng.standard_normal((ny, d)).astype(np.float32)
        for metric in (O.L2, O.IP):
            a = O.knn(x, y, 17, metric)
            b = O.knn(x, y, 17, metric, fast=True)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)), \
                (nx, ny, d, metric, O.has_avx512())
