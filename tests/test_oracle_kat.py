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
