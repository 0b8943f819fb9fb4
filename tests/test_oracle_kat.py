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
