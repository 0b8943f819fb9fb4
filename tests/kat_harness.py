"""Materialise the reference's SQL known-answer tests (tests/golden/kats.json)
into part data and check a search implementation against them.

A `search_fn(rows, nonempty, granularity, queries, k, metric, filter_bits,
row_exists_bits) -> (ids[nq,k], dist[nq,k])` is one part's
vectorScanWithoutIndex (MergeTreeVSManager.cpp:960-1536); the harness applies
the SQL around it: per-part results merged across parts, WHERE on the distance,
ORDER BY ... LIMIT.
"""
import json
import os

import numpy as np

FLT_MAX = np.float32(3.4028235e38)
METRIC = {"L2": 0, "IP": 1, "Cosine": 2}
_HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases():
    with open(os.path.join(_HERE, "golden", "kats.json")) as f:
        return json.load(f)["cases"]


def build_table(table, d=3):
    ids, vecs, nonempty = [], [], []
    for seg in table["segments"]:
        for n in range(seg["start"], seg["start"] + seg["count"]):
            ids.append(n)
            if seg["vec"] == "nnn":
                vecs.append([n, n, n])
                nonempty.append(1)
            elif seg["vec"] == "n_n3_n1":
                vecs.append([n, n + 3, n + 1])
                nonempty.append(1)
            else:  # empty array -> FLT_MAX fill (MergeTreeVSManager.cpp:1381)
                vecs.append([FLT_MAX] * d)
                nonempty.append(0)
    return (np.array(ids, np.int64), np.array(vecs, np.float32),
            np.array(nonempty, np.uint8))


def bits(mask):
    return np.packbits(np.asarray(mask, np.uint8), bitorder="little")


def run_case(case, search_fn):
    """Return the rows the SQL would print: [(id, dist)] or [(id, qi, dist)]."""
    ids, rows, nonempty = build_table(case["table"])
    parts = case["table"].get("parts", [[0, len(ids)]])
    queries = np.array(case["queries"], np.float32)
    k = case["k"]
    metric = METRIC[case["metric"]]
    results = []  # (qi, dist, id)
    for p0, p1 in parts:
        pid = ids[p0:p1]
        flt = None
        if "prewhere_ids" in case:
            sel = np.isin(pid, np.array(case["prewhere_ids"], np.int64))
            flt = bits(sel)
        rex = None
        if "deleted_ids" in case:
            rex = bits(~np.isin(pid, np.array(case["deleted_ids"], np.int64)))
        out_ids, out_dist = search_fn(rows[p0:p1], nonempty[p0:p1], case["table"]["granularity"],
                                      queries, k, metric, flt, rex)
        out_ids, out_dist = np.asarray(out_ids), np.asarray(out_dist)
        for qi in range(len(queries)):
            for j in range(k):
                if out_ids[qi, j] >= 0:
                    results.append((qi, np.float32(out_dist[qi, j]), int(pid[out_ids[qi, j]])))
    if "where_dist_lt" in case:
        results = [r for r in results if r[1] < case["where_dist_lt"]]
    desc = metric == 1
    out = []
    for qi in range(len(queries)):
        rq = [r for r in results if r[0] == qi]
        rq.sort(key=lambda r: ((-r[1] if desc else r[1]), r[2]))
        out.extend(rq[:k])
    if case.get("batch"):
        return [(r[2], r[0], r[1]) for r in out]
    return [(r[2], r[1]) for r in out]


def check_case(case, search_fn):
    got = run_case(case, search_fn)
    exp = case["expect"]
    assert len(got) == len(exp), f"{case['name']}: {len(got)} rows, expected {len(exp)}"
    for g, e in zip(got, exp):
        if case.get("batch"):
            assert (g[0], g[1]) == (e[0], e[1]), f"{case['name']}: got {g}, expected {e}"
            assert g[2] == np.float32(e[2]), f"{case['name']}: got {g}, expected {e}"
        else:
            assert g[0] == e[0], f"{case['name']}: got {g}, expected {e}"
            assert g[1] == np.float32(e[1]), f"{case['name']}: got {g} ({g[1]!r}), expected {e}"


# ---- binary vectors (KAT 00038, tests/golden/binary_kats.json) -------------

def load_binary_cases():
    with open(os.path.join(_HERE, "golden", "binary_kats.json")) as f:
        return json.load(f)["cases"]


def build_binary_table(table):
    n = table["n"]
    ids = np.arange(n, dtype=np.int64)
    codes = np.repeat((ids % 256).astype(np.uint8)[:, None], 4, axis=1)  # char(n, n, n, n)
    return ids, codes


def run_binary_case(case, search_fn):
    """search_fn(codes, granularity, queries_u8, k, metric_name, filter_bits,
    row_exists_bits) -> (ids[nq,k], dist[nq,k] float32): one part's
    vectorScanWithoutIndex<BinaryVector>; the SQL ORDER BY ... LIMIT is applied
    here (one part)."""
    ids, codes = build_binary_table(case["table"])
    queries = np.array(case["queries"], np.uint8)
    k = case["k"]
    flt = bits(np.isin(ids, np.array(case["prewhere_ids"], np.int64))) if "prewhere_ids" in case else None
    rex = bits(~np.isin(ids, np.array(case["deleted_ids"], np.int64))) if "deleted_ids" in case else None
    out_ids, out_dist = search_fn(codes, case["table"]["granularity"], queries, k, case["metric"], flt, rex)
    out_ids, out_dist = np.asarray(out_ids), np.asarray(out_dist)
    res = []
    for qi in range(len(queries)):
        rq = [(int(ids[out_ids[qi, j]]), qi, np.float32(out_dist[qi, j])) for j in range(k) if out_ids[qi, j] >= 0]
        rq.sort(key=lambda r: (r[2], r[0]))
        res.extend(rq[:k])
    if case.get("batch"):
        return res
    return [(r[0], r[2]) for r in res]


def check_binary_case(case, search_fn):
    got = run_binary_case(case, search_fn)
    exp = case["expect"]
    assert len(got) == len(exp), f"{case['name']}: {len(got)} rows, expected {len(exp)}"
    for g, e in zip(got, exp):
        if case.get("batch"):
            assert (g[0], g[1]) == (e[0], e[1]) and g[2] == np.float32(e[2]), f"{case['name']}: got {g}, expected {e}"
        else:
            assert g[0] == e[0] and g[1] == np.float32(e[1]), f"{case['name']}: got {g} ({g[1]!r}), expected {e}"
