"""Regenerate tests/golden/kats.json from the reference's SQL known-answer tests.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box); the committed kats.json is what tests use.

Each case restates one `tests/queries/2_vector_search/<name>.{sh,sql}` script
as data: the table (rows derived from the id column exactly as the INSERTs
build them), index_granularity, parts, the query vectors, metric, k (LIMIT),
PREWHERE predicate (as the set of ids it selects), lightweight deletes, and the
expected (id, distance) rows copied from the matching `.reference` file.
"""
import json
import os
import re

REF = "/root/reference/tests/queries/2_vector_search"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")

# tables -------------------------------------------------------------------
# 'nnn': [n, n, n]; 'n_n3_n1': [n, n+3, n+1]; 'empty': []
T_PREPARE_INDEX = {  # helpers/00000_prepare_index.sh
    "segments": [{"start": 0, "count": 100, "vec": "nnn"}], "granularity": 1024}
T_PREPARE_INDEX_2 = {  # helpers/00000_prepare_index_2.sh
    "segments": [{"start": 0, "count": 10, "vec": "nnn"},
                 {"start": 10, "count": 20, "vec": "empty"},
                 {"start": 30, "count": 10000, "vec": "nnn"}], "granularity": 128}
T_EMPTY = {  # helpers/00000_prepare_data_with_empty_vectors.sh (OPTIMIZE -> 1 part)
    "segments": [{"start": 0, "count": 10, "vec": "nnn"},
                 {"start": 10, "count": 20, "vec": "empty"},
                 {"start": 30, "count": 400, "vec": "nnn"}], "granularity": 1024}


def ids_where(pred, n):
    return [i for i in range(n) if pred(i)]


def parse_rows(path, skip=0, take=None, batch=False):
    rows = []
    with open(path) as f:
        lines = [ln.rstrip("\n") for ln in f]
    lines = [ln for ln in lines if ln and not ln.startswith("--")]
    for ln in lines[skip: None if take is None else skip + take]:
        parts = ln.split("\t")
        if batch:
            m = re.match(r"\((\d+),(.*)\)", parts[-1])
            rows.append([int(parts[0]), int(m.group(1)), m.group(2)])
        else:
            rows.append([int(parts[0]), parts[-1]])
    return rows


def main():
    cases = []
    r = lambda name: os.path.join(REF, name + ".reference")

    cases.append(dict(name="00001_mqvs_distance", table=T_PREPARE_INDEX, metric="L2",
                      queries=[[0.1, 0.1, 0.1]], k=10,
                      expect=parse_rows(r("00001_mqvs_distance"), 0, 10)))
    batch_table = {"segments": [{"start": 0, "count": 100, "vec": "nnn"}], "granularity": 8192,
                   "parts": [[0, 50], [50, 100]]}
    bq = [[0.1, 0.1, 0.1], [0.2, 0.2, 0.2], [50.1, 50.1, 50.1]]
    with open(r("00002_mqvs_batch_distance")) as f:
        body = f.read().split("-- batch_distance of metric_type=IP")
    l2_lines = [ln for ln in body[0].splitlines() if "\t" in ln]
    ip_lines = [ln for ln in body[1].splitlines() if "\t" in ln]

    def batch_rows(lines):
        out = []
        for ln in lines:
            p = ln.split("\t")
            m = re.match(r"\((\d+),(.*)\)", p[-1])
            out.append([int(p[0]), int(m.group(1)), m.group(2)])
        return out
    cases.append(dict(name="00002_mqvs_batch_distance_L2", table=batch_table, metric="L2",
                      queries=bq, k=10, batch=True, expect=batch_rows(l2_lines)))
    cases.append(dict(name="00002_mqvs_batch_distance_IP", table=batch_table, metric="IP",
                      queries=bq, k=10, batch=True, expect=batch_rows(ip_lines)))
    cases.append(dict(name="00003_mqvs_distance_with_prewhere", table=T_PREPARE_INDEX, metric="L2",
                      queries=[[1.0, 1.0, 1.0]], k=20,
                      prewhere_ids=ids_where(lambda i: i < 10 or i > 60, 100),
                      expect=parse_rows(r("00003_mqvs_distance_with_prewhere"))))
    cases.append(dict(name="00004_mqvs_filter_by_distance", table=T_PREPARE_INDEX, metric="L2",
                      queries=[[0.1, 0.1, 0.1]], k=10, where_dist_lt=10.0,
                      expect=parse_rows(r("00004_mqvs_filter_by_distance"), 0, 2)))
    cases.append(dict(name="00008_mqvs_empty_vector", table=T_EMPTY, metric="L2",
                      queries=[[20.0, 20.0, 20.0]], k=10,
                      expect=parse_rows(r("00008_mqvs_empty_vector"), 0, 10)))
    cases.append(dict(name="00009_mqvs_brute_force_search_prewhere_0", table=T_PREPARE_INDEX_2,
                      metric="L2", queries=[[10020.1] * 3], k=100,
                      prewhere_ids=ids_where(lambda i: i > 5000 or i in (9, 31, 999, 1), 10030),
                      expect=parse_rows(r("00009_mqvs_brute_force_search_prewhere_0"))))
    cases.append(dict(name="00010_mqvs_brute_force_search_prewhere_1", table=T_PREPARE_INDEX_2,
                      metric="L2", queries=[[10020.1] * 3], k=100,
                      prewhere_ids=ids_where(lambda i: i < 100 or i > 10000, 10030),
                      expect=parse_rows(r("00010_mqvs_brute_force_search_prewhere_1"))))
    cases.append(dict(name="00011_mqvs_brute_force_search_where", table=T_PREPARE_INDEX_2,
                      metric="L2", queries=[[10020.0] * 3], k=100,
                      prewhere_ids=ids_where(lambda i: i < 50 or i in (51, 55, 99, 100, 9999), 10030),
                      expect=parse_rows(r("00011_mqvs_brute_force_search_where"))))
    cases.append(dict(name="00012_mqvs_brute_force_search", table=T_PREPARE_INDEX_2, metric="L2",
                      queries=[[10020.1] * 3], k=100,
                      expect=parse_rows(r("00012_mqvs_brute_force_search"))))
    with open(r("00014_mqvs_distance_cosine_bruteforce")) as f:
        cos = [[int(a), b] for a, b in (ln.split("\t") for ln in f.read().splitlines() if ln)]
    cases.append(dict(name="00014_mqvs_distance_cosine_bruteforce",
                      table={"segments": [{"start": 0, "count": 1000, "vec": "n_n3_n1"}],
                             "granularity": 1024},
                      metric="Cosine", queries=[[8.0, 11.0, 9.0]], k=5, expect=cos))
    cases.append(dict(name="00016_mqvs_lightweight_delete_with_vector",
                      table={"segments": [{"start": 0, "count": 2100, "vec": "nnn"}],
                             "granularity": 1024},
                      metric="L2", queries=[[0.1, 0.1, 0.1]], k=10, deleted_ids=[2],
                      expect=parse_rows(r("00016_mqvs_lightweight_delete_with_vector"), 2, 10)))
    cases.append(dict(name="00032_mqvs_lightweight_delete_small_ranges",
                      table={"segments": [{"start": 0, "count": 100, "vec": "nnn"}],
                             "granularity": 3},
                      metric="L2", queries=[[1.0, 1.0, 1.0]], k=10, deleted_ids=[2, 3, 8],
                      expect=parse_rows(r("00032_mqvs_lightweight_delete_small_ranges"), 2, 10)))
    with open(r("00038_mqvs_brute_force_setting")) as f:
        lines = f.read().splitlines()
    i = lines.index("enable_brute_force_vector_search = 1")
    bf = [[int(a), b] for a, b in (ln.split("\t") for ln in lines[i + 1:i + 6])]
    cases.append(dict(name="00038_mqvs_brute_force_setting",
                      table={"segments": [{"start": 0, "count": 100, "vec": "nnn"}],
                             "granularity": 8192},
                      metric="L2", queries=[[1.0, 1.0, 1.0]], k=5, expect=bf))
    for c in cases:
        c["source"] = "tests/queries/2_vector_search/" + re.sub(r"_(L2|IP)$", "", c["name"])
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_kats.py", "cases": cases}, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()
