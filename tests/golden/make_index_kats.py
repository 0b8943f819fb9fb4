"""Regenerate tests/golden/index_kats.json from the reference's MSTG SQL tests.

Run in the build container only (it reads /root/reference, absent on the GPU
box); tests use the committed JSON.  Each case restates one SELECT of
`tests/queries/2_vector_search/00028_mqvs_index_mstg_build_search.sql` or
`00029_mqvs_fallback_to_flat.sql` as data: the table formula (rows are
rebuilt in the test exactly as the INSERT computes them), the query vector
(Float64 literal -> Float32), metric, k (LIMIT), the ids a WHERE keeps, the
lightweight-deleted ids, and the expected (id, distance) rows copied from the
matching `.reference` file.
"""
import json
import os
import re

REF = "/root/reference/tests/queries/2_vector_search"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "index_kats.json")


def queries_in(sql_path):
    text = open(sql_path).read()
    return [[float(x) for x in m.split(",")] for m in re.findall(r"distance(?:\('[^']*'\))?\(vector, \[([^\]]+)\]\)", text)]


def result_blocks(ref_path, k):
    rows = []
    for ln in open(ref_path):
        parts = ln.rstrip("\n").split("\t")
        if len(parts) == 2 and re.fullmatch(r"\d+", parts[0]) and re.fullmatch(r"[-0-9.e+]+", parts[1]):
            rows.append([int(parts[0]), parts[1]])
    return [rows[i:i + k] for i in range(0, len(rows), k)]


def main():
    cases = []
    q28 = queries_in(os.path.join(REF, "00028_mqvs_index_mstg_build_search.sql"))
    b28 = result_blocks(os.path.join(REF, "00028_mqvs_index_mstg_build_search.reference"), 5)
    assert len(q28) == 4 and len(b28) == 4, (len(q28), len(b28))
    base = dict(table="mstg768", n=1000, d=768, granularity=1024, k=5)
    # MSTG('disk_mode=1'): default metric (L2)
    cases.append(dict(base, name="00028_l2", metric="L2", query=q28[0], where_not=[], deleted=[],
                      params="", expect=b28[0]))
    cases.append(dict(base, name="00028_cosine_alpha4", metric="Cosine", query=q28[1], where_not=[],
                      deleted=[], params="alpha=4", expect=b28[1]))
    cases.append(dict(base, name="00028_cosine_where", metric="Cosine", query=q28[2], where_not=[0],
                      deleted=[], params="alpha=4", expect=b28[2]))
    cases.append(dict(base, name="00028_cosine_lwd", metric="Cosine", query=q28[3], where_not=[],
                      deleted=[0, 2], params="alpha=4", expect=b28[3]))
    q29 = queries_in(os.path.join(REF, "00029_mqvs_fallback_to_flat.sql"))
    b29 = result_blocks(os.path.join(REF, "00029_mqvs_fallback_to_flat.reference"), 5)
    base = dict(table="shift8", n=1000, d=8, granularity=1024, k=5)
    for i, (q, e) in enumerate(zip(q29, b29)):
        cases.append(dict(base, name=f"00029_cosine_{i}", metric="Cosine", query=q, where_not=[], deleted=[],
                          params="", expect=e))
    doc = {"tables": {
        "mstg768": "row n, col x: float32(0.00001 * (n*768 + x + 1) * (-1 if x % 2 == 0 else 1)) (Float64 arithmetic)",
        "shift8": "row n: [n, n+7, n+6, n+5, n+4, n+3, n+2, n+1]"},
        "source": "tests/queries/2_vector_search/00028_mqvs_index_mstg_build_search.{sql,reference}, "
                  "00029_mqvs_fallback_to_flat.{sql,reference}",
        "cases": cases}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
