"""Regenerate tests/golden/binary_kats.json from the reference's binary-vector
known-answer test (tests/queries/2_vector_search/00038_mqvs_binary_vector_feature).

Run in the build container only (it reads /root/reference, absent on the GPU
box); tests use the committed JSON.  The table is restated as data:
`FixedString(4)` codes char(n, n, n, n) (each byte n mod 256) for ids 0..1023,
one part, default index_granularity 8192.  Query literals: char(a, b, c, d) ->
bytes; unbin('0101...') -> 0x55 x 4; unhex('FFFFFFFF') -> 0xFF x 4.
The BinaryFLAT sections are brute force too (same expectations); the
BINARYMSTG sections are an approximate graph index and are not restated.
"""
import json
import os
import re

REF = "/root/reference/tests/queries/2_vector_search/00038_mqvs_binary_vector_feature.reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "binary_kats.json")

Q_MAIN = [100, 101, 102, 103]
Q_BATCH = [[0x55] * 4, [0, 255, 1, 254], [0xFF] * 4]


def sections(path):
    out, cur = {}, None
    with open(path) as f:
        for ln in f:
            ln = ln.rstrip("\n")
            if ln.startswith("-- "):
                cur = ln[3:]
                out[cur] = []
            elif cur is not None and ln:
                out[cur].append(ln)
    return out


def rows(lines, batch=False):
    res = []
    for ln in lines:
        parts = ln.split("\t")
        if len(parts) != 2:
            continue  # 'sleep' output and system.vector_indices rows
        if batch:
            m = re.match(r"\((\d+),(.*)\)", parts[1])
            res.append([int(parts[0]), int(m.group(1)), m.group(2)])
        else:
            res.append([int(parts[0]), parts[1]])
    return res


def main():
    sec = sections(REF)
    table = {"n": 1024, "code": "nnnn", "granularity": 8192}
    cases = []
    for metric in ("Hamming", "Jaccard"):
        cases.append(dict(name=f"00038_brute_force_{metric}", table=table, metric=metric, queries=[Q_MAIN],
                          k=20, expect=rows(sec[f"Brute Force ({metric})"])))
        cases.append(dict(name=f"00038_batch_{metric}", table=table, metric=metric, queries=Q_BATCH, k=10,
                          batch=True, expect=rows(sec[f"Batch distance ({metric})"], batch=True)))
        cases.append(dict(name=f"00038_filter_{metric}", table=table, metric=metric, queries=[Q_MAIN], k=20,
                          prewhere_ids=list(range(101, 120)), expect=rows(sec[f"Search with filter ({metric})"])))
        cases.append(dict(name=f"00038_binaryflat_{metric}", table=table, metric=metric, queries=[Q_MAIN],
                          k=10, expect=rows(sec[f"BinaryFLAT ({metric})"])))
    lwd = rows(sec["LWD"])
    cases.append(dict(name="00038_lwd_Hamming", table=table, metric="Hamming", queries=[Q_MAIN], k=10,
                      deleted_ids=list(range(200)), expect=lwd[:10]))
    with open(OUT, "w") as f:
        json.dump({"source": "tests/queries/2_vector_search/00038_mqvs_binary_vector_feature.{sql,reference}",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} cases -> {OUT}")


if __name__ == "__main__":
    main()
