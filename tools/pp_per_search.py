#!/usr/bin/env python3
"""Per-search sums of the batch-scan launches in a rocprofv3 kernel trace of
the bench (its --kernel-trace run).  A search is one batch-probe launch
(`k_scan_p4m<..., true, ...>`) followed by its main-scan segments
(`k_scan_p4m<..., false, ...>`); the main-scan launches are summed per search.
  python tools/pp_per_search.py gpurun_out/r04/prof/run_kernel_trace.csv > profiles/r04/bench_p4m_per_search.txt"""
import csv
import sys


def main(path, kernel="k_scan_p4m"):
    ev = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if kernel not in name:
                continue
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            ev.append((t0, (t1 - t0) / 1e6, "true" in name.split("(")[0]))
    ev.sort()
    searches, cur = [], None
    for _, ms, probe in ev:
        if probe:
            cur = {"probe_ms": ms, "main": []}
            searches.append(cur)
        elif cur is not None:
            cur["main"].append(ms)
    print(f"{kernel} launches of the rocprofv3 --kernel-trace run of the bench")
    print("(bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-index --no-configs --no-config1-points):")
    print("per search: the batch probe, then the main-scan segments; search 0 = warmup, then the timed steps.")
    print("search  main_sum_ms  probe_ms  main per-launch ms")
    for i, s in enumerate(searches):
        print(i, round(sum(s["main"]), 3), round(s["probe_ms"], 3), [round(x, 3) for x in s["main"]])


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
