#!/usr/bin/env python3
"""Per-search sums of the batch-scan launches (k_scan_p4 by default) in a
rocprofv3 kernel trace (the bench's rocprof run: six main-scan launches per
search).
  python tools/pp_per_search.py gpurun_out/r03/prof/run_kernel_trace.csv [kernel] > profiles/r03/bench_p4_per_search.txt"""
import csv
import sys


def main(path, kernel="k_scan_p4", per_search=6):
    durs = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                durs.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
    durs.sort()
    ms = [d for _, d in durs]
    print(f"{kernel} launches of the rocprofv3 --kernel-trace run of the bench")
    print("(bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-index --no-configs --no-config1-points):")
    print("six launches (main-scan segments) per search; search 0 = warmup, then the timed steps.")
    print("search  sum_ms  per-launch ms")
    for s in range(len(ms) // per_search):
        part = ms[s * per_search:(s + 1) * per_search]
        print(s, round(sum(part), 3), [round(x, 3) for x in part])


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
