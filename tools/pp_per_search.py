#!/usr/bin/env python3
"""Per-search sums of the k_scan_hi_pp launches in a rocprofv3 kernel trace
(tools/gpu_r02.sh's rocprof run: six main-scan launches per search).
  python tools/pp_per_search.py gpurun_out/prof/run_kernel_trace.csv > profiles/r02/bench_pp_per_search.txt"""
import csv
import sys


def main(path, per_search=6):
    durs = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if "k_scan_hi_pp" in row["Kernel_Name"]:
                durs.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
    durs.sort()
    ms = [d for _, d in durs]
    print("k_scan_hi_pp launches of the rocprofv3 --kernel-trace run of tools/gpu_r02.sh")
    print("(bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-small --no-index --no-configs):")
    print("six launches (main-scan segments) per search; search 0 = warmup, 1-3 = the timed steps.")
    print("search  sum_ms  per-launch ms")
    for s in range(len(ms) // per_search):
        part = ms[s * per_search:(s + 1) * per_search]
        print(s, round(sum(part), 3), [round(x, 3) for x in part])


if __name__ == "__main__":
    main(sys.argv[1])
