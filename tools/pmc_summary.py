#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel name (substring filter) over every
dispatch in the given counter_collection.csv files:
    python tools/pmc_summary.py k_scan_mx gpurun_out/pmcmx_a1/.../*counter_collection.csv"""
import collections
import csv
import sys


def main():
    pat, files = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    for k, v in agg.items():
        print(k, "dispatches", len(disp[k]))
        for c, x in sorted(v.items()):
            print("   %-28s %.4g" % (c, x))
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
            print("   L2 hit rate %.3f" % (h / max(h + m, 1)))


if __name__ == "__main__":
    main()
