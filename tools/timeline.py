#!/usr/bin/env python3
"""Kernel timeline of one call from a rocprofv3 --kernel-trace CSV: the
dispatches from the --nth occurrence of kernel --start up to the next one
(or the end), with the gap before each and its duration (us).

  python tools/timeline.py gpurun_out/x/run_kernel_trace.csv --start k_query_prep --nth -2
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", required=True, help="substring of the kernel that opens a call")
    ap.add_argument("--nth", type=int, default=-1, help="which occurrence (python index)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.start in r["Kernel_Name"]]
    if not idx:
        raise SystemExit("no dispatch of " + a.start)
    k = idx[a.nth]
    nxt = [i for i in idx if i > k]
    win = rows[k:nxt[0]] if nxt else rows[k:]
    t0 = prev = int(win[0]["Start_Timestamp"])
    busy = 0
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print("%8.1f  gap %7.1f  dur %7.1f  q%s  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3,
                                                    r.get("Queue_Id", "?"), r["Kernel_Name"][:80]))
        prev = max(prev, e)
    print("span %.1f us, kernels %.1f us" % ((prev - t0) / 1e3, busy / 1e3))


if __name__ == "__main__":
    main()
