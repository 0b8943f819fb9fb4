#!/usr/bin/env python3
"""Kernel timeline of one call from a rocprofv3 --kernel-trace CSV: the
dispatches from the --nth occurrence of kernel --start up to the next one
(or the end), with the gap before each and its duration (us).

  python tools/timeline.py gpurun_out/x/run_kernel_trace.csv --start k_query_prep --nth -2

--api run_hip_api_trace.csv (a --hip-runtime-trace of the same run): also
list the host's HIP calls of the window (from 300 us before its first
dispatch), each with its start and duration on the same clock, and for each
dispatch the time its launch call returned ("launched"), so that a GPU gap
shows whether the host had not yet issued the next work.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", required=True, help="substring of the kernel that opens a call")
    ap.add_argument("--nth", type=int, default=-1, help="which occurrence (python index)")
    ap.add_argument("--api", default=None, help="hip_api_trace.csv of the same run")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.start in r["Kernel_Name"]]
    if not idx:
        raise SystemExit("no dispatch of " + a.start)
    k = idx[a.nth]
    nxt = [i for i in idx if i > k]
    win = rows[k:nxt[0]] if nxt else rows[k:]
    t0 = prev = int(win[0]["Start_Timestamp"])
    api = []
    if a.api:
        api = sorted(csv.DictReader(open(a.api)), key=lambda r: int(r["Start_Timestamp"]))
    launch = {r["Correlation_Id"]: int(r["End_Timestamp"]) for r in api}
    busy = 0
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        la = launch.get(r.get("Correlation_Id"))
        lt = "  launched %8.1f" % ((la - t0) / 1e3) if la is not None else ""
        print("%8.1f  gap %7.1f  dur %7.1f  q%s%s  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3,
                                                      r.get("Queue_Id", "?"), lt, r["Kernel_Name"][:80]))
        prev = max(prev, e)
    print("span %.1f us, kernels %.1f us" % ((prev - t0) / 1e3, busy / 1e3))
    if api:
        print("host HIP calls:")
        for r in api:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < t0 - 300000 or s > prev:
                continue
            print("%8.1f  dur %7.1f  tid %s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Thread_Id", "?"),
                                                  r.get("Function", r.get("Operation", "?"))))


if __name__ == "__main__":
    main()
