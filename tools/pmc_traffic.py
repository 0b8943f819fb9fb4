#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into per-search HBM
traffic of the main-scan kernel, for bench.py's roofline.traffic.

FETCH_SIZE on gfx950 reports half the bytes of a wide coalesced stream
(MI355X_MICROARCH.md, HBM section): bytes = 2 * FETCH_SIZE * 1024 +
WRITE_SIZE * 1024.  Launches are grouped by kernel template; `--searches`
is how many searches the profiled command ran (to get per-search figures).

  python tools/pmc_traffic.py gpurun_out --searches 4 --out profiles/r01/pmc_traffic.json
"""
import argparse
import collections
import csv
import json
import os
import re


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", help="directory holding pmc1/ pmc2/ pmc3/ (gpurun_out)")
    ap.add_argument("--searches", type=int, required=True)
    ap.add_argument("--nq", type=int, default=None, help="batch size of the profiled searches")
    ap.add_argument("--kernel", default="k_scan_(?:hi|p4)")
    ap.add_argument("--last", type=int, default=0,
                    help="keep only the last N dispatches of each kernel per pass (drops e.g. an index "
                         "build's own scans that precede the profiled searches)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    dur = collections.defaultdict(dict)
    for tag in ("pmc1", "pmc2", "pmc3"):
        p = os.path.join(args.root, tag, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rows = load(p)
        if args.last:
            ids = collections.defaultdict(set)
            for r in rows:
                m = re.search(args.kernel + r"[_a-z]*(?:<([^>]*)>)?", r["Kernel_Name"])
                if m:
                    ids[m.group(0)].add(int(r["Dispatch_Id"]))
            keep = {k: set(sorted(v)[-args.last:]) for k, v in ids.items()}
        for r in rows:
            m = re.search(args.kernel + r"[_a-z]*(?:<([^>]*)>)?", r["Kernel_Name"])
            if not m:
                continue
            key = m.group(0)
            if args.last and int(r["Dispatch_Id"]) not in keep[key]:
                continue
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[key][tag].add(r["Dispatch_Id"])
            dur[(key, tag)][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {"source": "rocprofv3 --pmc (separate passes: SQ/GRBM, FETCH_SIZE, WRITE_SIZE+TCC)",
           "fetch_correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)",
           "searches": args.searches, "nq": args.nq, "kernels": {}}
    if args.last:
        out["last_dispatches"] = args.last
    for key, c in agg.items():
        k = {}
        launches = max(len(v) for v in disp[key].values())
        k["launches"] = launches
        durs = [v for (kk, tag), dd in dur.items() if kk == key for v in dd.values()]
        if durs:
            k["avg_launch_ms"] = round(sum(durs) / len(durs) / 1e6, 4)
        if "FETCH_SIZE" in c:
            rd = 2.0 * c["FETCH_SIZE"] * 1024
            wr = c.get("WRITE_SIZE", 0.0) * 1024
            k["hbm_read_bytes_per_search"] = rd / args.searches
            k["hbm_write_bytes_per_search"] = wr / args.searches
            k["hbm_bytes_per_search"] = (rd + wr) / args.searches
        if "GRBM_GUI_ACTIVE" in c:
            t = sum(dur[(key, "pmc1")].values()) / 1e9
            k["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3)
            k["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4), 4)
            wc = c["SQ_WAVE_CYCLES"]
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in c:
                    k[n.lower() + "_frac"] = round(c[n] / wc, 4)
        if "TCC_HIT_sum" in c:
            k["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if "SQ_LDS_BANK_CONFLICT" in c:
            k["lds_bank_conflict_cycles"] = c["SQ_LDS_BANK_CONFLICT"]
        out["kernels"][key] = k
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
