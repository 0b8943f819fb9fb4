#!/usr/bin/env python3
"""Binary-vector brute force (Hamming / Jaccard) on one GPU: per-search time
and scan bandwidth for a list of batch sizes.  Codes are random bits generated
on the device (torch), `--n` rows of `--bits` bits; one JSON line per setting.
Scan bytes = n * bits / 8 (the code column, read once per query pass)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--bits", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--nq", default="1,8,64,1000")
    ap.add_argument("--metric", default="Hamming,Jaccard")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_timing
    mq.init(0)
    nb = args.bits // 8
    g = torch.Generator(device="cuda").manual_seed(1)
    codes = torch.randint(0, 256, (args.n, nb), dtype=torch.uint8, device="cuda", generator=g)
    seg = mq.BinaryVectorScanSegment.from_codes(codes, metric="Hamming")
    del codes
    torch.cuda.empty_cache()
    set_timing(True)
    for metric in args.metric.split(","):
        for nq in [int(x) for x in args.nq.split(",")]:
            q = torch.randint(0, 256, (nq, nb), dtype=torch.uint8, device="cuda", generator=g)
            ids = torch.empty((nq, args.k), dtype=torch.int64, device="cuda")
            dist = torch.empty((nq, args.k), dtype=torch.float32, device="cuda")
            seg.search(q, args.k, metric, out=(ids, dist))
            best, st_best = 1e30, None
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                seg.search(q, args.k, metric, out=(ids, dist))
                torch.cuda.synchronize()
                w = (time.perf_counter() - t0) * 1e3
                if w < best:
                    best, st_best = w, _lib.last_search_stats()
            scan_ms = st_best["probe_ms"] + st_best["main_ms"]
            byts = args.n * nb
            print(json.dumps({"metric": metric, "n": args.n, "bits": args.bits, "nq": nq, "k": args.k,
                              "wall_ms": round(best, 3), "qps": round(nq / best * 1e3, 1),
                              "scan_ms": round(scan_ms, 3),
                              "scan_GBps": round(byts / (scan_ms * 1e-3) / 1e9, 1),
                              "Gpairs_per_s": round(args.n * nq / (scan_ms * 1e-3) / 1e9, 2),
                              **{kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in st_best.items()}}),
                  flush=True)
    seg.free()


if __name__ == "__main__":
    main()
