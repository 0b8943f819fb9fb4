#!/usr/bin/env python3
"""A/B of the IVF scan's query-group size (MQVS_IVF_QG) on one index: per
setting and group size, ms per search (nq queries, `reps` timed) and recall@10
against FLAT."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--mode", type=int, default=3)
    ap.add_argument("--settings", default="nprobe=128;nprobe=512")
    ap.add_argument("--qgs", default="32,64")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd.vector_index import last_index_stats
    from myscaledb_amd.vector_scan import generate_device, set_timing
    mq.init(0)
    set_timing(True)
    seed = 0x5EED0001
    seg = mq.VectorScanSegment.generate(seed, args.mode, args.n, args.d, "Cosine", 8192)
    idx = mq.VectorIndex.build(seg, "MSTG", "")
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    generate_device(seed, args.mode, args.n, args.nq, args.d, q)
    gt = seg.search(q, args.k)[0].cpu().numpy()
    for sp in args.settings.split(";"):
        for qg in args.qgs.split(","):
            os.environ["MQVS_IVF_QG"] = qg
            ids, _ = idx.search(q, args.k, sp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ids, _ = idx.search(q, args.k, sp)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.reps
            st = last_index_stats()
            got = ids.cpu().numpy()
            r10 = float(np.mean([len(set(got[i, :10]) & set(gt[i, :10])) for i in range(args.nq)]) / 10)
            print(json.dumps({"mode": args.mode, "search": sp, "qg": int(qg), "ms": round(ms, 3),
                              "recall_at_10": r10, "scan_ms": round(st["scan_ms"], 3),
                              "select_ms": round(st["select_ms"], 3), "plane_bytes": st["plane_bytes"]}), flush=True)


if __name__ == "__main__":
    main()
