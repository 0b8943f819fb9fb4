#!/usr/bin/env python3
"""nq sweep on one GPU: per-launch kernel times and roofline fractions for the
scan kernels (10M x 768 by default).  Prints one JSON line per config."""
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
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--nqs", default="1,4,16,19,20,64,256,1000")
    ap.add_argument("--metrics", default="Cosine,L2")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", type=int, default=2, help="generator mode (0 ints, 1 gauss, 2 mixture)")
    ap.add_argument("--sels", default="", help="PREWHERE selectivities, e.g. 1,0.5,0.1,0.01 "
                    "(uniform random bitmap per selectivity; empty = no filter)")
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device, set_timing
    mq.init(0)
    for metric in args.metrics.split(","):
        seg = mq.VectorScanSegment.generate(0x5EED0001, args.mode, args.n, args.d, metric, 8192)
        sels = [float(x) for x in args.sels.split(",")] if args.sels else [None]
        for sel, nq in [(s_, nq_) for s_ in sels for nq_ in [int(x) for x in args.nqs.split(",")]]:
            q = torch.empty((nq, args.d), dtype=torch.float32, device="cuda")
            generate_device(0x5EED0002, args.mode, 0, nq, args.d, q)
            flt = None
            if sel is not None:
                rng = np.random.default_rng(3)
                bits = np.packbits(rng.random(args.n) < sel, bitorder="little")
                flt = torch.from_numpy(bits).cuda()
            seg.search(q, args.k, filter_bitmap=flt)
            set_timing(True)
            sts, walls = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                seg.search(q, args.k, filter_bitmap=flt)
                walls.append((time.perf_counter() - t0) * 1e3)
                sts.append(_lib.last_search_stats())
            set_timing(False)
            st = min(sts, key=lambda s: s["main_ms"])
            main_rows, d = st["main_rows"], args.d
            gbs = (4.0 * main_rows * d) / (st["main_ms"] * 1e-3) / 1e9
            tfs = 2.0 * nq * main_rows * d / (st["main_ms"] * 1e-3) / 1e12
            print(json.dumps({
                "metric": metric, "n": args.n, "d": args.d, "nq": nq, "selectivity": sel,
                "wall_ms": round(min(walls), 3),
                "qps": round(nq / (min(walls) / 1e3), 1),
                "probe_ms": round(st["probe_ms"], 3), "probe_select_ms": round(st["probe_select_ms"], 3),
                "main_ms": round(st["main_ms"], 3), "refine_ms": round(st["refine_ms"], 3),
                "final_ms": round(st["final_ms"], 3),
                "main_bf16x3_TFLOPs": round(3 * tfs, 1),
                "total_ms": round(st["total_ms"], 3), "probe_rows": st["probe_rows"],
                "main_GBps": round(gbs, 1), "main_hbm_frac": round(gbs / 8000.0, 3),
                "main_TFLOPs": round(tfs, 2), "main_fp32_frac": round(tfs / 157.3, 3),
                "path": st["path"], "rescans": st["rescans"], "segments": st["segments"]}),
                  flush=True)
        seg.free()


if __name__ == "__main__":
    main()
