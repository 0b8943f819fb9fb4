#!/usr/bin/env python3
"""Index path (MSTG-type) sweep on one GPU: build time, then QPS and
recall@10 against the FLAT ground truth for a list of search settings.
Prints one JSON line per setting (BASELINE configs[2] by default:
10M x 768 Cosine, Gaussian mixture, nq 1000, k 100)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--metric", default="Cosine")
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--build", default="", help="index params, e.g. nlist=10000")
    ap.add_argument("--search", default="alpha=1;alpha=2;alpha=3;alpha=4",
                    help="';'-separated search param strings")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--query-seed", type=lambda x: int(x, 0), default=0x5EED0001)
    ap.add_argument("--rerank-all", action="store_true",
                    help="re-rank every num_reorder candidate (MQVS_F_RERANK_ALL: no bound pruning)")
    ap.add_argument("--dbg", action="store_true",
                    help="load the measurement build libmqvs_dbg.so (reads MQVS_* A/B switches)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import myscaledb_amd as mq
    if args.dbg:
        from myscaledb_amd import _lib as _mq_lib
        _mq_lib.use_measurement_build()
    from myscaledb_amd.vector_index import last_index_stats
    from myscaledb_amd.vector_scan import generate_device
    mq.init(0)
    t0 = time.perf_counter()
    seg = mq.VectorScanSegment.generate(0x5EED0001, args.mode, args.n, args.d, args.metric, 8192)
    torch.cuda.synchronize()
    t_seg = time.perf_counter() - t0
    t0 = time.perf_counter()
    idx = mq.VectorIndex.build(seg, "MSTG", args.build)
    t_build = time.perf_counter() - t0
    info = idx.info()
    print(json.dumps({"event": "build", "n": args.n, "d": args.d, "metric": args.metric,
                      "segment_s": round(t_seg, 2), "build_s": round(t_build, 2), **info}), flush=True)
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    # held-out draws of the part's own distribution: generator rows past the part
    # (--query-seed other than the base seed: a different mixture)
    generate_device(args.query_seed, args.mode, args.n if args.query_seed == 0x5EED0001 else 0, args.nq, args.d, q)
    gt_ids, _ = seg.search(q, args.k)
    gt = gt_ids.cpu().numpy()
    ids = torch.empty((args.nq, args.k), dtype=torch.int64, device="cuda")
    dist = torch.empty((args.nq, args.k), dtype=torch.float32, device="cuda")
    from myscaledb_amd.vector_scan import set_timing
    for sp in [s for s in args.search.split(";") if s is not None]:
        idx.search(q, args.k, sp, out=(ids, dist), rerank_all=args.rerank_all)
        walls, sts = [], []
        # stage times from searches with the timing events on; walls without
        set_timing(True)
        for _ in range(3):
            idx.search(q, args.k, sp, out=(ids, dist), rerank_all=args.rerank_all)
            sts.append(last_index_stats())
        set_timing(False)
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.search(q, args.k, sp, out=(ids, dist), rerank_all=args.rerank_all)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
        got = ids.cpu().numpy()
        r10 = float(np.mean([len(set(got[i, :10]) & set(gt[i, :10])) for i in range(args.nq)]) / 10)
        r100 = float(np.mean([len(set(got[i]) & set(gt[i])) for i in range(args.nq)]) / args.k)
        st = min(sts, key=lambda s: s["total_ms"])
        w = min(walls)
        print(json.dumps({
            "search": sp, "rerank_all": args.rerank_all, "nq": args.nq, "k": args.k, "wall_ms": round(w, 3),
            "qps": round(args.nq / (w / 1e3), 1), "recall_at_10": round(r10, 4),
            "recall_at_100": round(r100, 4),
            **{key: (round(v, 4) if isinstance(v, float) else v) for key, v in st.items()},
            "scan_GBps": round(st["plane_bytes"] / (st["scan_ms"] * 1e-3) / 1e9, 1) if st["scan_ms"] > 0 else None,
        }), flush=True)
    idx.free()
    seg.free()


if __name__ == "__main__":
    main()
