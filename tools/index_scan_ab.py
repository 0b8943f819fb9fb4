#!/usr/bin/env python3
"""A/B of index-search switches on one built index (measurement build
libmqvs_dbg.so, which reads MQVS_* variables per call): a 10M x 768 cosine
part of generator mode --mode, the MSTG-type index over it, then for each
';'-separated setting of --tunes (comma-separated VAR=value pairs, "" = the
defaults) --reps batches of --nq queries at --search, interleaved round-robin
so clock drift hits every setting alike.  Prints one JSON line per setting:
median / min wall per batch, the per-stage times of a timed batch, and
whether ids and distances equal the first setting's bit for bit."""
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
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--mode", type=int, default=3)
    ap.add_argument("--search", default="nprobe=1")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--tunes", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from myscaledb_amd import _lib
    _lib.use_measurement_build()
    import myscaledb_amd as mq
    from myscaledb_amd.vector_index import last_index_stats
    from myscaledb_amd.vector_scan import generate_device, set_timing
    mq.init(0)
    seed = 0x5EED0001
    seg = mq.VectorScanSegment.generate(seed, args.mode, args.n, args.d, "Cosine", 8192)
    idx = mq.VectorIndex.build(seg, "MSTG", "")
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    generate_device(seed, args.mode, args.n, args.nq, args.d, q)
    tunes = [t.strip() for t in args.tunes.split(";")]
    envs = []
    for t in tunes:
        e = {}
        for kv in filter(None, t.split(",")):
            k, v = kv.split("=")
            e[k.strip()] = v.strip()
        envs.append(e)
    keys = sorted({k for e in envs for k in e})

    def apply(e):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(e)

    walls = [[] for _ in envs]
    stages, outs = [], []
    for i, e in enumerate(envs):
        apply(e)
        for _ in range(2):
            ids, dist = idx.search(q, args.k, args.search)
        torch.cuda.synchronize()
        outs.append((ids.cpu().numpy(), dist.cpu().numpy()))
        set_timing(True)
        idx.search(q, args.k, args.search)
        torch.cuda.synchronize()
        stages.append(last_index_stats())
        set_timing(False)
    for _ in range(args.reps):
        for i, e in enumerate(envs):
            apply(e)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.search(q, args.k, args.search)
            torch.cuda.synchronize()
            walls[i].append((time.perf_counter() - t0) * 1e3)
    for i, t in enumerate(tunes):
        st = stages[i]
        print(json.dumps({
            "tune": t, "mode": args.mode, "search": args.search, "nlist": idx.info()["nlist"],
            "wall_med_ms": round(float(np.median(walls[i])), 4), "wall_min_ms": round(min(walls[i]), 4),
            "qps_med": round(args.nq / np.median(walls[i]) * 1e3),
            "coarse_ms": round(st["coarse_ms"], 4), "plan_ms": round(st["plan_ms"], 4),
            "scan_ms": round(st["scan_ms"], 4), "select_ms": round(st["select_ms"], 4),
            "rerank_ms": round(st["rerank_ms"], 4), "items": st["items"],
            "bitwise_eq_first": bool(np.array_equal(outs[i][0], outs[0][0])
                                     and np.array_equal(outs[i][1].view(np.uint32), outs[0][1].view(np.uint32))),
        }), flush=True)


if __name__ == "__main__":
    main()
