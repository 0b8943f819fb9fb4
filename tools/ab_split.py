#!/usr/bin/env python3
"""A/B of the batch pre-filter splits on one GPU (10M x 768 by default): per
(metric, generator mode, nq) the wall time, kernel times and survivor counts of
each split, with the ids / distances of every split compared bit for bit to
the exact path (mqvs_set_batch_mode(1): fp32 MFMA for nq >= 20, the exact VALU
scan below).  One JSON line per (split, metric, mode, nq).
Env overrides per arm: --tunes 'MQVS_HI_TUNE=2,4,4;MQVS_HI_TUNE=2,4,3'."""
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
    ap.add_argument("--nqs", default="1,16,64,1000")
    ap.add_argument("--metrics", default="Cosine")
    ap.add_argument("--modes", default="2")
    ap.add_argument("--splits", default="2,6")
    ap.add_argument("--tunes", default="", help="';'-separated ENV=VALUE settings, each its own arm")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sels", default="", help="PREWHERE selectivities in percent (attr < T over a uniform attr "
                                               "in [0, 100), the configs[4] shape); empty: no filter")
    ap.add_argument("--no-exact", action="store_true")
    ap.add_argument("--qseed", type=lambda s: int(s, 0), default=0x5EED0002)
    ap.add_argument("--dbg", action="store_true",
                    help="load the measurement build libmqvs_dbg.so (reads MQVS_* A/B switches)")
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    if args.dbg:
        from myscaledb_amd import _lib as _mq_lib
        _mq_lib.use_measurement_build()
    from myscaledb_amd.vector_scan import generate_device, set_timing, set_prefilter, set_batch_mode, pack_bitmap
    mq.init(0)
    tunes = [t for t in args.tunes.split(";") if t] or [""]
    nqs = [int(x) for x in args.nqs.split(",")]
    for metric in args.metrics.split(","):
        for mode in [int(x) for x in args.modes.split(",")]:
            truth = {}
            for split in [int(x) for x in args.splits.split(",")]:
                set_prefilter(split)
                t0 = time.perf_counter()
                seg = mq.VectorScanSegment.generate(0x5EED0001, mode, args.n, args.d, metric, 8192)
                torch.cuda.synchronize()
                build_s = time.perf_counter() - t0
                attr = None
                sels = [int(x) for x in args.sels.split(",") if x] or [None]
                if sels != [None]:
                    attr = np.random.default_rng(0x5EED0003).integers(0, 100, size=args.n, dtype=np.uint8)
                for nq, sel in [(a, b) for a in nqs for b in sels]:
                    q = torch.empty((nq, args.d), dtype=torch.float32, device="cuda")
                    generate_device(args.qseed, mode, 0, nq, args.d, q)
                    kw = {}
                    if sel is not None:
                        kw["filter_bitmap"] = torch.from_numpy(pack_bitmap(attr < sel)).cuda()
                    if not args.no_exact and (nq, sel) not in truth:
                        set_batch_mode(1)
                        ids, dist = seg.search(q, args.k, **kw)
                        torch.cuda.synchronize()
                        truth[(nq, sel)] = (ids.cpu().numpy(), dist.cpu().numpy())
                        set_batch_mode(0)
                    for tune in tunes:
                        for kv in [x for x in tune.split("+") if x]:  # ('+' joins several settings)
                            key, val = kv.split("=", 1)
                            os.environ[key] = val
                        ids, dist = seg.search(q, args.k, **kw)
                        torch.cuda.synchronize()
                        same = None
                        if (nq, sel) in truth:
                            tr = truth[(nq, sel)]
                            same = bool(np.array_equal(ids.cpu().numpy(), tr[0]) and np.array_equal(
                                dist.cpu().numpy().view(np.uint32), tr[1].view(np.uint32)))
                        # walls without the per-kernel events; the breakdown from timed runs
                        walls, sts = [], []
                        for _ in range(args.reps):
                            torch.cuda.synchronize()
                            t0 = time.perf_counter()
                            seg.search(q, args.k, **kw)
                            torch.cuda.synchronize()
                            walls.append((time.perf_counter() - t0) * 1e3)
                        set_timing(True)
                        for _ in range(args.reps):
                            seg.search(q, args.k, **kw)
                            sts.append(_lib.last_search_stats())
                        set_timing(False)
                        for kv in [x for x in tune.split("+") if x]:
                            del os.environ[kv.split("=", 1)[0]]
                        st = min(sts, key=lambda s: s["total_ms"])
                        print(json.dumps({
                            "split": split, "tune": tune, "metric": metric, "mode": mode, "nq": nq, "sel": sel,
                            "n": args.n, "d": args.d, "k": args.k, "bitwise_eq_exact": same,
                            "wall_ms": round(min(walls), 3), "wall_med_ms": round(float(np.median(walls)), 3),
                            "qps": round(nq / (min(walls) / 1e3), 1),
                            "total_ms": round(st["total_ms"], 3), "main_ms": round(st["main_ms"], 3),
                            "probe_ms": round(st["probe_ms"], 3), "probe_select_ms": round(st["probe_select_ms"], 3),
                            "refine_ms": round(st["refine_ms"], 3), "final_ms": round(st["final_ms"], 3),
                            "segments": st["segments"], "path": st["path"], "prefilter": st["prefilter"],
                            "rescans": st["rescans"], "survivors_max": st["survivors_max"],
                            "survivors_mean": round(st["survivors_total"] / max(nq, 1), 1),
                            "candidates_max": st["candidates_max"], "seg_build_s": round(build_s, 2)}),
                            flush=True)
                seg.free()
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
