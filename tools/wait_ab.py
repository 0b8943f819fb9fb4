#!/usr/bin/env python3
"""End-to-end latency of the bench's fixed-cost points under each host wait
mode (mqvs_set_wait_mode): configs[4] 1 % (50M x 768 L2, nq 1, device
pointers) and configs[1] nq 1 (10M x 768 cosine), timed as bench.py times
them (torch.cuda.synchronize() around each search, median of --reps),
the modes interleaved round-robin so clock drift hits each alike."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cases", default="sel1,nq1")
    a = ap.parse_args()
    import numpy as np
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device
    mq.init(0)
    modes = {"runtime": _lib.WAIT_RUNTIME, "hybrid": _lib.WAIT_HYBRID, "block": _lib.WAIT_BLOCK}
    k = 100
    for case in a.cases.split(","):
        if case == "sel1":
            n, d, metric, gmode = 50_000_000, 768, "L2", 1
        else:
            n, d, metric, gmode = 10_000_000, 768, "Cosine", 1
        seg = mq.VectorScanSegment.generate(0x5EED0001, gmode, n, d, metric=metric, granule=8192)
        kw = {}
        if case == "sel1":
            rng = np.random.default_rng(3)
            kw["filter_bitmap"] = torch.from_numpy(mq.pack_bitmap(rng.random(n) < 0.01)).cuda()
        q = torch.empty((1, d), dtype=torch.float32, device="cuda")
        generate_device(0x5EED0002, gmode, 0, 1, d, q)
        ids = torch.empty((1, k), dtype=torch.int64, device="cuda")
        dst = torch.empty((1, k), dtype=torch.float32, device="cuda")
        res = {m: [] for m in modes}
        for _ in range(a.rounds):
            for m, v in modes.items():
                _lib.set_wait_mode(v, 50)
                seg.search(q, k, out=(ids, dst), **kw)
                for _ in range(a.reps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    seg.search(q, k, out=(ids, dst), **kw)
                    torch.cuda.synchronize()
                    res[m].append((time.perf_counter() - t0) * 1e3)
        _lib.set_wait_mode(_lib.WAIT_HYBRID, 50)
        print(json.dumps({"case": case, **{m: round(float(np.median(v)), 4) for m, v in res.items()},
                          **{m + "_p10": round(float(np.percentile(v, 10)), 4) for m, v in res.items()}}), flush=True)
        seg.free()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
