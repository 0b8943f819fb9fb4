#!/usr/bin/env python3
"""Rows in HBM vs in pinned host memory (mqvs_segment_set_rows_host) on the
bench part (10M x 768 cosine, N(0,1)): HBM bytes of the segment and the
search time at nq 1 / 16 / 1000 (median of --reps, device-resident queries),
results compared bit for bit.  One JSON line per (residency, nq)."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--nqs", default="1,16,1000")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd.vector_scan import generate_device
    mq.init(0)
    seg = mq.VectorScanSegment.generate(0x5EED0001, args.mode, args.n, args.d, "Cosine", 8192)
    want = {}
    try:
        for host in (False, True):
            seg.set_rows_host(host)
            info = seg.info()
            for nq in [int(x) for x in args.nqs.split(",")]:
                q = torch.empty((nq, args.d), dtype=torch.float32, device="cuda")
                generate_device(0x5EED0002, args.mode, 0, nq, args.d, q)
                ids = torch.empty((nq, args.k), dtype=torch.int64, device="cuda")
                dst = torch.empty((nq, args.k), dtype=torch.float32, device="cuda")
                seg.search(q, args.k, out=(ids, dst))
                torch.cuda.synchronize()
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    seg.search(q, args.k, out=(ids, dst))
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) * 1e3)
                got = (ids.cpu().numpy(), dst.cpu().numpy().view(np.uint32))
                if not host:
                    want[nq] = got
                same = bool(np.array_equal(got[0], want[nq][0]) and np.array_equal(got[1], want[nq][1]))
                print(json.dumps({"rows": "host" if host else "hbm", "nq": nq, "ms_median": round(statistics.median(ts), 3),
                                  "qps": round(nq / (statistics.median(ts) * 1e-3), 1),
                                  "segment_hbm_bytes": info["hbm_bytes"], "same_bits_as_hbm": same}), flush=True)
    finally:
        seg.free()


if __name__ == "__main__":
    main()
