#!/usr/bin/env python3
"""configs[4] gather-source A/B: at low PREWHERE
selectivity, the bf16-plane gather (pre-filter + exact re-rank; a gathered row
reads 24 x 64-B pieces, each half of a 128-B line shared with its block
neighbour) against the exact fp32 gather over the row-major rows (3072 B per
row = 24 whole lines, no pre-filter, no re-rank: MQVS_F_EXACT + forced
gather).  Same part and bitmap for both; the outputs must be bit-identical.
One JSON line per (selectivity, nq, path)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--sel", default="1,2,5,10")
    ap.add_argument("--nq", default="1,16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--k", type=int, default=100)
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device, pack_bitmap, set_timing
    mq.init(0)
    seg = mq.VectorScanSegment.generate(0x5EED0001, 1, args.n, args.d, "L2", 8192)
    attr = np.random.default_rng(0x5EED0003).integers(0, 100, size=args.n, dtype=np.uint8)
    for sel in [int(x) for x in args.sel.split(",")]:
        bm = torch.from_numpy(pack_bitmap(attr < sel)).cuda()
        for nq in [int(x) for x in args.nq.split(",")]:
            q = torch.empty((nq, args.d), dtype=torch.float32, device="cuda")
            generate_device(0x5EED0002, 1, 0, nq, args.d, q)
            outs = {}
            for path, kw in (("bf16_gather", {"gather": True}), ("fp32_gather", {"gather": True, "exact": True})):
                ids = torch.empty((nq, args.k), dtype=torch.int64, device="cuda")
                dst = torch.empty((nq, args.k), dtype=torch.float32, device="cuda")
                for _ in range(3):
                    seg.search(q, args.k, filter_bitmap=bm, out=(ids, dst), **kw)
                walls = []
                for _ in range(args.reps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    seg.search(q, args.k, filter_bitmap=bm, out=(ids, dst), **kw)
                    torch.cuda.synchronize()
                    walls.append((time.perf_counter() - t0) * 1e3)
                set_timing(True)
                sts = []
                for _ in range(5):
                    seg.search(q, args.k, filter_bitmap=bm, out=(ids, dst), **kw)
                    torch.cuda.synchronize()
                    sts.append(_lib.last_search_stats())
                set_timing(False)
                st = sorted(sts, key=lambda s: s["total_ms"])[2]
                outs[path] = (ids.cpu().numpy(), dst.cpu().numpy())
                sel_rows = int((attr < sel).sum())
                ms = float(np.median(walls))
                print(json.dumps({"sel_pct": sel, "nq": nq, "path": path, "ms": round(ms, 4),
                                  "main_ms": round(st["main_ms"], 4), "total_kernel_ms": round(st["total_ms"], 4),
                                  "stats_path": st["path"], "gather": st["gather"], "rows_scanned": st["rows_scanned"],
                                  "selected_rows": sel_rows,
                                  "bf16_plane_gbs_e2e": round(2.0 * sel_rows * 768 / (ms * 1e-3) / 1e9, 1),
                                  "fp32_rows_gbs_e2e": round(4.0 * sel_rows * args.d / (ms * 1e-3) / 1e9, 1)}),
                      flush=True)
            a, b = outs["bf16_gather"], outs["fp32_gather"]
            same = np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
            print(json.dumps({"sel_pct": sel, "nq": nq, "bitwise_equal": bool(same)}), flush=True)
    seg.free()


if __name__ == "__main__":
    main()
