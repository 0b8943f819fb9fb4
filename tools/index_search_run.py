#!/usr/bin/env python3
"""One index workload for rocprofv3 PMC passes (tools/gpu_pmc.sh): a 10M x 768
cosine part of generator mode --mode, the MSTG-type index over it, then
--searches searches of --nq held-out queries at --search.
The k_ivf_scan counters / --searches are the per-search HBM bytes that
bench.py's index roofline takes as `traffic` (--index-pmc)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--search", default="nprobe=2")
    ap.add_argument("--searches", type=int, default=2)
    ap.add_argument("--info-out", default=None)
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd.vector_scan import generate_device
    mq.init(0)
    seed = 0x5EED0001
    seg = mq.VectorScanSegment.generate(seed, args.mode, args.n, args.d, "Cosine", 8192)
    idx = mq.VectorIndex.build(seg, "MSTG", "")
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    generate_device(seed, args.mode, args.n, args.nq, args.d, q)
    for _ in range(args.searches):
        idx.search(q, args.k, args.search)
    torch.cuda.synchronize()
    print("ok", args.mode, args.search, idx.info()["nlist"])
    if args.info_out:  # the index actually built (the summary records it; bench.py matches it)
        import json
        with open(args.info_out, "w") as f:
            json.dump({"mode": args.mode, "search": args.search, "nlist": idx.info()["nlist"]}, f)


if __name__ == "__main__":
    main()
