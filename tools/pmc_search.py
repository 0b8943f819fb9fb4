#!/usr/bin/env python3
"""A fixed number of searches for rocprofv3 --pmc passes (tools/gpu_pmc.sh):
one warm-up, then --searches timed ones, on a part generated in HBM.  Pass
--searches + 1 to tools/pmc_traffic.py.

  bash tools/gpu_pmc.sh python tools/pmc_search.py --nq 1 --searches 4
  python tools/pmc_traffic.py gpurun_out --searches 5 --nq 1 --out profiles/r03/pmc_nq1.json
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SEED_BASE, SEED_QUERY = 0x5EED0001, 0x5EED0002


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--metric", default="Cosine")
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--granule", type=int, default=8192)
    ap.add_argument("--searches", type=int, default=2)
    ap.add_argument("--selectivity", type=int, default=None,
                    help="PREWHERE attr < T over a uniform attr in [0, 100) (configs[4] shape)")
    ap.add_argument("--dbg", action="store_true",
                    help="load the measurement build libmqvs_dbg.so (reads MQVS_* A/B switches)")
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    if args.dbg:
        from myscaledb_amd import _lib as _mq_lib
        _mq_lib.use_measurement_build()
    from myscaledb_amd.vector_scan import generate_device, pack_bitmap
    mq.init(0)
    seg = mq.VectorScanSegment.generate(SEED_BASE, args.mode, args.n, args.d, args.metric, args.granule)
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    generate_device(SEED_QUERY, args.mode, 0, args.nq, args.d, q)
    kw = {}
    if args.selectivity is not None:
        attr = np.random.default_rng(0x5EED0003).integers(0, 100, size=args.n, dtype=np.uint8)
        kw["filter_bitmap"] = torch.from_numpy(pack_bitmap(attr < args.selectivity)).cuda()
    ids = torch.empty((args.nq, args.k), dtype=torch.int64, device="cuda")
    dst = torch.empty((args.nq, args.k), dtype=torch.float32, device="cuda")
    for _ in range(args.searches + 1):
        seg.search(q, args.k, out=(ids, dst), **kw)
    torch.cuda.synchronize()
    seg.free()
    print(f"pmc_search: {args.searches + 1} searches, nq {args.nq}, {args.metric}, n {args.n}", flush=True)


if __name__ == "__main__":
    main()
