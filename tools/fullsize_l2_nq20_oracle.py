#!/usr/bin/env python3
"""configs[1]'s part under L2 at nq 20 (the BLAS-branch formula) against the
oracle's scan of 16 row-range parts on 16 threads, merged by the reference's
cross-part merge: ids and distance bits.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd.vector_scan import generate_device
    from oracle import oracle as O
    mq.init(0)
    n, d, k, mode, nq = 10_000_000, 768, 100, 1, 20
    seg = mq.VectorScanSegment.generate(0x5EED0001, mode, n, d, "L2", 8192)
    q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
    generate_device(0x5EED0002, mode, 0, nq, d, q)
    gi, gd = seg.search(q, k)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    seg.free()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    rows = np.empty((n, d), np.float32)
    step = 1 << 20
    t = torch.empty((step, d), dtype=torch.float32, device="cuda")
    for r0 in range(0, n, step):
        m = min(step, n - r0)
        generate_device(0x5EED0001, mode, r0, m, d, t[:m])
        rows[r0:r0 + m] = t[:m].cpu().numpy()
    oi, od = O.scan_parts(rows, q.cpu().numpy(), k, O.L2, 8192, 16, 16)
    print(json.dumps({"ids_equal": bool(np.array_equal(gi, oi)),
                      "dist_bitwise_equal": bool(np.array_equal(gd.view(np.uint32), od.view(np.uint32))),
                      "id_mismatch_slots": int((gi != oi).sum())}), flush=True)


if __name__ == "__main__":
    main()
