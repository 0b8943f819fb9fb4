#!/usr/bin/env python3
"""Column ingest on one GPU: a part's Array(Float32) column as ClickHouse LZ4
files (1 MiB blocks) -> resident segment.  Reports the GPU decode rate
(decompressed bytes / time of the decode + copy-loop kernels, HIP-event free:
wall time of mqvs_segment_create_from_column with the streams already in HBM,
minus a segment created from resident rows, i.e. the prepare step), and the
oracle's single-thread CPU decode of a sample (the reference reads and
decompresses a part single-threaded, VIWithDataPart.h:350)."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--kind", default="gauss,quantised")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dbg", action="store_true",
                    help="load the measurement build libmqvs_dbg.so (reads MQVS_* A/B switches)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import myscaledb_amd as mq
    if args.dbg:
        from myscaledb_amd import _lib as _mq_lib
        _mq_lib.use_measurement_build()
    from oracle import oracle as O
    mq.init(0)
    n, d = args.n, args.d
    block = 1 << 20
    for kind in args.kind.split(","):
        rng = np.random.default_rng(1)
        rows = rng.standard_normal((n, d), dtype=np.float32)
        if kind == "quantised":
            rows = np.round(rows, 1)
        raw = rows.tobytes()
        # compress 64-block slices in parallel (framing is per block, so the
        # concatenation equals one sequential stream)
        step = 64 * block
        with ThreadPoolExecutor(16) as ex:
            parts = list(ex.map(lambda o: O.compress_stream(raw[o:o + step], block), range(0, len(raw), step)))
        db = b"".join(parts)
        sb = O.compress_stream(np.full(n, d, np.uint64).tobytes(), block)
        tdb = torch.frombuffer(bytearray(db), dtype=torch.uint8).cuda()
        tsb = torch.frombuffer(bytearray(sb), dtype=torch.uint8).cuda()
        trows = torch.from_numpy(rows).cuda()
        torch.cuda.synchronize()
        best_col, best_rows, best_nov = 1e30, 1e30, 1e30
        for _ in range(args.reps):
            t0 = time.perf_counter()
            seg = mq.VectorScanSegment.from_column(tdb, tsb, n, d, metric="L2")
            best_col = min(best_col, time.perf_counter() - t0)
            seg.free()
            t0 = time.perf_counter()
            seg = mq.VectorScanSegment.from_column(tdb, tsb, n, d, metric="L2", verify_checksum=False)
            best_nov = min(best_nov, time.perf_counter() - t0)
            seg.free()
            t0 = time.perf_counter()
            seg = mq.VectorScanSegment.from_rows(trows, metric="L2")
            best_rows = min(best_rows, time.perf_counter() - t0)
            seg.free()
        decode = max(best_col - best_rows, 1e-9)
        t0 = time.perf_counter()
        sample = parts[0]
        O.decompress_stream(sample, step)
        cpu_s = time.perf_counter() - t0
        print(json.dumps({"kind": kind, "n": n, "d": d, "decompressed_bytes": len(raw), "compressed_bytes": len(db),
                          "ratio": round(len(raw) / len(db), 3), "from_column_s": round(best_col, 4),
                          "from_rows_s": round(best_rows, 4), "decode_s": round(decode, 4),
                          "from_column_no_checksum_s": round(best_nov, 4),
                          "checksum_s": round(max(best_col - best_nov, 0.0), 4),
                          "decode_GBps": round(len(raw) / decode / 1e9, 1),
                          "cpu_oracle_1thread_GBps": round(min(step, len(raw)) / cpu_s / 1e9, 3)}), flush=True)
        del tdb, tsb, trows


if __name__ == "__main__":
    main()
