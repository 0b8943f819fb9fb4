#!/usr/bin/env python3
"""Host CPU time of waiting threads.

The reference runs up to 2 x physical cores scans at once
(ScanThreadLimiter.h:25-58, MergeTreeVSManager.cpp:974-975); each waits for its
GPU work.  For every wait mode of mqvs_set_wait_mode and 1 / 16 / 64 threads,
each thread runs --reps searches of one case on the 10M x 768 cosine part
(host query arrays, as the ClickHouse seam passes them) and measures its own
CPU time (time.thread_time: the C call runs on the calling thread; ctypes
releases the GIL).  Prints one JSON line per (mode, case, threads):
  cpu_ms_per_search   thread CPU time per search
  wall_ms_per_search  the thread's wall time per search (latency under load)
  cpu_frac            sum of thread CPU / sum of thread wall
Cases: nq1, nq1000 (k 100) and sel1 (nq 1, a 1 % PREWHERE filter: the mid-call
wait for the selected-row count).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--threads", default="1,16,64")
    ap.add_argument("--modes", default="runtime,hybrid,block")
    ap.add_argument("--cases", default="nq1,nq1000,sel1,nq1000d")
    ap.add_argument("--reps", type=int, default=0, help="searches per thread (0: per case default)")
    ap.add_argument("--spin-us", type=int, default=50)
    args = ap.parse_args()
    import numpy as np
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device
    mq.init(0)
    seg = mq.VectorScanSegment.generate(0x5EED0001, 1, args.n, args.d, metric="Cosine", granule=8192)
    rng = np.random.default_rng(1)
    flt = mq.pack_bitmap(rng.random(args.n) < 0.01)
    queries = {}
    for nq in (1, 1000):  # held-out generator rows, as host arrays
        t = torch.empty((nq, args.d), dtype=torch.float32, device="cuda")
        generate_device(0x5EED0001, 1, args.n, nq, args.d, t)
        queries[nq] = t.cpu().numpy()
    cases = {"nq1": (1, None, 40), "nq1000": (1000, None, 4), "sel1": (1, flt, 60), "nq1000d": (1000, None, 4)}
    dq1000 = torch.from_numpy(queries[1000]).cuda()  # nq1000d: device queries and outputs (no host copies)
    modes = {"runtime": _lib.WAIT_RUNTIME, "hybrid": _lib.WAIT_HYBRID, "block": _lib.WAIT_BLOCK}
    # warm every path once (workspaces of the main thread, kernels loaded)
    for nq, f, _ in cases.values():
        seg.search(queries[nq], 100, filter_bitmap=f)
    seg.search(dq1000, 100)
    for mode in args.modes.split(","):
        _lib.set_wait_mode(modes[mode], args.spin_us)
        for case in args.cases.split(","):
            nq, f, reps = cases[case]
            reps = args.reps or reps
            for nt in (int(x) for x in args.threads.split(",")):
                cpu, wall, errs = [0.0] * nt, [0.0] * nt, []
                start = threading.Barrier(nt)

                def worker(i):
                    try:
                        mq.init(0)
                        qa = dq1000 if case == "nq1000d" else queries[nq]
                        seg.search(qa, 100, filter_bitmap=f)  # this thread's workspace
                        start.wait()
                        c0, w0 = time.thread_time(), time.perf_counter()
                        for _ in range(reps):
                            seg.search(qa, 100, filter_bitmap=f)
                        cpu[i] = time.thread_time() - c0
                        wall[i] = time.perf_counter() - w0
                        _lib.check(_lib.lib.mqvs_thread_release())
                    except Exception as e:  # noqa: BLE001
                        errs.append(repr(e))

                th = [threading.Thread(target=worker, args=(i,)) for i in range(nt)]
                t0 = time.perf_counter()
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                total = time.perf_counter() - t0
                rec = {"mode": mode, "spin_us": args.spin_us if mode == "hybrid" else None, "case": case,
                       "threads": nt, "reps": reps,
                       "cpu_ms_per_search": round(1e3 * sum(cpu) / (nt * reps), 4),
                       "wall_ms_per_search": round(1e3 * sum(wall) / (nt * reps), 4),
                       "cpu_frac": round(sum(cpu) / max(sum(wall), 1e-12), 4),
                       "qps_total": round(nt * reps * nq / total, 1), "errors": errs[:2]}
                print(json.dumps(rec), flush=True)
    _lib.set_wait_mode(_lib.WAIT_HYBRID, 50)


if __name__ == "__main__":
    main()
