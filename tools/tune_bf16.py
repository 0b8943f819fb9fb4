#!/usr/bin/env python3
"""A/B workgroup shapes / schedule variants of the pre-filter scans in ONE
process (interleaved rounds), on the bench workload (10M x 768 cosine,
nq=1000 by default).  A config is "WQ,QB,VAR" or "bf:WQ,QB,VAR" for the split-3
bf16 scan (kernels_bf16_scan.hip, MQVS_BF16_TUNE) and "mx:WQ,QB,VAR" for the
split-6 MX scan (kernels_mx.hip, MQVS_MX_TUNE); "mx:default" / "bf:default"
take the library's own choice; a suffix "@xG" sets MQVS_MX_XCD=G.  Every config must return the same bits as the
first.  Prints one JSON line per config: min / median main-scan ms and the
split-3-equivalent TFLOP/s (3 x 2 nq n d per scan, whatever the split)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--configs", default="2,4,0;2,4,4;2,4,7")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-check", action="store_true",
                    help="timing-only diagnostic variants (wrong results by design)")
    args = ap.parse_args()
    import torch
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device, set_timing
    mq.init(0)
    from myscaledb_amd.vector_scan import set_prefilter
    variants = args.configs.split(";")
    segs = {}
    for kind, split in (("bf", 3), ("mx", 6)):
        if any(v.startswith(kind + ":") or (kind == "bf" and ":" not in v) for v in variants):
            set_prefilter(split)
            segs[kind] = mq.VectorScanSegment.generate(0x5EED0001, 2, args.n, args.d, "Cosine", 8192)
    set_prefilter(2)
    q = torch.empty((args.nq, args.d), dtype=torch.float32, device="cuda")
    generate_device(0x5EED0002, 2, 0, args.nq, args.d, q)
    ref = None
    times = {v: [] for v in variants}
    rescans = {v: 0 for v in variants}
    set_timing(True)
    for rnd in range(args.rounds + 1):
        for v in variants:
            kind, cfg = v.split(":") if ":" in v else ("bf", v)
            env = "MQVS_MX_TUNE" if kind == "mx" else "MQVS_BF16_TUNE"
            os.environ.pop("MQVS_MX_TUNE", None)
            os.environ.pop("MQVS_BF16_TUNE", None)
            os.environ.pop("MQVS_MX_XCD", None)
            if "@x" in cfg:  # "@xG": MX workgroup -> XCD grouping G (kernels_mx.hip)
                cfg, g = cfg.split("@x")
                os.environ["MQVS_MX_XCD"] = g
            if cfg != "default":
                os.environ[env] = cfg
            ids, dist = segs[kind].search(q, args.k)
            st = _lib.last_search_stats()
            rescans[v] += st["rescans"]
            if ref is None:
                ref = (ids.clone(), dist.clone())
            elif not args.no_check and not (torch.equal(ids, ref[0]) and torch.equal(dist, ref[1])):
                print(json.dumps({"config": v, "error": "results differ from config %s" % variants[0]}),
                      flush=True)
                return 1
            if rnd > 0:
                times[v].append(st["main_ms"])
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    set_timing(False)
    flop = 3 * 2.0 * args.nq * (args.n - st["probe_rows"]) * args.d
    for v in variants:
        t = times[v]
        print(json.dumps({"config": v, "nq": args.nq, "main_ms_min": round(min(t), 3),
                          "main_ms_med": round(statistics.median(t), 3),
                          "bf16x3_TFLOPs_med": round(flop / (statistics.median(t) * 1e-3) / 1e12, 1),
                          "rescans": rescans[v]}), flush=True)
    for sg in segs.values():
        sg.free()
    return 0


if __name__ == "__main__":
    sys.exit(main())
