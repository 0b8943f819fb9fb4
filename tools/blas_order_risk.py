#!/usr/bin/env python3
"""Parity risk of the unpinned BLAS-branch summation order.

The oracle restates faiss's BLAS branch (nq >= 20, exhaustive_*_blas,
BruteForceSearch.h:80-87) as ONE fp32 fma chain over k per element
(oracle/mqvs_oracle.c, orc_gemm_dot).  A real sgemm may block K.  This tool
counts, for a configs[1]-shaped search, the queries whose top-k ids or
distance bits change when every element is instead summed in K blocks of 64
or 256 (each block an fma chain, the blocks added in order:
orc_gemm_dot_blocked).

Method: the exact fp32 path (mqvs_set_batch_mode(1)) returns each query's
top-kc (kc > k) under the chain.  Every candidate's chain value is recomputed
on the CPU (must equal the GPU's bits) and so are its blocked values; the
top-k under each order is re-selected from the kc candidates with the
reference key (distance, then row id).  Rows outside the top-kc cannot enter:
the tool checks, per query, that the gap between the k-th and kc-th chain
distances exceeds twice the largest |chain - blocked| difference seen, and
reports how many queries satisfy it.

  python tools/blas_order_risk.py --n 10000000 --nq 1000 --out profiles/r03/blas_order_risk.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED_BASE, SEED_QUERY = 0x5EED0001, 0x5EED0002


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--kc", type=int, default=160)
    ap.add_argument("--metric", default="Cosine")
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--granule", type=int, default=8192)
    ap.add_argument("--blocks", default="64,256")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from oracle import oracle as O
    import myscaledb_amd as mq
    from myscaledb_amd.vector_scan import set_batch_mode
    mq.init(0)
    t0 = time.time()
    seg = mq.VectorScanSegment.generate(SEED_BASE, args.mode, args.n, args.d, args.metric, args.granule)
    q = O.generate(SEED_QUERY, args.mode, 0, args.nq, args.d)
    set_batch_mode(1)
    try:
        ids, dist = seg.search(q, args.kc, args.metric)
    finally:
        set_batch_mode(0)
        seg.free()
    t_gpu = time.time() - t0
    metric = O.METRICS[args.metric]
    blocks = [int(b) for b in args.blocks.split(",")]
    changed_ids = {b: 0 for b in blocks}
    changed_bits = {b: 0 for b in blocks}
    changed_slots = {b: 0 for b in blocks}
    max_diff = {b: 0.0 for b in blocks}
    chain_mismatch = 0
    window_ok = 0
    nchunks = -(-args.n // args.granule)
    t1 = time.time()
    for qi in range(args.nq):
        x = q[qi:qi + 1]
        variants, mu, lam = [], None, None
        if metric == O.COSINE:
            v, seen = x.copy(), {}
            for step in range(nchunks):
                v = O.normalize(v)
                key = v.tobytes()
                if key in seen:
                    mu, lam = seen[key], step - seen[key]
                    break
                seen[key] = step
                variants.append(v)

        def variant(chunk):
            if mu is None or chunk < mu:
                return variants[min(chunk, len(variants) - 1)][0]
            return variants[mu + (chunk - mu) % lam][0]

        cand = ids[qi]
        cand = cand[cand >= 0]
        vals = {"chain": []}
        for b in blocks:
            vals[b] = []
        for r in cand:
            y = O.generate(SEED_BASE, args.mode, int(r), 1, args.d)[0]
            if metric == O.COSINE:
                y = O.normalize(y[None, :])[0]
                xv = variant(int(r) // args.granule)
            else:
                xv = x[0]
            for key in ["chain"] + blocks:
                ip = O.gemm_dot(xv, y) if key == "chain" else O.gemm_dot_blocked(xv, y, key)
                if metric == O.COSINE:
                    dd = np.float32(1.0) - ip
                elif metric == O.IP:
                    dd = ip
                else:
                    xn, yn = O.norm_l2sqr(xv), O.norm_l2sqr(y)
                    dd = max((xn + yn) - np.float32(2.0) * ip, np.float32(0))
                vals[key].append(np.float32(dd))

        def topk(v):
            v = np.asarray(v, np.float32)
            order = sorted(range(len(cand)), key=(lambda i: (-v[i], cand[i])) if metric == O.IP
                           else (lambda i: (v[i], cand[i])))[:args.k]
            return cand[order], v[order]

        ci, cd = topk(vals["chain"])
        gi, gd = ids[qi][:args.k], dist[qi][:args.k]
        if not (np.array_equal(ci, gi) and np.array_equal(cd.view(np.uint32), gd.view(np.uint32))):
            chain_mismatch += 1
        worst = 0.0
        for b in blocks:
            bi, bd = topk(vals[b])
            diff = float(np.max(np.abs(np.asarray(vals[b], np.float64) - np.asarray(vals["chain"], np.float64))))
            worst = max(worst, diff)
            max_diff[b] = max(max_diff[b], diff)
            if not np.array_equal(bi, ci):
                changed_ids[b] += 1
            if not np.array_equal(bd.view(np.uint32), cd.view(np.uint32)):
                changed_bits[b] += 1
            changed_slots[b] += int(np.sum((bi != ci) | (bd.view(np.uint32) != cd.view(np.uint32))))
        if len(cand) >= args.kc:
            gap = abs(float(dist[qi][args.kc - 1]) - float(dist[qi][args.k - 1]))
            window_ok += gap > 2 * worst
    res = {
        "config": {"n": args.n, "d": args.d, "nq": args.nq, "k": args.k, "metric": args.metric,
                   "generator_mode": args.mode, "granule_rows": args.granule, "candidates_per_query": args.kc},
        "model": "sgemm K blocking: each K block an fp32 fma chain from zero, blocks added in order "
                 "(orc_gemm_dot_blocked); reference assumption = one fma chain (orc_gemm_dot)",
        "chain_recompute_mismatches": chain_mismatch,
        "window_ok_queries": window_ok,
        "per_block": {str(b): {"queries_ids_changed": changed_ids[b], "queries_bits_changed": changed_bits[b],
                               "slots_changed": changed_slots[b], "slots_total": args.nq * args.k,
                               "max_abs_distance_diff": max_diff[b]} for b in blocks},
        "seconds": {"gpu": round(t_gpu, 1), "cpu": round(time.time() - t1, 1)},
    }
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        os.makedirs(os.path.dirname(os.path.join(ROOT, args.out)), exist_ok=True)
        with open(os.path.join(ROOT, args.out), "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
