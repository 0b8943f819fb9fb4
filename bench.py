#!/usr/bin/env python3
"""bench.py -- MI355X brute-force vector scan, BASELINE.json configs[1]:
FLAT cosine over 10M x 768 Float32, batch of 1000 queries, top-100.

One step = one batch search of `--nq` queries over the whole part (every rank
scans its granule-aligned row-range shard; with N > 1 the per-shard top-k are
all-gathered over RCCL and merged inside libmqvs, mqvs_sharded_search).  Strong
scaling: the 10M-row part is fixed and split over N GPUs.  Inputs are generated
in HBM (counter-based generator, the oracle's bit-identical twin) before the
timed region.

`--gpus N` (N > 1) without a launcher's WORLD_SIZE starts
`torch.distributed.run --nproc-per-node N` on this script as a CHILD process
before anything touches the GPU, and exits with its return code; rank 0's JSON
line reaches stdout through the inherited descriptor.  With N > 1 the line
also carries BASELINE configs[3] (FLAT IP, 1536-d, 12.5M rows per GPU: the
full 100M part at N = 8, a labelled 12.5M x N subset below) searched through
the same sharded path.

Prints ONE JSON line on rank 0 (see the driver contract in the task README).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

SEED_BASE, SEED_QUERY = 0x5EED0001, 0x5EED0002
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, f32 MFMA (= VALU) dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, bf16 MFMA dense peak (no sparsity)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, HBM3E spec peak
ROOT = os.path.dirname(os.path.abspath(__file__))
PMC_DEFAULT = "profiles/r05/pmc_traffic.json"
PMC_NQ1_DEFAULT = "profiles/r05/pmc_nq1.json"
BLAS_RISK_DEFAULT = "profiles/r03/blas_order_risk.json"


def seg_dpad(d):
    """Row stride (elements) of the resident bf16 planes (mqvs.hip, kBfK = 64)."""
    return (d + 63) // 64 * 64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch only: every rank prints its RANK / LOCAL_RANK / WORLD_SIZE and exits (no GPU)")
    ap.add_argument("--no-config3-sharded", action="store_true",
                    help="N > 1: skip the configs[3] (100M x 1536 IP over 8 GPUs) leg")
    ap.add_argument("--loopback", type=int, default=0,
                    help="rehearse the N-rank sequence of --gpus N on ONE GPU: N virtual ranks (threads) over a "
                         "loopback communicator (mqvs_comm_init_loopback); prints the N-rank lines")
    ap.add_argument("--config3-rows", type=int, default=0,
                    help="configs[3] rows per rank (default: 12.5M per GPU, the full 100M part at N = 8)")
    ap.add_argument("--inject-leg-failure", default="",
                    help="testing: 'config3:R' makes rank R fail the configs[3] leg (fail-soft drill)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--metric", default="Cosine")
    ap.add_argument("--mode", type=int, default=1, help="0 exact ints, 1 gauss, 2 gaussian mixture (4096 centres, noise 0.25), 3 hard mixture (65536 centres, noise 1.0)")
    ap.add_argument("--granule", type=int, default=8192)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the full-size exact-path comparison")
    ap.add_argument("--no-small", action="store_true", help="skip the nq = 1 / 4 / 16 / 64 sweep")
    ap.add_argument("--pmc", default=None, help="rocprofv3 PMC summary JSON for roofline.traffic")
    ap.add_argument("--pmc-nq1", default=None, help="rocprofv3 PMC summary JSON of the nq = 1 scan (roofline.nq1)")
    ap.add_argument("--no-index", action="store_true", help="skip the index (configs[2]) leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs[3] shard / configs[4] hybrid leg")
    ap.add_argument("--no-config1-points", action="store_true",
                    help="skip the extra configs[1] points (L2 metric, second distribution)")
    ap.add_argument("--read-sweep-gib", type=float, default=8.0,
                    help="buffer of the HBM read sweep (mqvs_measure_read_bandwidth); 0 = skip")
    ap.add_argument("--index-settings", default="nprobe=1;nprobe=2;nprobe=4;nprobe=8;nprobe=16",
                    help="';'-separated mqvs_index_search parameter strings timed by the index leg")
    ap.add_argument("--index-mode", type=int, default=2,
                    help="index distribution (generator mode; 2 = 4096 centres, noise 0.25)")
    ap.add_argument("--index-hard-mode", type=int, default=3,
                    help="second index distribution (generator mode, 3 = 65536 centres, noise 1.0; -1 = none)")
    ap.add_argument("--index-hard-settings",
                    default="nprobe=1;nprobe=2;nprobe=4;nprobe=8",
                    help="settings timed on the second distribution")
    ap.add_argument("--index-pmc", default=None,
                    help="JSON {mode: pmc_traffic.py output} of k_ivf_scan at each distribution's operating point")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# oracle-side helpers (CPU baseline leg + sample verification only)

def _oracle():
    from oracle import oracle as O
    return O


def verify_sample(O, ids, dist, q_host, args, n_probe_rows=20000):
    """Size-independent exactness check at full size: the returned distances
    are bit-identical to the oracle formula for those rows, and no sampled
    other row beats the k-th result (full reference key incl. ties)."""
    metric = O.METRICS[args.metric]
    rng = np.random.default_rng(1)
    blas = args.nq >= 20
    ok = True
    checked = 0
    for qi in (0, args.nq // 2):
        q = q_host[qi:qi + 1].copy()
        # cosine: the query re-normalised once per chunk (VIWithDataPart.h:358),
        # the chain followed to its repeat (mu, lambda) or to the last chunk
        variants, mu, lam = [], None, None
        if metric == O.COSINE:
            v, seen = q.copy(), {}
            for step in range(-(-args.n // args.granule)):
                v = O.normalize(v)
                key = v.tobytes()
                if key in seen:
                    mu, lam = seen[key], step - seen[key]
                    break
                seen[key] = step
                variants.append(v)

        def variant(chunk):
            if mu is None or chunk < mu:
                return variants[min(chunk, len(variants) - 1)]
            return variants[mu + (chunk - mu) % lam]

        def dist_of(rows_idx):
            rows = np.concatenate([O.generate(SEED_BASE, args.mode, int(r), 1, args.d)
                                   for r in rows_idx]) if len(rows_idx) else np.zeros((0, args.d), np.float32)
            out = []
            for r, y in zip(rows_idx, rows):
                if metric == O.COSINE:
                    yn = O.normalize(y[None, :])[0]
                    qv = variant(int(r) // args.granule)[0]
                    ip = O.gemm_dot(qv, yn) if blas else O.inner_product(qv, yn)
                    out.append((np.float32(1.0) - np.float32(ip), ip))
                elif metric == O.IP:
                    ip = O.gemm_dot(q[0], y) if blas else O.inner_product(q[0], y)
                    out.append((np.float32(ip), ip))
                else:
                    if blas:
                        xn, yn2 = O.norm_l2sqr(q[0]), O.norm_l2sqr(y)
                        dd = (xn + yn2) - np.float32(2.0) * O.gemm_dot(q[0], y)
                        dd = max(dd, np.float32(0))
                    else:
                        dd = O.l2sqr(q[0], y)
                    out.append((np.float32(dd), dd))
            return out

        got_ids = ids[qi]
        got = dist_of(got_ids[got_ids >= 0])
        for (dd, _), g in zip(got, dist[qi][got_ids >= 0]):
            ok &= np.float32(dd).view(np.uint32) == np.float32(g).view(np.uint32)
        # sampled challengers must not beat the k-th result
        kth_d = dist[qi][args.k - 1]
        sample = rng.choice(args.n, size=n_probe_rows, replace=False)
        sample = sample[~np.isin(sample, got_ids)]
        ch = dist_of(sample[:2000])
        for r, (dd, _) in zip(sample[:2000], ch):
            if metric == O.IP:
                ok &= not (dd > kth_d or (dd == kth_d and r < got_ids[args.k - 1]))
            else:
                ok &= not (dd < kth_d)
        checked += 1
    return bool(ok), checked


def host_cpu():
    """CPU model and physical core count of this host (lscpu -p, else
    /proc/cpuinfo), and the CPU share this process may use (affinity mask,
    capped by OMP_NUM_THREADS: the GPU box gives each GPU a 16-CPU share)."""
    import subprocess
    model, cores = "unknown", None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
        out = subprocess.run(["lscpu", "-p=SOCKET,CORE"], capture_output=True, text=True, timeout=10).stdout
        cores = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")}) or None
    except Exception:  # noqa: BLE001
        pass
    if cores is None or model == "unknown":
        try:
            seen, phys = set(), None
            with open("/proc/cpuinfo") as f:
                for line in f:
                    k, _, v = line.partition(":")
                    k, v = k.strip(), v.strip()
                    if k == "model name" and model == "unknown":
                        model = v
                    elif k == "physical id":
                        phys = v
                    elif k == "core id":
                        seen.add((phys, v))
            cores = cores or len(seen) or os.cpu_count()
        except OSError:
            cores = cores or os.cpu_count()
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return model, cores, share


def cpu_baseline(O, args):
    """The reference's CPU path restated by the oracle (bit-identical to it:
    faiss knn semantics, per-granule searchWrapper merge, cross-part merge),
    with its threading shape -- one thread per data part
    (VIWithDataPart.h:350), parts in parallel -- timed on a bounded row sample
    of the same workload and extrapolated per query to the full part.  The
    nq >= 20 distance chains run in an AVX-512 register-blocked micro-kernel
    (6 rows x 64 queries, still one fma chain per element).  Reported: the
    P-thread rate (P = min(physical cores, this process's CPU share)), the
    1-thread rate, the CPU model / core count and a STREAM triad figure."""
    model, phys, share = host_cpu()
    threads = max(1, min(phys or share, share))
    metric = O.METRICS[args.metric]
    q = O.generate(SEED_QUERY, args.mode, 0, args.nq, args.d)
    # one thread, one part of two granules
    rows1 = min(args.n, 2 * args.granule)
    base = O.generate(SEED_BASE, args.mode, 0, rows1, args.d)
    O.scan_parts(base[: args.granule], q, args.k, metric, args.granule, 1, 1)  # warm
    t0 = time.perf_counter()
    O.scan_parts(base, q, args.k, metric, args.granule, 1, 1)
    t1 = time.perf_counter() - t0
    one = args.nq * rows1 / t1
    # P parts x 1 thread
    rows = 4096 * threads
    base = O.generate(SEED_BASE, args.mode, 0, rows, args.d)
    t0 = time.perf_counter()
    O.scan_parts(base, q, args.k, metric, args.granule, threads, threads)
    t_cal = time.perf_counter() - t0
    target = int(rows * max(1.0, args.cpu_seconds / max(t_cal, 1e-3)))
    target = max(rows, min(target, 2_000_000, args.n))
    if target > rows:
        base = O.generate(SEED_BASE, args.mode, 0, target, args.d)
    reps, t = 0, 0.0
    while t < args.cpu_seconds and reps < 50:  # ~10-30 s of CPU work
        t0 = time.perf_counter()
        O.scan_parts(base, q, args.k, metric, args.granule, threads, threads)
        t += time.perf_counter() - t0
        reps += 1
    dist_per_s = args.nq * target * reps / t
    del base
    triad = O.stream_triad(1 << 26, threads, 5)
    return {
        "value": round(dist_per_s / args.n, 3),
        "unit": "queries/s (extrapolated to the full part)",
        "cores": threads,
        "kind": "port",
        "sample": f"{args.nq} queries x first {target} rows ({args.d}-d, {args.metric}) x {reps} passes, "
                  f"{threads} parts x 1 thread, {t:.1f} s; {dist_per_s / 1e6:.1f} M distances/s",
        "mdist_per_s": round(dist_per_s / 1e6, 2),
        "one_thread": {"qps": round(one / args.n, 3), "mdist_per_s": round(one / 1e6, 2),
                       "sample": f"{args.nq} queries x {rows1} rows, 1 part x 1 thread, {t1:.2f} s"},
        "cpu_model": model, "physical_cores": phys, "cpu_share": share,
        "avx512_microkernel": O.has_avx512(),
        "stream_triad_gbs": round(triad, 1), "stream_triad_threads": threads,
        "algorithmic_gflops": round(dist_per_s * 2 * args.d / 1e9, 1),
    }


INDEX_PMC_DEFAULT = os.path.join(ROOT, "profiles", "r05", "index_pmc.json")


def index_points(mq, seg, mode, settings, args):
    """An MSTG-type index (mqvs_index_build) over `seg`, searched with nq
    held-out generator rows of the same distribution, top-k.  Each setting:
    one warmup, then `steps` timed searches (device sync on both sides);
    recall@10 against the exact FLAT result of the same queries."""
    import torch
    from myscaledb_amd.vector_index import last_index_stats
    from myscaledb_amd.vector_scan import generate_device
    n, d, nq, k = seg.n, args.d, args.nq, args.k
    t0 = time.perf_counter()
    idx = mq.VectorIndex.build(seg, "MSTG", "")
    build_s = time.perf_counter() - t0
    info = idx.info()
    qi = torch.empty((nq, d), dtype=torch.float32, device="cuda")
    generate_device(SEED_BASE, mode, n, nq, d, qi)  # generator rows past the part
    gt = seg.search(qi, k)[0].cpu().numpy()
    ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    points = []
    from myscaledb_amd.vector_scan import set_timing
    for sp in [x for x in settings.split(";") if x]:
        idx.search(qi, k, sp, out=(ids, dst))
        torch.cuda.synchronize()
        # the per-stage kernel times from searches with the timing events on;
        # the wall-clock loop runs without them (as the FLAT legs)
        sts = []
        set_timing(True)
        try:
            for _ in range(3):
                idx.search(qi, k, sp, out=(ids, dst))
                sts.append(last_index_stats())
        finally:
            set_timing(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            idx.search(qi, k, sp, out=(ids, dst))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        got = ids.cpu().numpy()
        r10 = float(np.mean([len(set(got[i, :10]) & set(gt[i, :10])) for i in range(nq)]) / 10)
        st = min(sts, key=lambda x: x["total_ms"])
        points.append({"search": sp, "ms_per_search": round(ms, 3), "qps": round(nq / (ms * 1e-3), 1),
                       "recall_at_10": round(r10, 4),
                       "kernel_ms": {x: round(st[x + "_ms"], 4) for x in ("coarse", "plan", "scan", "select",
                                                                          "rerank")},
                       "scan_plane_bytes": st["plane_bytes"], "nprobe": st["nprobe"],
                       "num_reorder": st["num_reorder"]})
    idx.free()
    ok = [p for p in points if p["recall_at_10"] >= 0.95]
    best = max(ok, key=lambda p: p["qps"]) if ok else max(points, key=lambda p: p["recall_at_10"])
    scan_gbs = best["scan_plane_bytes"] / (best["kernel_ms"]["scan"] * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": "k_ivf_scan (bf16 MFMA list scan)",
            "achieved": round(scan_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(scan_gbs / HBM_PEAK_GBS, 4),
            "bytes_definition": "bf16 list-plane bytes per search (every work item streams its list)",
            "traffic": None}
    pmc_path = args.index_pmc or INDEX_PMC_DEFAULT
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pm = json.load(f).get(str(mode))
        ks = [v for key, v in (pm or {}).get("kernels", {}).items() if "k_ivf_scan" in key]
        same_index = pm is not None and pm.get("nlist") in (None, info["nlist"])  # (older summaries: no nlist)
        if ks and all("hbm_bytes_per_search" in v for v in ks) and pm.get("search") == best["search"] and same_index:
            # every k_ivf_scan launch of a search: the coarse quantizer's scan
            # of the centroids and the list scan (reads: list plane; writes:
            # one 8-B approximate value per (query, probed position))
            rd = sum(v["hbm_read_bytes_per_search"] for v in ks)
            wr = sum(v["hbm_write_bytes_per_search"] for v in ks)
            roof["traffic"] = round(rd + wr)
            roof["traffic_read"] = round(rd)
            roof["traffic_write"] = round(wr)
            roof["read_over_plane_bytes"] = round(rd / best["scan_plane_bytes"], 3)
            roof["traffic_source"] = os.path.relpath(pmc_path, ROOT)
    return {"generator_mode": mode, "qps": best["qps"], "recall_at_10": best["recall_at_10"],
            "search": best["search"], "meets_0_95": bool(ok), "build_s": round(build_s, 2), "nlist": info["nlist"],
            "index_hbm_bytes": info["hbm_bytes"], "roofline": roof, "points": points}


def index_leg(mq, seg, args):
    """BASELINE configs[2]: the index on a clustered distribution (mode 2:
    4096 centres; the bench part itself when it has that mode) and on a
    second, IVF-hostile one (mode 3: 65536 centres with noise as large as the
    centres) of the same size.  (On the bench's default N(0,1) part no
    partition index has recall: its neighbours carry no structure.)"""
    import torch
    n, d, nq, k = args.n, args.d, args.nq, args.k
    dists = []
    for mode, settings in ((args.index_mode, args.index_settings), (args.index_hard_mode, args.index_hard_settings)):
        if mode < 0 or any(x["generator_mode"] == mode for x in dists):
            continue
        if mode == args.mode:
            dists.append(index_points(mq, seg, mode, settings, args))
            continue
        hseg = mq.VectorScanSegment.generate(SEED_BASE, mode, n, d, args.metric, args.granule)
        try:
            dists.append(index_points(mq, hseg, mode, settings, args))
        finally:
            hseg.free()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    main = dists[0]
    return {
        "workload": f"MSTG-type IVF index, {n // 1_000_000}M x {d} {args.metric}, batch {nq}, top-{k}, "
                    "recall@10 >= 0.95 (BASELINE configs[2]); held-out queries of each distribution",
        **{x: main[x] for x in ("qps", "recall_at_10", "search", "build_s", "nlist", "index_hbm_bytes", "roofline",
                                "points", "generator_mode")},
        "distributions": dists,
    }


def _pmc_kernel(path, want, nq=None, sum_all=False):
    """The per-search PMC figures of kernel `want` from a committed
    tools/pmc_traffic.py summary (None when absent or for another nq).
    sum_all: the HBM bytes of every matching template (probe + main scan)."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pmc = json.load(f)
    if nq is not None and pmc.get("nq") not in (None, nq):
        return None
    hits = [(name, k) for name, k in pmc.get("kernels", {}).items() if want in name and "hbm_bytes_per_search" in k]
    if not hits:
        return None
    name, kinfo = max(hits, key=lambda h: h[1]["hbm_bytes_per_search"])
    out = dict(kinfo, kernel=name, source=os.path.relpath(path, ROOT))
    if sum_all:
        out["hbm_bytes_per_search"] = sum(k["hbm_bytes_per_search"] for _, k in hits)
        out["kernel"] = " + ".join(n for n, _ in hits)
    return out


def roofline(st, main_ms, nq, d, args):
    """The dominant kernel's roofline from one search's stats: all main-scan
    launches of the search, timed with HIP events on the search stream."""
    rows = st["main_rows"]
    dp = seg_dpad(d)
    sec = main_ms * 1e-3
    pf = st.get("prefilter", 0)
    want = None
    if st["path"] == 2 and pf == 2:
        # bf16-hi pre-filter (kernels_hi.hip / kernels_p4.hip): ONE bf16 MFMA
        # product per fp32 MAC over the row-blocked bf16 plane (2 B per element)
        plane = 2.0 * rows * dp
        flop = 2.0 * nq * rows * dp
        if nq <= 64:
            want = "k_scan_hi_reg" if nq <= 32 else "k_scan_hi<"
            kern = "k_scan_hi_reg (bf16 16x16x32, operands straight from HBM into registers)" if nq <= 32 else \
                "k_scan_hi<metric,APPEND,WQ=1,QB=2,NBUF=3>"
            roof = {"bound": "hbm", "kernel": kern, "achieved": round(plane / sec / 1e9, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(plane / sec / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                    "bytes_definition": "bf16 plane bytes of the scanned rows (2 * rows * dpad), read once"}
        else:
            qt = 256 if nq > 128 else 128
            stream = 2.0 * rows * dp * -(-nq // qt) + 2.0 * nq * dp * -(-rows // 256)
            if st.get("batch_kernel"):
                want = "k_scan_p4m"
                kern = ("k_scan_p4m<metric,NBUF=4> (one wave per SIMD, 128x128 rows x queries per wave as 8x8 blocks "
                        "of bf16 16x16x32, 256 AGPR accumulators, LDS-DMA ring)")
            else:
                want = "k_scan_hi<"
                kern = "k_scan_hi<metric,APPEND,WQ=2,QB=4,NBUF=4> (bf16 32x32x16)"
            roof = {"bound": "mfma", "kernel": kern,
                    "achieved": round(flop / sec / 1e12, 2), "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(flop / sec / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                    "flop_definition": "executed bf16 MFMA flops = 2 * nq * rows * dpad (hi * hi)",
                    "algorithmic_fp32_tflops": round(2.0 * nq * rows * d / sec / 1e12, 2),
                    "hbm_frac_plane": round(plane / sec / 1e9 / HBM_PEAK_GBS, 4),
                    "l2_to_lds_tb_s": round(stream / sec / 1e12, 2),
                    "l2_to_lds_bytes": stream}
        roof["per_search"] = {"rows": rows, "flop": flop, "plane_bytes": plane, "ms": round(main_ms, 3),
                              "launches": st["segments"]}
    elif st["path"] == 1:
        flop = 2.0 * nq * rows * d
        roof = {"bound": "mfma", "kernel": "k_scan_mfma (fp32, APPEND)", "achieved": round(flop / sec / 1e12, 2),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(flop / sec / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                "per_search": {"rows": rows, "flop": flop, "ms": round(main_ms, 3), "launches": st["segments"]}}
    else:
        byts = 4.0 * rows * d + 4.0 * nq * d
        roof = {"bound": "hbm", "kernel": "k_scan_small (APPEND)", "achieved": round(byts / sec / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(byts / sec / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None, "per_search": {"rows": rows, "bytes": byts, "ms": round(main_ms, 3)}}
    pm = _pmc_kernel(args.pmc or os.path.join(ROOT, PMC_DEFAULT), want, nq) if want else None
    if pm:
        # HBM bytes of the same kernel from a committed rocprofv3 --pmc run of
        # this workload (tools/gpu_pmc.sh + tools/pmc_traffic.py), per search
        roof["traffic"] = round(pm["hbm_bytes_per_search"])
        roof["traffic_unit"] = "HBM bytes per search (all main-scan launches)"
        roof["traffic_source"] = pm["source"]
        if "per_search" in roof and roof["per_search"].get("plane_bytes"):
            roof["traffic_over_plane"] = round(pm["hbm_bytes_per_search"] / roof["per_search"]["plane_bytes"], 3)
        for extra in ("clock_ghz", "mfma_busy_frac", "l2_hit_rate", "avg_launch_ms"):
            if extra in pm:
                roof["pmc_" + extra] = pm[extra]
    return roof


def exact_check(mq_scan, seg, q, k, ids, dst, **kw):
    """Outside the timed region: the same batch on the exact fp32 path
    (mqvs_set_batch_mode(1): fp32 MFMA fma chains over every row for nq >= 20,
    the faiss sequential formula below) and the timed path's output compared
    on ALL queries -- ids and distance bits -- plus recall@10 of the timed
    path against it."""
    mq_scan.set_batch_mode(1)
    try:
        ei, ed = seg.search(q, k, **kw)
    finally:
        mq_scan.set_batch_mode(0)
    gi, gd = ids.cpu().numpy(), dst.cpu().numpy()
    ei, ed = ei.cpu().numpy(), ed.cpu().numpy()
    k10 = min(10, k)
    r10 = float(np.mean([len(set(gi[i, :k10]) & set(ei[i, :k10])) for i in range(gi.shape[0])]) / k10)
    return {"queries": int(gi.shape[0]), "ids_equal": bool(np.array_equal(gi, ei)),
            "dist_bitwise_equal": bool(np.array_equal(gd.view(np.uint32), ed.view(np.uint32))),
            "recall_at_10": round(r10, 6)}


def small_batch_leg(mq_scan, seg, args, nqs=(1, 4, 16, 64), reps=10):
    """SURVEY 8(d) config 1 nq sweep below the batch: per nq, the end-to-end
    search time (device pointers, host sync per search), the main-scan kernel
    time, the HBM rate of the bf16 plane and its fraction of 8 TB/s, SURVEY's
    fp32 T* over T, and bit-equality with the exact path on every query."""
    import torch
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device
    n, d, k = args.n, args.d, args.k
    out = []
    for nq in nqs:
        q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
        generate_device(SEED_QUERY, args.mode, 0, nq, d, q)
        ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        for _ in range(3):
            seg.search(q, k, out=(ids, dst))
        # end-to-end walls without the per-kernel timing events; the kernel
        # breakdown (main-scan time) from separate timed searches
        walls, sts = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            seg.search(q, k, out=(ids, dst))
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
        mq_scan.set_timing(True)
        for _ in range(reps):
            seg.search(q, k, out=(ids, dst))
            torch.cuda.synchronize()
            sts.append(_lib.last_search_stats())
        mq_scan.set_timing(False)
        ms = float(np.median(walls))
        stt = sorted(sts, key=lambda s_: s_["total_ms"])[len(sts) // 2]
        chk = exact_check(mq_scan, seg, q, k, ids, dst)
        plane = 2.0 * n * seg_dpad(d) if stt["path"] == 2 and stt.get("prefilter") == 2 else 4.0 * n * d
        t_star = (4.0 * n * d + 4.0 * nq * d + 12.0 * nq * k) / (HBM_PEAK_GBS * 1e9) * 1e3
        out.append({"nq": nq, "ms_per_search": round(ms, 3), "qps": round(nq / (ms * 1e-3), 1),
                    "main_ms": round(stt["main_ms"], 3), "kernel_total_ms": round(stt["total_ms"], 3),
                    "path": stt["path"], "prefilter": stt.get("prefilter"),
                    "bytes_read": plane,
                    "main_gbs": round(plane * (stt["main_rows"] / n) / (stt["main_ms"] * 1e-3) / 1e9, 1),
                    "end_to_end_gbs": round(plane / (ms * 1e-3) / 1e9, 1),
                    "hbm_frac_main": round(plane * (stt["main_rows"] / n) / (stt["main_ms"] * 1e-3) / 1e9
                                           / HBM_PEAK_GBS, 4),
                    "hbm_frac_end_to_end": round(plane / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "survey_t_star_ms": round(t_star, 3), "survey_t_star_over_t": round(t_star / ms, 3),
                    "survivors_max": stt["survivors_max"],
                    "exact": chk})
    return out


def config1_points(mq, mq_scan, args):
    """Further configs[1] points: the same 10M x 768
    batch of 1000 under the L2 metric, and cosine on the other generator
    distribution (mode 2 when the headline runs mode 1), each on its own part
    generated in HBM after the main part is freed: QPS, main-scan time,
    survivors, rescans and the exact-path check on every query."""
    import torch
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import generate_device
    n, d, nq, k, g = args.n, args.d, args.nq, args.k, args.granule
    other = 2 if args.mode != 2 else 1
    out = []
    for metric, mode in (("L2", args.mode), (args.metric, other)):
        seg = mq.VectorScanSegment.generate(SEED_BASE, mode, n, d, metric, g)
        try:
            q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
            generate_device(SEED_QUERY, mode, 0, nq, d, q)
            ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
            dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
            for _ in range(2):
                seg.search(q, k, out=(ids, dst))
            walls, sts = [], []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                seg.search(q, k, out=(ids, dst))
                torch.cuda.synchronize()
                walls.append((time.perf_counter() - t0) * 1e3)
            mq_scan.set_timing(True)
            for _ in range(3):
                seg.search(q, k, out=(ids, dst))
                torch.cuda.synchronize()
                sts.append(_lib.last_search_stats())
            mq_scan.set_timing(False)
            ms = float(np.median(walls))
            st = sorted(sts, key=lambda s_: s_["total_ms"])[len(sts) // 2]
            flop = 2.0 * nq * st["main_rows"] * seg_dpad(d)
            out.append({"workload": f"FLAT {metric} {n // 1_000_000}M x {d}, batch {nq}, top-{k}, generator mode {mode}",
                        "metric": metric, "generator_mode": mode, "ms_per_search": round(ms, 3),
                        "qps": round(nq / (ms * 1e-3), 1), "main_ms": round(st["main_ms"], 3),
                        "main_bf16_frac": round(flop / (st["main_ms"] * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4),
                        "batch_kernel": st.get("batch_kernel"), "survivors_max": st["survivors_max"],
                        "survivors_mean": round(st["survivors_total"] / nq, 1), "candidates_max": st["candidates_max"],
                        "rescans": st["rescans"], "exact_check": exact_check(mq_scan, seg, q, k, ids, dst)})
        finally:
            seg.free()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    return out


def configs_leg(mq, mq_scan, args):
    """BASELINE configs[3] (one of the 8 granule-aligned row-range shards of
    the 100M x 1536 IP part: what each GPU of the 8-GPU configuration holds)
    and configs[4] (50M x 768 L2, PREWHERE attr < T at 100 / 50 / 10 / 1 %), on their
    own parts generated in HBM after the main part is freed.  Per point: the
    median end-to-end search time (device pointers), the main-scan time and
    the bf16-plane bytes it read, and the exact-path check on every query."""
    import torch
    from myscaledb_amd import _lib
    from myscaledb_amd.sharded import shard_rows
    from myscaledb_amd.vector_scan import generate_device, pack_bitmap
    k = 100

    def point(seg, nq, d, mode, reps, plane_rows, **kw):
        q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
        generate_device(SEED_QUERY, mode, 0, nq, d, q)
        ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        seg.search(q, k, out=(ids, dst), **kw)
        walls, sts = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            seg.search(q, k, out=(ids, dst), **kw)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
        mq_scan.set_timing(True)
        for _ in range(reps):
            seg.search(q, k, out=(ids, dst), **kw)
            torch.cuda.synchronize()
            sts.append(_lib.last_search_stats())
        mq_scan.set_timing(False)
        ms = float(np.median(walls))
        st = sorted(sts, key=lambda s_: s_["total_ms"])[len(sts) // 2]
        plane = 2.0 * plane_rows * seg_dpad(d)
        return {"nq": nq, "ms_per_search": round(ms, 3), "qps": round(nq / (ms * 1e-3), 1),
                "main_ms": round(st["main_ms"], 3), "gather": st["gather"], "rows_scanned": st["rows_scanned"],
                "plane_bytes_read": plane, "end_to_end_gbs": round(plane / (ms * 1e-3) / 1e9, 1),
                "rescans": st["rescans"], "exact": exact_check(mq_scan, seg, q, k, ids, dst, **kw)}

    out = {}
    d3 = 1536
    r0, r1 = shard_rows(100_000_000, args.granule, 3, 8)
    seg = mq.VectorScanSegment.generate(SEED_BASE, 1, r1 - r0, d3, "IP", args.granule, row_offset=r0)
    try:
        out["config3_shard"] = {
            "workload": f"FLAT IP, rows [{r0}, {r1}) of 100M x 1536 (one of 8 row-range shards), N(0,1), top-{k}",
            "points": [point(seg, nq, d3, 1, 5 if nq == 1000 else 10, r1 - r0) for nq in (1, 16, 1000)]}
    finally:
        seg.free()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    n4, d4 = 50_000_000, 768
    seg = mq.VectorScanSegment.generate(SEED_BASE, 1, n4, d4, "L2", args.granule)
    try:
        attr = np.random.default_rng(0x5EED0003).integers(0, 100, size=n4, dtype=np.uint8)
        pts = []
        for sel in (100, 50, 10, 1):  # SURVEY 8(d) config 4 sweep
            mask = attr < sel
            bm = torch.from_numpy(pack_bitmap(mask)).cuda()
            for nq in ((1, 16) if sel <= 10 else (1,)):
                e = point(seg, nq, d4, 1, 10, int(mask.sum()), filter_bitmap=bm)
                e["selectivity_pct"] = sel
                pts.append(e)
        out["config4_hybrid"] = {
            "workload": f"FLAT L2 50M x 768, WHERE attr < T (uniform attr in [0, 100)), top-{k}",
            "points": pts}
    finally:
        seg.free()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


# ---------------------------------------------------------------------------
# ranks: one process per GPU (torch.distributed) or, for the one-GPU
# rehearsal, one thread per virtual rank of a loopback communicator

class LegError(Exception):
    """A leg step failed on some rank: every rank raises it together."""


class DistCtx:
    """Rank of a torch.distributed job (one process per GPU)."""

    def __init__(self, rank, world):
        import torch.distributed as tdist
        self.tdist, self.rank, self.world = tdist, rank, world

    def barrier(self):
        self.tdist.barrier()

    def max(self, x):
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device="cuda")
        self.tdist.all_reduce(t, op=self.tdist.ReduceOp.MAX)
        return float(t.item())

    def all_ok(self, ok):
        return self.max(0.0 if ok else 1.0) == 0.0

    def first_error(self, err):
        """The lowest failing rank's error message (None when every rank is
        fine), the same on every rank."""
        objs = [None] * self.world
        self.tdist.all_gather_object(objs, err)
        return next((f"rank {r}: {e}" for r, e in enumerate(objs) if e), None)

    def process_wide(self, fn):
        fn()  # (every process holds its own library state)


class LoopShared:
    def __init__(self, n, timeout=900.0):
        import threading
        self.n = n
        self.bar = threading.Barrier(n, timeout=timeout)
        self.vals = [0.0] * n
        self.errs = [None] * n


class LoopCtx:
    """Virtual rank r of a loopback group: a thread of this process.  The
    library's process-wide switches (timing, batch mode) are set once by rank
    0 between barriers.  A barrier times out (BrokenBarrierError) rather than
    hang when a rank dies outside a step."""

    def __init__(self, shared, rank):
        self.sh, self.rank, self.world = shared, rank, shared.n

    def barrier(self):
        self.sh.bar.wait()

    def max(self, x):
        self.sh.vals[self.rank] = float(x)
        self.sh.bar.wait()
        m = max(self.sh.vals)
        self.sh.bar.wait()
        return m

    def all_ok(self, ok):
        return self.max(0.0 if ok else 1.0) == 0.0

    def first_error(self, err):
        self.sh.errs[self.rank] = err
        self.sh.bar.wait()
        e = next((f"rank {r}: {x}" for r, x in enumerate(self.sh.errs) if x), None)
        self.sh.bar.wait()
        return e

    def process_wide(self, fn):
        self.sh.bar.wait()
        if self.rank == 0:
            fn()
        self.sh.bar.wait()


def step_all(ctx, fn, what):
    """fn() on every rank, then one collective status: all ranks return, or
    all raise LegError together (a rank's failure before a collective would
    otherwise leave the others waiting in it)."""
    try:
        r, err = fn(), None
    except Exception as e:  # noqa: BLE001
        r, err = None, f"{what}: {type(e).__name__}: {e}"
    first = ctx.first_error(err)
    if first is not None:
        raise LegError(first)
    return r


def sharded_point(ctx, comm, seg, q, k, reps, mq_scan):
    """One batch size through mqvs_sharded_search on every rank: the first
    call runs the validated path, the timed ones the one-sync fast path; the
    time is the slowest rank's.  Then the same sharded search on the exact
    fp32 path of every rank (mqvs_set_batch_mode(1)) and the timed output
    compared with it on ALL queries (ids and distance bits, every rank)."""
    import torch
    nq = q.shape[0]
    ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    for _ in range(2):
        comm.sharded_search(seg, q, k, out=(ids, dst))
    before = comm.stats()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        comm.sharded_search(seg, q, k, out=(ids, dst))
    torch.cuda.synchronize()
    ms = ctx.max((time.perf_counter() - t0) * 1e3 / reps)
    after = comm.stats()
    ctx.process_wide(lambda: mq_scan.set_batch_mode(1))
    try:
        ei, ed = comm.sharded_search(seg, q, k)
    finally:
        ctx.process_wide(lambda: mq_scan.set_batch_mode(0))
    same = bool(torch.equal(ids, ei)) and bool(torch.equal(dst.view(torch.int32), ed.view(torch.int32)))
    all_same = ctx.max(0.0 if same else 1.0) == 0.0
    return {"nq": nq, "ms_per_search": round(ms, 3), "qps": round(nq / (ms * 1e-3), 1),
            "fast_path_calls": after["fast_calls"] - before["fast_calls"],
            "redo_calls": after["redo_calls"] - before["redo_calls"],
            "exact": {"queries": nq, "ids_and_dist_bits_equal_on_every_rank": all_same}}


def sharded_legs(ctx, mq, mq_scan, comm, seg, args):
    """N > 1, on every rank (collectives): the small batches of the configs[1]
    part through the sharded path, then BASELINE configs[3] -- FLAT IP over a
    1536-d part, 12.5M rows per GPU generated in HBM: the full 100M x 1536
    part at N >= 8, a 12.5M x N subset below (100M needs >= 8
    shards of this size; the loopback rehearsal uses --config3-rows per
    virtual rank) -- at nq 1 / 16 / 1000, each point checked against the exact
    path on every query.  A leg that fails on any rank is recorded as
    {"error": ...} on every rank (step_all) and the next leg runs."""
    import torch
    from myscaledb_amd.sharded import shard_rows
    from myscaledb_amd.vector_scan import generate_device
    rank, world = ctx.rank, ctx.world
    out = {}

    def small():
        pts = []
        for nq in (1, 16):
            q = step_all(ctx, lambda: _queries(args.mode, nq, args.d), "small-batch queries")
            e = step_all(ctx, lambda: sharded_point(ctx, comm, seg, q, args.k, 20, mq_scan), f"sharded nq {nq}")
            plane = 2.0 * args.n * seg_dpad(args.d)
            e["aggregate_plane_tb_s"] = round(plane / (e["ms_per_search"] * 1e-3) / 1e12, 3)
            pts.append(e)
        return pts

    try:
        out["small_batch_sharded"] = small()
    except LegError as e:
        out["small_batch_sharded"] = {"error": str(e)}
    if args.no_config3_sharded:
        return out
    d3 = 1536
    per = args.config3_rows or 12_500_000
    total = 100_000_000 if (world >= 8 and not args.config3_rows) else per * world
    r0, r1 = shard_rows(total, args.granule, rank, world)
    seg3 = None

    def gen3():
        if args.inject_leg_failure == f"config3:{rank}":
            raise RuntimeError("injected failure (--inject-leg-failure)")
        return mq.VectorScanSegment.generate(SEED_BASE, 1, r1 - r0, d3, "IP", args.granule, row_offset=r0)

    try:
        seg3 = step_all(ctx, gen3, "config3 shard generation")
        pts = []
        for nq in (1, 16, 1000):
            q = step_all(ctx, lambda: _queries(1, nq, d3), "config3 queries")
            e = step_all(ctx, lambda: sharded_point(ctx, comm, seg3, q, 100, 5 if nq == 1000 else 10, mq_scan),
                         f"config3 nq {nq}")
            plane = 2.0 * total * seg_dpad(d3)
            e["plane_bytes_read"] = plane
            e["aggregate_plane_tb_s"] = round(plane / (e["ms_per_search"] * 1e-3) / 1e12, 3)
            e["frac_of_n_x_8tbs"] = round(plane / (e["ms_per_search"] * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)
            pts.append(e)
        out["config3_sharded"] = {
            "workload": (f"FLAT IP {total / 1e6:g}M x {d3} (N(0,1)) over {world} ranks, top-100, "
                         + ("BASELINE configs[3] at full size" if total == 100_000_000 else
                            f"scaled subset of BASELINE configs[3]'s 100M rows: {per / 1e6:g}M rows per rank")),
            "rows": total, "rows_per_rank0": r1 - r0 if rank == 0 else None, "full_size": total == 100_000_000,
            "points": pts}
    except LegError as e:
        out["config3_sharded"] = {"error": str(e)}
    finally:
        if seg3 is not None:
            seg3.free()
        torch.cuda.synchronize()
    return out


def _queries(mode, nq, d):
    import torch
    from myscaledb_amd.vector_scan import generate_device
    q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
    generate_device(SEED_QUERY, mode, 0, nq, d, q)
    return q


def launch_ranks(args):
    """`--gpus N` run directly (the driver's N > 1 contract starts us under
    torch.distributed.run itself): start that launcher as a child process --
    never exec, and before any GPU call -- and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


# keys of the line's `roofline` kept first (the driver's record keeps about
# 20 keys of a nested dict): the north-star nq = 1 scalars right after the
# contract's own; everything else goes to `roofline_detail`
ROOF_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
             "nq1_frac_8tbs", "nq1_frac_end_to_end_8tbs", "nq1_ms", "nq1_ms_end_to_end", "nq1_pmc_over_plane",
             "nq1_exact", "traffic_over_plane", "pmc_mfma_busy_frac", "pmc_clock_ghz", "survey_t_star_over_t",
             "l2_to_lds_tb_s", "traffic_source", "flop_definition")


def split_roofline(roof):
    """(roofline with at most 20 keys in ROOF_KEYS order, the rest)."""
    head = {k: roof[k] for k in ROOF_KEYS if k in roof}
    if "kernel" in head and isinstance(head["kernel"], str) and len(head["kernel"]) > 100:
        head["kernel"] = head["kernel"][:97] + "..."
    rest = {k: v for k, v in roof.items() if k not in head or k == "kernel"}
    return head, rest


def emit(result):
    out = dict(result)
    if "roofline" in out:
        head, rest = split_roofline(out["roofline"])
        out["roofline"] = head
        out["roofline_detail"] = rest
    print(json.dumps(out), flush=True)


def run_leg(result, name, fn):
    """An optional single-GPU leg: its failure is recorded in the line
    instead of losing the line."""
    try:
        result[name] = fn()
    except Exception as e:  # noqa: BLE001
        result[name] = {"error": f"{type(e).__name__}: {e}"}
        import torch
        torch.cuda.synchronize()


def headline(args, ms, st, roof, exact, n_ranks, exchange, world, extra_config=None):
    n, d, nq, k, g = args.n, args.d, args.nq, args.k, args.granule
    qps = nq / (ms / 1000.0)
    pf = st.get("prefilter") if st["path"] == 2 else None
    compute = ("bf16-hi MFMA pre-filter (one bf16 product, rigorous error bound from measured residual norms) + "
               "exact f32 fma-chain re-rank of the survivors") if pf == 2 else (
        "f32 MFMA fma chain" if st["path"] == 1 else "f32 VALU, product then add")
    cfg = {"workload": f"FLAT {args.metric} {n // 1_000_000}M x {d} Float32, batch {nq}, "
                       f"top-{k} (BASELINE configs[1])",
           "n": n, "d": d, "nq": nq, "k": k, "metric": args.metric, "generator_mode": args.mode,
           "granule_rows": g, "parallelism": f"row-range shards x{world}", "exchange": exchange}
    cfg.update(extra_config or {})
    return {
        "metric": "QPS (FLAT brute force, batch top-k)",
        "value": round(qps, 2),
        "unit": "queries/s",
        "n_gpus": n_ranks,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "roofline": roof,
        "compute": compute,
        "data": "synthetic (counter-based %s, generated in HBM)" % {
            0: "exact integers in [-8, 8]", 1: "N(0,1)", 2: "gaussian mixture, 4096 centres",
            3: "gaussian mixture, 65536 centres, unit noise"}[args.mode],
        "config": cfg,
        "mdist_per_s": round(nq * n / (ms / 1000.0) / 1e6, 1),
        "recall_at_10": exact["recall_at_10"] if exact and "recall_at_10" in exact else None,
        "exact_check": exact,
        "stats_last_step": {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in st.items()},
    }


def rank_main(ctx, args, comm, exchange, loopback=0):
    """N > 1 (processes over RCCL, or threads over the loopback transport):
    each rank searches its granule-aligned row-range shard of the configs[1]
    part, the per-shard top-k are exchanged and merged inside libmqvs.  Rank
    0 prints the headline line as soon as it is measured, then the line again
    with the optional legs (a leg failing on any rank is recorded, not fatal)."""
    import torch
    import myscaledb_amd as mq
    import myscaledb_amd.vector_scan as mq_scan
    from myscaledb_amd import _lib
    from myscaledb_amd.sharded import shard_rows
    from myscaledb_amd.vector_scan import merge_shards
    rank, world = ctx.rank, ctx.world
    n, d, nq, k, g = args.n, args.d, args.nq, args.k, args.granule
    r0, r1 = shard_rows(n, g, rank, world)
    seg = mq.VectorScanSegment.generate(SEED_BASE, args.mode, r1 - r0, d, args.metric, g, row_offset=r0)
    q = _queries(args.mode, nq, d)
    f_ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    f_dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    if comm is None:
        # (torch.distributed fallback exchange: the library's communicator
        # could not be set up)
        import torch.distributed as tdist
        ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        g_ids = torch.empty((world, nq, k), dtype=torch.int64, device="cuda")
        g_dst = torch.empty((world, nq, k), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    def step():
        if comm is not None:
            comm.sharded_search(seg, q, k, out=(f_ids, f_dst))
            return
        seg.search(q, k, out=(ids, dst))
        tdist.all_gather_into_tensor(g_ids, ids)
        tdist.all_gather_into_tensor(g_dst, dst)
        merge_shards(g_ids, g_dst, args.metric, out=(f_ids, f_dst))

    for _ in range(args.warmup):
        step()
    ctx.process_wide(lambda: mq_scan.set_timing(True))
    before = comm.stats() if comm is not None else None
    stats = []
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        stats.append(_lib.last_search_stats())
    torch.cuda.synchronize()
    ctx.barrier()
    ms = ctx.max((time.perf_counter() - t0) * 1000.0 / args.steps)
    ctx.process_wide(lambda: mq_scan.set_timing(False))
    after = comm.stats() if comm is not None else None

    main_ms = float(np.mean([s["main_ms"] for s in stats]))
    st = stats[-1]
    roof = roofline(st, main_ms, nq, d, args)
    t_star = max((4.0 * n * d + 4.0 * nq * d + 12.0 * nq * k) / (HBM_PEAK_GBS * 1e9),
                 2.0 * nq * n * d / (FP32_MFMA_PEAK_TFLOPS * 1e12))
    roof["survey_t_star_ms"] = round(t_star * 1e3, 3)
    roof["survey_t_star_over_t"] = round(t_star * 1e3 / ms, 3)

    # exactness at full size, outside the timed region: the timed (merged)
    # output against the same sharded search on every rank's exact fp32 path
    exact = None
    if not args.no_verify:
        def check():
            ctx.process_wide(lambda: mq_scan.set_batch_mode(1))
            try:
                if comm is not None:
                    xi, xd = comm.sharded_search(seg, q, k)
                else:
                    ei, ed = seg.search(q, k)
                    tdist.all_gather_into_tensor(g_ids, ei)
                    tdist.all_gather_into_tensor(g_dst, ed)
                    xi, xd = merge_shards(g_ids, g_dst, args.metric)
            finally:
                ctx.process_wide(lambda: mq_scan.set_batch_mode(0))
            gi, gd, xi, xd = f_ids.cpu().numpy(), f_dst.cpu().numpy(), xi.cpu().numpy(), xd.cpu().numpy()
            k10 = min(10, k)
            return {"queries": nq, "ids_equal": bool(np.array_equal(gi, xi)),
                    "dist_bitwise_equal": bool(np.array_equal(gd.view(np.uint32), xd.view(np.uint32))),
                    "recall_at_10": round(float(np.mean([len(set(gi[i, :k10]) & set(xi[i, :k10]))
                                                         for i in range(nq)]) / k10), 6)}
        try:
            exact = step_all(ctx, check, "exact check")
        except LegError as e:
            exact = {"error": str(e)}

    result = None
    if rank == 0:
        extra = {"loopback_virtual_ranks": loopback} if loopback else {}
        result = headline(args, ms, st, roof, exact, 1 if loopback else world, exchange, world, extra)
        if loopback:
            result["metric"] = "QPS (FLAT brute force, batch top-k) -- loopback rehearsal of the N-rank path on 1 GPU"
            result["note"] = (f"{loopback} virtual ranks (threads) share ONE GPU: the value is not a scaling "
                              "point; it exercises the sharded code path end to end")
        if comm is not None:
            result["fast_path_calls"] = after["fast_calls"] - before["fast_calls"]
            result["redo_calls"] = after["redo_calls"] - before["redo_calls"]
        emit(result)  # the headline first: a later leg cannot lose it
    legs = sharded_legs(ctx, mq, mq_scan, comm, seg, args) if comm is not None else {}
    if rank == 0:
        result.update(legs)
        emit(result)
    ctx.barrier()
    seg.free()
    return 0


def loopback_main(args):
    """--loopback N: the N-rank sequence of `--gpus N` on ONE GPU -- one
    process, mqvs_comm_init_loopback(N), one thread (and HIP stream) per
    virtual rank, the exchange done as device copies by the same
    mqvs_sharded_search code an RCCL communicator runs."""
    import threading
    import torch
    torch.cuda.set_device(0)
    import myscaledb_amd as mq
    from myscaledb_amd import _lib
    from myscaledb_amd.sharded import LoopbackComm
    mq.init(0)
    if not args.config3_rows:
        args.config3_rows = 1_500_000  # (N virtual ranks share one GPU's HBM)
    comms = LoopbackComm.group(args.loopback)
    shared = LoopShared(args.loopback)
    errs = []

    def worker(r):
        try:
            mq.init(0)
            with torch.cuda.stream(torch.cuda.Stream()):
                rank_main(LoopCtx(shared, r), args, comms[r],
                          f"mqvs_sharded_search over a {args.loopback}-rank loopback communicator "
                          "(device copies between host barriers)", loopback=args.loopback)
            _lib.check(_lib.lib.mqvs_thread_release())
        except BaseException as e:  # noqa: BLE001
            errs.append(f"rank {r}: {type(e).__name__}: {e}")
            shared.bar.abort()

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(args.loopback)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for c in comms:
        c.free()
    if errs:
        print("\n".join(errs), file=sys.stderr, flush=True)
        return 1
    return 0


def single_main(args):
    import torch
    import myscaledb_amd as mq
    import myscaledb_amd.vector_scan as mq_scan
    from myscaledb_amd import _lib
    from myscaledb_amd.vector_scan import set_timing
    n, d, nq, k, g = args.n, args.d, args.nq, args.k, args.granule
    seg = mq.VectorScanSegment.generate(SEED_BASE, args.mode, n, d, args.metric, g)
    q = _queries(args.mode, nq, d)
    ids = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    dst = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        seg.search(q, k, out=(ids, dst))  # returns after its stream drained
    set_timing(True)
    stats = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        seg.search(q, k, out=(ids, dst))
        stats.append(_lib.last_search_stats())
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    set_timing(False)
    ms = (t1 - t0) * 1000.0 / args.steps

    main_ms = float(np.mean([s["main_ms"] for s in stats]))
    st = stats[-1]
    roof = roofline(st, main_ms, nq, d, args)
    # T* = max(bytes / HBM, flops / fp32 MFMA) for the whole step
    t_star = max((4.0 * n * d + 4.0 * nq * d + 12.0 * nq * k) / (HBM_PEAK_GBS * 1e9),
                 2.0 * nq * n * d / (FP32_MFMA_PEAK_TFLOPS * 1e12))
    roof["survey_t_star_ms"] = round(t_star * 1e3, 3)
    roof["survey_t_star_over_t"] = round(t_star * 1e3 / ms, 3)
    # exactness at full size, outside the timed region: the timed path's
    # output against the exact fp32 path on every query
    exact = None if args.no_verify else exact_check(mq_scan, seg, q, k, ids, dst)
    result = headline(args, ms, st, roof, exact, 1, None, 1)

    if args.read_sweep_gib > 0:
        # the measured HBM read peak of this device (same process, same GPU):
        # the denominator of frac_measured_peak below
        def sweep():
            gbs, bms = mq_scan.measure_read_bandwidth(int(args.read_sweep_gib * (1 << 30)), 5)
            return {"gbs": round(gbs, 1), "bytes": int(args.read_sweep_gib * (1 << 30)),
                    "best_ms": round(bms, 3), "frac_of_8tbs": round(gbs / HBM_PEAK_GBS, 4),
                    "kernel": "best of k_read_sweep (16 B per lane, 4 loads in flight, grid-stride, "
                              "8 workgroups per CU) and k_read_slices (a contiguous slice per "
                              "workgroup, 8 or 16 non-temporal 16-B loads in flight per lane, "
                              "2-8 workgroups per CU)"}
        run_leg(result, "hbm_read_sweep", sweep)
    if not args.no_small:
        run_leg(result, "small_batch", lambda: small_batch_leg(mq_scan, seg, args))
        p1 = [x for x in result["small_batch"] if x.get("nq") == 1] if isinstance(result["small_batch"], list) else []
        if p1:
            # the north-star nq = 1 point: HBM-bound scan of the
            # bf16 plane, against 8 TB/s and the measured read peak
            p1 = p1[0]
            plane = p1["bytes_read"]
            nq1 = {"ms": p1["main_ms"], "ms_end_to_end": p1["ms_per_search"], "plane_bytes": plane,
                   "kernel": "k_scan_hi_reg (bf16 16x16x32, operands straight from HBM into registers)",
                   "achieved_gbs": p1["main_gbs"], "frac_8tbs": p1["hbm_frac_main"],
                   "frac_end_to_end_8tbs": p1["hbm_frac_end_to_end"], "exact": p1["exact"]["ids_equal"] and
                   p1["exact"]["dist_bitwise_equal"]}
            sw = result.get("hbm_read_sweep")
            if isinstance(sw, dict) and "gbs" in sw:
                nq1["measured_peak_gbs"] = sw["gbs"]
                nq1["frac_measured_peak"] = round(p1["main_gbs"] / sw["gbs"], 4)
            pm = _pmc_kernel(args.pmc_nq1 or os.path.join(ROOT, PMC_NQ1_DEFAULT), "k_scan_hi_reg", 1, sum_all=True)
            if pm:
                nq1["pmc_hbm_bytes"] = round(pm["hbm_bytes_per_search"])
                nq1["pmc_over_plane"] = round(pm["hbm_bytes_per_search"] / plane, 4)
                nq1["pmc_source"] = pm["source"]
            result["roofline"]["nq1"] = nq1
            # (scalars in the roofline dict: the driver's record keeps its
            # first ~20 keys, ROOF_KEYS orders them)
            for key, val in (("nq1_ms", nq1["ms"]), ("nq1_ms_end_to_end", nq1["ms_end_to_end"]),
                             ("nq1_frac_8tbs", nq1["frac_8tbs"]),
                             ("nq1_frac_end_to_end_8tbs", nq1["frac_end_to_end_8tbs"]),
                             ("nq1_pmc_over_plane", nq1.get("pmc_over_plane")),
                             ("nq1_frac_measured_peak", nq1.get("frac_measured_peak")),
                             ("nq1_exact", nq1["exact"])):
                result["roofline"][key] = val
    if not args.no_cpu:
        # the CPU leg: the oracle (the reference's CPU path restated) timed on
        # the host cores, and -- as the checker only -- its formula on sampled
        # rows of the timed output (pins the exact path)
        def cpu():
            O = _oracle()
            cb = cpu_baseline(O, args)
            cb["one_thread_qps"] = cb["one_thread"]["qps"]
            if not args.no_verify:
                ok, nchk = verify_sample(O, ids.cpu().numpy(), dst.cpu().numpy(), q.cpu().numpy(), args)
                result["oracle_sample"] = {"queries": nchk, "bitwise_and_no_better_sample": ok}
            return cb
        run_leg(result, "cpu_baseline", cpu)
    if not args.no_index:
        run_leg(result, "index", lambda: index_leg(mq, seg, args))
    risk = os.path.join(ROOT, BLAS_RISK_DEFAULT)
    if os.path.exists(risk):
        # parity risk of the unpinned BLAS-branch order (tools/blas_order_risk.py,
        # committed run of this config): queries whose top-k would change if
        # faiss's sgemm blocked K
        with open(risk) as f:
            rk = json.load(f)
        result["blas_order_risk"] = dict(rk, source=os.path.relpath(risk, ROOT))
    seg.free()  # (room for the next parts)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if not args.no_config1_points:
        run_leg(result, "config1_points", lambda: config1_points(mq, mq_scan, args))
    if not args.no_configs:
        run_leg(result, "configs", lambda: configs_leg(mq, mq_scan, args))
    emit(result)


def main():
    args = parse()
    if args.loopback:
        if args.dry_run:
            print(json.dumps({"dry_run": True, "loopback": args.loopback}), flush=True)
            return
        sys.exit(loopback_main(args))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        print(json.dumps({"dry_run": True, "rank": rank, "local_rank": local, "world_size": world,
                          "gpus_arg": args.gpus}), flush=True)
        return
    import torch
    torch.cuda.set_device(local)
    import myscaledb_amd as mq
    if world == 1:
        mq.init(local)
        single_main(args)
        return
    import torch.distributed as tdist
    tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    mq.init(local)
    # libmqvs's own exchange (mqvs_sharded_search: RCCL all-gather of the
    # per-shard top-k + device merge); torch.distributed's all_gather +
    # mqvs_merge_shards if that communicator cannot be set up
    comm, exchange = None, None
    try:
        from myscaledb_amd.sharded import RcclComm
        comm = RcclComm.from_process_group()
        exchange = (f"mqvs_sharded_search (libmqvs RCCL communicator of {comm.nranks} ranks: header all-gather + "
                    "one group of per-rank top-k all-gathers, device merge, one host sync per search)")
    except Exception as e:  # noqa: BLE001
        comm, exchange = None, f"torch.distributed all_gather + mqvs_merge_shards ({type(e).__name__})"
    try:
        rank_main(DistCtx(rank, world), args, comm, exchange)
    finally:
        if comm is not None:
            comm.free()
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
