"""Multi-GPU decomposition (myscaledb_amd/sharded.py) on CPU:
granule-aligned row-range shards, per-shard bitmap slices, the all-gather of
per-shard top-k and the cross-part merge -- world_size 2 over gloo, local
searches and merges done by the oracle.  The sharded answer must equal the
single-part oracle scan bit for bit (L2 / IP; cosine shards are covered on
the GPU by test_gpu_parity.py::test_merge_shards_matches_single_part)."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O


def test_shard_rows_cover_part():
    from myscaledb_amd.sharded import shard_rows
    for n, g, w in ((10_000_000, 8192, 8), (12345, 512, 3), (100, 1000, 4), (0, 64, 2), (4096, 4096, 2)):
        prev = 0
        for r in range(w):
            r0, r1 = shard_rows(n, g, r, w)
            assert r0 == prev and r0 <= r1 and (r0 % g == 0 or r0 == n)
            prev = r1
        assert prev == n


def test_slice_bitmap():
    from myscaledb_amd.sharded import slice_bitmap
    rng = np.random.default_rng(0)
    n = 1003
    bits = rng.random(n) > 0.5
    packed = np.packbits(bits, bitorder="little")
    for r0, r1 in ((0, 1003), (8, 500), (16, 1003), (3, 77), (512, 1000)):
        got = np.unpackbits(slice_bitmap(packed, n, r0, r1), bitorder="little")[:r1 - r0]
        assert np.array_equal(got, bits[r0:r1].astype(np.uint8)), (r0, r1)
    assert slice_bitmap(None, n, 0, 5) is None


N, D, NQ, K, GRAN = 9000, 24, 7, 30, 1024
FLT_MAX = np.float32(3.4028235e38)


def _part(metric_mode):
    rows = O.generate(71, metric_mode, 0, N, D)
    q = O.generate(72, metric_mode, 0, NQ, D)
    rng = np.random.default_rng(9)
    flt = np.packbits(rng.random(N) > 0.25, bitorder="little")
    rex = np.packbits(rng.random(N) > 0.1, bitorder="little")
    return rows, q, flt, rex


def _worker(rank, world, port, metric, mode, use_bitmaps, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from myscaledb_amd.sharded import ShardedScan
        rows, q, flt, rex = _part(mode)
        if not use_bitmaps:
            flt = rex = None

        scan = None

        def local(queries, k, f, e):
            r0, r1 = scan.r0, scan.r1
            ids, dist_ = O.vector_scan(rows[r0:r1], queries, k, metric, GRAN, filter_bits=f,
                                       row_exists_bits=e)
            return np.where(ids >= 0, ids + r0, -1), dist_

        def merge(si, sd):
            # row-range shards of ONE part: (distance, row) order, i.e. what
            # mqvs_merge_shards does by default (not the cross-part multimap,
            # which reverses exact IP ties)
            nq, k = si.shape[1], si.shape[2]
            oi = np.full((nq, k), -1, np.int64)
            od = np.full((nq, k), np.float32(1.17549435e-38) if metric == O.IP else FLT_MAX, np.float32)
            for j in range(nq):
                ent = [(float(sd[s, j, p]), int(si[s, j, p])) for s in range(si.shape[0])
                       for p in range(k) if si[s, j, p] >= 0]
                ent.sort(key=lambda e: ((-e[0] if metric == O.IP else e[0]), e[1]))
                for p, (dv, idv) in enumerate(ent[:k]):
                    oi[j, p], od[j, p] = idv, dv
            return oi, od

        scan = ShardedScan(N, GRAN, metric, local_search=local, merge=merge)
        ids, dist_ = scan.search(q, K, flt, rex)
        if rank == 0:
            np.savez(out_path, ids=ids, dist=dist_)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("metric,mode,bitmaps", [(O.L2, 0, False), (O.L2, 1, True), (O.IP, 1, False),
                                                 (O.IP, 0, True)])
def test_sharded_gloo_world2_equals_single_part(tmp_path, metric, mode, bitmaps):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(2, _free_port(), metric, mode, bitmaps, out), nprocs=2, join=True)
    res = np.load(out)
    rows, q, flt, rex = _part(mode)
    if not bitmaps:
        flt = rex = None
    io, do = O.vector_scan(rows, q, K, metric, GRAN, filter_bits=flt, row_exists_bits=rex)
    assert np.array_equal(res["ids"], io)
    assert np.array_equal(res["dist"].view(np.uint32), do.view(np.uint32))
