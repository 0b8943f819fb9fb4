"""Multi-GPU decomposition (myscaledb_amd/sharded.py) on CPU:
granule-aligned row-range shards, per-shard bitmap slices, the all-gather of
per-shard top-k and the cross-part merge -- world_size 2 over gloo, local
searches and merges done by the oracle.  The sharded answer must equal the
single-part oracle scan bit for bit, for L2 / IP / cosine, with PREWHERE
filters, deletes and empty arrays (cosine: the shard's chunk-ordinal base)."""
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


def _part(metric_mode, empties=False, gran=GRAN):
    rows = O.generate(71, metric_mode, 0, N, D)
    q = O.generate(72, metric_mode, 0, NQ, D)
    rng = np.random.default_rng(9)
    keep = rng.random(N) > 0.25
    skip = 0 if gran > GRAN else 1          # coarse granules: shard 1 starts at chunk 1
    keep[skip * gran:(skip + 1) * gran] = False   # a chunk of shard 0 filtered out entirely
    flt = np.packbits(keep, bitorder="little")
    rex = np.packbits(rng.random(N) > 0.1, bitorder="little")
    ne = None
    if empties:
        ne = (rng.random(N) > 0.2).astype(np.uint8)
        e = 0 if gran > GRAN else 2
        ne[e * gran:(e + 1) * gran] = 0     # an all-empty chunk before shard 1
        rows[ne == 0] = FLT_MAX
    return rows, q, flt, rex, ne


def _worker(rank, world, port, metric, mode, use_bitmaps, empties, gran, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from myscaledb_amd.sharded import ShardedScan
        rows, q, flt, rex, ne = _part(mode, empties, gran)
        if not use_bitmaps:
            flt = rex = None

        scan = None

        def local(queries, k, f, e, ord_base):
            r0, r1 = scan.r0, scan.r1
            if metric == O.COSINE:
                # the reference's query object after ord_base searched chunks
                for _ in range(ord_base):
                    queries = O.normalize(queries)
            ids, dist_ = O.vector_scan(rows[r0:r1], queries, k, metric, gran, filter_bits=f,
                                       row_exists_bits=e, nonempty=None if ne is None else ne[r0:r1])
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

        scan = ShardedScan(N, gran, metric, local_search=local, merge=merge, nonempty=ne)
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


@pytest.mark.parametrize("metric,mode,bitmaps,empties,gran", [
    (O.L2, 0, False, False, GRAN), (O.L2, 1, True, True, GRAN), (O.IP, 1, False, False, GRAN),
    (O.IP, 0, True, False, GRAN), (O.COSINE, 1, False, False, GRAN), (O.COSINE, 1, True, False, GRAN),
    (O.COSINE, 2, True, True, GRAN), (O.COSINE, 1, False, True, GRAN),
    (O.COSINE, 1, True, False, 3000), (O.COSINE, 2, False, True, 3000)])
def test_sharded_gloo_world2_equals_single_part(tmp_path, metric, mode, bitmaps, empties, gran):
    """Cosine cases: shard 0 holds a fully filtered-out chunk, or shard 1 is
    preceded by an all-empty chunk -- the reference skips those chunks, so
    shard 1's query-variant ordinals start below row_offset / granule."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(2, _free_port(), metric, mode, bitmaps, empties, gran, out), nprocs=2,
             join=True)
    res = np.load(out)
    rows, q, flt, rex, ne = _part(mode, empties, gran)
    if not bitmaps:
        flt = rex = None
    io, do = O.vector_scan(rows, q, K, metric, gran, filter_bits=flt, row_exists_bits=rex, nonempty=ne)
    assert np.array_equal(res["ids"], io)
    assert np.array_equal(res["dist"].view(np.uint32), do.view(np.uint32))


def test_chunk_ordinal_base():
    from myscaledb_amd.sharded import chunk_ordinal_base
    g, n = 100, 1000
    assert chunk_ordinal_base(300, g, n) == 3
    ne = np.ones(n, np.uint8)
    ne[100:200] = 0
    assert chunk_ordinal_base(300, g, n, nonempty=ne) == 2
    keep = np.ones(n, bool)
    keep[0:100] = False
    f = np.packbits(keep, bitorder="little")
    assert chunk_ordinal_base(300, g, n, nonempty=ne, filter_bits=f) == 1
    live = np.ones(n, bool)
    live[200:300] = False
    e = np.packbits(live, bitorder="little")
    assert chunk_ordinal_base(300, g, n, nonempty=ne, filter_bits=f, row_exists_bits=e) == 0
    # deletes alone do not skip chunks (searchWrapper masks them after the search)
    assert chunk_ordinal_base(300, g, n, row_exists_bits=e) == 3
