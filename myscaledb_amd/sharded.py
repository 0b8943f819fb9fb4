"""Row-range sharding of one data part over GPUs.

One process per GPU (`torch.distributed`, backend "nccl" = RCCL over xGMI).
Rank g owns the granule-aligned row range `shard_rows(n, granule, g, G)` of
the part as its own resident segment (row_offset = range start, so ids are
part-global and the cosine chunk ordinals continue across shards).  A search
is a local top-k on every rank, ONE all-gather of the per-shard (ids, dist)
lists (nq*k*12 bytes per rank), and a merge by distance, then shard (= row
order), then position (mqvs_merge_shards).  The result equals the single-GPU
search of the whole part -- a shard is not a data part, so the reference's
cross-part multimap order (MergeTreeBaseSearchManager.cpp:207-297, which
reverses exact IP ties between parts) is the wrong rule here; it is
available as merge_shards(..., part_merge=True) for genuinely different parts.

The local search and the merge are injectable so the decomposition can be
exercised with the gloo backend on CPU (tests/test_sharded.py); the defaults
are the HIP path (VectorScanSegment.search, mqvs_merge_shards).
"""
from __future__ import annotations

import math

import numpy as np


def shard_rows(n: int, granule: int, rank: int, world: int) -> tuple[int, int]:
    """[r0, r1) of rank's shard: whole granules, as even as possible."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank / world size")
    nchunks = math.ceil(n / granule) if n > 0 else 0
    c0, c1 = nchunks * rank // world, nchunks * (rank + 1) // world
    return min(c0 * granule, n), min(c1 * granule, n)


def slice_bitmap(bits, n: int, r0: int, r1: int):
    """Rows [r0, r1) of an LSB-first n-bit bitmap, re-packed from bit 0."""
    if bits is None:
        return None
    b = np.asarray(bits, dtype=np.uint8)
    if r0 % 8 == 0:
        out = b[r0 // 8:(r1 + 7) // 8].copy()
        tail = (r1 - r0) % 8
        if tail and out.size:
            out[-1] &= np.uint8((1 << tail) - 1)
        return out
    flat = np.unpackbits(b, bitorder="little")[:n]
    return np.packbits(flat[r0:r1], bitorder="little")


def chunk_ordinal_base(r0: int, granule: int, n: int, nonempty=None, filter_bits=None,
                       row_exists_bits=None) -> int:
    """How many granule chunks before row r0 the reference searches (and so
    re-normalises a cosine query for): a chunk is searched iff it holds a
    non-empty row that, under a PREWHERE filter, also passes it and is not
    deleted (MergeTreeVSManager.cpp:960-1536; the device twin is
    kernels_misc.hip k_chunk_active)."""
    nch = r0 // granule
    if nch == 0:
        return 0
    if nonempty is None and filter_bits is None:
        return nch
    m = r0  # rows of the chunks before the shard
    ok = np.ones(m, bool) if nonempty is None else np.asarray(nonempty, bool)[:m].copy()
    if filter_bits is not None:
        ok &= np.unpackbits(np.asarray(filter_bits, np.uint8), bitorder="little")[:m].astype(bool)
        if row_exists_bits is not None:
            ok &= np.unpackbits(np.asarray(row_exists_bits, np.uint8), bitorder="little")[:m].astype(bool)
    return int(ok.reshape(nch, granule).any(axis=1).sum())


class ShardedScan:
    """A part sharded over the ranks of a process group.

    local_search(queries, k, filter_bits, row_exists_bits, ord_base) -> (ids[nq,k], dist[nq,k])
        ids part-global (the shard's row_offset applied), -1 padded;
        ord_base = chunk_ordinal_base of the shard (cosine query variant)
    merge(ids[S,nq,k], dist[S,nq,k]) -> (ids[nq,k], dist[nq,k])
    nonempty: the PART's per-row non-empty flags (n bytes) or None.
    """

    def __init__(self, n: int, granule: int, metric, local_search=None, merge=None,
                 segment=None, group=None, nonempty=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n, self.granule, self.metric = n, granule, metric
        self.nonempty = nonempty
        self.r0, self.r1 = shard_rows(n, granule, self.rank, self.world)
        self.segment = segment
        if local_search is None:
            if segment is None:
                raise ValueError("need a segment or a local_search function")
            local_search = self._segment_search
        if merge is None:
            from .vector_scan import merge_shards
            merge = lambda i, d: merge_shards(i, d, metric)  # noqa: E731
        self.local_search = local_search
        self.merge = merge

    @classmethod
    def generate(cls, seed, mode, n, d, metric, granule, group=None):
        """Each rank generates its own shard in HBM (counter-based generator)."""
        import torch.distributed as dist
        from .vector_scan import VectorScanSegment
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        r0, r1 = shard_rows(n, granule, rank, world)
        seg = VectorScanSegment.generate(seed, mode, r1 - r0, d, metric, granule, row_offset=r0)
        return cls(n, granule, metric, segment=seg, group=group)

    def _segment_search(self, queries, k, filter_bits, row_exists_bits, ord_base):
        return self.segment.search(queries, k, self.metric, filter_bits, row_exists_bits,
                                   ord_base=ord_base)

    def search(self, queries, k, filter_bits=None, row_exists_bits=None):
        """Sharded top-k over the whole part; every rank returns the merged
        result.  Bitmaps are the PART's (n bits); each rank uses its slice."""
        import torch
        f = slice_bitmap(filter_bits, self.n, self.r0, self.r1)
        e = slice_bitmap(row_exists_bits, self.n, self.r0, self.r1)
        base = chunk_ordinal_base(self.r0, self.granule, self.n, self.nonempty, filter_bits,
                                  row_exists_bits)
        ids, dist = self.local_search(queries, k, f, e, base)
        if self.world == 1:
            return self.merge(ids[None], dist[None]) if self.r1 - self.r0 < self.n else (ids, dist)
        on_device = torch.is_tensor(ids) and ids.is_cuda
        ti = ids if torch.is_tensor(ids) else torch.from_numpy(np.ascontiguousarray(ids))
        td = dist if torch.is_tensor(dist) else torch.from_numpy(np.ascontiguousarray(dist))
        gi = [torch.empty_like(ti) for _ in range(self.world)]
        gd = [torch.empty_like(td) for _ in range(self.world)]
        # ids and distances travel together: one gather of a 12-byte record
        # would need a packed dtype; two small gathers (nq*k*8 + nq*k*4 bytes)
        # are latency-bound either way
        self.dist.all_gather(gi, ti, group=self.group)
        self.dist.all_gather(gd, td, group=self.group)
        si, sd = torch.stack(gi), torch.stack(gd)
        if not on_device:
            si, sd = si.numpy(), sd.numpy()
        return self.merge(si, sd)


class RcclComm:
    """libmqvs's own RCCL communicator (mqvs_comm_*): one rank per GPU, the
    exchange of mqvs_sharded_search.  unique_id() runs on one rank; its 128
    bytes reach the others out of band (here: a torch.distributed broadcast)."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        import ctypes
        from . import _lib
        self._lib = _lib
        self.nranks, self.rank = nranks, rank
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.mqvs_comm_init(nranks, rank, buf, ctypes.byref(h)))
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        buf = (ctypes.c_uint8 * 128)()
        _lib.check(_lib.lib.mqvs_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_process_group(cls, group=None):
        """Every rank of a torch.distributed group joins one communicator."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = cls.unique_id() if rank == 0 else bytes(128)
        if world > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
            t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
            dist.broadcast(t, src=0, group=group)
            uid = bytes(t.cpu().tolist())
        return cls(world, rank, uid)

    def sharded_search(self, segment, queries, k, filter_bitmap=None, row_exists=None, out=None, metric=None,
                       stream=None):
        """mqvs_sharded_search: this rank's shard (`segment`, row_offset = its
        first row) searched, the per-rank top-k all-gathered over RCCL and
        merged on the device; every rank returns the merged [nq, k] result.
        Bitmaps are the shard's own (its n bits).  Device tensors run on
        `stream` (default: torch's current stream, so inputs written by
        earlier torch kernels are ready)."""
        from .vector_scan import _host_f32, _host_u8, _is_torch, _ptr, metric_id
        from ._lib import F_DEVICE_PTRS
        m = segment.metric if metric is None else metric_id(metric)
        if _is_torch(queries):
            import torch
            assert queries.is_cuda and queries.is_contiguous() and queries.dtype == torch.float32, \
                "queries: a contiguous float32 CUDA tensor"
            for b in (filter_bitmap, row_exists):
                assert b is None or (b.is_cuda and b.is_contiguous() and b.dtype == torch.uint8), \
                    "bitmaps: contiguous uint8 CUDA tensors"
            nq = queries.shape[0]
            if out is None:
                ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
                dist = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
            else:
                ids, dist = out
                assert ids.is_cuda and ids.is_contiguous() and ids.dtype == torch.int64
                assert dist.is_cuda and dist.is_contiguous() and dist.dtype == torch.float32
            if stream is None:
                stream = torch.cuda.current_stream(queries.device).cuda_stream
            self._lib.check(self._lib.lib.mqvs_sharded_search(
                self._h, segment._h, _ptr(queries), nq, k, m, _ptr(filter_bitmap), _ptr(row_exists), _ptr(ids),
                _ptr(dist), F_DEVICE_PTRS, stream))
            return ids, dist
        q = _host_f32(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        ids = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        self._lib.check(self._lib.lib.mqvs_sharded_search(
            self._h, segment._h, _ptr(q), nq, k, m, _ptr(_host_u8(filter_bitmap)), _ptr(_host_u8(row_exists)),
            _ptr(ids), _ptr(dist), 0, stream))
        return ids, dist

    def stats(self):
        """{'fast_calls': searches that synchronised the host once, 'redo_calls':
        those of them re-run on the validated path} (mqvs_comm_stats)."""
        import ctypes
        f, r = ctypes.c_int64(), ctypes.c_int64()
        self._lib.check(self._lib.lib.mqvs_comm_stats(self._h, ctypes.byref(f), ctypes.byref(r)))
        return {"fast_calls": f.value, "redo_calls": r.value}

    def free(self):
        if getattr(self, "_h", None):
            self._lib.check(self._lib.lib.mqvs_comm_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001
            pass


class LoopbackComm(RcclComm):
    """One rank of a loopback communicator group (mqvs_comm_init_loopback):
    N virtual ranks in this process on the current GPU, the exchanges done as
    device copies.  Each rank's sharded_search must run on its own thread
    (the ranks meet at host barriers); the search code is the RCCL one."""

    def __init__(self, handle):  # noqa: D401  (built by group())
        from . import _lib
        self._lib = _lib
        self._h = handle

    @classmethod
    def group(cls, nranks: int):
        import ctypes
        from . import _lib
        hs = (ctypes.c_void_p * nranks)()
        _lib.check(_lib.lib.mqvs_comm_init_loopback(nranks, hs))
        ranks = []
        for r in range(nranks):
            c = cls(ctypes.c_void_p(hs[r]))
            c.nranks, c.rank = nranks, r
            ranks.append(c)
        return ranks
