"""Host-side mirror of MyScaleDB's brute-force vector-scan operator over libmqvs.

Names and contracts follow the reference so the parity tests read like its own:

* ``try_brute_force_search``  -- VectorIndex::tryBruteForceSearch<FloatVector>
  (src/VectorIndex/Common/BruteForceSearch.h:62-111); faiss result layout.
* ``VectorScanSegment``       -- one data part's Array(Float32) column, registered
  once and resident in HBM (replaces the per-granule copy loop of
  MergeTreeVSManager.cpp:1366-1393).
* ``BinaryVectorScanSegment`` / ``try_brute_force_search_binary`` -- the same for
  FixedString(N) binary columns, Hamming / Jaccard
  (tryBruteForceSearch<BinaryVector>, BruteForceSearch.h:94-110;
  MergeTreeVSManager.cpp:1188-1273, 1395-1425).
* ``vector_scan_without_index`` -- MergeTreeVSManager::vectorScanWithoutIndex<Float>
  (MergeTreeVSManager.cpp:960-1536) incl. searchWrapper (:1538-1680); returns
  the same result columns (label UInt32, [vector_id UInt32,] distance Float32)
  with the -1 labels dropped (:1502-1532).

Inputs are numpy arrays (host) or torch tensors already on the GPU (device
pointers passed straight through the C-ABI).  Every call runs the HIP kernels;
there is no CPU path in this package.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import (F_ASYNC, F_DEVICE_PTRS, F_EXACT, F_GATHER_ALWAYS, F_GATHER_NEVER, F_NO_CHECKSUM,
                   F_PART_MERGE, F_TIMING, METRICS, check, lib)

FLT_MAX = np.float32(3.4028235e38)
FLT_MIN = np.float32(1.1754944e-38)
DEFAULT_GRANULE = 8192  # MergeTreeSettings.h index_granularity


def metric_id(metric) -> int:
    if isinstance(metric, (int, np.integer)):
        return int(metric)
    try:
        return METRICS[metric]
    except KeyError:
        raise _lib.NotImplementedMetric(_lib.ERR_NOT_IMPLEMENTED,
                                        f"Metric {metric} not implemented in brute force search")


def _is_torch(a):
    return type(a).__module__.startswith("torch")


def _ptr(a):
    if a is None:
        return None
    if _is_torch(a):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


def _host_f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _host_u8(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.uint8)


def pack_bitmap(mask) -> np.ndarray:
    """bool/0-1 per row -> LSB-first uint8 bitmap (Search::DenseBitmap byte layout)."""
    return np.packbits(np.asarray(mask, dtype=np.uint8), bitorder="little")


def init(device: int = 0):
    check(lib.mqvs_init(device))


class VectorScanSegment:
    """A data part's vector column resident in HBM.

    rows: (n, d) float32 (numpy, or a torch CUDA tensor); rows whose Array is
    empty must be FLT_MAX-filled and flagged 0 in ``nonempty``.
    """

    def __init__(self, handle, n, d, metric, granule, row_offset):
        self._h = handle
        self.n, self.d, self.metric, self.granule, self.row_offset = n, d, metric, granule, row_offset

    @classmethod
    def from_rows(cls, rows, metric="L2", granule=DEFAULT_GRANULE, nonempty=None, row_offset=0):
        m = metric_id(metric)
        h = ctypes.c_void_p()
        if _is_torch(rows):
            assert rows.is_cuda and rows.is_contiguous()
            n, d = rows.shape
            ne = None
            if nonempty is not None:
                ne = nonempty
            check(lib.mqvs_segment_create_device(_ptr(rows), n, d, m, granule, _ptr(ne),
                                                 row_offset, ctypes.byref(h)))
        else:
            rows = _host_f32(rows)
            n, d = rows.shape
            ne = _host_u8(nonempty)
            check(lib.mqvs_segment_create(_ptr(rows), n, d, m, granule, _ptr(ne), row_offset,
                                          ctypes.byref(h)))
        return cls(h, n, d, m, granule, row_offset)

    @classmethod
    def from_column(cls, data_bin, sizes_bin, n, d, metric="L2", granule=DEFAULT_GRANULE, row_offset=0,
                    verify_checksum=True):
        """A part's Array(Float32) column from its compressed files, decoded on
        the GPU (mqvs_segment_create_from_column): data_bin = `<col>.bin`
        bytes, sizes_bin = `<col>.size0.bin` bytes (bytes / numpy uint8, or
        torch uint8 CUDA tensors).  Block checksums are verified unless
        verify_checksum=False (CompressedReadBufferBase's disable_checksum)."""
        m = metric_id(metric)
        h = ctypes.c_void_p()
        if _is_torch(data_bin):
            flags = F_DEVICE_PTRS
            dp, dn = _ptr(data_bin), data_bin.numel()
            sp, sn = _ptr(sizes_bin), sizes_bin.numel()
            keep = None
        else:
            flags = 0
            a = np.frombuffer(bytes(data_bin), np.uint8) if isinstance(data_bin, (bytes, bytearray)) \
                else _host_u8(data_bin)
            b = np.frombuffer(bytes(sizes_bin), np.uint8) if isinstance(sizes_bin, (bytes, bytearray)) \
                else _host_u8(sizes_bin)
            keep = (a, b)
            dp, dn, sp, sn = _ptr(a), a.size, _ptr(b), b.size
        if not verify_checksum:
            flags |= F_NO_CHECKSUM
        check(lib.mqvs_segment_create_from_column(dp, dn, sp, sn, n, d, m, granule, row_offset, flags,
                                                  ctypes.byref(h)))
        del keep
        return cls(h, n, d, m, granule, row_offset)

    @classmethod
    def generate(cls, seed, mode, n, d, metric="L2", granule=DEFAULT_GRANULE, row_offset=0):
        """Synthetic part from the counter-based generator (mode 0 exact, 1 gauss, 2 mixture, 3 hard mixture)."""
        m = metric_id(metric)
        h = ctypes.c_void_p()
        check(lib.mqvs_segment_generate(seed, mode, n, d, m, granule, row_offset, ctypes.byref(h)))
        return cls(h, n, d, m, granule, row_offset)

    def info(self):
        n, d, m, g, o = (ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(),
                         ctypes.c_int64())
        b = ctypes.c_size_t()
        check(lib.mqvs_segment_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(m),
                                    ctypes.byref(g), ctypes.byref(o), ctypes.byref(b)))
        sp, pb, ok = ctypes.c_int32(), ctypes.c_size_t(), ctypes.c_int32()
        check(lib.mqvs_segment_prefilter(self._h, ctypes.byref(sp), ctypes.byref(pb), ctypes.byref(ok)))
        rh = ctypes.c_int32()
        check(lib.mqvs_segment_rows_host(self._h, ctypes.byref(rh)))
        return dict(n=n.value, d=d.value, metric=m.value, granule=g.value, row_offset=o.value,
                    hbm_bytes=b.value, prefilter=sp.value, plane_bytes=pb.value, approx_ok=bool(ok.value),
                    rows_host=bool(rh.value))

    def set_rows_host(self, host: bool = True):
        """mqvs_segment_set_rows_host: the Float32 rows to pinned host memory
        (HBM keeps the bf16 plane; same results, survivors re-ranked over
        PCIe) or back into HBM."""
        check(lib.mqvs_segment_set_rows_host(self._h, 1 if host else 0))

    def device_rows_ptr(self) -> int:
        p = ctypes.c_void_p()
        check(lib.mqvs_segment_rows(self._h, ctypes.byref(p)))
        return p.value

    def search(self, queries, k, metric=None, filter_bitmap=None, row_exists=None, out=None,
               async_=False, stream=None, ord_base=None, exact=False, gather=None, timing=False):
        """Raw mqvs_search: (ids[nq,k] int64, dist[nq,k] float32), -1 padded.
        ord_base: cosine chunk-ordinal base of a row-range shard
        (mqvs_search_ex; None = every earlier chunk searched).
        Per-call path flags (same bits on every path): exact=True scans every
        row in fp32 (MQVS_F_EXACT); gather=False / True forces the masked /
        gathered PREWHERE scan; timing=True fills the stats' kernel times.
        async_=True (device tensors): returns before the stream drains; check
        the outcome with async_check()."""
        m = self.metric if metric is None else metric_id(metric)
        base = -1 if ord_base is None else int(ord_base)
        extra = (F_EXACT if exact else 0) | (F_TIMING if timing else 0) | \
            (0 if gather is None else F_GATHER_ALWAYS if gather else F_GATHER_NEVER)

        def call(qp, nq, fp, ep, ip, dp, flags, st):
            check(lib.mqvs_search_ex(self._h, qp, nq, k, m, fp, ep, base, ip, dp, flags | extra, st))

        if _is_torch(queries):
            import torch
            assert queries.is_cuda and queries.is_contiguous() and queries.dtype == torch.float32
            nq = queries.shape[0]
            if out is None:
                ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
                dist = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
            else:
                ids, dist = out
            flags = F_DEVICE_PTRS | (F_ASYNC if async_ else 0)
            call(_ptr(queries), nq, _ptr(filter_bitmap), _ptr(row_exists), _ptr(ids), _ptr(dist), flags,
                 ctypes.c_void_p(stream) if stream else None)
            return ids, dist
        q = _host_f32(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        if q.shape[1] != self.d:
            raise _lib.MqvsError(_lib.ERR_LOGICAL,
                                 f"query dimension {q.shape[1]} != column dimension {self.d}")
        ids = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        call(_ptr(q), nq, _ptr(_host_u8(filter_bitmap)), _ptr(_host_u8(row_exists)), _ptr(ids),
             _ptr(dist), 0, None)
        return ids, dist

    def rerank(self, queries, candidates, k, metric=None, row_exists=None):
        """mqvs_rerank (computeTopDistanceSubset contract, VIWithDataPart.cpp:838-856):
        candidates[nq, ncand] segment-local rows (-1 = none) -> exact top-k
        (ids, dist) with mqvs_search's formula, order key and padding."""
        m = self.metric if metric is None else metric_id(metric)
        q = _host_f32(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        c = np.ascontiguousarray(np.asarray(candidates, dtype=np.int64).reshape(nq, -1))
        ids = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        check(lib.mqvs_rerank(self._h, _ptr(q), nq, _ptr(c), c.shape[1], k, m,
                              _ptr(_host_u8(row_exists)), _ptr(ids), _ptr(dist), 0, None))
        return ids, dist

    def free(self):
        if self._h:
            check(lib.mqvs_segment_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def try_brute_force_search(x, y, d, k, nx, ny, metric):
    """VectorIndex::tryBruteForceSearch: returns (result_id[nx*k], distance[nx*k])."""
    m = metric_id(metric)
    x = _host_f32(x).reshape(-1)
    y = _host_f32(y).reshape(-1)
    ids = np.empty(nx * k, np.int64)
    dist = np.empty(nx * k, np.float32)
    check(lib.mqvs_knn_raw(_ptr(x), _ptr(y), d, k, nx, ny, m, _ptr(ids), _ptr(dist)))
    return ids, dist


class BinaryVectorScanSegment:
    """A data part's FixedString(N) binary vector column resident in HBM.

    codes: (n, N) uint8 (numpy, or a torch CUDA uint8 tensor); dimension = 8N
    bits.  metric: the column's binary_vector_search_metric_type (Hamming or
    Jaccard); a search may pass the other one."""

    def __init__(self, handle, n, nbytes, metric, granule, row_offset):
        self._h = handle
        self.n, self.nbytes, self.d = n, nbytes, 8 * nbytes
        self.metric, self.granule, self.row_offset = metric, granule, row_offset

    @classmethod
    def from_codes(cls, codes, metric="Hamming", granule=DEFAULT_GRANULE, row_offset=0):
        m = metric_id(metric)
        h = ctypes.c_void_p()
        if _is_torch(codes):
            assert codes.is_cuda and codes.is_contiguous()
            n, nb = codes.shape
            check(lib.mqvs_segment_create_binary(_ptr(codes), n, 8 * nb, m, granule, row_offset, F_DEVICE_PTRS,
                                                 ctypes.byref(h)))
        else:
            codes = _host_u8(codes)
            n, nb = codes.shape
            check(lib.mqvs_segment_create_binary(_ptr(codes), n, 8 * nb, m, granule, row_offset, 0,
                                                 ctypes.byref(h)))
        return cls(h, n, nb, m, granule, row_offset)

    def search(self, queries, k, metric=None, filter_bitmap=None, row_exists=None, out=None, async_=False,
               stream=None):
        """mqvs_search_binary: (ids[nq,k] int64, dist[nq,k] float32), ascending,
        -1 / FLT_MAX padded."""
        m = self.metric if metric is None else metric_id(metric)
        if _is_torch(queries):
            import torch
            assert queries.is_cuda and queries.is_contiguous() and queries.dtype == torch.uint8
            nq = queries.shape[0]
            if out is None:
                ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
                dist = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
            else:
                ids, dist = out
            flags = F_DEVICE_PTRS | (F_ASYNC if async_ else 0)
            check(lib.mqvs_search_binary(self._h, _ptr(queries), nq, k, m, _ptr(filter_bitmap), _ptr(row_exists),
                                         _ptr(ids), _ptr(dist), flags, ctypes.c_void_p(stream) if stream else None))
            return ids, dist
        q = _host_u8(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        if q.shape[1] != self.nbytes:
            raise _lib.MqvsError(_lib.ERR_LOGICAL,
                                 f"query length {q.shape[1]} bytes != column FixedString({self.nbytes})")
        ids = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        check(lib.mqvs_search_binary(self._h, _ptr(q), nq, k, m, _ptr(_host_u8(filter_bitmap)),
                                     _ptr(_host_u8(row_exists)), _ptr(ids), _ptr(dist), 0, None))
        return ids, dist

    def free(self):
        if self._h:
            check(lib.mqvs_segment_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def try_brute_force_search_binary(x, y, d, k, nx, ny, metric):
    """tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110): x, y
    uint8 codes of d bits; returns (result_id[nx*k], distance[nx*k]) where the
    distance buffer holds int32 counts for Hamming (faiss::hammings_knn_mc via
    reinterpret_cast<int32_t*>) and float32 for Jaccard."""
    m = metric_id(metric)
    x = _host_u8(x).reshape(-1)
    y = _host_u8(y).reshape(-1)
    ids = np.empty(nx * k, np.int64)
    dist = np.empty(nx * k, np.float32)
    check(lib.mqvs_knn_binary_raw(_ptr(x), _ptr(y), d, k, nx, ny, m, _ptr(ids), _ptr(dist)))
    if m == _lib.METRIC_HAMMING:
        dist = dist.view(np.int32)
    return ids, dist


def vector_scan_without_index(segment: VectorScanSegment, query_vector, k, metric=None,
                              filter_bitmap=None, row_exists=None, is_batch=False):
    """MergeTreeVSManager::vectorScanWithoutIndex result columns.

    Returns (label, distance) or, for batch, (label, vector_id, distance) with
    the reference's emission order: query-major, best first, -1 labels dropped.
    """
    if isinstance(segment, BinaryVectorScanSegment):
        q = _host_u8(query_vector)
    else:
        q = _host_f32(query_vector)
    if q.ndim == 1:
        q = q[None, :]
    ids, dist = segment.search(q, k, metric, filter_bitmap, row_exists)
    flat_ids, flat_dist = ids.reshape(-1), dist.reshape(-1)
    keep = flat_ids > -1
    label = flat_ids[keep].astype(np.uint32)
    distance = flat_dist[keep]
    if is_batch:
        vector_id = (np.arange(flat_ids.size) // k)[keep].astype(np.uint32)
        return label, vector_id, distance
    return label, distance


def merge_shards(ids, dist, metric, out=None, async_=False, stream=None, part_merge=False):
    """Merge per-shard results [nshards, nq, k] -> [nq, k] (mqvs_merge_shards).
    part_merge=True: lists are different data parts, merged with the
    reference's cross-part multimap order (MergeTreeBaseSearchManager.cpp:207-297;
    exact IP ties come out last-inserted first); default: row-range shards of
    one part (result == the unsharded part)."""
    m = metric_id(metric)
    pm = F_PART_MERGE if part_merge else 0
    nshards, nq, k = ids.shape
    if _is_torch(ids):
        import torch
        if out is None:
            oi = torch.empty((nq, k), dtype=torch.int64, device=ids.device)
            od = torch.empty((nq, k), dtype=torch.float32, device=ids.device)
        else:
            oi, od = out
        flags = F_DEVICE_PTRS | (F_ASYNC if async_ else 0) | pm
        check(lib.mqvs_merge_shards(nshards, nq, k, m, _ptr(ids.contiguous()), _ptr(dist.contiguous()),
                                    _ptr(oi), _ptr(od), flags,
                                    ctypes.c_void_p(stream) if stream else None))
        return oi, od
    ids = np.ascontiguousarray(ids, np.int64)
    dist = _host_f32(dist)
    oi = np.empty((nq, k), np.int64)
    od = np.empty((nq, k), np.float32)
    check(lib.mqvs_merge_shards(nshards, nq, k, m, _ptr(ids), _ptr(dist), _ptr(oi), _ptr(od), pm,
                                None))
    return oi, od


def generate_device(seed, mode, row0, n, d, out_tensor, stream=None):
    check(lib.mqvs_generate_device(seed, mode, row0, n, d, _ptr(out_tensor),
                                   ctypes.c_void_p(stream) if stream else None))


def async_check(stream=None):
    """mqvs_async_check: raises MqvsError(LOGICAL_ERROR) when one of this
    thread's async searches since the last check needed a host-driven
    fallback (its results are invalid: repeat it without async_)."""
    check(lib.mqvs_async_check(ctypes.c_void_p(stream) if stream else None))


def set_timing(enabled: bool):
    check(lib.mqvs_set_timing(1 if enabled else 0))


def set_gather_mode(mode: int):
    """Selective PREWHERE: 0 scan all rows + mask, 1 gather the selected rows
    when few pass (default: <= 60% on the bf16 pre-filter, <= 30% on the exact
    small-batch kernel), 2 always gather (mqvs_set_gather_mode)."""
    check(lib.mqvs_set_gather_mode(int(mode)))


def set_scratch_budget(nbytes: int) -> int:
    """Device scratch per buffer of one call (large-k sorts, candidate lists);
    larger calls run in query sub-batches with the same bits
    (mqvs_set_scratch_budget).  Returns the previous value; 0 only reads it."""
    return int(lib.mqvs_set_scratch_budget(int(nbytes)))


def measure_read_bandwidth(nbytes: int = 8 << 30, reps: int = 5):
    """Achievable HBM read rate (GB/s) of the current device by a STREAM-like
    read sweep (mqvs_measure_read_bandwidth); returns (gbs, best_ms)."""
    g, m = ctypes.c_double(), ctypes.c_double()
    check(lib.mqvs_measure_read_bandwidth(int(nbytes), int(reps), ctypes.byref(g), ctypes.byref(m)))
    return g.value, m.value


def set_prefilter(split: int):
    """Pre-filter planes of segments created after the call: 2 = bf16 hi
    plane (default), 0 = none -- batches then run the exact fp32 MFMA path
    (mqvs_set_prefilter).  Both return the same bits."""
    check(lib.mqvs_set_prefilter(int(split)))


def set_batch_mode(mode: int):
    """nq >= 20: 0 = bf16 MFMA pre-filter + exact fp32 re-rank (default),
    1 = fp32 MFMA over every row.  Both return identical bits."""
    check(lib.mqvs_set_batch_mode(int(mode)))
