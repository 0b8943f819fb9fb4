"""Host-side mirror of MyScaleDB's vector-index seam over libmqvs (index path).

* ``VectorIndex.build``   -- Search::createVectorIndex<..., FloatVector>(name,
  IndexType::MSTG, metric, dim, total_vec, params, ...) + VectorIndex::build
  (src/VectorIndex/Common/VIWithDataPart.cpp:416-447, VIWithDataPart.h:295-339).
* ``VectorIndex.search``  -- VectorIndex::search(queries, k, params,
  first_stage_only, filter) as VIWithColumnInPart::search calls it
  (VIWithDataPart.cpp:858-957; the filter is PREWHERE ∩ the delete bitmap,
  :903-908).
* ``VectorIndex.compute_top_distance_subset`` -- stage 2 of a two-stage
  search, VIWithColumnInPart::computeTopDistanceSubset (VIWithDataPart.cpp:838-856):
  mqvs_rerank on the index's segment.

The MSTG library is absent from the reference snapshot; the index here is the
library's own GPU design with MSTG's parameter surface (``alpha``,
``metric_type``), see include/mqvs.h.  Every call runs HIP kernels; there is
no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import F_ASYNC, F_DEVICE_PTRS, F_FIRST_STAGE, F_RERANK_ALL, check, lib
from .vector_scan import VectorScanSegment, _host_f32, _host_u8, _is_torch, _ptr


def _params(p) -> bytes:
    if p is None:
        return b""
    if isinstance(p, dict):
        p = ",".join(f"{k}={v}" for k, v in p.items())
    return p.encode()


class VectorIndex:
    """An MSTG-type index over a resident segment (the segment must outlive it)."""

    def __init__(self, handle, segment: VectorScanSegment):
        self._h = handle
        self.segment = segment

    @classmethod
    def build(cls, segment: VectorScanSegment, index_type="MSTG", params=None):
        h = ctypes.c_void_p()
        check(lib.mqvs_index_build(segment._h, index_type.encode(), _params(params), ctypes.byref(h)))
        return cls(h, segment)

    def set_row_ids_map(self, row_ids_map):
        """Decoupled part (VIWithMeta::row_ids_map): source-part row -> row of
        the decoupled part; later searches return decoupled-part row ids
        (transferToNewRowIds, VIWithDataPart.cpp:56-67).  None clears it."""
        if row_ids_map is None:
            check(lib.mqvs_index_set_row_ids_map(self._h, None, 0, 0))
            return
        if _is_torch(row_ids_map):
            check(lib.mqvs_index_set_row_ids_map(self._h, _ptr(row_ids_map), row_ids_map.numel(), F_DEVICE_PTRS))
            return
        m = np.ascontiguousarray(row_ids_map, np.uint64)
        check(lib.mqvs_index_set_row_ids_map(self._h, _ptr(m), m.size, 0))

    def info(self):
        st = _lib.IndexInfo()
        check(lib.mqvs_index_info(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in _lib.IndexInfo._fields_}

    def centroids(self):
        """The coarse step's centroid table, float32[nlist, dim]."""
        info = self.info()
        c = np.empty((info["nlist"], info["dim"]), np.float32)
        check(lib.mqvs_index_centroids(self._h, _ptr(c), c.size))
        return c

    def probes(self, queries, params=None):
        """The lists a search with `params` probes, int64[nq, nprobe] (no order)."""
        q = _host_f32(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        pr = _params(params)
        info = self.info()
        # nprobe as the search resolves it: run the coarse step into a buffer
        # of every list, then trim to the count the stats report
        buf = np.full((nq, info["nlist"]), -1, np.int64)
        check(lib.mqvs_index_probes(self._h, _ptr(q), nq, pr, _ptr(buf)))
        npb = _lib.last_index_stats()["nprobe"]
        return buf.reshape(-1)[: nq * npb].reshape(nq, npb).copy()

    def search(self, queries, k, params=None, filter_bitmap=None, row_exists=None, first_stage_only=False,
               out=None, async_=False, stream=None, rerank_all=False):
        """(ids[nq,k] int64, dist[nq,k] float32), reference order, -1 padded.
        first_stage_only: the k best rows by the approximate distance (stage 1
        of a two-stage search; re-rank with compute_top_distance_subset).
        rerank_all: re-rank every num_reorder candidate (MQVS_F_RERANK_ALL; the
        default bound pruning gives the same results)."""
        fs = (F_FIRST_STAGE if first_stage_only else 0) | (F_RERANK_ALL if rerank_all else 0)
        pr = _params(params)
        if _is_torch(queries):
            import torch
            assert queries.is_cuda and queries.is_contiguous() and queries.dtype == torch.float32
            nq = queries.shape[0]
            if out is None:
                ids = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
                dist = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
            else:
                ids, dist = out
            flags = F_DEVICE_PTRS | (F_ASYNC if async_ else 0) | fs
            check(lib.mqvs_index_search(self._h, _ptr(queries), nq, k, pr, _ptr(filter_bitmap), _ptr(row_exists),
                                        _ptr(ids), _ptr(dist), flags, ctypes.c_void_p(stream) if stream else None))
            return ids, dist
        q = _host_f32(queries)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        if q.shape[1] != self.segment.d:
            raise _lib.MqvsError(_lib.ERR_LOGICAL, "The dimension of searched index and input doesn't match.")
        ids = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        check(lib.mqvs_index_search(self._h, _ptr(q), nq, k, pr, _ptr(_host_u8(filter_bitmap)),
                                    _ptr(_host_u8(row_exists)), _ptr(ids), _ptr(dist), fs, None))
        return ids, dist

    def compute_top_distance_subset(self, queries, first_stage_ids, top_k, row_exists=None):
        """Exact re-rank of stage-1 ids (segment-local rows, -1 = none)."""
        ids = np.asarray(first_stage_ids, np.int64)
        local = np.where(ids >= 0, ids - self.segment.row_offset, -1)
        return self.segment.rerank(queries, local, top_k, row_exists=row_exists)

    def free(self):
        if self._h:
            check(lib.mqvs_index_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def last_index_stats():
    return _lib.last_index_stats()


def decoupled_filter(new_filter, new_rows, inverted_row_ids_map, inverted_row_sources_map, own_id, old_rows):
    """getRealBitmap (VIUtils.cpp:479-497) on the GPU: a PREWHERE bitmap over
    the decoupled part's rows -> the bitmap over one source part's rows."""
    nf = _host_u8(new_filter)
    inv = None if inverted_row_ids_map is None else np.ascontiguousarray(inverted_row_ids_map, np.uint64)
    src = None if inverted_row_sources_map is None else np.ascontiguousarray(inverted_row_sources_map, np.uint8)
    out = np.zeros((old_rows + 7) // 8, np.uint8)
    check(lib.mqvs_decoupled_filter(_ptr(nf), new_rows, _ptr(inv), _ptr(src), 0 if inv is None else inv.size,
                                    own_id, _ptr(out), old_rows, 0, None))
    return out
