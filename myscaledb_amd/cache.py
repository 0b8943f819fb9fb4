"""Device-resident LRU of data parts (mqvs_cache_*), the GPU counterpart of
the reference's VICacheManager (src/VectorIndex/Cache/VICacheManager.h:82-114,
over DB::LRUResourceCache): entries keyed by a CacheKey string, weighed by
their HBM bytes, held while in use, evicted least-recently-used first."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check, lib
from .vector_index import VectorIndex
from .vector_scan import VectorScanSegment


def _borrow_segment(h):
    n, d, m, g, o = (ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64())
    check(lib.mqvs_segment_info(h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(m), ctypes.byref(g),
                                ctypes.byref(o), None))
    seg = VectorScanSegment(h, n.value, d.value, m.value, g.value, o.value)
    seg.free = lambda: None  # owned by the cache
    return seg


class PartCache:
    def __init__(self, max_bytes: int):
        h = ctypes.c_void_p()
        check(lib.mqvs_cache_create(int(max_bytes), ctypes.byref(h)))
        self._h = h

    def put(self, key: str, segment: VectorScanSegment, index: VectorIndex | None = None):
        """The cache takes ownership of the segment (and index): the Python
        objects stop owning their handles."""
        check(lib.mqvs_cache_put(self._h, key.encode(), segment._h, index._h if index else None))
        segment._h = None
        if index is not None:
            index._h = None

    def acquire(self, key: str):
        """(segment, index-or-None) held until release(), or None on a miss."""
        s, i = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib.mqvs_cache_acquire(self._h, key.encode(), ctypes.byref(s), ctypes.byref(i)))
        if not s.value:
            return None
        seg = _borrow_segment(s)
        idx = None
        if i.value:
            idx = VectorIndex(i, seg)
            idx.free = lambda: None
        return seg, idx

    def release(self, key: str, segment: VectorScanSegment):
        check(lib.mqvs_cache_release(self._h, key.encode(), segment._h))

    def remove(self, key: str):
        check(lib.mqvs_cache_remove(self._h, key.encode()))

    def stats(self):
        st = _lib.CacheStats()
        check(lib.mqvs_cache_stats(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in _lib.CacheStats._fields_}

    def free(self):
        if self._h:
            check(lib.mqvs_cache_free(self._h))
            self._h = None
