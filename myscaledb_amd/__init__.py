"""myscaledb_amd -- MI355X-native brute-force vector-scan path for MyScaleDB.

The product is libmqvs.so (HIP kernels for gfx950 + the C-ABI in
include/mqvs.h).  This package is its Python-side mirror of the reference
operator surface (vector_scan) plus the multi-GPU row-range sharding
(sharded).  Importing it loads libmqvs.so and fails loudly if it is missing.
"""
from . import _lib  # noqa: F401  (loads libmqvs.so, raises if absent)
from .vector_scan import (  # noqa: F401
    BinaryVectorScanSegment,
    VectorScanSegment,
    init,
    merge_shards,
    pack_bitmap,
    try_brute_force_search,
    try_brute_force_search_binary,
    vector_scan_without_index,
)
from .vector_index import VectorIndex  # noqa: F401

__all__ = ["BinaryVectorScanSegment", "try_brute_force_search_binary", "VectorScanSegment", "init", "merge_shards", "pack_bitmap",
           "try_brute_force_search", "vector_scan_without_index", "VectorIndex"]
