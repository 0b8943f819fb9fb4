"""ctypes binding of libmqvs.so (include/mqvs.h).

The shared library is built in-tree (myscaledb_amd/libmqvs.so, see
__graft_entry__.build / myscaledb_amd/csrc/Makefile).  There is no fallback:
if the library is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The release library; nothing in the environment selects another one.  The
# measurement build (libmqvs_dbg.so, `make dbg`: kernels that read A/B switches
# from the environment) is loaded only by a tool that calls
# use_measurement_build() explicitly, before its first library call.
LIB_PATH = os.path.join(_HERE, "libmqvs.so")
DBG_LIB_PATH = os.path.join(_HERE, "libmqvs_dbg.so")

# include/mqvs.h
METRIC_L2, METRIC_IP, METRIC_COSINE, METRIC_HAMMING, METRIC_JACCARD = 0, 1, 2, 4, 5
METRICS = {"L2": METRIC_L2, "IP": METRIC_IP, "COSINE": METRIC_COSINE, "Cosine": METRIC_COSINE,
           "cosine": METRIC_COSINE, "l2": METRIC_L2, "ip": METRIC_IP,
           "Hamming": METRIC_HAMMING, "HAMMING": METRIC_HAMMING, "hamming": METRIC_HAMMING,
           "Jaccard": METRIC_JACCARD, "JACCARD": METRIC_JACCARD, "jaccard": METRIC_JACCARD}
OK = 0
ERR_NOT_IMPLEMENTED, ERR_LOGICAL, ERR_ILLEGAL_COLUMN, ERR_BAD_ARGUMENTS, ERR_MEMORY_LIMIT, \
    ERR_DEVICE, ERR_CHECKSUM = 1, 2, 3, 4, 5, 6, 7
F_DEVICE_PTRS = 0x1
F_ASYNC = 0x2
F_PART_MERGE = 0x4
F_FIRST_STAGE = 0x8
F_NO_CHECKSUM = 0x10
F_EXACT = 0x20
F_GATHER_NEVER = 0x40
F_GATHER_ALWAYS = 0x80
F_TIMING = 0x100
F_RERANK_ALL = 0x200
WAIT_RUNTIME, WAIT_HYBRID, WAIT_BLOCK = 0, 1, 2

# Exported C symbols: every one of these is declared in include/mqvs.h.
SYMBOLS = [
    "mqvs_abi_version", "mqvs_init", "mqvs_device_count", "mqvs_last_error",
    "mqvs_thread_release", "mqvs_shutdown", "mqvs_segment_create", "mqvs_segment_create_device",
    "mqvs_segment_generate", "mqvs_segment_free", "mqvs_segment_info", "mqvs_segment_prefilter", "mqvs_segment_rows",
    "mqvs_segment_set_rows_host", "mqvs_segment_rows_host",
    "mqvs_search", "mqvs_search_ex", "mqvs_knn_raw", "mqvs_rerank", "mqvs_merge_shards", "mqvs_generate_device",
    "mqvs_last_search_stats", "mqvs_set_timing", "mqvs_set_batch_mode", "mqvs_set_gather_mode", "mqvs_set_prefilter",
    "mqvs_set_scratch_budget", "mqvs_measure_read_bandwidth", "mqvs_set_workspace_budget", "mqvs_workspace_stats",
    "mqvs_index_build", "mqvs_index_free", "mqvs_index_info", "mqvs_index_search", "mqvs_index_last_stats",
    "mqvs_index_centroids", "mqvs_index_probes",
    "mqvs_segment_create_binary", "mqvs_search_binary", "mqvs_knn_binary_raw",
    "mqvs_segment_create_from_column", "mqvs_async_check",
    "mqvs_comm_unique_id", "mqvs_comm_init", "mqvs_comm_init_loopback", "mqvs_comm_free", "mqvs_sharded_search", "mqvs_comm_stats",
    "mqvs_index_set_row_ids_map", "mqvs_decoupled_filter",
    "mqvs_cache_create", "mqvs_cache_free", "mqvs_cache_put", "mqvs_cache_acquire", "mqvs_cache_release",
    "mqvs_cache_remove", "mqvs_cache_stats", "mqvs_inject_fault", "mqvs_set_wait_mode",
]


class SearchStats(ctypes.Structure):
    _fields_ = [("probe_ms", ctypes.c_double), ("probe_select_ms", ctypes.c_double),
                ("main_ms", ctypes.c_double), ("refine_ms", ctypes.c_double),
                ("final_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("rows_scanned", ctypes.c_int64),
                ("probe_rows", ctypes.c_int64), ("main_rows", ctypes.c_int64),
                ("nq", ctypes.c_int32), ("k", ctypes.c_int32),
                ("path", ctypes.c_int32), ("rescans", ctypes.c_int32),
                ("segments", ctypes.c_int32), ("gather", ctypes.c_int32),
                ("prefilter", ctypes.c_int32), ("batch_kernel", ctypes.c_int32),
                ("survivors_total", ctypes.c_int64), ("survivors_max", ctypes.c_int32),
                ("candidates_max", ctypes.c_int32)]


class IndexInfo(ctypes.Structure):
    _fields_ = [("nlist", ctypes.c_int64), ("npos", ctypes.c_int64), ("max_list", ctypes.c_int64),
                ("rows_indexed", ctypes.c_int64), ("metric", ctypes.c_int32), ("dim", ctypes.c_int32),
                ("hbm_bytes", ctypes.c_size_t), ("build_ms", ctypes.c_double)]


class CacheStats(ctypes.Structure):
    _fields_ = [("items", ctypes.c_int64), ("bytes", ctypes.c_size_t), ("max_bytes", ctypes.c_size_t),
                ("hits", ctypes.c_int64), ("misses", ctypes.c_int64), ("evictions", ctypes.c_int64),
                ("pinned", ctypes.c_int64), ("expired_held", ctypes.c_int64)]


class WorkspaceStats(ctypes.Structure):
    _fields_ = [("budget", ctypes.c_size_t), ("held", ctypes.c_size_t), ("peak", ctypes.c_size_t),
                ("waits", ctypes.c_int64), ("trims", ctypes.c_int64), ("over_budget", ctypes.c_int64),
                ("active", ctypes.c_int32), ("workspaces", ctypes.c_int32)]


class IndexSearchStats(ctypes.Structure):
    _fields_ = [("coarse_ms", ctypes.c_double), ("plan_ms", ctypes.c_double),
                ("scan_ms", ctypes.c_double), ("select_ms", ctypes.c_double),
                ("rerank_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("values", ctypes.c_int64), ("items", ctypes.c_int64),
                ("plane_bytes", ctypes.c_int64), ("pairs", ctypes.c_int64),
                ("nq", ctypes.c_int32), ("k", ctypes.c_int32),
                ("nprobe", ctypes.c_int32), ("num_reorder", ctypes.c_int32),
                ("reranked", ctypes.c_int64), ("pick_overflow", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


def _share_hip_runtime_with_torch():
    """PyTorch-ROCm wheels bundle their own libamdhip64.so.7.  If libmqvs.so is
    loaded first, the dynamic linker binds that soname to /opt/rocm's runtime
    and torch then finds no GPU in the same process.  Loading torch first makes
    libmqvs.so bind to the runtime torch already loaded, so the process has one
    HIP runtime.  (Processes without torch use /opt/rocm's.)"""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _load(path=LIB_PATH):
    _share_hip_runtime_with_torch()
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the HIP path has no CPU fallback)")
    L = ctypes.CDLL(path)
    P, I32, I64, U32, U64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                             ctypes.c_uint64)
    sig = {
        "mqvs_abi_version": ([], ctypes.c_int),
        "mqvs_init": ([ctypes.c_int], ctypes.c_int),
        "mqvs_device_count": ([P], ctypes.c_int),
        "mqvs_last_error": ([], ctypes.c_char_p),
        "mqvs_thread_release": ([], ctypes.c_int),
        "mqvs_shutdown": ([], ctypes.c_int),
        "mqvs_segment_create": ([P, I64, I32, I32, I64, P, I64, P], ctypes.c_int),
        "mqvs_segment_create_device": ([P, I64, I32, I32, I64, P, I64, P], ctypes.c_int),
        "mqvs_segment_generate": ([U64, I32, I64, I32, I32, I64, I64, P], ctypes.c_int),
        "mqvs_segment_free": ([P], ctypes.c_int),
        "mqvs_segment_info": ([P, P, P, P, P, P, P], ctypes.c_int),
        "mqvs_segment_prefilter": ([P, P, P, P], ctypes.c_int),
        "mqvs_segment_rows": ([P, P], ctypes.c_int),
        "mqvs_segment_set_rows_host": ([P, ctypes.c_int32], ctypes.c_int),
        "mqvs_segment_rows_host": ([P, P], ctypes.c_int),
        "mqvs_search": ([P, P, I32, I32, I32, P, P, P, P, U32, P], ctypes.c_int),
        "mqvs_search_ex": ([P, P, I32, I32, I32, P, P, I64, P, P, U32, P], ctypes.c_int),
        "mqvs_knn_raw": ([P, P, I64, I64, I64, I64, I32, P, P], ctypes.c_int),
        "mqvs_rerank": ([P, P, I32, P, I32, I32, I32, P, P, P, U32, P], ctypes.c_int),
        "mqvs_merge_shards": ([I32, I32, I32, I32, P, P, P, P, U32, P], ctypes.c_int),
        "mqvs_generate_device": ([U64, I32, I64, I64, I32, P, P], ctypes.c_int),
        "mqvs_last_search_stats": ([P], ctypes.c_int),
        "mqvs_set_timing": ([ctypes.c_int], ctypes.c_int),
        "mqvs_set_batch_mode": ([ctypes.c_int], ctypes.c_int),
        "mqvs_set_gather_mode": ([ctypes.c_int], ctypes.c_int),
        "mqvs_set_scratch_budget": ([ctypes.c_size_t], ctypes.c_size_t),
        "mqvs_set_workspace_budget": ([ctypes.c_size_t], ctypes.c_size_t),
        "mqvs_workspace_stats": ([P, ctypes.c_int32], ctypes.c_int),
        "mqvs_measure_read_bandwidth": ([ctypes.c_size_t, ctypes.c_int32, P, P], ctypes.c_int),
        "mqvs_set_prefilter": ([ctypes.c_int], ctypes.c_int),
        "mqvs_inject_fault": ([I32, I32], ctypes.c_int),
        "mqvs_set_wait_mode": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "mqvs_index_build": ([P, ctypes.c_char_p, ctypes.c_char_p, P], ctypes.c_int),
        "mqvs_index_free": ([P], ctypes.c_int),
        "mqvs_index_info": ([P, P], ctypes.c_int),
        "mqvs_index_search": ([P, P, I32, I32, ctypes.c_char_p, P, P, P, P, U32, P], ctypes.c_int),
        "mqvs_index_last_stats": ([P], ctypes.c_int),
        "mqvs_index_centroids": ([P, P, I64], ctypes.c_int),
        "mqvs_index_probes": ([P, P, I32, ctypes.c_char_p, P], ctypes.c_int),
        "mqvs_segment_create_binary": ([P, I64, I32, I32, I64, I64, U32, P], ctypes.c_int),
        "mqvs_search_binary": ([P, P, I32, I32, I32, P, P, P, P, U32, P], ctypes.c_int),
        "mqvs_knn_binary_raw": ([P, P, I64, I64, I64, I64, I32, P, P], ctypes.c_int),
        "mqvs_segment_create_from_column": ([P, I64, P, I64, I64, I32, I32, I64, I64, U32, P], ctypes.c_int),
        "mqvs_async_check": ([P], ctypes.c_int),
        "mqvs_comm_unique_id": ([P], ctypes.c_int),
        "mqvs_comm_init": ([I32, I32, P, P], ctypes.c_int),
        "mqvs_comm_init_loopback": ([I32, P], ctypes.c_int),
        "mqvs_comm_free": ([P], ctypes.c_int),
        "mqvs_sharded_search": ([P, P, P, I32, I32, I32, P, P, P, P, U32, P], ctypes.c_int),
        "mqvs_comm_stats": ([P, P, P], ctypes.c_int),
        "mqvs_index_set_row_ids_map": ([P, P, I64, U32], ctypes.c_int),
        "mqvs_decoupled_filter": ([P, I64, P, P, I64, U32, P, I64, U32, P], ctypes.c_int),
        "mqvs_cache_create": ([ctypes.c_size_t, P], ctypes.c_int),
        "mqvs_cache_free": ([P], ctypes.c_int),
        "mqvs_cache_put": ([P, ctypes.c_char_p, P, P], ctypes.c_int),
        "mqvs_cache_acquire": ([P, ctypes.c_char_p, P, P], ctypes.c_int),
        "mqvs_cache_release": ([P, ctypes.c_char_p, P], ctypes.c_int),
        "mqvs_cache_remove": ([P, ctypes.c_char_p], ctypes.c_int),
        "mqvs_cache_stats": ([P, P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


class _Lib:
    """The loaded library's functions (attribute access forwards to the CDLL)."""

    def __init__(self, cdll, path):
        self._cdll, self.path = cdll, path

    def __getattr__(self, name):
        return getattr(self._cdll, name)


lib = _Lib(_load(), LIB_PATH)


def use_measurement_build():
    """For measurement tools only (tools/ab_split.py --dbg and the like): route
    every later call of this process to libmqvs_dbg.so, whose kernels read A/B
    switches (some of them diagnostic builds with wrong results) from the
    environment.  The product path and the tests never call this."""
    lib._cdll, lib.path = _load(DBG_LIB_PATH), DBG_LIB_PATH


# DB::ErrorCodes the reference throws for the same conditions
CLICKHOUSE_CODE = {ERR_NOT_IMPLEMENTED: 48, ERR_LOGICAL: 49, ERR_ILLEGAL_COLUMN: 44,
                   ERR_BAD_ARGUMENTS: 36, ERR_MEMORY_LIMIT: 241, ERR_DEVICE: 1001, ERR_CHECKSUM: 40}
CODE_NAME = {ERR_NOT_IMPLEMENTED: "NOT_IMPLEMENTED", ERR_LOGICAL: "LOGICAL_ERROR",
             ERR_ILLEGAL_COLUMN: "ILLEGAL_COLUMN", ERR_BAD_ARGUMENTS: "BAD_ARGUMENTS",
             ERR_MEMORY_LIMIT: "MEMORY_LIMIT_EXCEEDED", ERR_DEVICE: "DEVICE_ERROR",
             ERR_CHECKSUM: "CHECKSUM_DOESNT_MATCH"}


class MqvsError(RuntimeError):
    """Mirror of DB::Exception(code, message) raised by the reference path."""

    def __init__(self, status, message):
        self.status = status
        self.code = CLICKHOUSE_CODE.get(status, 1001)
        self.name = CODE_NAME.get(status, "UNKNOWN")
        super().__init__(f"{self.name} ({self.code}): {message}")


class NotImplementedMetric(MqvsError):
    pass


def check(rc):
    if rc != OK:
        msg = lib.mqvs_last_error()
        msg = msg.decode() if msg else ""
        cls = NotImplementedMetric if rc == ERR_NOT_IMPLEMENTED else MqvsError
        raise cls(rc, msg)
    return rc


def last_search_stats():
    st = SearchStats()
    check(lib.mqvs_last_search_stats(ctypes.byref(st)))
    return {f: getattr(st, f) for f, _ in SearchStats._fields_}


def workspace_stats(reset_peak=False):
    """mqvs_workspace_stats as a dict (bytes and counters of the workspace budget)."""
    st = WorkspaceStats()
    check(lib.mqvs_workspace_stats(ctypes.byref(st), 1 if reset_peak else 0))
    return {f: getattr(st, f) for f, _ in WorkspaceStats._fields_}


def set_wait_mode(mode, spin_us=-1):
    """mqvs_set_wait_mode: how calling threads wait for their GPU work
    (WAIT_RUNTIME / WAIT_HYBRID / WAIT_BLOCK); returns the previous mode."""
    rc = lib.mqvs_set_wait_mode(int(mode), int(spin_us))
    if rc < 0:
        check(-rc)
    return rc


def set_workspace_budget(nbytes):
    """mqvs_set_workspace_budget: returns the previous cap (0 leaves it unchanged)."""
    return lib.mqvs_set_workspace_budget(int(nbytes))


def last_index_stats():
    st = IndexSearchStats()
    check(lib.mqvs_index_last_stats(ctypes.byref(st)))
    return {f: getattr(st, f) for f, _ in IndexSearchStats._fields_}
