"""ctypes loader for the CPU oracle (oracle/_build/libmqvs_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package (myscaledb_amd/).
The C sources (mqvs_oracle.c) restate the reference functions they cite.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmqvs_oracle.so")

L2, IP, COSINE, HAMMING, JACCARD = 0, 1, 2, 4, 5
METRICS = {"L2": L2, "IP": IP, "Cosine": COSINE, "COSINE": COSINE, "Hamming": HAMMING, "Jaccard": JACCARD}

_lib = None


def build(quiet: bool = True) -> str:
    """Compile the oracle with the committed Makefile (gcc)."""
    out = subprocess.run(["make", "-C", _HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I64 = ctypes.c_int64
        L.orc_knn.argtypes = [P, P, I64, I64, I64, I64, ctypes.c_int, P, P]
        L.orc_knn_fast.argtypes = L.orc_knn.argtypes
        L.orc_search_without_index.argtypes = L.orc_knn.argtypes
        L.orc_normalize.argtypes = [P, I64, I64]
        L.orc_vector_scan.argtypes = [P, P, I64, I64, P, I64, P, I64, I64, ctypes.c_int, P, P, P, P]
        L.orc_vector_scan_fast.argtypes = L.orc_vector_scan.argtypes
        L.orc_scan_parts.argtypes = [P, I64, I64, I64, P, I64, I64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, P, P]
        L.orc_merge_parts.argtypes = [I64, I64, ctypes.c_int, P, P, P, P, P]
        L.orc_hamming_knn.argtypes = [P, P, I64, I64, I64, I64, P, P]
        L.orc_jaccard_knn.argtypes = [P, P, I64, I64, I64, I64, P, P]
        L.orc_jaccard.argtypes = [P, P, I64]
        L.orc_jaccard.restype = ctypes.c_float
        L.orc_knn_binary.argtypes = [P, P, I64, I64, I64, I64, ctypes.c_int, P, P]
        L.orc_vector_scan_binary.argtypes = [P, I64, I64, P, I64, P, I64, I64, ctypes.c_int, P, P, P, P]
        L.orc_lz4_decompress.argtypes = [P, I64, P, I64]
        L.orc_lz4_compress.argtypes = [P, I64, P, I64]
        L.orc_lz4_compress.restype = I64
        L.orc_compress_stream.argtypes = [P, I64, I64, ctypes.c_int, P, I64]
        L.orc_compress_stream.restype = I64
        L.orc_decompress_stream.argtypes = [P, I64, P, I64, ctypes.c_int]
        L.orc_cityhash128.argtypes = [P, I64, P]
        L.orc_decompress_stream.restype = I64
        L.orc_array_rows.argtypes = [P, I64, P, I64, I64, P, P]
        L.orc_generate.argtypes = [ctypes.c_uint64, ctypes.c_int, I64, I64, I64, P]
        L.orc_gemm_dot.argtypes = [P, P, I64]
        L.orc_gemm_dot.restype = ctypes.c_float
        L.orc_gemm_dot_blocked.argtypes = [P, P, I64, I64]
        L.orc_gemm_dot_blocked.restype = ctypes.c_float
        L.orc_norm_l2sqr.argtypes = [P, I64]
        L.orc_norm_l2sqr.restype = ctypes.c_float
        L.orc_l2sqr.argtypes = [P, P, I64]
        L.orc_l2sqr.restype = ctypes.c_float
        L.orc_inner_product.argtypes = [P, P, I64]
        L.orc_inner_product.restype = ctypes.c_float
        for f in ("orc_knn", "orc_knn_fast", "orc_search_without_index", "orc_vector_scan",
                  "orc_vector_scan_fast", "orc_scan_parts"):
            getattr(L, f).restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def knn(x, y, k, metric, fast=False):
    """tryBruteForceSearch (BruteForceSearch.h:62-111)."""
    x, y = _f32(x), _f32(y)
    nx, d = x.shape
    ny = y.shape[0]
    ids = np.empty((nx, k), np.int64)
    dist = np.empty((nx, k), np.float32)
    fn = lib().orc_knn_fast if fast else lib().orc_knn
    rc = fn(_p(x), _p(y), d, k, nx, ny, metric, _p(ids), _p(dist))
    if rc:
        raise NotImplementedError("metric not implemented in brute force search")
    return ids, dist


def search_without_index(x, y, k, metric):
    """VIWithColumnInPart::searchWithoutIndex; copies (the C function mutates)."""
    x, y = _f32(x).copy(), _f32(y).copy()
    nx, d = x.shape
    ids = np.empty((nx, k), np.int64)
    dist = np.empty((nx, k), np.float32)
    rc = lib().orc_search_without_index(_p(x), _p(y), d, k, nx, y.shape[0], metric, _p(ids), _p(dist))
    if rc:
        raise NotImplementedError
    return ids, dist


def normalize(a):
    a = _f32(a).copy()
    lib().orc_normalize(_p(a), a.shape[0], a.shape[1])
    return a


def vector_scan(rows, queries, k, metric, mark_rows, nonempty=None, filter_bits=None,
                row_exists_bits=None, fast=False):
    """MergeTreeVSManager::vectorScanWithoutIndex over one part.

    rows: (n, d) float32 (FLT_MAX-filled where the array is empty);
    nonempty: (n,) uint8 or None; filter_bits/row_exists_bits: packed LSB-first
    uint8 bitmaps (np.packbits(..., bitorder='little')) or None;
    mark_rows: int or list of rows per mark.
    """
    rows, queries = _f32(rows), _f32(queries)
    n, d = rows.shape
    nq = queries.shape[0]
    if np.isscalar(mark_rows):
        mr = np.full(max(1, -(-n // int(mark_rows))), int(mark_rows), np.int64)
    else:
        mr = np.ascontiguousarray(mark_rows, np.int64)
    ne = None if nonempty is None else np.ascontiguousarray(nonempty, np.uint8)
    fb = None if filter_bits is None else np.ascontiguousarray(filter_bits, np.uint8)
    rb = None if row_exists_bits is None else np.ascontiguousarray(row_exists_bits, np.uint8)
    ids = np.empty((nq, k), np.int64)
    dist = np.empty((nq, k), np.float32)
    fn = lib().orc_vector_scan_fast if fast else lib().orc_vector_scan
    rc = fn(_p(rows), _p(ne), n, d, _p(mr), len(mr), _p(queries), nq, k, metric, _p(fb), _p(rb),
            _p(ids), _p(dist))
    if rc:
        raise NotImplementedError
    return ids, dist


def _u8(a):
    return np.ascontiguousarray(a, np.uint8)


def knn_binary(x, y, k, metric):
    """tryBruteForceSearch<BinaryVector> (BruteForceSearch.h:94-110) on code
    arrays x (nx, N) and y (ny, N) uint8.  Hamming: int32 distances (the
    reference's reinterpret of the float buffer); Jaccard: float32."""
    x, y = _u8(x), _u8(y)
    nx, nb = x.shape
    ny = y.shape[0]
    ids = np.empty((nx, k), np.int64)
    dist = np.empty((nx, k), np.int32 if metric == HAMMING else np.float32)
    if lib().orc_knn_binary(_p(x), _p(y), nb * 8, k, nx, ny, metric, _p(ids), _p(dist)):
        raise NotImplementedError
    return ids, dist


def vector_scan_binary(codes, queries, k, metric, mark_rows, filter_bits=None, row_exists_bits=None):
    """vectorScanWithoutIndex<BinaryVector> over one part: codes (n, N) uint8
    (FixedString(N)); returns ids (nq, k) and float32 distances."""
    codes, queries = _u8(codes), _u8(queries)
    n, nb = codes.shape
    nq = queries.shape[0]
    if np.isscalar(mark_rows):
        mr = np.full(max(1, -(-n // int(mark_rows))), int(mark_rows), np.int64)
    else:
        mr = np.ascontiguousarray(mark_rows, np.int64)
    fb = None if filter_bits is None else _u8(filter_bits)
    rb = None if row_exists_bits is None else _u8(row_exists_bits)
    ids = np.empty((nq, k), np.int64)
    dist = np.empty((nq, k), np.float32)
    if lib().orc_vector_scan_binary(_p(codes), n, nb, _p(mr), len(mr), _p(queries), nq, k, metric, _p(fb),
                                    _p(rb), _p(ids), _p(dist)):
        raise NotImplementedError
    return ids, dist


def compress_stream(data: bytes | np.ndarray, block_size=1 << 20, method=0x82) -> bytes:
    """ClickHouse CompressedWriteBuffer framing + LZ4 (test data), CityHash128 block checksums."""
    src = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else _u8(data.view(np.uint8))
    cap = int(src.size + src.size // 200 + 64 * (src.size // block_size + 1) + 1024)
    out = np.empty(cap, np.uint8)
    n = lib().orc_compress_stream(_p(src), src.size, block_size, method, _p(out), cap)
    if n < 0:
        raise ValueError("compress_stream failed")
    return out[:n].tobytes()


def decompress_stream(blob: bytes, cap: int, verify: bool = True) -> bytes:
    src = np.frombuffer(blob, np.uint8)
    out = np.empty(max(cap, 1), np.uint8)
    n = lib().orc_decompress_stream(_p(src), src.size, _p(out), cap, int(verify))
    if n == -2:
        raise ValueError("CHECKSUM_DOESNT_MATCH")
    if n < 0:
        raise ValueError("CANNOT_DECOMPRESS")
    return out[:n].tobytes()


def cityhash128(data) -> tuple:
    """CityHash_v1_0_2::CityHash128 (oracle restatement): (low64, high64)."""
    src = np.frombuffer(bytes(data), np.uint8)
    h = np.zeros(2, np.uint64)
    lib().orc_cityhash128(_p(src) if src.size else None, src.size, _p(h))
    return int(h[0]), int(h[1])


def checksum_bytes(data) -> bytes:
    """The 16 checksum bytes ClickHouse stores before a compressed block."""
    lo, hi = cityhash128(data)
    return lo.to_bytes(8, "little") + hi.to_bytes(8, "little")


def array_rows(data_f32, sizes_u64, d):
    """MergeTreeVSManager.cpp:1381-1393: (rows[n,d] float32, nonempty[n] uint8)."""
    data = _f32(data_f32).reshape(-1)
    sizes = np.ascontiguousarray(sizes_u64, np.uint64)
    n = sizes.size
    rows = np.empty((n, d), np.float32)
    ne = np.empty(n, np.uint8)
    if lib().orc_array_rows(_p(data), data.size, _p(sizes), n, d, _p(rows), _p(ne)):
        raise ValueError("array sizes do not match the data stream")
    return rows, ne


def scan_parts(rows, queries, k, metric, granule, parts, threads):
    rows, queries = _f32(rows), _f32(queries)
    n, d = rows.shape
    nq = queries.shape[0]
    ids = np.empty((nq, k), np.int64)
    dist = np.empty((nq, k), np.float32)
    lib().orc_scan_parts(_p(rows), n, d, granule, _p(queries), nq, k, metric, parts, threads,
                         _p(ids), _p(dist))
    return ids, dist


def has_avx512() -> bool:
    return bool(lib().orc_has_avx512())


def stream_triad(n=1 << 26, threads=1, reps=5) -> float:
    """STREAM triad GB/s (doubles, 24 B per element) on `threads` threads."""
    f = lib().orc_stream_triad
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    return float(f(n, threads, reps))


def merge_parts(labels, dists, metric):
    labels = np.ascontiguousarray(labels, np.int64)
    dists = _f32(dists)
    nparts, k = labels.shape
    op = np.empty(k, np.int64)
    ol = np.empty(k, np.int64)
    od = np.empty(k, np.float32)
    lib().orc_merge_parts(nparts, k, metric, _p(labels), _p(dists), _p(op), _p(ol), _p(od))
    return op, ol, od


def generate(seed, mode, row0, n, d):
    out = np.empty((n, d), np.float32)
    lib().orc_generate(seed, mode, row0, n, d, _p(out))
    return out


def l2sqr(x, y):
    x, y = _f32(x), _f32(y)
    return np.float32(lib().orc_l2sqr(_p(x), _p(y), x.shape[0]))


def inner_product(x, y):
    x, y = _f32(x), _f32(y)
    return np.float32(lib().orc_inner_product(_p(x), _p(y), x.shape[0]))


def gemm_dot(x, y):
    """fma-chain dot (the BLAS-branch sgemm element, nq >= 20)."""
    x, y = _f32(x), _f32(y)
    return np.float32(lib().orc_gemm_dot(_p(x), _p(y), x.shape[0]))


def gemm_dot_blocked(x, y, kb):
    """sgemm-style K-blocked element (blocks of kb, each an fma chain, summed
    in order): the BLAS-order parity-risk model, not the reference formula."""
    x, y = _f32(x), _f32(y)
    return np.float32(lib().orc_gemm_dot_blocked(_p(x), _p(y), x.shape[0], int(kb)))


def norm_l2sqr(x):
    x = _f32(x)
    return np.float32(lib().orc_norm_l2sqr(_p(x), x.shape[0]))
