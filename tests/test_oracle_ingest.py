"""Column-ingest oracle (CPU, test infrastructure): ClickHouse compressed-block
framing, LZ4 block decoding and the Array(Float32) -> rows copy loop.

Reference: CompressedReadBufferBase.cpp:115-160 (framing), CompressionInfo.h
(method bytes), LZ4_decompress_faster.cpp:480-640 (LZ4 block format),
MergeTreeVSManager.cpp:1381-1393 (copy loop).  No compressed fixture ships
with the reference, so the decoder is pinned by hand-built blocks that follow
the LZ4 block format and by compress -> decompress round trips.
"""
import ctypes
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O


def frame(payload: bytes, usize: int, method=0x82) -> bytes:
    body = struct.pack("<BII", method, 9 + len(payload), usize) + payload
    return O.checksum_bytes(body) + body


# Block checksum (CompressedReadBufferBase.cpp:37-45, CityHash128 v1.0.2):
# pinned by golden vectors from the reference's own city.cc
# (tests/golden/cityhash102.json, made by tests/golden/make_cityhash.py) and,
# when oracle/_ref is built, against that build directly.
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "cityhash102.json")
REF_CITY = os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref", "libcityref.so")


def golden_data(n):
    return ((np.arange(n, dtype=np.int64) * 131 + n * 7 + 3) & 255).astype(np.uint8).tobytes()


def test_cityhash_golden_vectors():
    """Oracle CityHash128 == the reference city.cc on every golden length
    (0..199 covers every short / murmur / tail branch; up to 1 MiB + 9)."""
    vec = json.load(open(GOLDEN))["vectors"]
    assert len(vec) >= 200
    for v in vec:
        lo, hi = O.cityhash128(golden_data(v["len"]))
        assert (f"{lo:016x}", f"{hi:016x}") == (v["lo"], v["hi"]), v["len"]


@pytest.mark.skipif(not os.path.exists(REF_CITY), reason="oracle/_ref not built (make -C oracle ref)")
def test_cityhash_vs_reference_build():
    ref = ctypes.CDLL(REF_CITY)
    ref.ref_cityhash128.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    rng = np.random.default_rng(9)
    for n in list(range(0, 300)) + [1023, 4096 + 9, 65536 + 37]:
        a = rng.integers(0, 256, n, dtype=np.uint8)
        h = np.zeros(2, np.uint64)
        ref.ref_cityhash128(a.ctypes.data if n else None, n, h.ctypes.data)
        assert O.cityhash128(a.tobytes()) == (int(h[0]), int(h[1])), n


@pytest.mark.parametrize("where", ["payload", "header", "stored"])
def test_checksum_mismatch_detected(where):
    """A flipped bit anywhere in a block -> CHECKSUM_DOESNT_MATCH before any
    decoding (CompressedReadBufferBase.cpp:192-196); verify=False decodes."""
    data = np.arange(5000, dtype=np.float32).tobytes()
    c = bytearray(O.compress_stream(data, 4096, 0x02))
    pos = {"payload": 25 + 100, "header": 16 + 5, "stored": 3}[where]
    c[pos] ^= 0x10
    with pytest.raises(ValueError, match="CHECKSUM"):
        O.decompress_stream(bytes(c), len(data))
    if where != "header":  # sizes intact: decodes without verification
        out = O.decompress_stream(bytes(c), len(data), verify=False)
        assert len(out) == len(data) and (out == data) == (where == "stored")


def test_lz4_hand_built_blocks():
    # literal "abcd", match offset 4 length 8 (overlapping copy), last literals "xyz01"
    blk = bytes([0x44]) + b"abcd" + struct.pack("<H", 4) + bytes([0x50]) + b"xyz01"
    out = O.decompress_stream(frame(blk, 17), 17)
    assert out == b"abcdabcdabcdxyz01"
    # offset 1: run-length replication; extended literal length (15 + 3 = 18)
    lit = bytes(range(65, 65 + 18))
    blk = bytes([0xF0 | 0x0F]) + bytes([3]) + lit + struct.pack("<H", 1) + bytes([5]) + bytes([0x50]) + b"END!!"
    want = lit + lit[-1:] * (15 + 5 + 4) + b"END!!"
    assert O.decompress_stream(frame(blk, len(want)), len(want)) == want
    # NONE method block
    assert O.decompress_stream(frame(b"plain", 5, 0x02), 5) == b"plain"


@pytest.mark.parametrize("bad", ["offset0", "offset_far", "truncated", "method"])
def test_lz4_malformed_rejected(bad):
    if bad == "offset0":
        blk = bytes([0x40]) + b"abcd" + struct.pack("<H", 0) + bytes([0x10]) + b"z"
        s = frame(blk, 9)
    elif bad == "offset_far":
        blk = bytes([0x40]) + b"abcd" + struct.pack("<H", 9) + bytes([0x10]) + b"z"
        s = frame(blk, 9)
    elif bad == "truncated":
        s = frame(bytes([0x50]) + b"abc", 5)
    else:
        s = frame(b"plain", 5, 0x90)
    with pytest.raises(ValueError):
        O.decompress_stream(s, 64)


@pytest.mark.parametrize("kind", ["gauss", "quantised", "zeros", "tiny"])
@pytest.mark.parametrize("block", [1 << 20, 65536, 4097])
def test_stream_round_trip(kind, block):
    rng = np.random.default_rng(5)
    if kind == "gauss":
        data = rng.standard_normal(300000).astype(np.float32).tobytes()
    elif kind == "quantised":
        data = np.round(rng.standard_normal(300000), 1).astype(np.float32).tobytes()
    elif kind == "zeros":
        data = bytes(200000)
    else:
        data = b"\x01\x02\x03"
    c = O.compress_stream(data, block)
    assert O.decompress_stream(c, len(data)) == data


def test_array_rows_copy_loop():
    """Empty arrays -> FLT_MAX rows flagged empty, short ones FLT_MAX-padded,
    long ones truncated (MergeTreeVSManager.cpp:1381-1393)."""
    sizes = np.array([3, 0, 1, 5], np.uint64)
    data = np.arange(9, dtype=np.float32)
    rows, ne = O.array_rows(data, sizes, 3)
    FM = np.float32(3.4028235e38)
    assert rows.tolist() == [[0, 1, 2], [FM, FM, FM], [3, FM, FM], [4, 5, 6]]
    assert ne.tolist() == [1, 0, 1, 1]
    with pytest.raises(ValueError):
        O.array_rows(data[:8], sizes, 3)
