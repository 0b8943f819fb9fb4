"""Column ingest on the GPU (mqvs_segment_create_from_column) vs the CPU
oracle: the decoded rows are bit-identical to the oracle's decode + copy loop
(MergeTreeVSManager.cpp:1381-1393), and searches over the ingested segment
equal the oracle's vectorScanWithoutIndex on those rows."""
import ctypes
import struct

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def device_rows(mq, seg):
    """Copy a segment's resident rows back (hipMemcpy D2H)."""
    ptr = seg.device_rows_ptr()
    out = np.empty((seg.n, seg.d), np.float32)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipDeviceSynchronize()
    rc = hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), ctypes.c_size_t(out.nbytes), 2)
    assert rc == 0
    return out


def column_files(data_f32, sizes, block=1 << 20, method=0x82):
    return (O.compress_stream(np.ascontiguousarray(data_f32, np.float32).tobytes(), block, method),
            O.compress_stream(np.ascontiguousarray(sizes, np.uint64).tobytes(), block, method))


@pytest.mark.parametrize("kind,block,method", [("gauss", 1 << 20, 0x82), ("quantised", 65536, 0x82),
                                               ("repeats", 4097, 0x82), ("gauss", 300000, 0x02),
                                               ("quantised", 1 << 20, 0x82), ("period24k", 1 << 20, 0x82),
                                               ("period40k", 1 << 20, 0x82), ("mixed", 1 << 20, 0x82),
                                               ("mixed", 70000, 0x82), ("sparse_rle", 1 << 20, 0x82),
                                               ("sparse_rle", 65536, 0x82)])
def test_gpu_ingest_dense(mq, kind, block, method):
    """periodNk: the rows repeat every N KiB, so nearly every match reaches
    back further than the decoder's 4 KiB LDS ring (its far-match path reads
    the block's flushed output), long matches included.  mixed: 16-float
    pieces of four kinds (fresh gaussian = literal runs of every length,
    quantised = short matches, copies of a recent piece = longer and
    overlapping matches, constant runs), so the decoder's groups of short
    sequences alternate with the wave-wide long-sequence paths.  sparse_rle:
    blocks compressed to >= 7/8 of their size take the token-at-a-time path,
    with overlapping and far matches."""
    rng = np.random.default_rng(11)
    n, d = 20000, 64
    if kind == "gauss":
        rows = rng.standard_normal((n, d)).astype(np.float32)
    elif kind == "quantised":
        rows = np.round(rng.standard_normal((n, d)), 1).astype(np.float32)
    elif kind.startswith("period"):
        period = (96 if kind == "period24k" else 156)  # rows of 256 B: 24576 / 39936 B
        base = rng.standard_normal((period, d)).astype(np.float32)
        base[::7] = np.round(base[::7], 1)
        rows = np.tile(base, (n // period + 1, 1))[:n].copy()
        rows[::97] += 1.0  # break some matches: fresh literals between far matches
    elif kind == "sparse_rle":
        # nearly incompressible (the decoder's one-token-at-a-time path): Gaussian
        # rows, every 37th with runs of one repeated float (overlapping matches,
        # off = 4) and every 53rd a copy of an earlier row (far matches)
        rows = rng.standard_normal((n, d)).astype(np.float32)
        rows[::37, 8:40] = rows[::37, 7:8]
        rows[53::53] = rows[:-53:53][: len(rows[53::53])]
    elif kind == "mixed":
        pieces = rng.integers(0, 4, n * d // 16)
        flat = np.round(rng.standard_normal(n * d), 1).astype(np.float32)
        g = rng.standard_normal(n * d).astype(np.float32)
        for i in np.nonzero(pieces == 0)[0]:
            flat[16 * i:16 * i + 16] = g[16 * i:16 * i + 16]
        for i in np.nonzero(pieces == 2)[0]:
            j = max(0, i - int(rng.integers(1, 40)))
            flat[16 * i:16 * i + 16] = flat[16 * j:16 * j + 16]
        for i in np.nonzero(pieces == 3)[0]:
            flat[16 * i:16 * i + 16] = flat[16 * i - 1] if i else 0.5
        rows = flat.reshape(n, d)
    else:  # long matches incl. overlapping ones (runs of equal values, repeated rows)
        base = np.repeat(rng.integers(-3, 4, (n // 8, d // 4)).astype(np.float32), 4, axis=1)
        rows = np.repeat(base, 8, axis=0)
    sizes = np.full(n, d, np.uint64)
    db, sb = column_files(rows, sizes, block, method)
    seg = mq.VectorScanSegment.from_column(db, sb, n, d, metric="L2", granule=8192)
    try:
        got = device_rows(mq, seg)
        assert np.array_equal(got.view(np.uint32), rows.view(np.uint32))
        q = rng.standard_normal((3, d)).astype(np.float32)
        ids, dist = seg.search(q, 20)
        ids_o, dist_o = O.vector_scan(rows, q, 20, O.L2, 8192)
        assert np.array_equal(ids, ids_o) and np.array_equal(dist.view(np.uint32), dist_o.view(np.uint32))
    finally:
        seg.free()


def test_gpu_ingest_ragged_cosine(mq):
    """Empty, short and long arrays; cosine with a PREWHERE filter: the
    reference's copy loop semantics end to end."""
    rng = np.random.default_rng(12)
    n, d = 30000, 48
    sizes = rng.choice([0, d, d, d, d - 5, d + 7], n).astype(np.uint64)
    sizes[: 8192] = np.where(sizes[:8192] == 0, d, sizes[:8192])
    sizes[8192:16384] = 0  # a whole granule of empty arrays (never searched)
    data = rng.standard_normal(int(sizes.sum())).astype(np.float32)
    db, sb = column_files(data, sizes, 1 << 18)
    rows, ne = O.array_rows(data, sizes, d)
    seg = mq.VectorScanSegment.from_column(db, sb, n, d, metric="Cosine", granule=8192)
    try:
        q = rng.standard_normal((4, d)).astype(np.float32)
        flt = np.packbits(rng.random(n) < 0.7, bitorder="little")
        for f in (None, flt):
            ids, dist = seg.search(q, 30, filter_bitmap=f)
            ids_o, dist_o = O.vector_scan(rows, q, 30, O.COSINE, 8192, nonempty=ne, filter_bits=f)
            assert np.array_equal(ids, ids_o)
            assert np.array_equal(dist.view(np.uint32), dist_o.view(np.uint32))
    finally:
        seg.free()


def test_gpu_ingest_device_streams(mq):
    import torch
    rng = np.random.default_rng(13)
    n, d = 5000, 32
    rows = rng.standard_normal((n, d)).astype(np.float32)
    db, sb = column_files(rows, np.full(n, d, np.uint64), 1 << 16)
    tdb = torch.frombuffer(bytearray(db), dtype=torch.uint8).cuda()
    tsb = torch.frombuffer(bytearray(sb), dtype=torch.uint8).cuda()
    seg = mq.VectorScanSegment.from_column(tdb, tsb, n, d, metric="IP")
    try:
        assert np.array_equal(device_rows(mq, seg).view(np.uint32), rows.view(np.uint32))
    finally:
        seg.free()


def _corrupt(db, what):
    b = bytearray(db)
    if what == "truncated":
        return bytes(b[:-7])
    if what == "method":
        b[16] = 0x90  # ZSTD
        return bytes(b)
    raise ValueError(what)


def _hand_block(offset):
    """12 bytes = 3 floats: literal "abcd", a 4-byte match at `offset`, last
    literals "wxyz" (LZ4 block format)."""
    blk = bytes([0x40]) + b"abcd" + struct.pack("<H", offset) + bytes([0x40]) + b"wxyz"
    body = struct.pack("<BII", 0x82, 9 + len(blk), 12) + blk
    return O.checksum_bytes(body) + body


def test_gpu_ingest_hand_built_lz4(mq):
    from myscaledb_amd import _lib
    sb = O.compress_stream(np.array([3], np.uint64).tobytes())
    seg = mq.VectorScanSegment.from_column(_hand_block(4), sb, 1, 3, metric="L2")
    try:
        want = np.frombuffer(b"abcdabcdwxyz", np.float32)
        assert np.array_equal(device_rows(mq, seg)[0].view(np.uint32), want.view(np.uint32))
    finally:
        seg.free()
    with pytest.raises(_lib.MqvsError) as e:  # match before the start of the block
        mq.VectorScanSegment.from_column(_hand_block(9), sb, 1, 3, metric="L2")
    assert e.value.status == _lib.ERR_ILLEGAL_COLUMN


@pytest.mark.parametrize("what,status", [("truncated", 3), ("method", 1), ("count", 3)])
def test_gpu_ingest_errors(mq, what, status):
    from myscaledb_amd import _lib
    rng = np.random.default_rng(14)
    n, d = 1000, 16
    rows = rng.standard_normal((n, d)).astype(np.float32)
    db, sb = column_files(rows, np.full(n, d, np.uint64), 1 << 14)
    nn = n
    if what == "count":
        nn = n + 1
    else:
        db = _corrupt(db, what)
    with pytest.raises(_lib.MqvsError) as e:
        mq.VectorScanSegment.from_column(db, sb, nn, d, metric="L2")
    assert e.value.status == status, str(e.value)


@pytest.mark.parametrize("stream,where", [("data", "payload"), ("data", "stored"), ("sizes", "payload")])
def test_gpu_ingest_checksum_mismatch(mq, stream, where):
    """CompressedReadBufferBase.cpp:192-196: a corrupted block fails with
    CHECKSUM_DOESNT_MATCH (status 7, ClickHouse code 40) before decoding;
    with verification disabled the (NONE-method) block decodes as stored."""
    from myscaledb_amd import _lib
    rng = np.random.default_rng(15)
    n, d = 3000, 16
    rows = rng.standard_normal((n, d)).astype(np.float32)
    db, sb = column_files(rows, np.full(n, d, np.uint64), 1 << 14, 0x02)
    b = bytearray(db if stream == "data" else sb)
    b[25 + 1000 if where == "payload" else 5] ^= 0x04
    db, sb = (bytes(b), sb) if stream == "data" else (db, bytes(b))
    with pytest.raises(_lib.MqvsError) as e:
        mq.VectorScanSegment.from_column(db, sb, n, d, metric="L2")
    assert e.value.status == _lib.ERR_CHECKSUM, str(e.value)
    assert _lib.CLICKHOUSE_CODE[e.value.status] == 40
    if stream == "data":
        seg = mq.VectorScanSegment.from_column(db, sb, n, d, metric="L2", verify_checksum=False)
        try:
            want = np.frombuffer(O.decompress_stream(db, rows.nbytes, verify=False), np.float32).reshape(n, d)
            assert np.array_equal(device_rows(mq, seg).view(np.uint32), want.view(np.uint32))
        finally:
            seg.free()


def test_gpu_checksum_every_block_length(mq):
    """Blocks of 1..400 payload bytes (hashed lengths 10..409: every
    CityMurmur / 128-byte-loop / tail branch) at every byte alignment, NONE and
    LZ4 alternating: the GPU CityHash128 must accept all of them (one wrong
    hash fails the ingest) and the rows must round-trip bit-exactly."""
    rng = np.random.default_rng(16)
    n, d = 700, 64
    rows = np.round(rng.standard_normal((n, d)), 1).astype(np.float32)
    raw = rows.tobytes()
    parts, o, blen = [], 0, 1
    while o < len(raw):
        take = min(blen, len(raw) - o)
        parts.append(O.compress_stream(raw[o:o + take], take, 0x02 if blen % 2 else 0x82))
        o += take
        blen = blen % 400 + 1
    db = b"".join(parts)
    sb = O.compress_stream(np.full(n, d, np.uint64).tobytes(), 1 << 20)
    assert O.decompress_stream(db, len(raw)) == raw
    seg = mq.VectorScanSegment.from_column(db, sb, n, d, metric="L2")
    try:
        assert np.array_equal(device_rows(mq, seg).view(np.uint32), rows.view(np.uint32))
    finally:
        seg.free()
