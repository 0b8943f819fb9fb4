// kernels_ingest.hip -- column ingest on the GPU: a
// MergeTree Array(Float32) column, as the bytes of its compressed files, is
// decoded in HBM into the rows matrix the scan reads.  It replaces the host
// read + copy loop of MergeTreeVSManager.cpp:1348-1393 (per granule:
// CompressedReadBuffer -> LZ4 -> ColumnArray -> vector_raw_data).
//
//   k_block_table   the chain of compressed blocks (CompressedReadBufferBase.cpp
//                   :115-160; CompressionInfo.h: 16-B checksum, method byte,
//                   UInt32 compressed size incl. the 9-B header, UInt32
//                   decompressed size).  One thread walks the headers; a
//                   1 MiB block costs one dependent 25-B read.
//   k_decode_blocks one 64-lane workgroup per block.  LZ4 (LZ4_decompress_faster
//                   .cpp:480-640 block format): the token stream is parsed in
//                   lock-step (uniform control flow) into groups of up to 64
//                   sequences, one per lane; a group's literal runs are then
//                   copied at once and its matches in dependency rounds
//                   (a lane per sequence).  Long literal runs go as whole
//                   output dwords (copy_literals), long matches 256 bytes per
//                   step.  Matches read from an 8 KiB LDS ring of the block's
//                   latest output, farther ones from the flushed output.
//   k_block_checksum CityHash128 v1.0.2 of every block (one lane per block),
//                   compared with the stored 16-B checksum.
//   k_sizes_scan_*  array sizes (UInt64 per row) -> element offsets.
//   k_array_rows    the copy loop of :1381-1393: FLT_MAX fill, first
//                   min(size, d) elements of a non-empty array, nonempty flag.
#include "mqvs_internal.h"
#include "tuning.h"

namespace mqvs {

// LDS ring of the block's latest output.  8 KiB (not the 64 KiB LZ4 window)
// so that twenty decode waves fit on a CU: the decode is latency-bound per
// wave, and a 64 KiB ring left two waves per CU.  Matches reaching further
// back (~6 % of them on quantised float columns) read the already-flushed
// output from global memory (far_byte).
constexpr int kRing = 4096;
constexpr int kFlush = 1024;  // unflushed output < kFlush + one step (< kRing - 256)
// a group holds sequences of at most kGrpLit literals and kGrpMatch match
// bytes: 64 of them write < kRing - kFlush - 256 bytes
constexpr int kGrpLit = 16, kGrpMatch = 27;
static_assert(64 * (kGrpLit + kGrpMatch) + kFlush + 256 < kRing, "group output must fit the ring");

__global__ void k_block_table(const uint8_t *src, int64_t n, IngestBlock *tab, int64_t max_blocks,
                              int64_t *out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t pos = 0, nb = 0, total = 0, status = 0;
    while (pos < n) {
        if (n - pos < 25 || nb >= max_blocks) {
            status = 1;
            break;
        }
        const uint8_t *h = src + pos + 16;
        const uint32_t method = h[0];
        const uint32_t csize = (uint32_t)h[1] | ((uint32_t)h[2] << 8) | ((uint32_t)h[3] << 16) | ((uint32_t)h[4] << 24);
        const uint32_t usize = (uint32_t)h[5] | ((uint32_t)h[6] << 8) | ((uint32_t)h[7] << 16) | ((uint32_t)h[8] << 24);
        if ((method != 0x82 && method != 0x02) || csize < 9 || pos + 16 + (int64_t)csize > n ||
            (method == 0x02 && csize - 9 != usize)) {
            status = method != 0x82 && method != 0x02 ? 2 : 1;
            break;
        }
        tab[nb].src = pos + 25;
        tab[nb].dst = total;
        tab[nb].csize = csize - 9;
        tab[nb].usize = usize;
        tab[nb].method = method;
        ++nb;
        total += usize;
        pos += 16 + csize;
    }
    out[0] = nb;
    out[1] = total;
    out[2] = status;
}

// all lanes see the same values (uniform parse); bytes of the compressed input
__device__ __forceinline__ uint32_t in_byte(const uint8_t *p, int64_t i) { return p[i]; }

// Literal run: output bytes [op, op + len) of the block <- s[0, len), also
// into the LDS ring.  Long runs (incompressible floats are one run per block)
// go by whole output dwords: two aligned source dwords per lane joined by
// v_alignbyte, 8 per lane in flight (2 KiB per wave); the ragged head and tail
// go byte by byte.  out must be 4-byte aligned for the dword path.
__device__ __forceinline__ void copy_literals(const uint8_t *s, const uint8_t *s_end, uint8_t *out, int64_t op,
                                              int64_t len, uint8_t *ring, int lane) {
    auto byte_copy = [&](int64_t b, int64_t e) {
        for (int64_t i = b + lane; i < e; i += 64) {
            const uint8_t v = s[i];
            out[op + i] = v;
            ring[(op + i) & (kRing - 1)] = v;
        }
    };
    if (len < 256 || ((uintptr_t)out & 3)) {
        byte_copy(0, len);
        return;
    }
    const int64_t head = (4 - (op & 3)) & 3;
    byte_copy(0, head);
    const int64_t p0 = op + head, nw = (len - head) >> 2;
    const uintptr_t sa = (uintptr_t)(s + head);
    const int sh = (int)(sa & 3);
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(sa & ~(uintptr_t)3);
    uint32_t *ow = reinterpret_cast<uint32_t *>(out + p0);
    uint32_t *rw = reinterpret_cast<uint32_t *>(ring);
    const int64_t r0 = p0 >> 2;
    constexpr int U = 8;
    for (int64_t w0 = 0; w0 < nw; w0 += 64 * U) {
        uint32_t lo[U], hi[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t w = w0 + u * 64 + lane;
            lo[u] = hi[u] = 0;
            if (w < nw) {
                lo[u] = sw[w];
                if (sh) {
                    const uint32_t *nx = sw + w + 1;
                    if ((const uint8_t *)nx + 4 <= s_end) {
                        hi[u] = *nx;
                    } else {  // the stream ends inside this dword: only its leading bytes exist
                        const uint8_t *b = (const uint8_t *)nx;
                        for (int k = 0; k < 4 && b + k < s_end; ++k) hi[u] |= (uint32_t)b[k] << (8 * k);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t w = w0 + u * 64 + lane;
            if (w < nw) {
                const uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi[u], lo[u], (uint32_t)sh) : lo[u];
                ow[w] = v;
                rw[(r0 + w) & (kRing / 4 - 1)] = v;
            }
        }
    }
    byte_copy(head + 4 * nw, len);
}

// A byte of this wave's own earlier, flushed output: the stores are waited
// for (vmcnt) by the caller; the load bypasses the non-coherent L1 (agent-
// scope atomic load of the containing dword).
__device__ __forceinline__ uint32_t far_byte(const uint8_t *out, int32_t pos) {
    const uintptr_t a = (uintptr_t)(out + pos);
    const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return (w >> (8 * (a & 3))) & 255u;
}

// The decoder stages a block's compressed bytes in LDS kChunk at a time (plus
// kLook bytes of look-ahead) and parses each chunk with all 64 lanes: the
// chunk is cut into 64 segments of kSeg bytes and lane i parses the tokens
// that START in segment i.  A lane cannot know where its first token starts,
// so it first parses speculatively from each of the segment's first kStarts
// bytes (pass A), recording each parse's first kSpec token positions with the
// output / record counts before them: an LZ4 parse started at an arbitrary
// byte mostly falls into the true token chain within a few tokens.  A uniform walk over the 64 lanes then
// chains the true entries -- segment i's entry is segment i-1's exit; when
// the entry is among lane i's recorded positions its exit and counts follow,
// otherwise the segment is re-parsed from the entry right there -- and each
// lane re-parses its segment from its true entry (pass B), writing one record
// per sequence (literal position and length, offset, match length, output
// position) to LDS.  The records then run in order, up to 64 at a time, one
// lane per sequence: every literal run at once (they depend on nothing), then
// the matches in rounds -- a match is copied in the first round in which no
// unfinished match before it writes its source bytes (the first unfinished
// one always can be), so each round makes progress.  A match reads
// byte src + (t mod off) for output byte t, so the replication of an
// overlapping match (off < length) needs no ordering of its own.  Sequences
// longer than kGrpLit / kGrpMatch end a group and take wave-wide paths.
// (The round-2 decoder parsed tokens one at a time in scalar registers: ~500
// cycles per sequence on quantised floats, 0.25 s for a 3 GB column.)
//
// Output goes to an LDS ring only and is flushed to global memory in runs of
// >= kFlush bytes with dword stores; unflushed bytes stay < kFlush + one
// group, so the ring never overwrites them and every byte further back than
// the ring is already in global memory (far matches read it there).  (One
// wave per workgroup: its LDS accesses complete in program order, so a read
// after a write sees it; the wave barriers only keep the compiler from moving
// them.)  Positions are 32-bit (larger blocks are rejected as malformed).
//
// DIAG (measurement builds only; wrong output): 1 = parse only (no copies);
// 2 = staging only, 4 = staging + pass A, 8 = staging + pass A + chain
// (2, 4, 8: no status)
constexpr int kChunk = 1024, kLook = 256, kSeg = kChunk / 64, kSpec = 4, kStarts = 4;
constexpr int kMaxRec = kChunk / 3 + 2;  // tokens starting in a chunk (>= 3 bytes each but the last)
template <int DIAG>
__global__ __launch_bounds__(64) void k_decode_blocks(const uint8_t *src, int64_t src_bytes, const IngestBlock *tab,
                                                      int64_t nblocks, uint8_t *dst, int *status) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint32_t cinw[(kChunk + kLook) / 4 + 2];
    __shared__ __attribute__((aligned(16))) uint4 recs[kMaxRec];
    __shared__ uint16_t roff[kMaxRec];
    const uint8_t *cin = reinterpret_cast<const uint8_t *>(cinw);
    const uint8_t *src_end = src + src_bytes;
    const int lane = threadIdx.x;
    for (int64_t bi = blockIdx.x; bi < nblocks; bi += gridDim.x) {
        const IngestBlock blk = tab[bi];
        const uint8_t *ip0 = src + blk.src;
        uint8_t *out = dst + blk.dst;
        if (blk.method == 0x02) {  // stored block: one literal run (the ring copy is unused)
            copy_literals(ip0, src_end, out, 0, blk.usize, ring, lane);
            continue;
        }
        bool bad = blk.csize >= (1u << 30) || blk.usize >= (1u << 30);
        const int32_t isz = bad ? 0 : (int32_t)blk.csize, osz = bad ? 0 : (int32_t)blk.usize;
        const int32_t mis = (int32_t)((uintptr_t)ip0 & 3);
        const uint8_t *pa = ip0 - mis;  // dword-aligned; stream bytes at [mis, mis + isz)
        const int32_t lim = mis + isz;
        int32_t cb = 0, clen = 0;  // LDS holds pa bytes [cb, cb + clen)
        // byte `pos` of the block's compressed stream (per lane; pos < isz)
        auto B = [&](int32_t pos) -> uint32_t {
            const int32_t r = mis + pos - cb;
            return (r >= 0 && r < clen) ? (uint32_t)cin[r] : (uint32_t)ip0[pos];
        };
        // one token at p: false when it runs past the stream (or, for a
        // speculative parse, past the staged bytes: a parse inside a long
        // literal run must not chase global memory); last = the literals-only
        // final sequence (its literals end the stream)
        auto tok = [&](int32_t p, int32_t &lip, int32_t &ll, int32_t &off, int32_t &ml, bool &last, int32_t &next,
                       bool spec) -> bool {
            bool miss = false;
            auto rd = [&](int32_t pos) -> uint32_t {
                const int32_t r = mis + pos - cb;
                if (r >= 0 && r < clen) return (uint32_t)cin[r];
                if (spec) {
                    miss = true;
                    return 0u;
                }
                return (uint32_t)ip0[pos];
            };
            const uint32_t t = rd(p);
            int32_t q = p + 1;
            ll = (int32_t)(t >> 4);
            if (ll == 15) {
                uint32_t b;
                do {
                    if (q >= isz) return false;
                    b = rd(q++);
                    ll += (int32_t)b;
                } while (b == 255 && ll < (1 << 30));
            }
            if (miss || ll > isz - q) return false;
            lip = q;
            q += ll;
            off = 0;
            ml = 0;
            last = q == isz;
            if (!last) {
                if (isz - q < 2) return false;
                off = (int32_t)(rd(q) | (rd(q + 1) << 8));
                q += 2;
                ml = (int32_t)(t & 15);
                if (ml == 15) {
                    uint32_t b;
                    do {
                        if (q >= isz) return false;
                        b = rd(q++);
                        ml += (int32_t)b;
                    } while (b == 255 && ml < (1 << 30));
                }
                ml += 4;
            }
            next = q;
            return !miss;
        };
        int32_t fl = 0;  // out[0, fl) written
        auto flush = [&](int32_t upto) {
            const int32_t oa = (int32_t)((uintptr_t)(out + fl) & 3);
            int32_t head = (4 - oa) & 3;
            if (head > upto - fl) head = upto - fl;
            if (lane < head) out[fl + lane] = ring[(fl + lane) & (kRing - 1)];
            const int32_t p0 = fl + head, nw = (upto - p0) >> 2;
            uint32_t *ow = reinterpret_cast<uint32_t *>(out + p0);
            for (int32_t w = lane; w < nw; w += 64) {
                const int32_t b = p0 + 4 * w;
                ow[w] = (uint32_t)ring[b & (kRing - 1)] | ((uint32_t)ring[(b + 1) & (kRing - 1)] << 8) |
                        ((uint32_t)ring[(b + 2) & (kRing - 1)] << 16) | ((uint32_t)ring[(b + 3) & (kRing - 1)] << 24);
            }
            const int32_t p1 = p0 + 4 * nw;
            if (lane < upto - p1) out[p1 + lane] = ring[(p1 + lane) & (kRing - 1)];
            fl = upto;
        };
        int32_t op = 0;  // output written to the ring so far (uniform)
        // a long sequence (wave-wide): literals [lip, lip + len) at op, then
        // its match
        auto big_literals = [&](int32_t lip, int32_t len) {
            if (len > 256) {
                flush(op);
                copy_literals(ip0 + lip, src_end, out, op, len, ring, lane);
                fl = op + len;
                return;
            }
            for (int32_t r = 0; r < len; r += 64)
                if (r + lane < len) ring[(op + r + lane) & (kRing - 1)] = (uint8_t)B(lip + r + lane);
        };
        auto big_match = [&](int32_t off, int32_t mlen) {
            if (off > kRing - 256) {
                // far match (off > mlen-step, so no replication within a
                // 256-byte step): from the flushed output
                for (int32_t d0 = 0; d0 < mlen; d0 += 256) {
                    if (op + d0 - fl >= kFlush) flush(op + d0);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the flushes landed)
                    const int32_t cnt = mlen - d0 < 256 ? mlen - d0 : 256;
                    uint32_t v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t i = u * 64 + lane;
                        v[u] = i < cnt ? far_byte(out, op + d0 + i - off) : 0u;
                    }
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t i = u * 64 + lane;
                        if (i < cnt) ring[(op + d0 + i) & (kRing - 1)] = (uint8_t)v[u];
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            } else {
                // chunks of up to 256 bytes: byte op + i equals byte op + i -
                // m off for any m >= 1, so chunk [d0, d0 + cnt) reads the
                // latest off bytes before it, all final
                for (int32_t d0 = 0; d0 < mlen; d0 += 256) {
                    __builtin_amdgcn_wave_barrier();
                    if (op + d0 - fl >= kFlush) {
                        flush(op + d0);
                        __builtin_amdgcn_wave_barrier();
                    }
                    const int32_t cnt = mlen - d0 < 256 ? mlen - d0 : 256;
                    uint8_t v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t i = u * 64 + lane;
                        v[u] = 0;
                        if (i < cnt) v[u] = ring[(op + d0 + i - (i / off + 1) * off) & (kRing - 1)];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int32_t i = u * 64 + lane;
                        if (i < cnt) ring[(op + d0 + i) & (kRing - 1)] = v[u];
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        };
        int32_t E = 0;  // the next true token position (uniform)
        bool done = false;
        // Nearly incompressible blocks (ratio below 8/7: a few long literal
        // runs, e.g. 167 sequences of ~6 KB per MiB of Gaussian floats): the
        // tokens one at a time, uniformly, from a 256-B window of the stream
        // held one dword per lane -- the chunked parse would stage and parse
        // a chunk per token.
        if ((int64_t)isz * 8 >= (int64_t)osz * 7) {
            int32_t wa = -(1 << 30);
            uint32_t wv = 0;
            auto wbyte = [&](int32_t pos) -> uint32_t {  // uniform pos < isz
                const int32_t x = mis + pos;
                if (x < wa || x >= wa + 256) {
                    wa = x & ~3;
                    const int32_t q = wa + 4 * lane;
                    wv = 0;
                    if (q + 4 <= lim) {
                        wv = *reinterpret_cast<const uint32_t *>(pa + q);
                    } else {
                        for (int k = 0; k < 4; ++k)
                            if (q + k < lim) wv |= (uint32_t)pa[q + k] << (8 * k);
                    }
                    wa = __builtin_amdgcn_readfirstlane(wa);
                }
                const int32_t o = x - wa;
                return ((uint32_t)__builtin_amdgcn_readlane((int)wv, o >> 2) >> (8 * (o & 3))) & 255u;
            };
            int32_t p = 0;
            while (!bad && !done) {
                p = __builtin_amdgcn_readfirstlane(p);
                op = __builtin_amdgcn_readfirstlane(op);
                fl = __builtin_amdgcn_readfirstlane(fl);
                if (p >= isz) {
                    bad = true;
                    break;
                }
                const uint32_t t = wbyte(p);
                int32_t q = p + 1, ll = (int32_t)(t >> 4);
                if (ll == 15) {
                    uint32_t b;
                    do {
                        if (q >= isz) {
                            bad = true;
                            break;
                        }
                        b = wbyte(q++);
                        ll += (int32_t)b;
                    } while (b == 255 && ll < (1 << 30));
                    if (bad) break;
                }
                if (ll > isz - q || ll > osz - op) {
                    bad = true;
                    break;
                }
                const int32_t lip = q;
                q += ll;
                if (op - fl >= kFlush) flush(op);
                big_literals(lip, ll);
                op += ll;
                if (q == isz) {  // the final, literals-only sequence
                    done = true;
                    break;
                }
                if (isz - q < 2) {
                    bad = true;
                    break;
                }
                const int32_t off = (int32_t)(wbyte(q) | (wbyte(q + 1) << 8));
                q += 2;
                int32_t ml = (int32_t)(t & 15);
                if (ml == 15) {
                    uint32_t b;
                    do {
                        if (q >= isz) {
                            bad = true;
                            break;
                        }
                        b = wbyte(q++);
                        ml += (int32_t)b;
                    } while (b == 255 && ml < (1 << 30));
                    if (bad) break;
                }
                ml += 4;
                if (off == 0 || off > op || ml > osz - op) {
                    bad = true;
                    break;
                }
                big_match(off, ml);
                op += ml;
                if (op - fl >= kFlush) flush(op);
                p = q;
            }
        }
        int32_t ncs = 0;
        for (int32_t cs = 0; cs < isz && !bad && !done; cs = ncs) {
            E = __builtin_amdgcn_readfirstlane(E);
            op = __builtin_amdgcn_readfirstlane(op);
            fl = __builtin_amdgcn_readfirstlane(fl);
            ncs = cs + kChunk;
            if (E >= cs + kChunk) continue;  // inside a long literal run
            // ---- stage [cs, cs + kChunk + kLook) of the stream
            __builtin_amdgcn_wave_barrier();
            cb = (mis + cs) & ~3;
            clen = lim - cb < kChunk + kLook + 4 ? lim - cb : kChunk + kLook + 4;
            {
                constexpr int kStageW = (kChunk + kLook) / 256 + 1;
                uint32_t v[kStageW];
#pragma unroll
                for (int u = 0; u < kStageW; ++u) {
                    const int32_t q = cb + 4 * (u * 64 + lane);
                    v[u] = 0;
                    if (q + 4 <= lim) {
                        v[u] = *reinterpret_cast<const uint32_t *>(pa + q);
                    } else {
                        for (int k = 0; k < 4; ++k)
                            if (q + k < lim) v[u] |= (uint32_t)pa[q + k] << (8 * k);
                    }
                }
#pragma unroll
                for (int u = 0; u < kStageW; ++u)
                    if (u * 64 + lane < (int)(sizeof(cinw) / 4)) cinw[u * 64 + lane] = v[u];
            }
            __builtin_amdgcn_wave_barrier();
            if (DIAG & 2) continue;
            const int32_t s0 = cs + kSeg * lane, s1 = s0 + kSeg;  // this lane's segment
            // ---- pass A: speculative parses of the segment from its first
            // kStarts bytes (one start per byte: on quantised floats, tokens
            // of 3 bytes, a parse started in the wrong byte phase stays in it
            // -- offsets below 4096 read as tokens without literals -- and
            // missed the true chain for 2 of 3 segments; from 4 starts the
            // true entry is a start or a recorded position for 99.9 %)
            int32_t rp[kStarts][kSpec], rc[kStarts][kSpec], xs[kStarts], ts[kStarts], ns[kStarts];
#pragma unroll
            for (int c = 0; c < kStarts; ++c) {
                int32_t x = s0 + c, t = 0, nn = 0;
#pragma unroll
                for (int j = 0; j < kSpec; ++j) {
                    rp[c][j] = -1;
                    rc[c][j] = 0;
                }
                if (s1 > E) {
                    while (x < s1 && x < isz) {
#pragma unroll
                        for (int j = 0; j < kSpec; ++j)
                            if (nn == j) {
                                rp[c][j] = x;
                                rc[c][j] = t;
                            }
                        int32_t lip, ll, off, ml, nx;
                        bool last;
                        if (!tok(x, lip, ll, off, ml, last, nx, true)) {
                            x = -1;  // runs off the stream: not the true chain
                            break;
                        }
                        t += ll + ml;
                        ++nn;
                        x = nx;
                        if (last) break;
                    }
                }
                xs[c] = x;
                ts[c] = t;
                ns[c] = nn;
            }
            if (DIAG & 4) {
                if (__ballot(xs[0] == 12345 && ts[1] == 7 && ns[2] == 9 && xs[3] == 3) != 0) bad = true;
                continue;
            }
            // ---- the true chain over the segments (uniform)
            // (segments without a true token start keep vE = isz: no pass B;
            // the walk visits only the segments the chain enters)
            int32_t vE = isz, vO = 0, vR = 0;
            int32_t R = 0, O = op;
            for (int i = (E - cs) / kSeg; i < 64 && E < isz && !bad; i = (E - cs) / kSeg) {
                const int32_t si = cs + kSeg * i, ei = si + kSeg;
                vE = lane == i ? E : vE;
                vO = lane == i ? O : vO;
                vR = lane == i ? R : vR;
                bool hit = false;
                const int32_t dl = E - si;
                if (dl < kStarts) {
                    // the common case: a parse started at the entry
                    int32_t hx = -1, ht = 0, hn = 0;
#pragma unroll
                    for (int c = 0; c < kStarts; ++c)
                        if (c == dl) {
                            hx = __builtin_amdgcn_readlane(xs[c], i);
                            ht = __builtin_amdgcn_readlane(ts[c], i);
                            hn = __builtin_amdgcn_readlane(ns[c], i);
                        }
                    if (hx >= 0) {
                        hit = true;
                        O += ht;
                        R += hn;
                        E = hx;
                    }
                }
                if (!hit) {
                    // a later recorded position of some parse
#pragma unroll
                    for (int c = 0; c < kStarts; ++c)
#pragma unroll
                        for (int j = 1; j < kSpec; ++j) {
                            if (hit) continue;
                            const int32_t nc = __builtin_amdgcn_readlane(ns[c], i);
                            const int32_t xc = __builtin_amdgcn_readlane(xs[c], i);
                            if (j < nc && xc >= 0 && __builtin_amdgcn_readlane(rp[c][j], i) == E) {
                                hit = true;
                                O += __builtin_amdgcn_readlane(ts[c], i) - __builtin_amdgcn_readlane(rc[c][j], i);
                                R += nc - j;
                                E = xc;
                            }
                        }
                }
                if (!hit) {
                    // no parse met the entry: re-parse the segment here
                    // (uniform arguments: every lane computes the same)
                    int32_t p = E;
                    while (p < ei && p < isz) {
                        int32_t lip, ll, off, ml, nx;
                        bool last;
                        if (!tok(p, lip, ll, off, ml, last, nx, false)) {
                            bad = true;
                            break;
                        }
                        O += ll + ml;
                        ++R;
                        p = __builtin_amdgcn_readfirstlane(nx);
                        if (last) break;
                    }
                    E = p;
                }
                E = __builtin_amdgcn_readfirstlane(E);
                O = __builtin_amdgcn_readfirstlane(O);
                R = __builtin_amdgcn_readfirstlane(R);
            }
            if (bad || R > kMaxRec) {
                bad = true;
                break;
            }
            if (DIAG & 8) {
                if (__ballot(vE == 12345 && vO == 7 && vR == 9) != 0) bad = true;
                E = cs + kChunk;
                continue;
            }
            // ---- pass B: records from the true entries
            bool lbad = false;
            {
                int32_t p = vE, o = vO, r = vR;
                while (p < s1 && p < isz) {
                    int32_t lip, ll, off, ml, nx;
                    bool last;
                    if (!tok(p, lip, ll, off, ml, last, nx, false) || ll > osz - o || (!last && (off == 0 || off > o + ll)) ||
                        ml > osz - o - ll || r >= kMaxRec) {
                        lbad = true;
                        break;
                    }
                    recs[r] = uint4{(uint32_t)lip, (uint32_t)o, (uint32_t)ll, (uint32_t)ml};
                    roff[r] = (uint16_t)off;
                    ++r;
                    o += ll + ml;
                    p = nx;
                    if (last) break;
                }
            }
            if (__ballot(lbad) != 0) {
                bad = true;
                break;
            }
            done = E >= isz;
            // the next chunk holding a token start
            ncs = E - E % kChunk > cs ? E - E % kChunk : cs + kChunk;
            __builtin_amdgcn_wave_barrier();
            if (DIAG & 1) {
                op = O;
                continue;
            }
            // ---- run the records, up to 64 at a time
            for (int32_t r0 = 0; r0 < R;) {
                r0 = __builtin_amdgcn_readfirstlane(r0);
                op = __builtin_amdgcn_readfirstlane(op);
                const int32_t jr = r0 + lane;
                uint4 rec = uint4{0u, (uint32_t)op, 0u, 0u};
                int32_t off = 0;
                if (jr < R) {
                    rec = recs[jr];
                    off = roff[jr];
                }
                const int32_t ll = (int32_t)rec.z, ml = (int32_t)rec.w;
                const bool live = jr < R;
                const uint64_t bm = __ballot(live && (ll > kGrpLit || ml > kGrpMatch));
                const int32_t avail = R - r0 < 64 ? R - r0 : 64;
                const int g = bm ? (int)__builtin_ctzll(bm) : avail;
                if (g > 0) {
                    const bool act = lane < g;
                    const int32_t dst_ = (int32_t)rec.y;  // the sequence's literals
                    const int32_t gl = act ? ll : 0, gm = act ? ml : 0;
                    const int32_t mdst = dst_ + gl;  // its match
                    const int32_t gend = __builtin_amdgcn_readlane(mdst + gm, g - 1);
                    // literal runs (bytes of the staged input, mostly)
                    for (int32_t t0 = 0; __ballot(gl > t0) != 0; t0 += 8) {
                        uint32_t v[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] = t0 + u < gl ? B((int32_t)rec.x + t0 + u) : 0u;
#pragma unroll
                        for (int u = 0; u < 8; ++u)
                            if (t0 + u < gl) ring[(dst_ + t0 + u) & (kRing - 1)] = (uint8_t)v[u];
                    }
                    // bytes below far_lim may be overwritten in the ring by
                    // this group: they come from the flushed output (all of
                    // it is: the unflushed tail is < kFlush bytes behind the
                    // group's start)
                    const int32_t far_lim = gend - kRing;
                    const int32_t srcp = mdst - off;
                    const bool far = gm > 0 && srcp < far_lim;
                    // far matches: their bytes, as dwords of the flushed
                    // output re-aligned to the source (off > gm: no
                    // replication), loaded before the rounds
                    uint32_t fw[kGrpMatch / 4 + 1];
#pragma unroll
                    for (int i = 0; i < kGrpMatch / 4 + 1; ++i) fw[i] = 0;
                    if (__ballot(far) != 0) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the flushes landed)
                        const uintptr_t fa = (uintptr_t)(out + (far ? srcp : 0));
                        const uint32_t *wp = reinterpret_cast<const uint32_t *>(fa & ~(uintptr_t)3);
                        const uint32_t sh = (uint32_t)(fa & 3);
                        uint32_t raw[kGrpMatch / 4 + 2];
#pragma unroll
                        for (int i = 0; i < kGrpMatch / 4 + 2; ++i)
                            raw[i] = far && 4 * i < gm + (int)sh
                                         ? __hip_atomic_load(wp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : 0u;
#pragma unroll
                        for (int i = 0; i < kGrpMatch / 4 + 1; ++i) fw[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
                    }
                    // A match is copied once no unfinished match writes its
                    // source bytes: the lanes before it whose match ends
                    // past its source start (a binary search over the lanes'
                    // ordered match ends), [kl, lane).  Literal bytes are all
                    // written already.
                    // (sources before the group -- far ones included -- and the
                    // replicated prefix of an overlapping match: no lanes)
                    const int32_t need_end = off < gm ? mdst : srcp + gm;
                    const int32_t mend = mdst + gm;
                    int kl = 0, kh = 0;  // lanes [kl, kh): match end > srcp, match start < need_end
#pragma unroll
                    for (int st = 32; st >= 1; st >>= 1) {
                        const int cl = kl + st - 1, ch = kh + st - 1;
                        const int32_t el = __shfl(mend, cl < 64 ? cl : 63);
                        const int32_t sh_ = __shfl(mdst, ch < 64 ? ch : 63);
                        if (kl + st <= lane && el <= srcp) kl += st;
                        if (kh + st <= lane && sh_ < need_end) kh += st;
                    }
                    auto below = [](int x) -> uint64_t { return x <= 0 ? 0ull : (~0ull >> (64 - x)); };
                    const uint64_t deps = kh > kl ? below(kh) & ~below(kl) : 0ull;
                    bool fin = gm == 0;
                    while (true) {
                        const uint64_t und = __ballot(!fin);
                        if (und == 0) break;
                        const bool go = !fin && (und & deps) == 0;
                        if (go) {
                            int32_t k = 0;  // (t mod off)
#pragma unroll
                            for (int c = 0; c < (kGrpMatch + 11) / 12; ++c) {
                                if (12 * c >= gm) break;
                                uint32_t v[12];
#pragma unroll
                                for (int u = 0; u < 12; ++u) {
                                    const int t = 12 * c + u;
                                    v[u] = 0;
                                    if (t < gm) {
                                        v[u] = far ? (fw[t >> 2] >> (8 * (t & 3))) & 255u
                                                   : (uint32_t)ring[(srcp + k) & (kRing - 1)];
                                        k = k + 1 == off ? 0 : k + 1;
                                    }
                                }
#pragma unroll
                                for (int u = 0; u < 12; ++u)
                                    if (12 * c + u < gm) ring[(mdst + 12 * c + u) & (kRing - 1)] = (uint8_t)v[u];
                            }
                        }
                        fin = fin || go;
                    }
                    __builtin_amdgcn_wave_barrier();
                    op = gend;
                    r0 += g;
                }
                if (bm) {  // the long sequence at lane g
                    const int32_t blip = __builtin_amdgcn_readlane((int)rec.x, g);
                    const int32_t bll = __builtin_amdgcn_readlane(ll, g), bml = __builtin_amdgcn_readlane(ml, g);
                    const int32_t boff = __builtin_amdgcn_readlane(off, g);
                    if (op - fl >= kFlush) flush(op);
                    big_literals(blip, bll);
                    op += bll;
                    if (bml > 0) {
                        big_match(boff, bml);
                        op += bml;
                    }
                    r0 += 1;
                }
                if (op - fl >= kFlush) flush(op);
            }
        }
        bad = bad || !done || op != osz;
        if (DIAG & 14) bad = false;
        __builtin_amdgcn_wave_barrier();
        if (!bad) flush(op);
        if (bad && lane == 0) atomicOr(status, 4);
        __syncthreads();
    }
}

// ---- block checksums: CityHash128 v1.0.2 ------------------------------------
// CompressedReadBufferBase.cpp:37-45, 192-196 validates every block before
// decompressing it: CityHash_v1_0_2::CityHash128 (contrib/cityhash102/src/
// city.cc:256-358) over the 9-B header + payload, against the 16 bytes stored
// before it.  CityHash is a sequential chain, so one lane hashes one block
// (1 MiB blocks: ~3k lanes for a 3 GB column).  Blocks start at arbitrary byte
// offsets: every 64-bit word is assembled from aligned dwords with
// v_alignbyte (the shift is fixed per block), and the next three 64-byte
// rounds' dwords are loaded while the current three are mixed.
namespace city {
constexpr uint64_t K0 = 0xc3a5c85c97cb3127ULL, K1 = 0xb492b66fbe98f273ULL, K2 = 0x9ae16a3b2f90404fULL,
                   K3 = 0xc949d7c7509e6557ULL;
__device__ __forceinline__ uint64_t ror(uint64_t v, int s) { return s ? (v >> s) | (v << (64 - s)) : v; }
__device__ __forceinline__ uint64_t mix47(uint64_t v) { return v ^ (v >> 47); }
__device__ __forceinline__ uint64_t pair(uint64_t lo, uint64_t hi) {  // Hash128to64
    constexpr uint64_t m = 0x9ddfea08eb382d69ULL;
    const uint64_t a = mix47((lo ^ hi) * m);
    return mix47((hi ^ a) * m) * m;
}
__device__ __forceinline__ uint32_t join(uint32_t lo, uint32_t hi, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
// unaligned little-endian loads; a dword is read only when it holds a needed byte
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t d0 = w[0], d1 = w[1], d2 = sh ? w[2] : 0u;
    return (uint64_t)join(d0, d1, sh) | ((uint64_t)join(d1, d2, sh) << 32);
}
__device__ __forceinline__ uint64_t ld32(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    return join(w[0], sh ? w[1] : 0u, sh);
}
__device__ uint64_t short_hash(const uint8_t *s, uint64_t len) {  // HashLen0to16
    if (len > 8) {
        const uint64_t a = ld64(s), b = ld64(s + len - 8);
        return pair(a, ror(b + len, (int)len)) ^ b;
    }
    if (len >= 4) return pair(len + (ld32(s) << 3), ld32(s + len - 4));
    if (len > 0) {
        const uint32_t y = (uint32_t)s[0] + ((uint32_t)s[len >> 1] << 8);
        const uint32_t z = (uint32_t)len + ((uint32_t)s[len - 1] << 2);
        return mix47(y * K2 ^ z * K3) * K2;
    }
    return K2;
}
// WeakHashLen32WithSeeds over words w0..w3
__device__ __forceinline__ void weak32(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint64_t a, uint64_t b,
                                       uint64_t &o1, uint64_t &o2) {
    a += w0;
    b = ror(b + a + w3, 21);
    const uint64_t c = a;
    a += w1 + w2;
    b += ror(a, 44);
    o1 = a + w3;
    o2 = b + c;
}
__device__ void murmur(const uint8_t *s, uint64_t len, uint64_t a, uint64_t b, uint64_t h[2]) {  // CityMurmur
    uint64_t c, d;
    if (len <= 16) {
        a = mix47(a * K1) * K1;
        c = b * K1 + short_hash(s, len);
        d = mix47(a + (len >= 8 ? ld64(s) : c));
    } else {
        c = pair(ld64(s + len - 8) + K1, a);
        d = pair(b + len, c + ld64(s + len - 16));
        a += d;
        for (int64_t l = (int64_t)len - 16; l > 0; l -= 16, s += 16) {
            a ^= mix47(ld64(s) * K1) * K1;
            a *= K1;
            b ^= a;
            c ^= mix47(ld64(s + 8) * K1) * K1;
            c *= K1;
            d ^= c;
        }
    }
    a = pair(a, c);
    b = pair(d, b);
    h[0] = a ^ b;
    h[1] = pair(b, a);
}
// 64 bytes at an aligned dword base + sh as 17 raw dwords
__device__ __forceinline__ void load_round(const uint32_t *w, uint32_t sh, uint32_t r[17]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = w[i];
    r[16] = sh ? w[16] : 0u;
}
__device__ void seeded(const uint8_t *s, uint64_t len, uint64_t x, uint64_t y, uint64_t h[2]) {  // CityHash128WithSeed
    if (len < 128) {
        murmur(s, len, x, y, h);
        return;
    }
    uint64_t z = len * K1;
    uint64_t v1 = ror(y ^ K1, 49) * K1 + ld64(s);
    uint64_t v2 = ror(v1, 42) * K1 + ld64(s + 8);
    uint64_t w1 = ror(y + z, 35) * K1 + x;
    uint64_t w2 = ror(x + ld64(s + 88), 53) * K1;
    const int64_t rounds = 2 * (int64_t)(len / 128);
    const uintptr_t a0 = (uintptr_t)s;
    const uint32_t sh = (uint32_t)(a0 & 3);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(a0 & ~(uintptr_t)3);
    // kAhead rounds in flight while kAhead rounds are mixed (3 x 17 dword
    // loads stay under the 63 outstanding vector loads a wave can count)
    constexpr int kAhead = 3;
    uint32_t cur[kAhead][17];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) load_round(base + 16 * (j < rounds ? j : rounds - 1), sh, cur[j]);
    for (int64_t r = 0; r < rounds; r += kAhead) {
        uint32_t nxt[kAhead][17];
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int64_t rr = r + kAhead + j;
            load_round(base + 16 * (rr < rounds ? rr : rounds - 1), sh, nxt[j]);
        }
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            if (r + j >= rounds) break;
            uint64_t q[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                q[i] = (uint64_t)join(cur[j][2 * i], cur[j][2 * i + 1], sh) |
                       ((uint64_t)join(cur[j][2 * i + 1], cur[j][2 * i + 2], sh) << 32);
            x = ror(x + y + v1 + q[2], 37) * K1;
            y = ror(y + v2 + q[6], 42) * K1;
            x ^= w2;
            y ^= v1;
            z = ror(z ^ w1, 33);
            weak32(q[0], q[1], q[2], q[3], v2 * K1, x + w1, v1, v2);
            weak32(q[4], q[5], q[6], q[7], z + w2, y, w1, w2);
            const uint64_t t = z;
            z = x;
            x = t;
        }
#pragma unroll
        for (int j = 0; j < kAhead; ++j)
#pragma unroll
            for (int i = 0; i < 17; ++i) cur[j][i] = nxt[j][i];
    }
    s += 64 * rounds;
    len -= 64 * (uint64_t)rounds;
    y += ror(w1, 37) * K0 + z;
    x += ror(v1 + z, 49) * K0;
    for (uint64_t done = 0; done < len;) {
        done += 32;
        y = ror(y - x, 42) * K0 + v2;
        w1 += ld64(s + len - done + 16);
        x = ror(x, 49) * K0 + w1;
        w1 += v1;
        const uint8_t *p = s + len - done;
        weak32(ld64(p), ld64(p + 8), ld64(p + 16), ld64(p + 24), v1, v2, v1, v2);
    }
    x = pair(x, v1);
    y = pair(y, w1);
    h[0] = pair(x + v2, w2) + y;
    h[1] = pair(x + w2, y + v2);
}
__device__ void hash128(const uint8_t *s, uint64_t len, uint64_t h[2]) {  // CityHash128
    if (len >= 16)
        seeded(s + 16, len - 16, ld64(s) ^ K3, ld64(s + 8), h);
    else if (len >= 8)
        seeded(nullptr, 0, ld64(s) ^ (len * K0), ld64(s + len - 8) ^ K1, h);
    else
        seeded(s, len, K0, K1, h);
}
}  // namespace city

__global__ __launch_bounds__(64) void k_block_checksum(const uint8_t *src, const IngestBlock *tab, int64_t nblocks,
                                                       int flag, int *status, uint64_t *hash_out) {
    const int64_t bi = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (bi >= nblocks) return;
    const IngestBlock b = tab[bi];
    const uint8_t *hdr = src + b.src - 9;  // the hash covers header + payload
    uint64_t h[2];
    city::hash128(hdr, (uint64_t)b.csize + 9, h);
    if (hash_out) {
        hash_out[2 * bi] = h[0];
        hash_out[2 * bi + 1] = h[1];
    }
    if (h[0] != city::ld64(hdr - 16) || h[1] != city::ld64(hdr - 8)) atomicOr(status, flag);
}

// ---- array sizes -> element offsets (exclusive scan over n UInt64) ----------
constexpr int kScanTile = 4096;  // sizes per workgroup (256 threads x 16)

__global__ __launch_bounds__(256) void k_sizes_partial(const uint64_t *sizes, int64_t n, int d, int64_t *tile_sum,
                                                       int64_t *stats) {
    __shared__ int64_t red[256];
    __shared__ int64_t cnt[256];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    int64_t s = 0, notd = 0;
    for (int i = threadIdx.x; i < kScanTile; i += 256) {
        const int64_t r = base + i;
        if (r < n) {
            s += (int64_t)sizes[r];
            notd += sizes[r] != (uint64_t)d;
        }
    }
    red[threadIdx.x] = s;
    cnt[threadIdx.x] = notd;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            red[threadIdx.x] += red[threadIdx.x + o];
            cnt[threadIdx.x] += cnt[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tile_sum[blockIdx.x] = red[0];
        if (cnt[0]) atomicAdd((unsigned long long *)&stats[0], (unsigned long long)cnt[0]);
    }
}

// exclusive prefix of the tile sums in place (one workgroup); total -> stats[1]
__global__ __launch_bounds__(1024) void k_sizes_top(int64_t *tile_sum, int64_t ntiles, int64_t *stats) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (ntiles + 1023) / 1024;
    const int64_t b = t * per, e = min(ntiles, b + per);
    int64_t s = 0;
    for (int64_t i = b; i < e; ++i) s += tile_sum[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        int64_t acc = 0;
        for (int i = 0; i < 1024; ++i) {
            const int64_t v = part[i];
            part[i] = acc;
            acc += v;
        }
        stats[1] = acc;
    }
    __syncthreads();
    int64_t run = part[t];
    for (int64_t i = b; i < e; ++i) {
        const int64_t v = tile_sum[i];
        tile_sum[i] = run;
        run += v;
    }
}

__global__ __launch_bounds__(256) void k_sizes_final(const uint64_t *sizes, int64_t n, const int64_t *tile_base,
                                                     int64_t *offsets) {
    __shared__ int64_t wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    // thread t owns sizes [base + 16 t, base + 16 t + 16)
    int64_t v[16], s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t r = base + 16 * t + i;
        v[i] = r < n ? (int64_t)sizes[r] : 0;
        s += v[i];
    }
    int64_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int64_t run = tile_base[blockIdx.x] + inc - s;
    for (int x = 0; x < w; ++x) run += wsum[x];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t r = base + 16 * t + i;
        if (r < n) offsets[r] = run;
        run += v[i];
    }
}

__global__ __launch_bounds__(256) void k_array_rows(const float *data, const int64_t *offsets, const uint64_t *sizes,
                                                    int64_t n, int d, float *rows, uint8_t *nonempty) {
    const float FLTMAX = 3.40282347e+38f;
    for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const int64_t sz = (int64_t)sizes[r], off = offsets[r];
        for (int j = threadIdx.x; j < d; j += 256) rows[r * d + j] = j < sz ? data[off + j] : FLTMAX;
        if (threadIdx.x == 0) nonempty[r] = sz > 0;
    }
}

// ---- launchers ----------------------------------------------------------------

void launch_block_table(const uint8_t *src, int64_t n, IngestBlock *tab, int64_t max_blocks, int64_t *out,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_block_table, dim3(1), dim3(1), 0, s, src, n, tab, max_blocks, out);
}

void launch_decode_blocks(const uint8_t *src, int64_t src_bytes, const IngestBlock *tab, int64_t nblocks, uint8_t *dst,
                          int *status, hipStream_t s) {
    if (nblocks <= 0) return;
    const int grid = (int)std::min<int64_t>(nblocks, 4096);
    // (diagnostics on the big stream only: the array sizes must decode)
    const int diag = kDebugTuning && nblocks > 64 ? tune_int("MQVS_LZ4_DIAG", 0) : 0;
    if (kDebugTuning && diag == 1)
        hipLaunchKernelGGL(k_decode_blocks<1>, dim3(grid), dim3(64), 0, s, src, src_bytes, tab, nblocks, dst, status);
    else if (kDebugTuning && diag == 2)
        hipLaunchKernelGGL(k_decode_blocks<2>, dim3(grid), dim3(64), 0, s, src, src_bytes, tab, nblocks, dst, status);
    else if (kDebugTuning && diag == 4)
        hipLaunchKernelGGL(k_decode_blocks<4>, dim3(grid), dim3(64), 0, s, src, src_bytes, tab, nblocks, dst, status);
    else if (kDebugTuning && diag == 8)
        hipLaunchKernelGGL(k_decode_blocks<8>, dim3(grid), dim3(64), 0, s, src, src_bytes, tab, nblocks, dst, status);
    else
        hipLaunchKernelGGL(k_decode_blocks<0>, dim3(grid), dim3(64), 0, s, src, src_bytes, tab, nblocks, dst, status);
}

void launch_block_checksum(const uint8_t *src, const IngestBlock *tab, int64_t nblocks, int flag, int *status,
                           uint64_t *hash_out, hipStream_t s) {
    if (nblocks <= 0) return;
    hipLaunchKernelGGL(k_block_checksum, dim3((unsigned)((nblocks + 63) / 64)), dim3(64), 0, s, src, tab, nblocks, flag,
                       status, hash_out);
}

// offsets[n] (exclusive); stats[0] += rows whose size != d, stats[1] = total
// elements (stats zeroed by the caller); scratch >= ceil(n / 4096) int64
void launch_sizes_scan(const uint64_t *sizes, int64_t n, int d, int64_t *offsets, int64_t *scratch, int64_t *stats,
                       hipStream_t s) {
    const int64_t tiles = std::max<int64_t>(1, (n + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(k_sizes_partial, dim3((unsigned)tiles), dim3(256), 0, s, sizes, n, d, scratch, stats);
    hipLaunchKernelGGL(k_sizes_top, dim3(1), dim3(1024), 0, s, scratch, tiles, stats);
    hipLaunchKernelGGL(k_sizes_final, dim3((unsigned)tiles), dim3(256), 0, s, sizes, n, scratch, offsets);
}

void launch_array_rows(const float *data, const int64_t *offsets, const uint64_t *sizes, int64_t n, int d,
                       float *rows, uint8_t *nonempty, hipStream_t s) {
    if (n <= 0) return;
    const int grid = (int)std::min<int64_t>(n, 65536);
    hipLaunchKernelGGL(k_array_rows, dim3(grid), dim3(256), 0, s, data, offsets, sizes, n, d, rows, nonempty);
}

}  // namespace mqvs
