// C entry point over the REFERENCE's own CityHash v1.0.2, compiled straight
// from /root/reference/contrib/cityhash102/src/city.cc by oracle/Makefile into
// oracle/_ref/libcityref.so (no reference source is copied).  Test
// infrastructure only: it pins the oracle's restatement (orc_cityhash128) and
// the GPU checksum kernel against the hash ClickHouse writes before every
// compressed block (CompressedWriteBuffer.cpp:44, CompressedReadBufferBase.cpp:37-45).
#include <city.h>

#include <cstdint>

extern "C" void ref_cityhash128(const uint8_t *s, int64_t len, uint64_t h[2]) {
    const CityHash_v1_0_2::uint128 r = CityHash_v1_0_2::CityHash128(reinterpret_cast<const char *>(s), (size_t)len);
    h[0] = r.first;
    h[1] = r.second;
}
