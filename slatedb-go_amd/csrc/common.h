// Shared definitions for the MI355X SST block codec (host + device).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/slatecodec.h"

static_assert(sizeof(slate_block_meta) == 16, "slate_block_meta must be 16 bytes");
static_assert(sizeof(slate_row) == 16, "slate_row must be 16 bytes");

namespace slate {

constexpr uint32_t kWave = 64;  // CDNA wavefront

// Snappy output is at most 64 bytes per 3 input bytes (copy2 tag), so a header
// length above 22x the payload can only end in golang/snappy's ErrCorrupt.
constexpr uint64_t kSnappyMaxExpansion = 22;

// A valid v0 row is >= 13 bytes plus a 2-byte offset (row.go:95-107): the number
// of row descriptors a decoded block of `len` bytes can need.
__host__ __device__ inline uint64_t row_capacity(uint64_t decoded_len) { return (decoded_len + 13) / 15; }

__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

__host__ __device__ inline uint16_t ld_be16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }
__host__ __device__ inline uint32_t ld_be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
__host__ __device__ inline uint64_t ld_be64(const uint8_t* p) {
  return (uint64_t(ld_be32(p)) << 32) | ld_be32(p + 4);
}
__host__ __device__ inline void st_be16(uint8_t* p, uint16_t v) { p[0] = uint8_t(v >> 8); p[1] = uint8_t(v); }
__host__ __device__ inline void st_be32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}
__host__ __device__ inline void st_be64(uint8_t* p, uint64_t v) { st_be32(p, uint32_t(v >> 32)); st_be32(p + 4, uint32_t(v)); }

// ---------------------------------------------------------------- CRC32-IEEE
// Reflected polynomial 0xEDB88320 (hash/crc32.ChecksumIEEE).  Slicing-by-4
// tables, and x^(8n) mod P constants for combining per-lane partial CRCs.
constexpr uint32_t kCrcPoly = 0xEDB88320u;

struct CrcTables {
  uint32_t t[4][256];
  constexpr CrcTables() : t{} {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int s = 1; s < 4; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};

// a * b mod P in the reflected representation (bit 31 = x^0); zlib's multmodp.
__host__ __device__ constexpr uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; i++) {
    if (a & 0x80000000u) p ^= b;
    a <<= 1;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

// x^(8n) mod P for n zero bytes.
__host__ __device__ constexpr uint32_t x8n(uint64_t n) {
  uint32_t r = 0x80000000u;    // x^0
  uint32_t sq = 0x00800000u;   // x^8
  while (n) {
    if (n & 1) r = gf2_mulmod(r, sq);
    sq = gf2_mulmod(sq, sq);
    n >>= 1;
  }
  return r;
}

// The block CRC splits a stripe of 64 lanes x Seg bytes, end-aligned to the
// message: lane l's partial R(0, seg_l) is shifted by the bytes after it.
constexpr uint32_t kCrcSeg = 64;
constexpr uint32_t kCrcStripe = kWave * kCrcSeg;  // 4096
template <uint32_t Seg>
struct CrcShiftT {
  uint32_t lane[kWave];  // x^(8 * Seg * (63 - l))
  uint32_t stripe;       // x^(8 * 64 * Seg)
  constexpr CrcShiftT() : lane{}, stripe(0) {
    uint32_t seg = 0x80000000u;
    for (int k = 0; k < 8 * int(Seg); k++) seg = (seg & 1) ? (seg >> 1) ^ kCrcPoly : seg >> 1;
    uint32_t acc = 0x80000000u;
    for (int l = int(kWave) - 1; l >= 0; l--) {
      lane[l] = acc;
      acc = gf2_mulmod(acc, seg);
    }
    stripe = acc;
  }
};
using CrcShift = CrcShiftT<kCrcSeg>;

// Host CRC (framing of small host-side pieces such as flatbuffer info).
uint32_t crc32_host(const uint8_t* p, size_t n);
uint32_t crc32_host16(const uint8_t* p, size_t n);  // slicing-by-16 (large host buffers)

}  // namespace slate
