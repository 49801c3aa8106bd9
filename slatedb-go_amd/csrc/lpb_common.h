// Helpers shared by the lane-per-block Snappy decoders (decode_lpb2.hip, decode_lpb3.hip):
// CRC32 slicing-by-16 tables and per-alignment CRC states, naturally aligned LDS window
// reads (gfx950 serialises misaligned LDS accesses lane by lane: tools/lds_cost_probe.hip),
// buffer resources.  Included by one translation unit each (anonymous namespace).
#pragma once
#include "common.h"
#include "wave_crc.h"

namespace slate {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

namespace {

constexpr uint32_t kOR = 128;           // lpb2 output ring bytes (ring_rd8/ring_rd16 default mask)
constexpr uint32_t kOOB = 0xFFFFFFF0u;  // buffer offset that is always out of range

// CRC register state that becomes 0xFFFFFFFF after `sh` zero bytes (sh < 16), and x^(8t) mod P.
struct CrcLeadTail {
  uint32_t init[16];
  uint32_t tail[16];
  constexpr CrcLeadTail() : init{}, tail{} {
    for (uint32_t sh = 0; sh < 16; sh++) {
      uint32_t s = 0xFFFFFFFFu;
      for (uint32_t b = 0; b < 8 * sh; b++) s = (s & 0x80000000u) ? (((s ^ kCrcPoly) << 1) | 1u) : (s << 1);
      init[sh] = s;
      tail[sh] = x8n(sh);
    }
  }
};
static __constant__ CrcLeadTail g_crc_lt = CrcLeadTail();

__device__ __forceinline__ uint32_t crc16_chunk(const uint32_t* tab, uint32_t c, const v4u& v) {
  return crc16_step(tab, c, v.x, v.y, v.z, v.w);
}

// Rings and natural alignment.  gfx950 executes ds_read/ds_write of 8 or 16 bytes at any
// byte address, but an access that is not naturally aligned is serialised lane by lane:
// ~64 CU-cycles per wave-instruction against 2-9 aligned, for b32, b64 and b128 alike
// (tools/lds_cost_probe.hip).  So every ring access here is naturally aligned: byte windows
// are cut out of aligned 8-byte reads with v_alignbyte, and 16 output bytes at any position
// are stored as five aligned dwords, the first merged with the bytes already in it (the
// lane keeps that dword in a register, Lane::T).  Each element wraps on its own, so the
// rings need no mirror copies.
__device__ __forceinline__ uint32_t be16_of(uint32_t w) { return ((w & 0xff) << 8) | ((w >> 8) & 0xff); }
// m8 = ring size - 8 (both rings are powers of two)
__device__ __forceinline__ v2u rd64(const uint8_t* ring, uint32_t a, uint32_t m8 = kOR - 8) {
  return *reinterpret_cast<const v2u*>(ring + (a & m8));
}
// z is a run-time zero (DecodeArgs::rt_zero): it keeps the compiler from fusing two b64
// accesses 8 bytes apart into ds_read2_b64 / ds_write2_b64, which cost ~55 CU-cycles per
// wave-instruction at these addresses (tools/lds_cost_probe.hip) against ~3 for two
// ds_read_b64.
__device__ __forceinline__ v4u rd128(const uint8_t* p, uint32_t z) {  // 8-byte aligned 16 bytes
  const v2u a = *reinterpret_cast<const v2u*>(p), b = *reinterpret_cast<const v2u*>(p + 8 + z);
  v4u r;
  r.x = a.x;
  r.y = a.y;
  r.z = b.x;
  r.w = b.y;
  return r;
}
__device__ __forceinline__ void wr128(uint8_t* p, const v4u& v, uint32_t z) {
  v2u a, b;
  a.x = v.x;
  a.y = v.y;
  b.x = v.z;
  b.y = v.w;
  *reinterpret_cast<v2u*>(p) = a;
  *reinterpret_cast<v2u*>(p + 8 + z) = b;
}
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t b) {
  return __builtin_amdgcn_alignbyte(hi, lo, b);
}
// ring bytes [p, p+8) (ring of 128 bytes, any p)
__device__ __forceinline__ v2u ring_rd8(const uint8_t* ring, uint32_t p, uint32_t m8 = kOR - 8) {
  const uint32_t a = p & m8;
  const v2u A = rd64(ring, a, m8), B = rd64(ring, a + 8, m8);
  const bool q = (p & 4) != 0;
  const uint32_t d0 = q ? A.y : A.x, d1 = q ? B.x : A.y, d2 = q ? B.y : B.x;
  const uint32_t b = p & 3;
  v2u r;
  r.x = alignb(d1, d0, b);
  r.y = alignb(d2, d1, b);
  return r;
}
// ring bytes [p, p+16)
__device__ __forceinline__ v4u ring_rd16(const uint8_t* ring, uint32_t p, uint32_t m8 = kOR - 8) {
  const uint32_t a = p & m8;
  const v2u A = rd64(ring, a, m8), B = rd64(ring, a + 8, m8), C = rd64(ring, a + 16, m8);
  const bool q = (p & 4) != 0;
  const uint32_t e0 = q ? A.y : A.x, e1 = q ? B.x : A.y, e2 = q ? B.y : B.x, e3 = q ? C.x : B.y,
                 e4 = q ? C.y : C.x;
  const uint32_t b = p & 3;
  v4u r;
  r.x = alignb(e1, e0, b);
  r.y = alignb(e2, e1, b);
  r.z = alignb(e3, e2, b);
  r.w = alignb(e4, e3, b);
  return r;
}
// the five dwords that put v at byte b (0..3) of a 20-byte window whose first dword keeps
// `head` below byte b
struct Win5 {
  uint32_t y0, y1, y2, y3, y4;
};
__device__ __forceinline__ Win5 shift_in(const v4u& v, uint32_t head, uint32_t b) {
  const uint32_t sel = 0x07060504u - b * 0x01010101u;  // v_perm: byte i <- byte (4 - b + i) of {hi:lo}
  const uint32_t keep = (1u << (8 * b)) - 1u;
  Win5 w;
  w.y0 = (head & keep) | (__builtin_amdgcn_perm(v.x, head, sel) & ~keep);
  w.y1 = __builtin_amdgcn_perm(v.y, v.x, sel);
  w.y2 = __builtin_amdgcn_perm(v.z, v.y, sel);
  w.y3 = __builtin_amdgcn_perm(v.w, v.z, sel);
  w.y4 = __builtin_amdgcn_perm(v.w, v.w, sel);
  return w;
}
__device__ __forceinline__ void wr32(uint8_t* ring, uint32_t a, uint32_t v) {
  *reinterpret_cast<uint32_t*>(ring + (a & (kOR - 4))) = v;
}
__device__ __forceinline__ void store_win(uint8_t* ring, uint32_t a4, const Win5& w) {
  wr32(ring, a4, w.y0);
  wr32(ring, a4 + 4, w.y1);
  wr32(ring, a4 + 8, w.y2);
  wr32(ring, a4 + 12, w.y3);
  wr32(ring, a4 + 16, w.y4);
}
// dword j (0..4) of the window, as bit-tested selects: an equality chain became a
// branch tree of divergent if-blocks
__device__ __forceinline__ uint32_t pick5(const Win5& w, uint32_t j) {
  const uint32_t a = (j & 1) ? w.y1 : w.y0, b = (j & 1) ? w.y3 : w.y2;
  const uint32_t r = (j & 2) ? b : a;
  return (j & 4) ? w.y4 : r;
}

// Cache policy (gfx950 CPol bits): 0 = default (allocates in L2: a lane reads its block's 128-byte
// lines 16 bytes at a time, so the line must stay for the next 7 accesses), 16 = sc1 (bypasses the
// CU's L1, for reads of this kernel's own output), 2 = nt (streaming).
template <int kAux>
__device__ __forceinline__ v4u bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAux);
}
// Stores are sc1 (write-through): the output is written in 64-byte runs, and default-policy
// partial-line writes made the XCD L2 fill the rest of each 128-byte line from HBM first
// (FETCH_SIZE 6.3 -> 4.3 KiB per block, tools/traffic_ablate.sh).
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, v4u v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// Resources must be in SGPRs (a VGPR resource turns every buffer op into a waterfall loop):
// the inputs are wave-uniform, readfirstlane makes that visible to the compiler.
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
  return (uint64_t(hi) << 32) | lo;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t b = uniform64(reinterpret_cast<uint64_t>(base));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes < kOOB ? uint32_t(bytes) : kOOB);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0, int(n), 0x00020000);
}

// Reads of this kernel's own output go around the CU's L1 (nt): a line another wave
// of this CU loaded earlier could be stale.
__device__ __forceinline__ uint32_t out_u8(const uint8_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint32_t out_be16(const uint8_t* p) { return (out_u8(p) << 8) | out_u8(p + 1); }
__device__ __forceinline__ uint32_t out_be32(const uint8_t* p) { return (out_be16(p) << 16) | out_be16(p + 2); }

// byte mask of dword j (bytes 4j..4j+3 of a chunk) keeping chunk bytes [lo, hi)
__device__ __forceinline__ uint32_t keep_mask(int32_t lo, int32_t hi, int32_t j) {
  const int32_t a = min(max(lo - 4 * j, 0), 4), b = min(max(hi - 4 * j, 0), 4);
  const uint64_t m = ((uint64_t(1) << (8 * b)) - 1) & ~((uint64_t(1) << (8 * a)) - 1);
  return uint32_t(m);
}

}  // namespace
}  // namespace slate
