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

#ifndef SLATE_LPB_OR
#define SLATE_LPB_OR 128
#endif
constexpr uint32_t kOR = SLATE_LPB_OR;  // lpb2 output ring bytes (ring_rd8/ring_rd16 default mask)
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

// CRC table lookups (decode_none.hip, decode_lpb2.hip).  A lookup's LDS address is (byte k of x) * 4 plus a table offset: one SDWA shift
// (src1_sel picks the byte) instead of an extract and a shift, and the table offset rides in the
// ds_read's immediate (the tables start at LDS address 0).
template <int K>
__device__ __forceinline__ uint32_t idx4(uint32_t x) {
  uint32_t r;
  if constexpr (K == 0)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(x));
  else if constexpr (K == 1)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(x));
  else if constexpr (K == 2)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(x));
  else
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(x));
  return r;
}
// The lookup's LDS address is formed from the integer: through the extern __shared__ array's
// symbol the compiler added its address (0) to every index with a v_add_u32 of its own.  The
// kernels that use these tables declare no static LDS, so the dynamic array starts at address 0.
typedef const __attribute__((address_space(3))) uint32_t lds_u32_t;
template <uint32_t kOff>
__device__ __forceinline__ uint32_t lut(const uint8_t* lds, uint32_t i4) {
  (void)lds;
  return *(lds_u32_t*)(kOff + i4);
}
// the four lookups of one dword against tables kT, kT - 1, kT - 2, kT - 3 (1 KiB each) at byte offset kBase
template <uint32_t kBase, int kT>
__device__ __forceinline__ void lut4(const uint8_t* lds, uint32_t x, uint32_t& a, uint32_t& b, uint32_t& c,
                                     uint32_t& d) {
  a = lut<kBase + 1024 * kT>(lds, idx4<0>(x));
  b = lut<kBase + 1024 * (kT - 1)>(lds, idx4<1>(x));
  c = lut<kBase + 1024 * (kT - 2)>(lds, idx4<2>(x));
  d = lut<kBase + 1024 * (kT - 3)>(lds, idx4<3>(x));
}
// the raw CRC register of a 16-byte chunk from a zero register (slicing-by-16, crc16_step)
__device__ __forceinline__ uint32_t crc_chunk0(const uint8_t* lds, const v4u& v) {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3, d0, d1, d2, d3;
  lut4<0, 15>(lds, v.x, a0, a1, a2, a3);
  lut4<0, 11>(lds, v.y, b0, b1, b2, b3);
  lut4<0, 7>(lds, v.z, c0, c1, c2, c3);
  lut4<0, 3>(lds, v.w, d0, d1, d2, d3);
  return xor3(xor3(a0, a1, a2), xor3(a3, b0, b1), xor3(xor3(b2, b3, c0), xor3(c1, c2, c3), xor3(d0, d1, xor3(d2, d3, 0u))));
}
// CRC register advance over zero bytes (decode_none.hip, encode.hip): tables in LDS after the
// slicing-by-16 tables, kAdvN x 4 KiB; table s advances by 32 << s bytes.
constexpr uint32_t kAdvN = 6;  // zero-byte advance tables for 32, 64, ..., 1024 bytes
// x^(8N) mod P for N = 32 << s: multiplying a raw CRC register by it advances the register over
// N zero bytes (zlib's crc32_combine arithmetic)
struct AdvConsts {
  uint32_t k[kAdvN];
  constexpr AdvConsts() : k{} {
    for (uint32_t s = 0; s < kAdvN; s++) k[s] = x8n(uint64_t(32) << s);
  }
};
static __constant__ AdvConsts g_adv = AdvConsts();

// register advanced over N zero bytes by four lookups: table s (N = 32 << s), t[j][i] = (i << 8j) * x^(8N)
template <int kS>
__device__ __forceinline__ uint32_t adv_tab(const uint8_t* lds, uint32_t c) {
  constexpr uint32_t o = kTab16Bytes + 4096 * kS;
  return xor3(lut<o>(lds, idx4<0>(c)), lut<o + 1024>(lds, idx4<1>(c)), lut<o + 2048>(lds, idx4<2>(c))) ^
         lut<o + 3072>(lds, idx4<3>(c));
}
// over 16 zero bytes: rows 12..15 of the slicing-by-16 tables (a chunk of zeros after c)
__device__ __forceinline__ uint32_t adv16(const uint8_t* lds, uint32_t c) {
  uint32_t a, b, d, e;
  lut4<0, 15>(lds, c, a, b, d, e);
  return xor3(a, b, d) ^ e;
}
template <int kShift>
__device__ __forceinline__ uint32_t row_shl(uint32_t v) {  // lane i <- lane i + kShift of its row of 16
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x100 + kShift, 0xf, 0xf, true));
}
// over t < 16 zero bytes: byte i < t of c is looked up after i steps and then carried over
// t - 1 - i more zero bytes (slicing row t - 1 - i); the bytes from t on only shift down
__device__ __forceinline__ uint32_t adv_small(const uint32_t* tab, uint32_t c, uint32_t t) {
  uint32_t r = t >= 4 ? 0u : c >> (8 * t);
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t v = tab[((t - 1 - i) & 15) * 256 + ((c >> (8 * i)) & 0xff)];
    r ^= i < t ? v : 0u;
  }
  return r;
}

// LDS table of the advance tables: entry i of table s = ((i & 255) << 8 * ((i >> 8) & 3)) * x^(8 * (32 << s))
__device__ __forceinline__ void load_adv_tables(uint32_t* adv) {
  for (uint32_t i = threadIdx.x; i < kAdvN * 1024; i += blockDim.x)
    adv[i] = gf2_mulmod((i & 255u) << (8 * ((i >> 8) & 3u)), g_adv.k[i >> 10]);
}

// c ? a : b as one v_cndmask_b32 on the lane mask of c: the compiler turned groups of selects
// on one condition into divergent branches (exec-mask save/restore around both arms)
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
#ifdef SLATE_NO_ASM_SEL
  return c ? a : b;
#endif
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(__builtin_amdgcn_ballot_w64(c)));
  return r;
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
  // v_perm: byte i <- byte (4 - b + i) of {hi:lo}; b * 0x01010101 as a byte broadcast (v_perm), not a
  // quarter-rate v_mul_lo_u32
  const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, b, 0u);
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
// A wave-uniform load of memory the running kernel never writes (plan arrays: in_off, out_off,
// row_base), as a scalar load.  The constant address space says so to the compiler; a plain load
// of a uniform address otherwise becomes a vector load + readfirstlane, and its s_waitcnt vmcnt(0)
// also drains every block load the wave has in flight.  p must be wave-uniform.
template <typename T>
__device__ __forceinline__ T sload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)(p);
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
