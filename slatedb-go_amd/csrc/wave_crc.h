// Wave-level CRC32-IEEE over bytes staged in LDS (shared by decode and encode).
#pragma once
#include "common.h"

namespace slate {

// Per translation unit (no relocatable device code): each TU gets its own copy.
static __constant__ CrcTables g_crc_tables = CrcTables();
static __constant__ CrcShift g_crc_shift = CrcShift();
static __constant__ CrcShiftT<16> g_crc_shift16 = CrcShiftT<16>();
static __constant__ CrcShiftT<32> g_crc_shift32 = CrcShiftT<32>();

constexpr uint32_t kTabBytes = 4096;  // 4 x 256 u32 slicing tables in LDS

// Slicing-by-16 tables: t[k][b] = the CRC of byte b followed by k zero bytes (t[0] is the
// classic table).  A 16-byte chunk then costs 16 independent lookups and one dependent
// step, instead of four dependent rounds of four.  Used by the lane-per-block kernels, one
// block per lane (decode_lpb2.hip, zstd_fast.hip).
struct CrcTables16 {
  uint32_t t[16][256];
  constexpr CrcTables16() : t{} {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int s = 1; s < 16; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
static __constant__ CrcTables16 g_crc16 = CrcTables16();
constexpr uint32_t kTab16Bytes = 16 * 256 * 4;

// v_bitop3_b32 with the truth table of a ^ b ^ c (the compiler re-chains plain XORs)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// the CRC register after the 16 bytes (x, y, z, w) (little-endian dwords), tables in LDS
__device__ __forceinline__ uint32_t crc16_step(const uint32_t* tab, uint32_t c, uint32_t vx, uint32_t vy, uint32_t vz,
                                               uint32_t vw) {
  const uint32_t x = c ^ vx;
#ifdef SLATE_CRC_TREE
  // the 16 lookups folded as a balanced tree of three-input XORs (4 levels instead of a
  // 15-deep chain)
  const uint32_t a0 = tab[15 * 256 + (x & 0xff)], a1 = tab[14 * 256 + ((x >> 8) & 0xff)],
                 a2 = tab[13 * 256 + ((x >> 16) & 0xff)], a3 = tab[12 * 256 + (x >> 24)];
  const uint32_t b0 = tab[11 * 256 + (vy & 0xff)], b1 = tab[10 * 256 + ((vy >> 8) & 0xff)],
                 b2 = tab[9 * 256 + ((vy >> 16) & 0xff)], b3 = tab[8 * 256 + (vy >> 24)];
  const uint32_t c0 = tab[7 * 256 + (vz & 0xff)], c1 = tab[6 * 256 + ((vz >> 8) & 0xff)],
                 c2 = tab[5 * 256 + ((vz >> 16) & 0xff)], c3 = tab[4 * 256 + (vz >> 24)];
  const uint32_t d0 = tab[3 * 256 + (vw & 0xff)], d1 = tab[2 * 256 + ((vw >> 8) & 0xff)],
                 d2 = tab[1 * 256 + ((vw >> 16) & 0xff)], d3 = tab[vw >> 24];
  const uint32_t e0 = xor3(a0, a1, a2), e1 = xor3(a3, b0, b1), e2 = xor3(b2, b3, c0), e3 = xor3(c1, c2, c3),
                 e4 = xor3(d0, d1, d2);
  const uint32_t r = xor3(xor3(e0, e1, e2), xor3(e3, e4, d3), 0u);
#else
  uint32_t r = tab[15 * 256 + (x & 0xff)] ^ tab[14 * 256 + ((x >> 8) & 0xff)] ^ tab[13 * 256 + ((x >> 16) & 0xff)] ^
               tab[12 * 256 + (x >> 24)];
  r ^= tab[11 * 256 + (vy & 0xff)] ^ tab[10 * 256 + ((vy >> 8) & 0xff)] ^ tab[9 * 256 + ((vy >> 16) & 0xff)] ^
       tab[8 * 256 + (vy >> 24)];
  r ^= tab[7 * 256 + (vz & 0xff)] ^ tab[6 * 256 + ((vz >> 8) & 0xff)] ^ tab[5 * 256 + ((vz >> 16) & 0xff)] ^
       tab[4 * 256 + (vz >> 24)];
  r ^= tab[3 * 256 + (vw & 0xff)] ^ tab[2 * 256 + ((vw >> 8) & 0xff)] ^ tab[1 * 256 + ((vw >> 16) & 0xff)] ^
       tab[vw >> 24];
#endif
  return r;
}

__device__ inline void load_crc_tables(uint32_t* tab) {
  const uint32_t* src = &g_crc_tables.t[0][0];
  for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) tab[i] = src[i];
  __syncthreads();
}

// 4 bytes at an arbitrary (possibly negative) byte offset of a 4-aligned LDS buffer.
__device__ inline uint32_t lds_u32(const uint8_t* base, int32_t off) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (off & ~3));
  return __builtin_amdgcn_alignbyte(w[1], w[0], uint32_t(off) & 3u);
}

__device__ inline uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

__device__ inline uint32_t crc_word(const uint32_t* tab, uint32_t c, uint32_t w) {
  c ^= w;
  return tab[768 + (c & 0xff)] ^ tab[512 + ((c >> 8) & 0xff)] ^ tab[256 + ((c >> 16) & 0xff)] ^ tab[c >> 24];
}

// R(init, msg[0..n)) with the CRC register semantics of crc32.ChecksumIEEE but
// without the final inversion: fold_init = true starts from 0xFFFFFFFF (folded
// into the first four bytes), false from 0.  n >= 4 when fold_init.
// 64 lanes x Seg-byte segments per (64 Seg)-byte stripe, end-aligned so each lane's shift
// x^(8*Seg*(63-l)) is a constant (CrcShiftT).  Seg 64 for long messages; short ones take
// Seg 16 or 32, so a 1 KiB message costs a lane 4 words instead of 16 (wave_crc32).
template <uint32_t Seg>
__device__ inline uint32_t wave_crc_seg(const uint32_t* tab, const uint8_t* lds, int32_t msg, uint32_t n, int lane,
                                        bool fold_init, const CrcShiftT<Seg>& sh) {
  constexpr uint32_t kStripe = kWave * Seg;
  uint32_t stripes = (n + kStripe - 1) / kStripe;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < stripes; k++) {
    if (k) acc = gf2_mulmod(acc, sh.stripe);
    int64_t p0 = int64_t(n) - int64_t(stripes - k) * kStripe + int64_t(lane) * Seg;
    uint32_t c = 0;
    if (p0 + int64_t(Seg) > 0) {
#pragma unroll 4
      for (uint32_t q = 0; q < Seg / 4; q++) {
        int64_t p = p0 + 4 * q;
        uint32_t w = 0;
        if (p > -4) {
          // p < 0: the message's first bytes shifted up (the same word as the aligned read around
          // msg + p with its leading bytes cleared, without touching bytes before msg: in HBM mode
          // those can lie before the buffer)
          w = p < 0 ? lds_u32(lds, msg) << (8 * uint32_t(-p)) : lds_u32(lds, int32_t(int64_t(msg) + p));
          if (fold_init && p < 4) {
            uint32_t m = 0;
            for (int b = 0; b < 4; b++) {
              int64_t pos = p + b;
              if (pos >= 0 && pos < 4) m |= 0xFFu << (8 * b);
            }
            w ^= m;
          }
        }
        c = crc_word(tab, c, w);
      }
    }
    acc ^= c;
  }
  return wave_xor(gf2_mulmod(acc, sh.lane[lane]));
}
__device__ inline uint32_t wave_crc_raw(const uint32_t* tab, const uint8_t* lds, int32_t msg, uint32_t n, int lane,
                                        bool fold_init) {
  if (n <= 64 * 16) return wave_crc_seg<16>(tab, lds, msg, n, lane, fold_init, g_crc_shift16);
  if (n <= 64 * 32) return wave_crc_seg<32>(tab, lds, msg, n, lane, fold_init, g_crc_shift32);
  return wave_crc_seg<kCrcSeg>(tab, lds, msg, n, lane, fold_init, g_crc_shift);
}

// crc32.ChecksumIEEE of msg[0..n) in LDS.
__device__ inline uint32_t wave_crc32(const uint32_t* tab, const uint8_t* lds, int32_t msg, uint32_t n, int lane) {
  if (n < 4) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < n; i++) c = tab[(c ^ lds[msg + int32_t(i)]) & 0xff] ^ (c >> 8);
    return ~c;
  }
  return ~wave_crc_raw(tab, lds, msg, n, lane, true);
}

}  // namespace slate
