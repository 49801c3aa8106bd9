// CodecZstd decode: compress.Decode = io.ReadAll(zstd.NewReader(buf)) (compression.go:146-153)
// with github.com/klauspost/compress v1.17.11, restated from RFC 8878.  oracle/zstd_oracle.c
// is the CPU restatement this follows check for check (status codes, their order, and the
// plan size rule: a frame's content size when its header has one, clamped by its blocks'
// bounds, else the bytes an in-order decode produces).
//
// One wave per stream.  Frame, block and sequence parsing is wave-uniform (every lane runs
// the same scalar chain; table reads at a uniform LDS address are broadcasts), the (up to)
// four Huffman literal streams decode on four lanes at once, copies and Huffman table fills
// are lane-parallel, and the FSE table builds (small, rare: most small blocks use the
// predefined tables, built once per workgroup) run on lane 0.  Literals are decoded into the
// tail of the output buffer and consumed front to back, so no separate literal buffer is
// needed: the write cursor never passes the unread literals (checked per sequence).
#pragma once
#include "common.h"
#include "wave_crc.h"

namespace slate {

constexpr uint32_t kZsBlockMax = 128u * 1024u;
constexpr uint64_t kZsMaxWindow = 1ull << 29;  // klauspost MaxWindowSize (64-bit)

struct ZsFse {
  uint8_t sym, nb;
  uint16_t base;
};
struct ZsScratch {     // per wave; the Huffman tree decode uses the fields before ll only
  uint16_t huf[2048];  // (nbits << 8) | symbol, indexed by the next tl stream bits
  ZsFse wt[64];
  int16_t norm[256];
  uint16_t next[256];
  uint8_t w[256];
  ZsFse ll[512], ml[512], of[256];
};
struct ZsShared {  // per workgroup: the predefined distributions (RFC 8878 3.1.1.3.2.2)
  ZsFse ll[64], ml[64], of[32];
};
constexpr uint32_t kZsScratch = (sizeof(ZsScratch) + 15) & ~15u;
constexpr uint32_t kZsHufScratch = (offsetof(ZsScratch, ll) + 15) & ~15u;  // zs_huf_read's part
constexpr uint32_t kZsShared = (sizeof(ZsShared) + 15) & ~15u;

__constant__ int16_t kZsLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                     2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kZsMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kZsOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t kZsLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                       20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kZsLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,
                                      1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kZsMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                       21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                       43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kZsMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

// Cross-lane LDS hand-off inside a wave: a compiler and hardware ordering point (the
// s_waitcnt / wave_barrier builtins alone do not order memory at the IR level).
__device__ inline void zs_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline uint32_t zrfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline int zrfl(int v) { return int(__builtin_amdgcn_readfirstlane(uint32_t(v))); }

// ----------------------------------------------------------------- bit access
// base is 4-aligned (LDS or global); offsets are bytes from base.
__device__ inline uint64_t zs_u64(const uint8_t* base, int32_t off) {
  return uint64_t(lds_u32(base, off)) | (uint64_t(lds_u32(base, off + 4)) << 32);
}
// k <= 56 bits of the little-endian bit string at absolute bit `bit`
__device__ inline uint64_t zs_bits(const uint8_t* base, int64_t bit, uint32_t k) {
  const uint64_t v = zs_u64(base, int32_t(bit >> 3)) >> (bit & 7);
  return v & ((1ull << k) - 1);
}
// Backward stream (RFC 8878 4.1): S = absolute bit of its first byte, pos = bits left
// (< 0 after an overread, whose bits read as zeros).
__device__ inline uint64_t zs_peek(const uint8_t* base, int64_t S, int64_t pos, uint32_t k) {
  if (k == 0 || pos <= 0) return 0;
  if (pos >= int64_t(k)) return zs_bits(base, S + pos - k, k);
  return zs_bits(base, S, uint32_t(pos)) << (k - uint32_t(pos));
}
// bits left in a backward stream base[off, off+n), or -1 (empty / zero last byte)
__device__ inline int64_t zs_bstart(const uint8_t* base, int32_t off, uint32_t n) {
  if (n == 0) return -1;
  const uint32_t last = base[off + int32_t(n) - 1];
  if (last == 0) return -1;
  return 8 * int64_t(n - 1) + (31 - __builtin_clz(last));
}
// forward stream base[off, off+n) zero padded: k <= 32 bits at bit bp
__device__ inline uint32_t zs_fbits(const uint8_t* base, int32_t off, uint32_t n, uint64_t bp, uint32_t k) {
  const uint64_t end = 8ull * n;
  if (bp >= end) return 0;
  uint32_t v = uint32_t(zs_bits(base, 8 * int64_t(off) + int64_t(bp), k));
  if (bp + k > end) v &= (1u << (end - bp)) - 1;
  return v;
}

// ------------------------------------------------------------------ FSE (lane 0)
// FSE_readNCount: bytes used or -1 (oracle zs_ncount)
__device__ int zs_ncount(const uint8_t* base, int32_t off, uint32_t n, int16_t* norm, int maxs, int maxal, int* al_out,
                         int* last) {
  if (n == 0) return -1;
  const int al = (base[off] & 15) + 5;
  if (al > maxal) return -1;
  uint64_t bp = 4;
  int remaining = (1 << al) + 1, threshold = 1 << al, nb = al + 1, s = 0;
  bool prev0 = false;
  for (int i = 0; i <= maxs; i++) norm[i] = 0;
  while (remaining > 1 && s <= maxs) {
    if (prev0) {
      int n0 = s;
      for (;;) {
        const uint32_t r = zs_fbits(base, off, n, bp, 2);
        bp += 2;
        n0 += int(r);
        if (r != 3) break;
      }
      if (n0 > maxs) return -1;
      s = n0;
      prev0 = false;
    }
    const uint32_t v = zs_fbits(base, off, n, bp, uint32_t(nb));
    const int max = (2 * threshold - 1) - remaining;
    int count;
    if (int(v & uint32_t(threshold - 1)) < max) {
      count = int(v & uint32_t(threshold - 1));
      bp += uint32_t(nb - 1);
    } else {
      count = int(v & uint32_t(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bp += uint32_t(nb);
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[s++] = int16_t(count);
    prev0 = count == 0;
    while (remaining < threshold && nb > 1) {
      nb--;
      threshold >>= 1;
    }
  }
  if (remaining != 1 || (bp + 7) / 8 > n) return -1;
  *al_out = al;
  *last = s - 1;
  return int((bp + 7) / 8);
}

// FSE decoding table (oracle zs_fse_build); 0 or -1
__device__ int zs_fse_build(ZsFse* t, const int16_t* norm, int last, int al, uint16_t* next) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t hi = size - 1;
  for (int s = 0; s <= last; s++) {
    const int c = norm[s];
    if (c == -1) {
      t[hi--].sym = uint8_t(s);
      next[s] = 1;
    } else {
      next[s] = uint16_t(c > 0 ? c : 0);
    }
  }
  uint32_t pos = 0;
  for (int s = 0; s <= last; s++)
    for (int i = 0; i < norm[s]; i++) {
      t[pos].sym = uint8_t(s);
      do pos = (pos + step) & mask;
      while (pos > hi);
    }
  if (pos != 0) return -1;
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t x = next[t[u].sym]++;
    const int nb = al - (31 - __builtin_clz(x));
    t[u].nb = uint8_t(nb);
    t[u].base = uint16_t((x << nb) - size);
  }
  return 0;
}

// the predefined tables, built once per workgroup by wave 0 (then __syncthreads)
__device__ void zs_shared_build(ZsShared* sh, ZsScratch* sc, int lane) {
  if (lane == 0) {
    for (int i = 0; i < 36; i++) sc->norm[i] = kZsLLDef[i];
    zs_fse_build(sh->ll, sc->norm, 35, 6, sc->next);
    for (int i = 0; i < 53; i++) sc->norm[i] = kZsMLDef[i];
    zs_fse_build(sh->ml, sc->norm, 52, 6, sc->next);
    for (int i = 0; i < 29; i++) sc->norm[i] = kZsOFDef[i];
    zs_fse_build(sh->of, sc->norm, 28, 5, sc->next);
  }
}

// ------------------------------------------------------------------ Huffman
// FSE-compressed weights (oracle zs_huf_read): the table description and build on lane 0,
// then the two-state decode wave-uniform out of registers: lane u holds table cell u and
// stream dword u (hb <= 127 bytes), so a symbol costs v_readlane + scalar bit arithmetic,
// no LDS round trip.  0 / -1, *nw = the number of decoded weights.
__device__ int zs_weights_fse(const uint8_t* base, int32_t off, uint32_t hb, ZsScratch* sc, int lane, int* nw_out) {
  int hs = 0, al = 0, last = 0;
  if (lane == 0) {
    hs = zs_ncount(base, off, hb, sc->norm, 255, 6, &al, &last);
    if (hs >= 0 && zs_fse_build(sc->wt, sc->norm, last, al, sc->next)) hs = -1;
  }
  hs = zrfl(hs);
  al = zrfl(al);
  if (hs < 0) return -1;
  zs_sync();
  const int32_t so = off + hs;
  const uint32_t bn = hb - uint32_t(hs);
  if (bn == 0) return -1;
  const uint32_t tab = lane < (1 << al) ? *reinterpret_cast<const uint32_t*>(&sc->wt[lane]) : 0u;
  const uint32_t win = uint32_t(lane) * 4 < bn ? lds_u32(base, so + 4 * lane) : 0u;
  auto byte_at = [&](uint32_t i) -> uint32_t {
    return (uint32_t(__builtin_amdgcn_readlane(win, int(i >> 2))) >> (8 * (i & 3))) & 0xFFu;
  };
  auto bits_at = [&](int64_t b, uint32_t k) -> uint32_t {  // k <= 24 bits at stream bit b >= 0
    const uint32_t d = uint32_t(b >> 5);
    const uint64_t v = uint64_t(uint32_t(__builtin_amdgcn_readlane(win, int(d)))) |
                       (uint64_t(uint32_t(__builtin_amdgcn_readlane(win, int(d + 1 < 64 ? d + 1 : 63)))) << 32);
    return uint32_t(v >> (b & 31)) & ((1u << k) - 1);
  };
  const uint32_t lastb = byte_at(bn - 1);
  if (lastb == 0) return -1;
  int64_t pos = 8 * int64_t(bn - 1) + (31 - __builtin_clz(lastb));
  auto rd = [&](uint32_t k) -> uint32_t {
    uint32_t v = 0;
    if (k && pos > 0) v = pos >= int64_t(k) ? bits_at(pos - k, k) : bits_at(0, uint32_t(pos)) << (k - uint32_t(pos));
    pos -= k;
    return v;
  };
  uint32_t s1 = rd(uint32_t(al)), s2 = rd(uint32_t(al));
  int nw = 0;
  for (;;) {  // two interleaved states until the stream overreads (FSE_decompress tail)
    if (nw > 253) return -1;
    uint32_t e = uint32_t(__builtin_amdgcn_readlane(tab, int(s1)));
    if (lane == 0) sc->w[nw] = uint8_t(e);
    nw++;
    s1 = (e >> 16) + rd((e >> 8) & 0xFF);
    if (pos < 0) {
      if (lane == 0) sc->w[nw] = uint8_t(__builtin_amdgcn_readlane(tab, int(s2)));
      nw++;
      break;
    }
    if (nw > 253) return -1;
    e = uint32_t(__builtin_amdgcn_readlane(tab, int(s2)));
    if (lane == 0) sc->w[nw] = uint8_t(e);
    nw++;
    s2 = (e >> 16) + rd((e >> 8) & 0xFF);
    if (pos < 0) {
      if (lane == 0) sc->w[nw] = uint8_t(__builtin_amdgcn_readlane(tab, int(s1)));
      nw++;
      break;
    }
  }
  *nw_out = nw;
  return 0;
}

// Huffman_Tree_Description at base[off, off+n): bytes used or -1; fills the decoding table (sc->huf,
// or huf_out when given: then sc->huf is never touched), *tl
__device__ int zs_huf_read(const uint8_t* base, int32_t off, uint32_t n, ZsScratch* sc, int lane, uint32_t* tl_out,
                           uint32_t dbg = 0, uint16_t* huf_out = nullptr) {  // dbg: profiling ablations (1<<25 no table fill, 1<<23 no weight decode)
  if (n < 1) return -1;
  const uint32_t hb = zrfl(uint32_t(base[off]));
  int nw, used;
  if (hb >= 128) {
    nw = int(hb) - 127;
    const uint32_t nbytes = (uint32_t(nw) + 1) / 2;
    if (1 + nbytes > n) return -1;
    for (int i = lane; i < nw; i += kWave) {
      const uint32_t b = base[off + 1 + i / 2];
      sc->w[i] = uint8_t((i & 1) ? (b & 15) : (b >> 4));
    }
    used = int(1 + nbytes);
  } else {
    if (1 + hb > n) return -1;
    int k = 0;
    if (dbg & (1u << 23)) {
      k = 255;  // profiling: weights left as they are
    } else if (zs_weights_fse(base, off + 1, hb, sc, lane, &k) < 0) {
      return -1;
    }
    nw = k;
    used = int(1 + hb);
  }
  zs_sync();
  // weight statistics (oracle zs_huf_read), lane-parallel: lane k counts weight k
  uint32_t cnt = 0, total = 0, bad = 0;
  for (int c0 = 0; c0 < nw; c0 += kWave) {
    const int i = c0 + lane;
    const uint32_t my = i < nw ? uint32_t(sc->w[i]) : 0u;
    bad |= my > 11 ? 1u : 0u;
    total += my ? (1u << (my - 1)) : 0u;
#pragma unroll
    for (uint32_t k = 1; k <= 11; k++) {
      const uint32_t c = uint32_t(__builtin_popcountll(__ballot(my == k)));
      cnt += (uint32_t(lane) == k) ? c : 0u;
    }
  }
  if (__ballot(bad != 0)) return -1;
  for (int o = 32; o >= 1; o >>= 1) total += uint32_t(__shfl_xor(int(total), o, 64));
  total = zrfl(total);
  if (total == 0) return -1;
  const uint32_t tl = 32 - __builtin_clz(total);  // highbit + 1
  if (tl > 11) return -1;
  const uint32_t rest = (1u << tl) - total;
  if (rest & (rest - 1)) return -1;
  const uint32_t lastw = 32 - __builtin_clz(rest);
  if (lane == 0) sc->w[nw] = uint8_t(lastw);
  cnt += (uint32_t(lane) == lastw) ? 1u : 0u;
  const uint32_t r1 = uint32_t(__builtin_amdgcn_readlane(cnt, 1));
  if (r1 < 2 || (r1 & 1)) return -1;
  // weight-major table, symbol order within a weight: lane k holds weight k's next slot
  uint32_t cur = 0, acc = 0;
  for (uint32_t k = 1; k <= tl; k++) {
    if (uint32_t(lane) == k) cur = acc;
    acc += uint32_t(__builtin_amdgcn_readlane(cnt, int(k))) << (k - 1);
  }
  zs_sync();
  for (int c0 = 0; c0 <= nw; c0 += kWave) {
    const int s = c0 + lane;
    const uint32_t my = s <= nw ? uint32_t(sc->w[s]) : 0u;
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t k = 1; k <= 11; k++) {
      const uint64_t m = __ballot(my == k);
      const uint32_t before = uint32_t(__builtin_amdgcn_readlane(cur, int(k)));
      const uint32_t rank = uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)));
      pos = (my == k) ? before + (rank << (k - 1)) : pos;
      cur += (uint32_t(lane) == k) ? (uint32_t(__builtin_popcountll(m)) << (k - 1)) : 0u;
    }
    if (my && !(dbg & (1u << 25))) {
      const uint16_t e = uint16_t(((tl + 1 - my) << 8) | uint32_t(s));
      uint16_t* huf = huf_out ? huf_out : sc->huf;
      for (uint32_t i = 0; i < (1u << (my - 1)); i++) huf[pos + i] = e;
    }
  }
  zs_sync();
  *tl_out = tl;
  return used;
}

// ----------------------------------------------------------------- sequences
struct ZsState {
  const ZsFse *ll, *of, *ml;  // current tables (nullptr: none yet in this frame)
  uint32_t ll_al, of_al, ml_al;
  uint32_t huf_valid, tl;
  uint32_t rep[3];
  uint32_t rep_used;  // a sequence took a repeat offset (the split payload path needs none)
};

// Symbol_Compression_Mode for one table type: bytes used or -1 (oracle zs_table).
__device__ int zs_table(uint32_t mode, const uint8_t* base, int32_t off, uint32_t n, ZsFse* own, const ZsFse* def,
                        uint32_t defal, int maxs, int maxal, ZsScratch* sc, const ZsFse** t, uint32_t* al, int lane) {
  if (mode == 0) {
    *t = def;
    *al = defal;
    return 0;
  }
  if (mode == 1) {
    if (n < 1) return -1;
    const uint32_t sym = zrfl(uint32_t(base[off]));
    if (int(sym) > maxs) return -1;
    if (lane == 0) {
      own[0].sym = uint8_t(sym);
      own[0].nb = 0;
      own[0].base = 0;
    }
    zs_sync();
    *t = own;
    *al = 0;
    return 1;
  }
  if (mode == 2) {
    int hs = 0, a = 0, last = 0;
    if (lane == 0) {
      hs = zs_ncount(base, off, n, sc->norm, maxs, maxal, &a, &last);
      if (hs >= 0 && zs_fse_build(own, sc->norm, last, a, sc->next)) hs = -1;
    }
    hs = zrfl(hs);
    a = zrfl(a);
    zs_sync();
    if (hs < 0) return -1;
    *t = own;
    *al = uint32_t(a);
    return hs;
  }
  return *t ? 0 : -1;  // repeat
}

// A compressed block at base[off, off+n) appended to out at *d (out == nullptr: sizes
// only).  fstart = the frame's first output byte.  Status codes as oracle zs_block.
// dbg: profiling ablations only (SLATE_DEBUG_MODE bits 17 skip the Huffman streams, 19 skip
// the sequence copies); 0 in production.
__device__ int zs_block(const uint8_t* base, int32_t off, uint32_t n, uint8_t* out, uint32_t cap, uint32_t* d,
                        uint32_t fstart, uint32_t bmax, ZsScratch* sc, const ZsShared* sh, ZsState& st, int lane,
                        uint32_t dbg = 0) {
  if (n < 1) return SLATE_E_ZSTD_CORRUPT;
  const uint32_t b0 = zrfl(uint32_t(base[off]));
  const uint32_t type = b0 & 3, sf = (b0 >> 2) & 3;
  uint32_t pos, nlit;
  const uint32_t d0 = *d;
  // literals go to the tail of the output buffer: out[lbase, lbase + nlit)
  uint32_t lbase = 0;
  auto bN = [&](int i) -> uint32_t { return zrfl(uint32_t(base[off + i])); };
  if (type <= 1) {
    uint32_t hs;
    if (sf == 1) {
      hs = 2;
      if (n < 2) return SLATE_E_ZSTD_CORRUPT;
      nlit = (b0 >> 4) + (bN(1) << 4);
    } else if (sf == 3) {
      hs = 3;
      if (n < 3) return SLATE_E_ZSTD_CORRUPT;
      nlit = (b0 >> 4) + (bN(1) << 4) + (bN(2) << 12);
    } else {
      hs = 1;
      nlit = b0 >> 3;
    }
    if (nlit > bmax) return SLATE_E_ZSTD_CORRUPT;
    if (type == 0 ? (n - hs < nlit) : (n - hs < 1)) return SLATE_E_ZSTD_CORRUPT;
    if (nlit > cap - d0) return SLATE_E_ZSTD_CORRUPT;  // the block cannot fit (the oracle fails at the end)
    lbase = cap - nlit;
    if (out) {
      if (type == 0) {
        for (uint32_t j = lane; j < nlit; j += kWave) out[lbase + j] = base[off + int32_t(hs + j)];
      } else {
        const uint8_t v = base[off + int32_t(hs)];
        for (uint32_t j = lane; j < nlit; j += kWave) out[lbase + j] = v;
      }
    }
    pos = hs + (type == 0 ? nlit : 1);
  } else {
    uint32_t hs, cs;
    const uint32_t streams = sf == 0 ? 1 : 4;
    if (sf <= 1) {
      hs = 3;
      if (n < 3) return SLATE_E_ZSTD_CORRUPT;
      const uint32_t h = b0 | (bN(1) << 8) | (bN(2) << 16);
      nlit = (h >> 4) & 0x3FF;
      cs = (h >> 14) & 0x3FF;
    } else if (sf == 2) {
      hs = 4;
      if (n < 4) return SLATE_E_ZSTD_CORRUPT;
      const uint32_t h = b0 | (bN(1) << 8) | (bN(2) << 16) | (bN(3) << 24);
      nlit = (h >> 4) & 0x3FFF;
      cs = (h >> 18) & 0x3FFF;
    } else {
      hs = 5;
      if (n < 5) return SLATE_E_ZSTD_CORRUPT;
      const uint64_t h = uint64_t(b0 | (bN(1) << 8) | (bN(2) << 16) | (bN(3) << 24)) | (uint64_t(bN(4)) << 32);
      nlit = uint32_t((h >> 4) & 0x3FFFF);
      cs = uint32_t((h >> 22) & 0x3FFFF);
    }
    if (nlit > bmax || n - hs < cs) return SLATE_E_ZSTD_CORRUPT;
    int32_t q = off + int32_t(hs);
    uint32_t qn = cs;
    if (type == 2) {
      uint32_t tl = 0;
      const int t = zs_huf_read(base, q, qn, sc, lane, &tl);
      if (t < 0) return SLATE_E_ZSTD_CORRUPT;
      st.huf_valid = 1;
      st.tl = tl;
      q += t;
      qn -= uint32_t(t);
    } else if (!st.huf_valid) {
      return SLATE_E_ZSTD_CORRUPT;
    }
    if (nlit > cap - d0) return SLATE_E_ZSTD_CORRUPT;
    lbase = cap - nlit;
    // stream l on lane l: bytes [sb, sb + sl), m literals to out[lbase + lo]
    uint32_t sb = 0, sl = 0, m = 0, lo = 0;
    if (streams == 1) {
      sb = uint32_t(q);
      sl = qn;
      m = nlit;
    } else {
      if (qn < 10) return SLATE_E_ZSTD_CORRUPT;
      const uint32_t l1 = bN(q - off) | (bN(q - off + 1) << 8), l2 = bN(q - off + 2) | (bN(q - off + 3) << 8),
                     l3 = bN(q - off + 4) | (bN(q - off + 5) << 8);
      if (l1 + l2 + l3 + 6 > qn) return SLATE_E_ZSTD_CORRUPT;
      const uint32_t l4 = qn - 6 - l1 - l2 - l3, seg = (nlit + 3) / 4;
      if (3 * seg > nlit) return SLATE_E_ZSTD_CORRUPT;
      const uint32_t s0 = uint32_t(q) + 6;
      sb = lane == 0 ? s0 : lane == 1 ? s0 + l1 : lane == 2 ? s0 + l1 + l2 : s0 + l1 + l2 + l3;
      sl = lane == 0 ? l1 : lane == 1 ? l2 : lane == 2 ? l3 : l4;
      m = lane < 3 ? seg : nlit - 3 * seg;
      lo = seg * uint32_t(lane < 3 ? lane : 3);
    }
    bool badl = false;
    if (uint32_t(lane) < streams && !(dbg & (1u << 17))) {
      int64_t bp = zs_bstart(base, int32_t(sb), sl);
      if (bp < 0) {
        badl = true;
      } else {
        const int64_t S = 8 * int64_t(sb);
        const uint32_t tl = st.tl;
        uint8_t* dst = out ? out + lbase + lo : nullptr;
        // 56-bit register window over stream bits [clo, clo + 56): one LDS refill per ~5
        // symbols instead of a bit fetch per symbol; the stream's first bits (an overread
        // pads with zeros) go through zs_peek
        const uint32_t tmask = (1u << tl) - 1;
        int64_t clo = 0;
        uint64_t cv = 0;
        bool have = false;
        for (uint32_t i = 0; i < m; i++) {
          const int64_t lo2 = bp - int64_t(tl);
          uint32_t v;
          if (have && lo2 >= clo) {
            v = uint32_t(cv >> (lo2 - clo)) & tmask;
          } else if (lo2 >= 0) {
            clo = bp > 56 ? bp - 56 : 0;
            cv = zs_bits(base, S + clo, 56);
            have = true;
            v = uint32_t(cv >> (lo2 - clo)) & tmask;
          } else {
            v = uint32_t(zs_peek(base, S, bp, tl));
          }
          const uint32_t e = sc->huf[v];
          if (dst) dst[i] = uint8_t(e);
          bp -= e >> 8;
        }
        badl = bp != 0;
      }
    }
    if (__ballot(badl)) return SLATE_E_ZSTD_CORRUPT;
    pos = hs + cs;
  }
  zs_sync();
  // Sequences_Section
  if (pos >= n) return SLATE_E_ZSTD_CORRUPT;
  const int32_t s = off + int32_t(pos);
  const uint32_t sn = n - pos;
  auto sB = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(base[s + int32_t(i)])); };
  uint32_t nseq, sp;
  const uint32_t c0 = sB(0);
  if (c0 < 128) {
    nseq = c0;
    sp = 1;
  } else if (c0 < 255) {
    if (sn < 2) return SLATE_E_ZSTD_CORRUPT;
    nseq = ((c0 - 128) << 8) + sB(1);
    sp = 2;
  } else {
    if (sn < 3) return SLATE_E_ZSTD_CORRUPT;
    nseq = sB(1) + (sB(2) << 8) + 0x7F00;
    sp = 3;
  }
  uint32_t lp = 0, o = d0;
  if (nseq == 0) {
    if (sp != sn) return SLATE_E_ZSTD_CORRUPT;
  } else {
    if (sp >= sn) return SLATE_E_ZSTD_CORRUPT;
    const uint32_t modes = sB(sp++);
    if (modes & 3) return SLATE_E_ZSTD_CORRUPT;
    int t = zs_table(modes >> 6, base, s + int32_t(sp), sn - sp, sc->ll, sh->ll, 6, 35, 9, sc, &st.ll, &st.ll_al, lane);
    if (t < 0) return SLATE_E_ZSTD_CORRUPT;
    sp += uint32_t(t);
    t = zs_table((modes >> 4) & 3, base, s + int32_t(sp), sn - sp, sc->of, sh->of, 5, 31, 8, sc, &st.of, &st.of_al, lane);
    if (t < 0) return SLATE_E_ZSTD_CORRUPT;
    sp += uint32_t(t);
    t = zs_table((modes >> 2) & 3, base, s + int32_t(sp), sn - sp, sc->ml, sh->ml, 6, 52, 9, sc, &st.ml, &st.ml_al, lane);
    if (t < 0) return SLATE_E_ZSTD_CORRUPT;
    sp += uint32_t(t);
    int64_t bp = zs_bstart(base, s + int32_t(sp), sn - sp);
    if (bp < 0) return SLATE_E_ZSTD_CORRUPT;
    const int64_t S = 8 * int64_t(s + int32_t(sp));
    auto rd = [&](uint32_t k) -> uint32_t {
      const uint32_t v = zrfl(uint32_t(zs_peek(base, S, bp, k)));
      bp -= k;
      return v;
    };
    uint32_t sll = rd(st.ll_al), sof = rd(st.of_al), sml = rd(st.ml_al);
    for (uint32_t i = 0; i < nseq; i++) {
      const ZsFse ell = st.ll[sll], eof = st.of[sof], eml = st.ml[sml];
      const uint32_t ofc = zrfl(uint32_t(eof.sym)), llc = zrfl(uint32_t(ell.sym)), mlc = zrfl(uint32_t(eml.sym));
      if (ofc > 31) return SLATE_E_ZSTD_CORRUPT;
      uint64_t ofv = (1ull << ofc);
      if (ofc > 24) {  // split wide offsets (peek reads <= 56 bits, but keep the pieces small)
        const uint32_t hi = rd(ofc - 24);
        ofv += (uint64_t(hi) << 24) + rd(24);
      } else {
        ofv += rd(ofc);
      }
      const uint32_t ml = kZsMLBase[mlc] + rd(kZsMLBits[mlc]);
      const uint32_t ll = kZsLLBase[llc] + rd(kZsLLBits[llc]);
      uint64_t offv;
      if (ofv > 3) {
        offv = ofv - 3;
        st.rep[2] = st.rep[1];
        st.rep[1] = st.rep[0];
        st.rep[0] = uint32_t(offv);
      } else {
        st.rep_used = 1;
        const uint32_t idx = uint32_t(ofv) - 1 + (ll == 0 ? 1u : 0u);
        offv = idx == 3 ? uint64_t(st.rep[0]) - 1 : (idx == 0 ? st.rep[0] : idx == 1 ? st.rep[1] : st.rep[2]);
        if (offv == 0) offv = 1;
        if (idx >= 2) st.rep[2] = st.rep[1];
        if (idx >= 1) {
          st.rep[1] = st.rep[0];
          st.rep[0] = uint32_t(offv);
        }
      }
      if (i + 1 < nseq) {
        sll = zrfl(uint32_t(ell.base)) + rd(zrfl(uint32_t(ell.nb)));
        sml = zrfl(uint32_t(eml.base)) + rd(zrfl(uint32_t(eml.nb)));
        sof = zrfl(uint32_t(eof.base)) + rd(zrfl(uint32_t(eof.nb)));
      }
      if (bp < 0) return SLATE_E_ZSTD_CORRUPT;
      if (ll > nlit - lp) return SLATE_E_ZSTD_CORRUPT;
      if (uint64_t(o - d0) + ll + ml > bmax || uint64_t(o) + ll + ml > cap) return SLATE_E_ZSTD_CORRUPT;
      // the write cursor must stay below the unread literals (the oracle fails at the block end)
      if (uint64_t(o) + ll + ml > uint64_t(lbase) + lp + ll) return SLATE_E_ZSTD_CORRUPT;
      if (out && !(dbg & (1u << 19))) {  // literals: dst <= src, 64 at a time, each chunk read before it is written
        for (uint32_t c = 0; c < ll; c += kWave) {
          const uint32_t j = c + uint32_t(lane);
          const uint8_t v = j < ll ? out[lbase + lp + j] : 0;
          __builtin_amdgcn_wave_barrier();
          if (j < ll) out[o + j] = v;
        }
      }
      lp += ll;
      o += ll;
      if (offv > o - fstart) return SLATE_E_ZSTD_CORRUPT;
      if (out && !(dbg & (1u << 19))) {
        const uint32_t off32 = uint32_t(offv);
        zs_sync();
        if (off32 >= ml) {
          for (uint32_t j = lane; j < ml; j += kWave) out[o + j] = out[o - off32 + j];
        } else {
          for (uint32_t j = lane; j < ml; j += kWave) out[o + j] = out[o - off32 + (j % off32)];
        }
        zs_sync();
      }
      o += ml;
    }
    if (bp != 0) return SLATE_E_ZSTD_CORRUPT;
  }
  const uint32_t rest = nlit - lp;
  if (uint64_t(o - d0) + rest > bmax || uint64_t(o) + rest > cap) return SLATE_E_ZSTD_CORRUPT;
  if (out) {
    for (uint32_t c = 0; c < rest; c += kWave) {
      const uint32_t j = c + uint32_t(lane);
      const uint8_t v = j < rest ? out[lbase + lp + j] : 0;
      __builtin_amdgcn_wave_barrier();
      if (j < rest) out[o + j] = v;
    }
    zs_sync();
  }
  *d = o + rest;
  return SLATE_OK;
}

// ------------------------------------------------------------------- XXH64
constexpr uint64_t kX64P1 = 0x9E3779B185EBCA87ull, kX64P2 = 0xC2B2AE3D27D4EB4Full, kX64P3 = 0x165667B19E3779F9ull,
                   kX64P4 = 0x85EBCA77C2B2AE63ull, kX64P5 = 0x27D4EB2F165667C5ull;
__device__ inline uint64_t x64rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ inline uint64_t x64round(uint64_t acc, uint64_t in) { return x64rotl(acc + in * kX64P2, 31) * kX64P1; }
__device__ inline uint64_t rfl64(uint64_t v) {
  return uint64_t(zrfl(uint32_t(v))) | (uint64_t(zrfl(uint32_t(v >> 32))) << 32);
}
// XXH64(seed 0) of base[off, off+n): the four stripe accumulators on lanes 0-3
__device__ uint64_t wave_xxh64(const uint8_t* base, uint32_t off, uint32_t n, int lane) {
  uint64_t h;
  if (n >= 32) {
    uint64_t v = lane == 0 ? kX64P1 + kX64P2 : (lane == 1 ? kX64P2 : (lane == 2 ? 0ull : 0ull - kX64P1));
    const uint32_t stripes = n / 32;
    if (lane < 4)
      for (uint32_t i = 0; i < stripes; i++) v = x64round(v, zs_u64(base, int32_t(off + 32 * i + 8 * uint32_t(lane))));
    uint64_t vv[4];
    for (int l = 0; l < 4; l++)
      vv[l] = uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v), l))) |  // (readlane returns int:
              (uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v >> 32), l))) << 32);  // no sign extension)
    h = x64rotl(vv[0], 1) + x64rotl(vv[1], 7) + x64rotl(vv[2], 12) + x64rotl(vv[3], 18);
    for (int l = 0; l < 4; l++) h = (h ^ x64round(0, vv[l])) * kX64P1 + kX64P4;
  } else {
    h = kX64P5;
  }
  h += n;
  uint32_t i = n & ~31u;
  for (; i + 8 <= n; i += 8) h = x64rotl(h ^ x64round(0, rfl64(zs_u64(base, int32_t(off + i)))), 27) * kX64P1 + kX64P4;
  if (i + 4 <= n) {
    h = x64rotl(h ^ uint64_t(zrfl(lds_u32(base, int32_t(off + i)))) * kX64P1, 23) * kX64P2 + kX64P3;
    i += 4;
  }
  for (; i < n; i++) h = x64rotl(h ^ uint64_t(zrfl(uint32_t(base[off + i]))) * kX64P5, 11) * kX64P1;
  h ^= h >> 33;
  h *= kX64P2;
  h ^= h >> 29;
  h *= kX64P3;
  h ^= h >> 32;
  return rfl64(h);
}

// ------------------------------------------------------------------- frames
struct ZsHdr {
  uint32_t hsize, has_fcs, checksum, status;
  uint64_t window, fcs;
};
// frame header after the magic at base[off, off+n) (oracle zs_header)
__device__ inline ZsHdr zs_header(const uint8_t* base, int32_t off, uint32_t n) {
  ZsHdr h{0, 0, 0, 0, 0, 0};
  if (n < 1) { h.status = SLATE_E_UNEXPECTED_EOF; return h; }
  auto B = [&](uint32_t i) -> uint64_t { return zrfl(uint32_t(base[off + int32_t(i)])); };
  const uint32_t fhd = uint32_t(B(0)), fcsf = fhd >> 6, ss = (fhd >> 5) & 1, dif = fhd & 3;
  if (fhd & 8) { h.status = SLATE_E_ZSTD_CORRUPT; return h; }
  const uint32_t dsz = dif == 3 ? 4 : dif, fl = fcsf == 0 ? ss : (2u << (fcsf - 1));
  h.hsize = 1 + (ss ? 0 : 1) + dsz + fl;
  if (n < h.hsize) { h.status = SLATE_E_UNEXPECTED_EOF; return h; }
  uint32_t q = 1;
  if (!ss) {
    const uint32_t wd = uint32_t(B(q++)), wl = 10 + (wd >> 3);
    h.window = (1ull << wl) + ((1ull << wl) >> 3) * (wd & 7);
  }
  uint32_t dict = 0;
  for (uint32_t i = 0; i < dsz; i++) dict |= uint32_t(B(q++)) << (8 * i);
  if (dict != 0) { h.status = SLATE_E_ZSTD_DICT; return h; }
  h.has_fcs = fl != 0;
  uint64_t f = 0;
  for (uint32_t i = 0; i < fl; i++) f |= B(q + i) << (8 * i);
  if (fl == 2) f += 256;
  h.fcs = f;
  if (ss) h.window = f;
  if (h.window > kZsMaxWindow) h.status = SLATE_E_ZSTD_CORRUPT;
  h.checksum = (fhd >> 2) & 1;
  return h;
}

__device__ inline uint32_t zs_le24(const uint8_t* base, int32_t off) {
  return zrfl(uint32_t(base[off]) | (uint32_t(base[off + 1]) << 8) | (uint32_t(base[off + 2]) << 16));
}

// One frame at base[off + *pos] (magic included; the stream is base[off, off+n)) into
// out at *d (oracle zs_frame).
__device__ int zs_frame(const uint8_t* base, int32_t off, uint32_t n, uint32_t* posp, uint8_t* out, uint32_t cap,
                        uint32_t* d, ZsScratch* sc, const ZsShared* sh, int lane, uint32_t dbg = 0) {
  uint32_t p = *posp + 4;
  const ZsHdr h = zs_header(base, off + int32_t(p), n - p);
  if (h.status) return int(h.status);
  p += h.hsize;
  const uint32_t bmax = uint32_t(h.window < kZsBlockMax ? h.window : kZsBlockMax);
  ZsState st{nullptr, nullptr, nullptr, 0, 0, 0, 0, 0, {1, 4, 8}};
  const uint32_t fstart = *d;
  for (;;) {
    if (n - p < 3) return SLATE_E_UNEXPECTED_EOF;
    const uint32_t bh = zs_le24(base, off + int32_t(p)), last = bh & 1, bt = (bh >> 1) & 3, bs = bh >> 3;
    p += 3;
    if (bt == 3) return SLATE_E_ZSTD_RESERVED_BLOCK;
    if (bs > bmax) return SLATE_E_ZSTD_CORRUPT;
    if (bt == 0) {
      if (n - p < bs) return SLATE_E_UNEXPECTED_EOF;
      if (bs > cap - *d) return SLATE_E_ZSTD_CORRUPT;
      if (out)
        for (uint32_t j = lane; j < bs; j += kWave) out[*d + j] = base[off + int32_t(p + j)];
      *d += bs;
      p += bs;
    } else if (bt == 1) {
      if (n - p < 1) return SLATE_E_UNEXPECTED_EOF;
      if (bs > cap - *d) return SLATE_E_ZSTD_CORRUPT;
      if (out) {
        const uint8_t v = base[off + int32_t(p)];
        for (uint32_t j = lane; j < bs; j += kWave) out[*d + j] = v;
      }
      *d += bs;
      p += 1;
    } else {
      if (n - p < bs) return SLATE_E_UNEXPECTED_EOF;
      const int r = zs_block(base, off + int32_t(p), bs, out, cap, d, fstart, bmax, sc, sh, st, lane, dbg);
      if (r) return r;
      p += bs;
    }
    if (last) break;
  }
  if (h.has_fcs && uint64_t(*d - fstart) != h.fcs) return SLATE_E_ZSTD_FRAME_SIZE;
  if (h.checksum) {
    if (n - p < 4) return SLATE_E_UNEXPECTED_EOF;
    if (out && !(dbg & (1u << 18))) {  // bit 18: skip the XXH64 (profiling only)
      zs_sync();
      const uint32_t want = zrfl(lds_u32(base, off + int32_t(p)));
      if (uint32_t(wave_xxh64(out, fstart, *d - fstart, lane)) != want) return SLATE_E_ZSTD_CHECKSUM;
    }
    p += 4;
  }
  *posp = p;
  return SLATE_OK;
}

// compress.Decode(CodecZstd) of base[off, off+n) into out[0, cap) (out == nullptr: sizes
// only); *out_len = bytes produced (also on failure).  oracle zs_frames.
__device__ int wave_zstd_decode(const uint8_t* base, int32_t off, uint32_t n, uint8_t* out, uint32_t cap, ZsScratch* sc,
                                const ZsShared* sh, int lane, uint32_t* out_len, uint32_t dbg = 0) {
  uint32_t pos = 0, d = 0;
  int st = SLATE_OK;
  while (pos < n) {
    if (n - pos < 4) { st = SLATE_E_UNEXPECTED_EOF; break; }
    const uint32_t magic = zrfl(lds_u32(base, off + int32_t(pos)));
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (n - pos < 8) { st = SLATE_E_UNEXPECTED_EOF; break; }
      const uint32_t sz = zrfl(lds_u32(base, off + int32_t(pos) + 4));
      if (sz > n - pos - 8) { st = SLATE_E_UNEXPECTED_EOF; break; }
      pos += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) { st = SLATE_E_ZSTD_MAGIC; break; }
    st = zs_frame(base, off, n, &pos, out, cap, &d, sc, sh, lane, dbg);
    if (st != SLATE_OK) break;
  }
  *out_len = d;
  return st;
}

// The plan size (oracle or_zstd_plan).
__device__ uint64_t wave_zstd_plan(const uint8_t* base, int32_t off, uint32_t n, ZsScratch* sc, const ZsShared* sh,
                                   int lane) {
  uint32_t pos = 0, d = 0;
  while (pos < n && n - pos >= 4) {
    const uint32_t magic = zrfl(lds_u32(base, off + int32_t(pos)));
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (n - pos < 8) break;
      const uint32_t sz = zrfl(lds_u32(base, off + int32_t(pos) + 4));
      if (sz > n - pos - 8) break;
      pos += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) break;
    const ZsHdr h = zs_header(base, off + int32_t(pos) + 4, n - pos - 4);
    if (h.status) break;
    if (!h.has_fcs) {
      if (zs_frame(base, off, n, &pos, nullptr, 0xFFFFFFFFu, &d, sc, sh, lane) != SLATE_OK) break;
      continue;
    }
    const uint32_t bmax = uint32_t(h.window < kZsBlockMax ? h.window : kZsBlockMax);
    uint32_t p = pos + 4 + h.hsize;
    uint64_t bound = 0;
    bool ok = true;
    for (;;) {
      if (n - p < 3) { ok = false; break; }
      const uint32_t bh = zs_le24(base, off + int32_t(p)), bt = (bh >> 1) & 3, bs = bh >> 3;
      p += 3;
      if (bt == 3 || bs > bmax) { ok = false; break; }
      const uint32_t adv = bt == 1 ? 1 : bs;
      if (n - p < adv) { ok = false; break; }
      bound += bt == 2 ? bmax : bs;
      p += adv;
      if (bh & 1) break;
    }
    const uint64_t add = h.fcs < bound ? h.fcs : bound;
    d = uint32_t(min(uint64_t(0xFFFFFFFFu), uint64_t(d) + add));
    if (!ok) break;
    if (h.checksum) {
      if (n - p < 4) break;
      p += 4;
    }
    pos = p;
  }
  return d;
}

}  // namespace slate
