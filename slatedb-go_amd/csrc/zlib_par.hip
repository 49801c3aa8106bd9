// Zlib index / filter payloads without flush points -- the streams compress/zlib's default writer
// (compression.go:96-103, level 6) and zlib's deflate produce, one run of deflate blocks -- inflated
// in parallel.  compress.Decode CodecZlib is io.ReadAll(zlib.NewReader(buf)) (compression.go:134-140);
// oracle/slate_oracle.c zlib_stream restates it and decode.hip wave_inflate is its exact GPU form.
//
// A deflate block's end is known only by decoding it, so block starts are found speculatively:
//   1. zp_scan: every bit position whose next bits could start a dynamic-Huffman block (BTYPE 2,
//      HLIT <= 29, HDIST <= 29, a complete code-length code) -- one thread per position;
//   2. zp_header: per survivor, the whole block header as flate reads it (code lengths through the
//      code-length code, repeat rules, literal/length and distance codes accepted by
//      huffmanDecoder.init, an end-of-block code) -- one thread per survivor;
//   3. zp_spec: per candidate, the block decoded without output (its end bit and decoded length),
//      one wave per candidate, tables in LDS;
//   4. zp_walk: one wave follows the true chain from the first block: dynamic blocks through the
//      candidates' results, stored blocks by LEN/NLEN, fixed-Huffman blocks decoded in place;
//   5. zp_emit: per block on the chain (one wave each), every decoded byte either its literal
//      value (val[x], pa[x] = x) or the byte its copy repeats (pa[x] = x - dist, global);
//   6. pointer doubling until every byte points at a literal, then a gather.
// Any check that fails (any error the serial decoder would report, a block longer than the
// speculation cap, a chain that does not end at the Adler-32 trailer, capacity limits) sets
// flag[0] and the caller hands the payload to the exact decoder, which then decodes and reports
// it: a success here is the serial decoder's success with the same bytes.
#include <hip/hip_runtime.h>

#include <utility>

#include "kernels.h"

namespace slate {
namespace {

constexpr uint32_t kZpTab = 10;             // primary decode table: 10-bit prefixes
constexpr uint32_t kZpMaxSyms = 1u << 18;   // symbols one block may hold here (longer: exact path)
constexpr uint32_t kZpWaves = 4;            // waves per workgroup in the per-block kernels
constexpr uint32_t kZpCandCap = 1u << 16;   // dynamic-header candidates
constexpr uint32_t kZpChainCap = 1u << 20;  // blocks on the chain

// One canonical code: the 10-bit table gives sym | len << 9 | 0x8000 for codes of at most 10 bits
// (indexed by the next 10 input bits, LSB first); 0 = a longer code or none (bit-serial path).
struct ZpHuff {
  uint16_t tab[1u << kZpTab];
  uint16_t sym[288];
  uint16_t count[16], first[16], index[16];
  uint32_t max, ok;
};
struct ZpWave {
  ZpHuff lit, dist;  // the code-length code is built in `dist` before the block's own codes
  uint8_t lens[320];
  uint32_t ring[128];  // input words, two halves of 64
};

__constant__ uint16_t kZpLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kZpLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kZpDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kZpDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kZpClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct ZpScratch {
  uint32_t* flag;  // [0] give up, [1] survivors, [2] candidates, [3] chain blocks, [4] decoded length
  uint32_t* surv;
  uint32_t* cand;
  uint32_t* cres;  // per candidate: end bit, decoded length, ok
  uint32_t* hkey;  // candidate position + 1 -> candidate index (open addressing)
  uint32_t* hval;
  uint32_t* chain;  // per block: start bit, type | final << 2, output offset, aux (candidate / stored byte)
  uint32_t surv_cap, hmask;
};

__host__ __device__ inline size_t zp_al(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline ZpScratch zp_carve(void* base, uint32_t nbits, size_t* bytes) {
  ZpScratch z;
  z.surv_cap = nbits / 256 + 4096;
  z.hmask = 2 * kZpCandCap - 1;
  uint8_t* q = static_cast<uint8_t*>(base);
  auto take = [&](size_t words) {
    uint32_t* r = reinterpret_cast<uint32_t*>(q);
    q += zp_al(words * 4);
    return r;
  };
  z.flag = take(16);
  z.surv = take(z.surv_cap);
  z.cand = take(kZpCandCap);
  z.cres = take(size_t(3) * kZpCandCap);
  z.hkey = take(size_t(z.hmask) + 1);
  z.hval = take(size_t(z.hmask) + 1);
  z.chain = take(size_t(4) * kZpChainCap);
  if (bytes) *bytes = size_t(q - static_cast<uint8_t*>(base));
  return z;
}

// 64 bits of the stream from bit p (LSB first); the buffer is readable 16 bytes past its end
__device__ inline uint64_t zp_bits64(const uint32_t* __restrict__ w, uint32_t p) {
  const uint32_t i = p >> 5, s = p & 31;
  const uint64_t lo = uint64_t(w[i]) | uint64_t(w[i + 1]) << 32;
  return s ? (lo >> s) | (uint64_t(w[i + 2]) << (64 - s)) : lo;
}

__device__ inline uint32_t zp_append(uint32_t* ctr, bool take, uint32_t cap, uint32_t* list, uint32_t v,
                                     uint32_t* fail) {
  const uint64_t m = __ballot(take);
  if (!m) return 0;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, uint32_t(__builtin_popcountll(m)));
  base = __shfl(base, leader, 64);
  if (take) {
    const uint32_t at = base + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)));
    if (at < cap) list[at] = v;
    else atomicOr(fail, 1u);
  }
  return 0;
}

// ---------------------------------------------------------------- 1. header scan
__global__ __launch_bounds__(256) void zp_scan_kernel(const uint32_t* __restrict__ w, uint32_t p0, uint32_t p1,
                                                      ZpScratch Z) {
  const uint32_t p = p0 + blockIdx.x * 256u + threadIdx.x;
  bool ok = p < p1;
  if (ok) {
    const uint64_t v = zp_bits64(w, p);
    ok = ((v >> 1) & 3) == 2 && ((v >> 3) & 31) <= 29 && ((v >> 8) & 31) <= 29;
    if (ok) {
      const uint32_t nclen = uint32_t((v >> 13) & 15) + 4;
      const uint64_t c = zp_bits64(w, p + 17);
      // Kraft sum of the code-length code in units of 2^-7 (lengths 1..7), complete = 128
      uint32_t kraft = 0;
      for (uint32_t i = 0; i < 19; i++) {
        const uint32_t l = i < nclen ? uint32_t(c >> (3 * i)) & 7 : 0u;
        kraft += l ? (128u >> l) : 0u;
      }
      ok = kraft == 128;
    }
  }
  zp_append(Z.flag + 1, ok, Z.surv_cap, Z.surv, p, Z.flag);
}

// ---------------------------------------------------------------- 2. full header check
// The block header at p as the serial decoder reads it; true when every check passes.  One lane,
// the code-length code through a 128-entry table in LDS.
__device__ bool zp_header_ok(const uint32_t* __restrict__ w, uint32_t p, uint32_t lim, uint8_t* cltab) {
  if (p + 17 > lim) return false;
  const uint64_t v = zp_bits64(w, p);
  const uint32_t nlit = uint32_t((v >> 3) & 31) + 257, ndist = uint32_t((v >> 8) & 31) + 1;
  const uint32_t nclen = uint32_t((v >> 13) & 15) + 4;
  uint32_t q = p + 17;
  if (q + 3 * nclen > lim) return false;
  const uint64_t c = zp_bits64(w, q);
  q += 3 * nclen;
  uint32_t cl[19];
  for (uint32_t i = 0; i < 19; i++) cl[i] = 0;
  for (uint32_t i = 0; i < 19; i++)
    if (i < nclen) cl[kZpClenOrder[i]] = uint32_t(c >> (3 * i)) & 7;
  // canonical code (complete: checked by the scan), table over 7-bit prefixes: sym | len << 5
  uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t i = 0; i < 19; i++) cnt[cl[i]]++;
  uint32_t next[8];
  uint32_t code = 0;
  cnt[0] = 0;
  for (uint32_t l = 1; l < 8; l++) {
    code = (code + cnt[l - 1]) << 1;
    next[l] = code;
  }
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t l = cl[i];
    if (!l) continue;
    const uint32_t cd = next[l]++;
    const uint32_t r = __builtin_bitreverse32(cd) >> (32 - l);
    for (uint32_t k = r; k < 128; k += (1u << l)) cltab[k] = uint8_t(i | (l << 5));
  }
  // the code lengths: Kraft sums (units of 2^-15) and nonzero counts of both codes
  uint32_t i = 0, prev = 0, klit = 0, kdist = 0, nzl = 0, nzd = 0, lmax1 = 0, dmax1 = 0, eob = 0;
  const uint32_t total = nlit + ndist;
  while (i < total) {
    if (q + 7 > lim + 7) return false;
    const uint64_t b = zp_bits64(w, q);
    const uint32_t e = cltab[b & 127];
    const uint32_t sym = e & 31, l = e >> 5;
    if (q + l > lim) return false;
    q += l;
    uint32_t rep = 1, val = sym;
    if (sym >= 16) {
      const uint64_t x = b >> l;
      if (sym == 16) {
        if (i == 0) return false;
        val = prev;
        rep = 3 + uint32_t(x & 3);
        q += 2;
      } else if (sym == 17) {
        val = 0;
        rep = 3 + uint32_t(x & 7);
        q += 3;
      } else {
        val = 0;
        rep = 11 + uint32_t(x & 127);
        q += 7;
      }
      if (q > lim || i + rep > total) return false;
    }
    for (uint32_t k = 0; k < rep; k++, i++) {
      if (val) {
        if (i < nlit) {
          klit += 32768u >> val;
          nzl++;
          lmax1 = val;
          if (i == 256) eob = 1;
        } else {
          kdist += 32768u >> val;
          nzd++;
          dmax1 = val;
        }
      }
    }
    prev = val;
  }
  // huffmanDecoder.init: complete, empty, or one code of length 1
  const bool lok = klit == 32768u || (nzl == 1 && lmax1 == 1);
  const bool dok = nzd == 0 || kdist == 32768u || (nzd == 1 && dmax1 == 1);
  return lok && dok && eob;
}

__global__ __launch_bounds__(256) void zp_header_kernel(const uint32_t* __restrict__ w, uint32_t lim, ZpScratch Z) {
  __shared__ uint8_t tabs[256 * 128];
  const uint32_t n = min(Z.flag[1], Z.surv_cap);
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t - threadIdx.x < n; t += gridDim.x * 256u) {
    const bool ok = t < n && zp_header_ok(w, Z.surv[t], lim, tabs + threadIdx.x * 128);
    zp_append(Z.flag + 2, ok, kZpCandCap, Z.cand, t < n ? Z.surv[t] : 0u, Z.flag);
  }
}

// ---------------------------------------------------------------- per-block decoding (one wave)
// Canonical tables from code lengths; ok = huffmanDecoder.init's acceptance.  Symbols of one
// length are ranked in symbol order with ballots; the 10-bit table is filled lane-strided by the
// bit-serial canonical decode of each prefix.
__device__ void zp_build(ZpHuff* h, const uint8_t* lens, uint32_t n, int lane) {
  uint32_t cnt = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + uint32_t(lane);
    const uint32_t my = i < n ? lens[i] : 0u;
    for (uint32_t l = 1; l < 16; l++) {
      const uint32_t k = uint32_t(__builtin_popcountll(__ballot(my == l)));
      cnt += (uint32_t(lane) == l) ? k : 0u;
    }
  }
  uint32_t max = 0, first = 0, idx = 0, c = 0;
  for (uint32_t l = 1; l < 16; l++) {
    const uint32_t k = __builtin_amdgcn_readlane(cnt, int(l));
    if (uint32_t(lane) == l) {
      h->count[l] = uint16_t(k);
      h->first[l] = uint16_t(first);
      h->index[l] = uint16_t(idx);
    }
    first = (first + k) << 1;
    idx += k;
    if (k) max = l;
  }
  for (uint32_t l = 1; l <= max; l++) c = (c << 1) + __builtin_amdgcn_readlane(cnt, int(l));
  if (lane == 0) {
    h->max = max;
    h->ok = (max == 0 || c == (1u << max) || (c == 1 && max == 1)) ? 1u : 0u;
  }
  uint32_t base = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += 64) {
    const uint32_t i = c0 + uint32_t(lane);
    const uint32_t my = i < n ? lens[i] : 0u;
    uint32_t pos = 0;
    for (uint32_t l = 1; l < 16; l++) {
      const uint64_t m = __ballot(my == l);
      const uint32_t before = __builtin_amdgcn_readlane(base, int(l));
      if (my == l) pos = before + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)));
      base += (uint32_t(lane) == l) ? uint32_t(__builtin_popcountll(m)) : 0u;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (my) h->sym[h->index[my] + pos] = uint16_t(i);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const uint32_t tmax = max < kZpTab ? max : kZpTab;
  for (uint32_t e = uint32_t(lane); e < (1u << kZpTab); e += 64) {
    uint32_t code = 0, ent = 0;
    for (uint32_t l = 1; l <= tmax; l++) {
      code |= (e >> (l - 1)) & 1u;
      const uint32_t f = h->first[l], k = h->count[l];
      if (code - f < k) {
        ent = uint32_t(h->sym[h->index[l] + code - f]) | (l << 9) | 0x8000u;
        break;
      }
      code <<= 1;
    }
    h->tab[e] = uint16_t(ent);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}

// Wave-uniform bit reader: words staged through an LDS ring (the half after next loaded into a
// register one half ahead), 33..64 bits buffered.  pos = the next unread bit; lim = input bits.
struct ZpBits {
  const uint32_t* w;
  uint32_t* ring;
  uint32_t nwords, pend, rw, nb, pos, lim;
  uint64_t bb;
  bool bad;
};

__device__ inline uint32_t zp_load_half(const ZpBits& b, uint32_t half, int lane) {
  const uint32_t i = half * 64u + uint32_t(lane);
  return i < b.nwords ? b.w[i] : 0u;
}

__device__ inline void zp_open(ZpBits& b, const uint32_t* w, uint32_t nwords, uint32_t* ring, uint32_t p,
                               uint32_t lim, int lane) {
  b.w = w;
  b.ring = ring;
  b.nwords = nwords;
  b.lim = lim;
  b.bad = false;
  const uint32_t w0 = p >> 5, h = w0 >> 6;
  ring[(h & 1) * 64 + lane] = zp_load_half(b, h, lane);
  ring[((h + 1) & 1) * 64 + lane] = zp_load_half(b, h + 1, lane);
  b.pend = zp_load_half(b, h + 2, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  b.bb = uint64_t(ring[w0 & 127]) >> (p & 31);
  b.nb = 32 - (p & 31);
  b.rw = w0 + 1;
  b.pos = p;
}

__device__ inline void zp_refill(ZpBits& b, int lane) {
  if (b.nb >= 32) return;
  if ((b.rw & 63) == 0) {  // entering half rw/64: the half after it (pend) goes into the ring
    const uint32_t h = b.rw >> 6;
    b.ring[((h + 1) & 1) * 64 + lane] = b.pend;
    b.pend = zp_load_half(b, h + 2, lane);
    __builtin_amdgcn_wave_barrier();
  }
  b.bb |= uint64_t(b.ring[b.rw & 127]) << b.nb;
  b.nb += 32;
  b.rw++;
}

__device__ inline uint32_t zp_take(ZpBits& b, uint32_t k) {
  const uint32_t v = uint32_t(b.bb) & ((1u << k) - 1u);
  b.bb >>= k;
  b.nb -= k;
  b.pos += k;
  if (b.pos > b.lim) b.bad = true;
  return v;
}

// the next symbol of h (refilled before); -1 when no code matches or the input ends
__device__ inline int zp_sym(ZpBits& b, const ZpHuff* h) {
  const uint32_t e = h->tab[uint32_t(b.bb) & ((1u << kZpTab) - 1)];
  if (e & 0x8000u) {
    zp_take(b, (e >> 9) & 15);
    return int(e & 511);
  }
  const uint32_t mx = h->max;
  uint32_t code = 0;
  for (uint32_t l = 1; l <= mx; l++) {
    code |= uint32_t(b.bb >> (l - 1)) & 1u;
    const uint32_t f = h->first[l], k = h->count[l];
    if (code - f < k) {
      zp_take(b, l);
      return int(h->sym[h->index[l] + code - f]);
    }
    code <<= 1;
  }
  return -1;
}

// Output of the emitting decode: val[x] / pa[x] for global byte x; literals gathered 64 at a
// time (lane k holds the k-th of the run) and written together.
struct ZpOut {
  uint8_t* val;
  uint32_t* pa;
  uint32_t x0;   // global offset of the block
  uint32_t x1;   // its end (the walk's decoded length): nothing is written at or past it
  uint32_t run;  // literals gathered (run start = x0 + d - run)
  uint32_t lit;  // this lane's literal
};

template <bool kEmit>
__device__ inline void zp_flush(ZpOut& o, uint32_t d, int lane) {
  if (!kEmit || o.run == 0) return;
  if (uint32_t(lane) < o.run) {
    const uint32_t x = o.x0 + d - o.run + uint32_t(lane);
    o.val[x] = uint8_t(o.lit);
    o.pa[x] = x;
  }
  o.run = 0;
}

// The header (BTYPE 2) or fixed tables, then the symbols up to end-of-block.  Returns false on any
// check the serial decoder would fail (or the symbol cap); *dlen = decoded bytes; b.pos = the bit
// after the block.  hdr: the block starts at b.pos with its 3 header bits.
template <bool kEmit>
__device__ bool zp_block(ZpBits& b, ZpWave* zw, const ZpHuff* fixl, const ZpHuff* fixd, ZpOut& o, uint32_t* dlen,
                         int lane) {
  zp_refill(b, lane);
  zp_take(b, 1);
  const uint32_t type = zp_take(b, 2);
  const ZpHuff *hl = fixl, *hd = fixd;
  if (type == 2) {
    zp_refill(b, lane);
    const uint32_t nlit = zp_take(b, 5) + 257, ndist = zp_take(b, 5) + 1, nclen = zp_take(b, 4) + 4;
    if (nlit > 286 || ndist > 30) return false;
    uint32_t cl = 0;
    for (uint32_t i = 0; i < 19; i++) {
      uint32_t v = 0;
      if (i < nclen) {
        zp_refill(b, lane);
        v = zp_take(b, 3);
      }
      if (uint32_t(lane) == kZpClenOrder[i]) cl = v;
    }
    if (lane < 19) zw->lens[lane] = uint8_t(cl);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    zp_build(&zw->dist, zw->lens, 19, lane);
    if (!zw->dist.ok || zw->dist.max == 0) return false;
    uint32_t i = 0, prev = 0;
    const uint32_t total = nlit + ndist;
    while (i < total) {
      zp_refill(b, lane);
      const int sym = zp_sym(b, &zw->dist);
      if (sym < 0) return false;
      if (sym < 16) {
        if (lane == 0) zw->lens[i] = uint8_t(sym);
        prev = uint32_t(sym);
        i++;
        continue;
      }
      uint32_t rep, val = 0;
      if (sym == 16) {
        if (i == 0) return false;
        val = prev;
        rep = 3 + zp_take(b, 2);
      } else if (sym == 17) {
        rep = 3 + zp_take(b, 3);
      } else {
        rep = 11 + zp_take(b, 7);
      }
      if (i + rep > total) return false;
      for (uint32_t j = uint32_t(lane); j < rep; j += 64) zw->lens[i + j] = uint8_t(val);
      prev = val;
      i += rep;
    }
    if (b.bad) return false;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (zw->lens[256] == 0) return false;
    zp_build(&zw->lit, zw->lens, nlit, lane);
    zp_build(&zw->dist, zw->lens + nlit, ndist, lane);
    if (!zw->lit.ok || !zw->dist.ok) return false;
    hl = &zw->lit;
    hd = &zw->dist;
  } else if (type != 1) {
    return false;
  }
  uint32_t d = 0;
  for (uint32_t nsym = 0; nsym < kZpMaxSyms; nsym++) {
    zp_refill(b, lane);
    const int sym = zp_sym(b, hl);
    if (sym < 0 || b.bad) return false;
    if (sym < 256) {
      if (kEmit) {
        if (o.x0 + d >= o.x1) return false;
        if (uint32_t(lane) == o.run) o.lit = uint32_t(sym);
        if (++o.run == 64) zp_flush<kEmit>(o, d + 1, lane);
      }
      d++;
      continue;
    }
    if (sym == 256) {
      zp_flush<kEmit>(o, d, lane);
      *dlen = d;
      return !b.bad;
    }
    const uint32_t s = uint32_t(sym) - 257;
    if (s >= 29) return false;
    const uint32_t len = kZpLenBase[s] + zp_take(b, kZpLenExtra[s]);
    zp_refill(b, lane);
    const int ds = zp_sym(b, hd);
    if (ds < 0 || ds >= 30) return false;
    const uint32_t dist = kZpDistBase[ds] + zp_take(b, kZpDistExtra[ds]);
    if (b.bad) return false;
    if (kEmit) {
      zp_flush<kEmit>(o, d, lane);
      const uint32_t x = o.x0 + d;
      if (dist > x) return false;  // reaches before the stream (flate: dist > bytes decoded)
      if (len > o.x1 - x) return false;
      for (uint32_t j = uint32_t(lane); j < len; j += 64) o.pa[x + j] = x + j - dist;
    }
    if (d + len < d) return false;
    d += len;
  }
  return false;  // longer than the cap: the exact path decodes it
}

__device__ void zp_fixed_build(ZpWave* zw, ZpHuff* fl, ZpHuff* fd, int lane) {
  for (uint32_t i = uint32_t(lane); i < 288; i += 64) zw->lens[i] = i < 144 ? 8 : (i < 256 ? 9 : (i < 280 ? 7 : 8));
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  zp_build(fl, zw->lens, 288, lane);
  for (uint32_t i = uint32_t(lane); i < 30; i += 64) zw->lens[i] = 5;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  zp_build(fd, zw->lens, 30, lane);
}

// ---------------------------------------------------------------- 3. speculative block decode
__global__ __launch_bounds__(64 * kZpWaves) void zp_spec_kernel(const uint32_t* __restrict__ w, uint32_t nwords,
                                                                 uint32_t lim, ZpScratch Z) {
  __shared__ ZpWave waves[kZpWaves];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  ZpWave* zw = &waves[wv];
  const uint32_t n = min(Z.flag[2], kZpCandCap);
  for (uint32_t c = blockIdx.x * kZpWaves + wv; c < n; c += gridDim.x * kZpWaves) {
    const uint32_t p = Z.cand[c];
    ZpBits b;
    zp_open(b, w, nwords, zw->ring, p, lim, lane);
    ZpOut o{};
    uint32_t dl = 0;
    const bool ok = zp_block<false>(b, zw, nullptr, nullptr, o, &dl, lane);
    if (lane == 0) {
      Z.cres[3 * c] = b.pos;
      Z.cres[3 * c + 1] = dl;
      Z.cres[3 * c + 2] = ok ? 1u : 0u;
      uint32_t h = (p * 2654435761u) & Z.hmask;
      for (;;) {
        const uint32_t prev = atomicCAS(&Z.hkey[h], 0u, p + 1);
        if (prev == 0 || prev == p + 1) {
          Z.hval[h] = c;
          break;
        }
        h = (h + 1) & Z.hmask;
      }
    }
  }
}

// ---------------------------------------------------------------- 4. the chain
__global__ __launch_bounds__(64) void zp_walk_kernel(const uint32_t* __restrict__ w, const uint8_t* __restrict__ in,
                                                     uint32_t nwords, uint32_t p0, uint32_t lim, uint32_t dend,
                                                     ZpScratch Z) {
  __shared__ ZpWave zw;
  __shared__ ZpHuff fix[2];
  const int lane = threadIdx.x & 63;
  if (Z.flag[0]) return;
  zp_fixed_build(&zw, &fix[0], &fix[1], lane);
  uint32_t p = p0, out = 0, k = 0;
  bool fail = false;
  for (;;) {
    if (k >= kZpChainCap || p + 3 > lim) {
      fail = true;
      break;
    }
    const uint32_t h3 = uint32_t(zp_bits64(w, p)) & 7;
    const uint32_t fin = h3 & 1, type = h3 >> 1;
    uint32_t aux = 0, dl = 0, nxt = 0;
    if (type == 0) {
      const uint32_t q = (p + 3 + 7) >> 3;  // LEN at the next byte boundary
      if (uint64_t(q) + 4 > lim / 8) {
        fail = true;
        break;
      }
      const uint32_t len = uint32_t(in[q]) | uint32_t(in[q + 1]) << 8;
      const uint32_t nlen = uint32_t(in[q + 2]) | uint32_t(in[q + 3]) << 8;
      if (len != (~nlen & 0xffffu) || uint64_t(q) + 4 + len > lim / 8) {
        fail = true;
        break;
      }
      aux = q + 4;
      dl = len;
      nxt = (q + 4 + len) * 8;
    } else if (type == 2) {
      uint32_t h = (p * 2654435761u) & Z.hmask, c = ~0u;
      for (;;) {
        const uint32_t key = Z.hkey[h];
        if (key == 0) break;
        if (key == p + 1) {
          c = Z.hval[h];
          break;
        }
        h = (h + 1) & Z.hmask;
      }
      if (c == ~0u || Z.cres[3 * c + 2] == 0) {
        fail = true;
        break;
      }
      aux = c;
      nxt = Z.cres[3 * c];
      dl = Z.cres[3 * c + 1];
    } else if (type == 1) {
      ZpBits b;
      zp_open(b, w, nwords, zw.ring, p, lim, lane);
      ZpOut o{};
      if (!zp_block<false>(b, &zw, &fix[0], &fix[1], o, &dl, lane)) {
        fail = true;
        break;
      }
      nxt = b.pos;
    } else {
      fail = true;
      break;
    }
    if (uint64_t(out) + dl > 0xFFFFFF00ull) {
      fail = true;
      break;
    }
    if (lane == 0) {
      Z.chain[4 * k] = p;
      Z.chain[4 * k + 1] = type | (fin << 2);
      Z.chain[4 * k + 2] = out;
      Z.chain[4 * k + 3] = aux;
    }
    out += dl;
    k++;
    p = nxt;
    if (fin) break;
  }
  // the Adler-32 trailer starts at the next byte boundary, which must be where the caller read it
  if (!fail && (p + 7) / 8 != dend) fail = true;
  if (lane == 0) {
    if (fail) Z.flag[0] = 1;
    Z.flag[3] = k;
    Z.flag[4] = out;
  }
}

// ---------------------------------------------------------------- 5. bytes
__global__ __launch_bounds__(64 * kZpWaves) void zp_emit_kernel(const uint32_t* __restrict__ w,
                                                                const uint8_t* __restrict__ in, uint32_t nwords,
                                                                uint32_t lim, ZpScratch Z, uint8_t* __restrict__ val,
                                                                uint32_t* __restrict__ pa) {
  __shared__ ZpWave waves[kZpWaves];
  __shared__ ZpHuff fix[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (Z.flag[0]) return;
  ZpWave* zw = &waves[wv];
  if (wv == 0) zp_fixed_build(zw, &fix[0], &fix[1], lane);
  __syncthreads();
  const uint32_t n = Z.flag[3], total = Z.flag[4];
  for (uint32_t k = blockIdx.x * kZpWaves + wv; k < n; k += gridDim.x * kZpWaves) {
    const uint32_t p = Z.chain[4 * k], type = Z.chain[4 * k + 1] & 3, x0 = Z.chain[4 * k + 2];
    const uint32_t aux = Z.chain[4 * k + 3];
    const uint32_t x1 = k + 1 < n ? Z.chain[4 * k + 6] : total;
    if (type == 0) {
      for (uint32_t j = uint32_t(lane); j < x1 - x0; j += 64) {
        val[x0 + j] = in[aux + j];
        pa[x0 + j] = x0 + j;
      }
      continue;
    }
    ZpBits b;
    zp_open(b, w, nwords, zw->ring, p, lim, lane);
    if (x1 < x0) {
      if (lane == 0) atomicOr(Z.flag, 1u);
      continue;
    }
    ZpOut o{val, pa, x0, x1, 0, 0};
    uint32_t dl = 0;
    const bool ok = zp_block<true>(b, zw, &fix[0], &fix[1], o, &dl, lane);
    if (!ok || dl != x1 - x0) {
      if (lane == 0) atomicOr(Z.flag, 1u);
    }
  }
}

// pointers are < n by construction (emit writes every byte of [0, n) with x or x - dist); a
// pointer outside is a defect and hands the payload to the exact path instead of reading past pa
__global__ void zp_ptr_kernel(uint32_t n, const uint32_t* __restrict__ ps, uint32_t* __restrict__ pd,
                              uint32_t* __restrict__ flag, uint32_t* __restrict__ changed, uint32_t r) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n || flag[0]) return;
  if (r > 0 && changed[r - 1] == 0) {
    pd[x] = ps[x];
    return;
  }
  const uint32_t a = ps[x];
  const uint32_t c = a < n ? ps[a] : a;
  if (c >= n) {
    atomicOr(flag, 1u);
    pd[x] = x;
    return;
  }
  pd[x] = c;
  if (__ballot(a != c) && (threadIdx.x & 63) == 0) changed[r] = 1u;
}

__global__ void zp_gather_kernel(uint32_t n, const uint32_t* __restrict__ flag, const uint8_t* __restrict__ val,
                                 const uint32_t* __restrict__ ps, uint8_t* __restrict__ out) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n || flag[0]) return;
  const uint32_t a = ps[x];
  out[x] = a < n ? val[a] : 0;
}

}  // namespace

size_t zlib_par_scratch_bytes(uint32_t clen) {
  size_t bytes = 0;
  zp_carve(nullptr, clen * 8u, &bytes);
  return bytes + 256;
}

const uint32_t* zlib_par_result(const void* scratch) {
  return static_cast<const uint32_t*>(scratch);  // flag[] is carved first
}

hipError_t launch_zlib_par_chain(hipStream_t st, const uint8_t* in, uint32_t clen, uint32_t p0, uint32_t dend,
                                 void* scratch, int num_cus) {
  if (clen >= (1u << 28) || (reinterpret_cast<uintptr_t>(in) & 3)) return hipErrorInvalidValue;
  const uint32_t lim = clen * 8u;
  const ZpScratch Z = zp_carve(scratch, lim, nullptr);
  hipError_t e = hipMemsetAsync(Z.flag, 0, 64, st);
  if (e == hipSuccess) e = hipMemsetAsync(Z.hkey, 0, (size_t(Z.hmask) + 1) * 4, st);
  if (e != hipSuccess) return e;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
  const uint32_t nwords = (clen + 3) / 4;
  const uint32_t p1 = dend * 8u;  // block headers start inside the deflate data
  if (p1 > p0) zp_scan_kernel<<<(p1 - p0 + 255) / 256, 256, 0, st>>>(w, p0, p1, Z);
  zp_header_kernel<<<uint32_t(num_cus) * 2, 256, 0, st>>>(w, lim, Z);
  zp_spec_kernel<<<uint32_t(num_cus) * 4, 64 * kZpWaves, 0, st>>>(w, nwords, lim, Z);
  zp_walk_kernel<<<1, 64, 0, st>>>(w, in, nwords, p0, lim, dend, Z);
  return hipGetLastError();
}

hipError_t launch_ptr_gather(hipStream_t st, uint32_t total, const uint8_t* val, uint32_t* pa, uint32_t* pb,
                             uint32_t* changed, uint32_t* flag, uint8_t* out) {
  if (total == 0) return hipSuccess;
  const uint32_t gb = (total + 255) / 256;
  hipError_t e = hipMemsetAsync(changed, 0, 64 * 4, st);
  if (e != hipSuccess) return e;
  uint32_t *ps = pa, *pd = pb;
  for (uint32_t r = 0; (1ull << r) < uint64_t(total); r++) {
    zp_ptr_kernel<<<gb, 256, 0, st>>>(total, ps, pd, flag, changed, r);
    std::swap(ps, pd);
  }
  zp_gather_kernel<<<gb, 256, 0, st>>>(total, flag, val, ps, out);
  return hipGetLastError();
}

hipError_t launch_zlib_par_bytes(hipStream_t st, const uint8_t* in, uint32_t clen, uint32_t total, void* scratch,
                                 uint8_t* val, uint32_t* pa, uint32_t* pb, uint32_t* changed, uint8_t* out,
                                 int num_cus) {
  const uint32_t lim = clen * 8u;
  const ZpScratch Z = zp_carve(scratch, lim, nullptr);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
  const uint32_t nwords = (clen + 3) / 4;
  zp_emit_kernel<<<uint32_t(num_cus) * 4, 64 * kZpWaves, 0, st>>>(w, in, nwords, lim, Z, val, pa);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ptr_gather(st, total, val, pa, pb, changed, Z.flag, out);
}

}  // namespace slate
