// compress.Encode for CodecLz4, CodecZlib and CodecZstd (internal/compress/compression.go:80-116:
// lz4.NewWriter, zlib.NewWriter, zstd.NewWriter(...).EncodeAll), for SST blocks (block.go:54-75),
// the bloom filter (bloom.go:52-67) and the index (flatbuf.go:126-139).
//
// The reference's encoders (github.com/pierrec/lz4/v4, compress/zlib, klauspost/compress/zstd)
// are third-party and absent here, so their exact bytes are not reproduced ("parity unpinned"):
// what is reproduced is the format -- every frame written here decodes, with the reference's
// readers as restated in oracle/ and with liblz4 / zlib / libzstd, to the input bytes -- which is
// what the SST readers (decode.go, compression.go:126-157) require.
//
// One LZ77 parse serves all three formats: the payload is cut into pieces of at most 64 KiB, each
// piece is parsed by the golang/snappy block encoder already used for CodecSnappy (snappy_enc.h,
// one wave per piece), and its tags are transcoded:
//   * LZ4: one independent LZ4 block per piece (token / literals / offset / match length,
//     end-of-block rules: the last 5 bytes literal, no match starting in the last 12);
//   * Zlib: one fixed-Huffman deflate block per piece (RFC 1951 3.2.6; matches split at 258,
//     distances above 32 KiB left literal), stored blocks when that is smaller, an empty stored
//     block after non-final pieces to byte-align them;
//   * Zstd: one compressed block per piece: raw literals section, sequences with the predefined
//     FSE distributions (RFC 8878 3.1.1.3.2.2), offsets never as repeat codes, raw block when
//     that is smaller.
// Literal bytes are taken from the raw piece (a 64-byte window across the lanes), so the
// transcoders only need the match positions from the tags.  A final pass per payload writes the
// frame: header, the pieces' bodies (or raw / stored forms), trailer (LZ4 XXH32 content checksum,
// Zlib Adler-32, Zstd XXH64) and, for blocks / filter / index, the BE32 CRC32 of the frame.
#include "common.h"
#include "encode.h"
#include "snappy_enc.h"
#include "wave_crc.h"

namespace slate {

namespace {

constexpr uint32_t kPieceMax = 65536;
constexpr uint32_t kSmallPiece = 4096;  // pieces up to this size: four waves per workgroup, LDS sequences
constexpr uint32_t kSmallSeqs = kSmallPiece / 4 + 2;

// ------------------------------------------------------------------ wave helpers
// bytes p.. of a global buffer through a 64-byte window held one byte per lane (wave-uniform p)
struct Win {
  const uint8_t* src;
  uint32_t n;
  uint32_t base = 0x80000000u, v = 0;
  __device__ uint32_t at(uint32_t p, uint32_t lane) {
    if (p - base >= 64u) {
      base = p;
      v = (p + lane < n) ? uint32_t(src[p + lane]) : 0u;
    }
    return __builtin_amdgcn_readlane(v, int(p - base));
  }
};

// serial byte writer (wave-uniform values; lane 0 stores)
struct BW {
  uint8_t* dst;
  uint32_t d, cap;
  bool over;
  __device__ void put(uint32_t lane, uint32_t b) {
    if (d < cap && lane == 0) dst[d] = uint8_t(b);
    over |= d >= cap;
    d++;
  }
};

// LSB-first bit writer (deflate, zstd), lane 0 stores whole bytes
struct Bits {
  uint64_t acc = 0;
  uint32_t nb = 0;
  __device__ void add(BW& w, uint32_t lane, uint64_t v, uint32_t k) {
    acc |= (k ? (v & ((uint64_t(1) << k) - 1)) : 0) << nb;
    nb += k;
    while (nb >= 8) {
      w.put(lane, uint32_t(acc & 0xff));
      acc >>= 8;
      nb -= 8;
    }
  }
  __device__ void pad(BW& w, uint32_t lane) {  // to the byte boundary (zero bits)
    if (nb) {
      w.put(lane, uint32_t(acc & 0xff));
      acc = 0;
      nb = 0;
    }
  }
};

// copy raw[a, a + len) to dst[d, d + len) across the lanes
__device__ inline void copy_bytes(uint8_t* dst, uint32_t d, uint32_t cap, const uint8_t* raw, uint32_t a, uint32_t len,
                                  uint32_t lane) {
  for (uint32_t k = lane; k < len; k += 64)
    if (d + k < cap) dst[d + k] = raw[a + k];
}

// ------------------------------------------------------------------ the LZ77 parse of a piece
// Matches from the golang/snappy tags of the piece: consecutive copies with the same offset that
// continue each other are merged.  next() returns false at the end of the tags.
struct Parse {
  Win w;
  uint32_t s = 0, d = 0;  // tag position, raw position
  uint32_t mpos = 0, mlen = 0, moff = 0;  // the pending match (mlen 0: none)
  __device__ bool tag(uint32_t lane, uint32_t* pos, uint32_t* len, uint32_t* off) {
    // the next copy tag; literal tags only advance d
    while (s < w.n) {
      const uint32_t c = w.at(s, lane), t = c & 3;
      if (t == 0) {
        uint32_t x = c >> 2, hl = 1;
        if (x >= 60) {
          const uint32_t nb = x - 59;
          x = 0;
          for (uint32_t k = 0; k < nb; k++) x |= w.at(s + 1 + k, lane) << (8 * k);
          hl += nb;
        }
        s += hl + x + 1;
        d += x + 1;
        continue;
      }
      uint32_t L, O;
      if (t == 1) {
        L = 4 + ((c >> 2) & 7);
        O = ((c & 0xe0) << 3) | w.at(s + 1, lane);
        s += 2;
      } else if (t == 2) {
        L = 1 + (c >> 2);
        O = w.at(s + 1, lane) | (w.at(s + 2, lane) << 8);
        s += 3;
      } else {
        L = 1 + (c >> 2);
        O = w.at(s + 1, lane) | (w.at(s + 2, lane) << 8) | (w.at(s + 3, lane) << 16) | (w.at(s + 4, lane) << 24);
        s += 5;
      }
      *pos = d;
      *len = L;
      *off = O;
      d += L;
      return true;
    }
    return false;
  }
  // the next merged match: (pos, len, off); false when none is left
  __device__ bool next(uint32_t lane, uint32_t* pos, uint32_t* len, uint32_t* off) {
    uint32_t p, l, o;
    while (tag(lane, &p, &l, &o)) {
      if (mlen && o == moff && p == mpos + mlen) {
        mlen += l;
        continue;
      }
      const bool had = mlen != 0;
      const uint32_t hp = mpos, hl = mlen, ho = moff;
      mpos = p;
      mlen = l;
      moff = o;
      if (had) {
        *pos = hp;
        *len = hl;
        *off = ho;
        return true;
      }
    }
    if (mlen) {
      *pos = mpos;
      *len = mlen;
      *off = moff;
      mlen = 0;
      return true;
    }
    return false;
  }
};

// ------------------------------------------------------------------ LZ4 block
__device__ inline void lz4_len(BW& w, uint32_t lane, uint32_t v) {  // v >= 15 already in the token
  v -= 15;
  while (v >= 255) {
    w.put(lane, 255);
    v -= 255;
  }
  w.put(lane, v);
}

__device__ uint32_t lz4_body(const uint8_t* tags, uint32_t tn, const uint8_t* raw, uint32_t n, uint8_t* dst, uint32_t cap,
                             uint32_t lane, bool* over) {
  BW w{dst, 0, cap, false};
  Parse P{Win{tags, tn}};
  uint32_t lit = 0, pos, len, off;
  auto seq = [&](uint32_t ll, uint32_t ml, uint32_t o, bool last) {
    const uint32_t tok = (min(ll, 15u) << 4) | (last ? 0u : min(ml - 4, 15u));
    w.put(lane, tok);
    if (ll >= 15) lz4_len(w, lane, ll);
    copy_bytes(dst, w.d, cap, raw, lit, ll, lane);
    w.over |= w.d + ll > cap;
    w.d += ll;
    if (last) return;
    w.put(lane, o & 0xff);
    w.put(lane, o >> 8);
    if (ml - 4 >= 15) lz4_len(w, lane, ml - 4);
  };
  while (P.next(lane, &pos, &len, &off)) {
    // LZ4 end-of-block rules: no match starts in the last 12 bytes, the last 5 bytes are literals
    if (n < 12 || pos > n - 12 || off > 65535) continue;
    if (pos + len > n - 5) len = n - 5 - pos;
    if (len < 4) continue;
    seq(pos - lit, len, off, false);
    lit = pos + len;
  }
  seq(n - lit, 0, 0, true);
  *over = w.over;
  return w.d;
}

// a match of the parse: Zstd (literal run before, length, offset) / deflate (position, length, offset)
struct Seq {
  uint32_t ll, ml, off;
};

// ------------------------------------------------------------------ deflate
__device__ __constant__ uint16_t kDLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                                  31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__device__ __constant__ uint8_t kDLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                                  2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__device__ __constant__ uint16_t kDDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                                   33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__device__ __constant__ uint8_t kDDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                                   6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// Huffman codes go out most significant bit first (RFC 1951 3.1.1): reversed into the LSB writer
__device__ inline uint32_t rev(uint32_t code, uint32_t len) { return __builtin_bitreverse32(code) >> (32 - len); }
__device__ inline void fixed_sym(Bits& b, BW& w, uint32_t lane, uint32_t sym) {
  uint32_t code, len;
  if (sym < 144) {
    code = 0x30 + sym;
    len = 8;
  } else if (sym < 256) {
    code = 0x190 + sym - 144;
    len = 9;
  } else if (sym < 280) {
    code = sym - 256;
    len = 7;
  } else {
    code = 0xC0 + sym - 280;
    len = 8;
  }
  b.add(w, lane, rev(code, len), len);
}
__device__ inline uint32_t fixed_bits(uint32_t sym) { return sym < 144 ? 8 : (sym < 256 ? 9 : (sym < 280 ? 7 : 8)); }

__device__ inline uint32_t dcode_len(uint32_t l) {  // length code index (0..28)
  uint32_t c = 0;
  while (c < 28 && kDLenBase[c + 1] <= l) c++;
  return c;
}
__device__ inline uint32_t dcode_dist(uint32_t dd) {
  uint32_t c = 0;
  while (c < 29 && kDDistBase[c + 1] <= dd) c++;
  return c;
}

// the deflate matches of a piece: lengths 3..258, distances <= 32768
template <typename F>
__device__ void deflate_matches(const uint8_t* tags, uint32_t tn, uint32_t lane, F&& emit) {
  Parse P{Win{tags, tn}};
  uint32_t pos, len, off;
  while (P.next(lane, &pos, &len, &off)) {
    if (off > 32768) continue;
    while (len) {
      const uint32_t take = len > 258 ? (len - 258 < 3 ? len - 3 : 258) : len;
      emit(pos, take, off);
      pos += take;
      len -= take;
    }
  }
}

// ---- dynamic Huffman (RFC 1951 3.2.7).  Per-wave scratch of the entropy stage (LDS).
constexpr uint32_t kDSyms = 286 + 30;  // literal / length codes, then distance codes
struct DFse {
  uint32_t freq[kDSyms];
  uint32_t A[kDSyms];          // the in-place Huffman array (sorted weights -> lengths)
  uint16_t order[kDSyms];      // symbols by ascending frequency
  uint16_t code[kDSyms];       // bit-reversed canonical codes
  uint8_t len[kDSyms];
  uint16_t rle[kDSyms];        // the code-length sequence, RLE-coded: symbol | extra << 5
  uint32_t cfreq[19];
  uint8_t clen[19];
  uint16_t ccode[19];
  uint32_t blc[17];
  uint32_t nextc[17];
};
constexpr uint32_t kDFseBytes = (sizeof(DFse) + 15) & ~15u;
constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Code lengths of a minimum-redundancy code over freq[0..n) limited to maxbits (Moffat-Katajainen
// in-place algorithm on the weights sorted by a wave-parallel rank, then zlib's overflow fix: leaves
// deeper than maxbits lifted, the Kraft sum restored by splitting shallower leaves, the lengths
// handed out shortest-first by frequency).  A single used symbol gets length 1.  len[] is written.
__device__ void huff_lengths(DFse* F, const uint32_t* freq, uint8_t* len, uint16_t* order, uint32_t n, uint32_t maxbits,
                             uint32_t lane) {
  // rank sort of the used symbols by (frequency, symbol)
  uint32_t used = 0;
  for (uint32_t s0 = 0; s0 < n; s0 += 64) {
    const uint32_t s = s0 + lane;
    const bool u = s < n && freq[s] != 0;
    used += uint32_t(__builtin_popcountll(__ballot(u)));
  }
  for (uint32_t s = lane; s < n; s += 64) {
    len[s] = 0;
    const uint32_t f = freq[s];
    if (!f) continue;
    uint32_t r = 0;
    for (uint32_t t = 0; t < n; t++) {
      const uint32_t g = freq[t];
      r += (g != 0 && (g < f || (g == f && t < s))) ? 1u : 0u;
    }
    order[r] = uint16_t(s);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0 && used) {
    uint32_t* A = F->A;
    if (used == 1) {
      len[order[0]] = 1;
    } else {
      const int m = int(used);
      for (int i = 0; i < m; i++) A[i] = freq[order[i]];
      // phase 1: internal node weights, parents
      A[0] += A[1];
      int root = 0, leaf = 2;
      for (int next = 1; next < m - 1; next++) {
        if (leaf >= m || A[root] < A[leaf]) {
          A[next] = A[root];
          A[root++] = uint32_t(next);
        } else {
          A[next] = A[leaf++];
        }
        if (leaf >= m || (root < next && A[root] < A[leaf])) {
          A[next] += A[root];
          A[root++] = uint32_t(next);
        } else {
          A[next] += A[leaf++];
        }
      }
      // phase 2: internal node depths
      A[m - 2] = 0;
      for (int next = m - 3; next >= 0; next--) A[next] = A[A[next]] + 1;
      // phase 3: leaf depths (ascending weight -> descending depth)
      int avail = 1, usedn = 0, depth = 0, r = m - 2, next = m - 1;
      while (avail > 0) {
        while (r >= 0 && int(A[r]) == depth) {
          usedn++;
          r--;
        }
        while (avail > usedn) {
          A[next--] = uint32_t(depth);
          avail--;
        }
        avail = 2 * usedn;
        depth++;
        usedn = 0;
      }
      // A[i] = the length of order[i] (A ascending in weight: A[0] the rarest, longest)
      uint32_t* bl = F->blc;
      for (uint32_t k = 0; k <= 16; k++) bl[k] = 0;
      uint32_t maxl = 0;
      for (int i = 0; i < m; i++) {
        const uint32_t l = A[i] > maxbits ? maxbits : A[i];
        maxl = A[i] > maxl ? A[i] : maxl;
        bl[l]++;
      }
      if (maxl > maxbits) {
        uint64_t kraft = 0;
        for (uint32_t l = 1; l <= maxbits; l++) kraft += uint64_t(bl[l]) << (maxbits - l);
        while (kraft > (uint64_t(1) << maxbits)) {
          uint32_t l = maxbits - 1;
          while (bl[l] == 0) l--;
          bl[l]--;
          bl[l + 1] += 2;
          bl[maxbits]--;
          kraft--;
        }
        // shortest lengths to the most frequent symbols
        int i = m - 1;
        for (uint32_t l = 1; l <= maxbits; l++)
          for (uint32_t k = 0; k < bl[l]; k++) A[i--] = l;
      }
      for (int i = 0; i < m; i++) len[order[i]] = uint8_t(A[i]);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// canonical codes (RFC 1951 3.2.2), bit-reversed for the LSB-first writer; one lane
__device__ void huff_codes(const uint8_t* len, uint16_t* code, uint32_t n, uint32_t* blc, uint32_t* next) {
  for (uint32_t k = 0; k <= 16; k++) blc[k] = 0;
  for (uint32_t s = 0; s < n; s++) blc[len[s]]++;
  blc[0] = 0;
  uint32_t c = 0;
  for (uint32_t b = 1; b <= 16; b++) {
    c = (c + blc[b - 1]) << 1;
    next[b] = c;
  }
  for (uint32_t s = 0; s < n; s++) {
    const uint32_t l = len[s];
    code[s] = l ? uint16_t(rev(next[l]++, l)) : 0;
  }
}

// A source of deflate matches (lengths 3..258, distances <= 32768) in order: the golang/snappy
// parse's copies (tags), or a list the chain parse built (Seq: ll = position, ml = length).
struct DSrc {
  const uint8_t* tags;
  uint32_t tn;
  const Seq* list;  // nullptr: the tags
  uint32_t nlist;
  template <typename F>
  __device__ void each(uint32_t lane, F&& emit) const {
    if (!list) {
      deflate_matches(tags, tn, lane, emit);
      return;
    }
    for (uint32_t i = 0; i < nlist; i++) {
      const Seq q = list[i];
      emit(uint32_t(__builtin_amdgcn_readfirstlane(q.ll)), uint32_t(__builtin_amdgcn_readfirstlane(q.ml)),
           uint32_t(__builtin_amdgcn_readfirstlane(q.off)));
    }
  }
};

// Greedy LZ77 parse with hash chains (3-byte minimum, zlib's match rules: lengths 3..258,
// distances <= 32768, up to kChain candidates per position) of a piece of at most kSmallPiece bytes
// staged in LDS (`raw`); matches into `out` (at most cap).  Candidates are compared 64 bytes at a
// time across the lanes.  The count, or ~0u when cap is exceeded.
constexpr uint32_t kChain = 32, kNice = 128, kHashBits = 12;
__device__ uint32_t chain_parse(const uint8_t* raw, uint32_t n, uint16_t* head, uint16_t* prev, Seq* out, uint32_t cap,
                                uint32_t lane) {
  for (uint32_t h = lane; h < (1u << kHashBits); h += 64) head[h] = 0xFFFF;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  auto hash = [&](uint32_t p) {
    const uint32_t v = uint32_t(raw[p]) | (uint32_t(raw[p + 1]) << 8) | (uint32_t(raw[p + 2]) << 16);
    return (v * 2654435761u) >> (32 - kHashBits);
  };
  auto insert = [&](uint32_t p) {
    const uint32_t h = hash(p);
    const uint32_t c = head[h];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      prev[p] = uint16_t(c);
      head[h] = uint16_t(p);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  uint32_t nm = 0, p = 0;
  while (p + 3 <= n) {
    const uint32_t lim = min(258u, n - p);
    uint32_t best = 0, boff = 0, c = head[hash(p)];
    for (uint32_t k = 0; k < kChain && c != 0xFFFF && best < kNice; k++) {
      uint32_t l = 0;
      for (;;) {  // common prefix of raw[c..] and raw[p..], 64 bytes per round
        const uint32_t i = l + lane;
        const bool same = i < lim && raw[c + i] == raw[p + i];
        const uint64_t miss = ~__ballot(same);
        if (miss) {
          l += uint32_t(__builtin_ctzll(miss));
          break;
        }
        l += 64;
      }
      if (l > best) {
        best = l;
        boff = p - c;
      }
      c = prev[c];
    }
    if (best >= 3) {
      if (nm >= cap) return ~0u;
      if (lane == 0) out[nm] = Seq{p, best, boff};
      nm++;
      for (uint32_t q = p; q < p + best && q + 3 <= n; q++) insert(q);
      p += best;
    } else {
      insert(p);
      p++;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return nm;
}

// One piece as deflate blocks: dynamic Huffman, fixed Huffman or stored, whichever is smallest; a
// non-final piece ends with an empty stored block (byte alignment for the next piece).
__device__ uint32_t deflate_body(const DSrc& src, const uint8_t* raw, uint32_t n, bool final, uint8_t* dst, uint32_t cap,
                                 DFse* F, uint32_t lane, bool* over) {
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // symbol frequencies (and the fixed form's size, in bits)
  for (uint32_t s = lane; s < kDSyms; s += 64) F->freq[s] = 0;
  sync();
  uint64_t fbits = 3 + 7, xbits = 0;  // fixed-form bits; extra bits (both Huffman forms)
  {
    uint32_t lit = 0;
    auto lits = [&](uint32_t a, uint32_t e) {
      uint32_t fb = 0;
      for (uint32_t q = a + lane; q < e; q += 64) {
        const uint32_t c = raw[q];
        atomicAdd(&F->freq[c], 1u);
        fb += fixed_bits(c);
      }
      for (int o = 32; o >= 1; o >>= 1) fb += uint32_t(__shfl_xor(int(fb), o, 64));
      fbits += uint32_t(__builtin_amdgcn_readfirstlane(fb));
    };
    src.each(lane, [&](uint32_t pos, uint32_t len, uint32_t off) {
      lits(lit, pos);
      const uint32_t lc = dcode_len(len), dc = dcode_dist(off);
      if (lane == 0) {
        F->freq[257 + lc]++;
        F->freq[286 + dc]++;
      }
      fbits += fixed_bits(257 + lc) + 5;
      xbits += kDLenExtra[lc] + kDDistExtra[dc];
      lit = pos + len;
    });
    lits(lit, n);
  }
  sync();
  if (lane == 0) {
    F->freq[256] = 1;
    bool anyd = false;
    for (uint32_t d = 0; d < 30; d++) anyd |= F->freq[286 + d] != 0;
    if (!anyd) F->freq[286] = 1;  // one distance code of length 1: no match uses it
  }
  sync();
  fbits += 7 + xbits;
  huff_lengths(F, F->freq, F->len, F->order, 286, 15, lane);
  huff_lengths(F, F->freq + 286, F->len + 286, F->order, 30, 15, lane);
  // the header: HLIT / HDIST, the code lengths RLE-coded (16: repeat the previous 3..6 times, 17 / 18:
  // 3..10 / 11..138 zeros), the code-length code
  uint32_t hlit = 257, hdist = 1, nrle = 0, hclen = 4;
  uint64_t dbits = 0;
  if (lane == 0) {
    for (uint32_t s = 257; s < 286; s++)
      if (F->len[s]) hlit = s + 1;
    for (uint32_t d = 1; d < 30; d++)
      if (F->len[286 + d]) hdist = d + 1;
    auto L = [&](uint32_t i) -> uint32_t { return i < hlit ? F->len[i] : F->len[286 + i - hlit]; };
    const uint32_t tot = hlit + hdist;
    for (uint32_t k = 0; k < 19; k++) F->cfreq[k] = 0;
    uint32_t i = 0;
    while (i < tot) {
      const uint32_t v = L(i);
      uint32_t r = 1;
      while (i + r < tot && L(i + r) == v) r++;
      uint32_t k = r;
      if (v == 0 && r >= 3) {
        while (k >= 3) {
          const uint32_t m = k < 138 ? k : 138;
          const uint32_t sym = m >= 11 ? 18u : 17u;
          F->rle[nrle++] = uint16_t(sym | ((m - (m >= 11 ? 11u : 3u)) << 5));
          F->cfreq[sym]++;
          k -= m;
        }
      } else if (v != 0 && r >= 4) {
        F->rle[nrle++] = uint16_t(v);
        F->cfreq[v]++;
        k = r - 1;
        while (k >= 3) {
          const uint32_t m = k < 6 ? k : 6;
          F->rle[nrle++] = uint16_t(16 | ((m - 3) << 5));
          F->cfreq[16]++;
          k -= m;
        }
      }
      for (; k > 0; k--) {
        F->rle[nrle++] = uint16_t(v);
        F->cfreq[v]++;
      }
      i += r;
    }
  }
  hlit = uint32_t(__builtin_amdgcn_readfirstlane(hlit));
  hdist = uint32_t(__builtin_amdgcn_readfirstlane(hdist));
  nrle = uint32_t(__builtin_amdgcn_readfirstlane(nrle));
  sync();
  huff_lengths(F, F->cfreq, F->clen, F->order, 19, 7, lane);
  if (lane == 0) {
    for (uint32_t k = 0; k < 19; k++)
      if (F->clen[kClOrder[k]]) hclen = k + 1 > hclen ? k + 1 : hclen;
    huff_codes(F->len, F->code, 286, F->blc, F->nextc);
    huff_codes(F->len + 286, F->code + 286, 30, F->blc, F->nextc);
    huff_codes(F->clen, F->ccode, 19, F->blc, F->nextc);
    dbits = 3 + 5 + 5 + 4 + 3 * hclen;
    for (uint32_t j = 0; j < nrle; j++) {
      const uint32_t sym = F->rle[j] & 31;
      dbits += F->clen[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
    }
    for (uint32_t s = 0; s < kDSyms; s++) dbits += uint64_t(F->freq[s]) * F->len[s];
    dbits += xbits;
  }
  hclen = uint32_t(__builtin_amdgcn_readfirstlane(hclen));
  dbits = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(dbits >> 32))) << 32) |
          __builtin_amdgcn_readfirstlane(uint32_t(dbits));
  sync();
  const uint64_t stored = 8ull * (n + 5 * ((n + 65534) / 65535 + (n == 0))) + 8;
  BW w{dst, 0, cap, false};
  Bits b;
  if (dbits <= fbits && dbits <= stored) {
    b.add(w, lane, final ? 1 : 0, 1);
    b.add(w, lane, 2, 2);  // BTYPE 10
    b.add(w, lane, hlit - 257, 5);
    b.add(w, lane, hdist - 1, 5);
    b.add(w, lane, hclen - 4, 4);
    for (uint32_t k = 0; k < hclen; k++) b.add(w, lane, F->clen[kClOrder[k]], 3);
    for (uint32_t j = 0; j < nrle; j++) {
      const uint32_t e = F->rle[j], sym = e & 31;
      b.add(w, lane, F->ccode[sym], F->clen[sym]);
      if (sym >= 16) b.add(w, lane, e >> 5, sym == 16 ? 2 : sym == 17 ? 3 : 7);
    }
    uint32_t lit = 0;
    auto lits = [&](uint32_t a, uint32_t e) {
      for (uint32_t q = a; q < e; q++) {
        const uint32_t c = raw[q];
        b.add(w, lane, F->code[c], F->len[c]);
      }
    };
    src.each(lane, [&](uint32_t pos, uint32_t len, uint32_t off) {
      lits(lit, pos);
      const uint32_t lc = dcode_len(len), dc = dcode_dist(off);
      b.add(w, lane, F->code[257 + lc], F->len[257 + lc]);
      b.add(w, lane, len - kDLenBase[lc], kDLenExtra[lc]);
      b.add(w, lane, F->code[286 + dc], F->len[286 + dc]);
      b.add(w, lane, off - kDDistBase[dc], kDDistExtra[dc]);
      lit = pos + len;
    });
    lits(lit, n);
    b.add(w, lane, F->code[256], F->len[256]);
  } else if (fbits <= stored) {
    b.add(w, lane, final ? 1 : 0, 1);
    b.add(w, lane, 1, 2);  // BTYPE 01
    uint32_t lit = 0;
    auto lits = [&](uint32_t a, uint32_t e) {
      for (uint32_t q = a; q < e; q++) fixed_sym(b, w, lane, raw[q]);
    };
    src.each(lane, [&](uint32_t pos, uint32_t len, uint32_t off) {
      lits(lit, pos);
      const uint32_t lc = dcode_len(len), dc = dcode_dist(off);
      fixed_sym(b, w, lane, 257 + lc);
      b.add(w, lane, len - kDLenBase[lc], kDLenExtra[lc]);
      b.add(w, lane, rev(dc, 5), 5);
      b.add(w, lane, off - kDDistBase[dc], kDDistExtra[dc]);
      lit = pos + len;
    });
    lits(lit, n);
    fixed_sym(b, w, lane, 256);
  } else {
    // stored blocks of at most 65535 bytes
    uint32_t a = 0;
    do {
      const uint32_t k = min(n - a, 65535u);
      const bool last = final && a + k == n;
      b.add(w, lane, last ? 1 : 0, 1);
      b.add(w, lane, 0, 2);
      b.pad(w, lane);
      w.put(lane, k & 0xff);
      w.put(lane, k >> 8);
      w.put(lane, ~k & 0xff);
      w.put(lane, (~k >> 8) & 0xff);
      copy_bytes(dst, w.d, cap, raw, a, k, lane);
      w.over |= w.d + k > cap;
      w.d += k;
      a += k;
    } while (a < n);
  }
  if (!final) {  // empty stored block: the next piece starts on a byte boundary
    b.add(w, lane, 0, 3);
    b.pad(w, lane);
    w.put(lane, 0);
    w.put(lane, 0);
    w.put(lane, 0xff);
    w.put(lane, 0xff);
  }
  b.pad(w, lane);
  *over = w.over;
  return w.d;
}

// ------------------------------------------------------------------ zstd (predefined FSE)
// RFC 8878 3.1.1.3.2.2 default distributions and the code tables (as decode.hip's zstd.h).
constexpr int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__device__ __constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                                20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__device__ __constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,
                                               1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__device__ __constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                                21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                                43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__device__ __constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                               0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

// FSE compression table (zstd's FSE_buildCTable over a normalized distribution): the state
// table and each symbol's (deltaNbBits, deltaFindState).
template <int N, int LOG>
struct FseCT {
  uint16_t state[1 << LOG];
  int32_t delta_find[N];
  uint32_t delta_nb[N];
  constexpr FseCT(const int16_t (&norm)[N]) : state{}, delta_find{}, delta_nb{} {
    constexpr uint32_t size = 1u << LOG, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t cumul[N + 1] = {};
    uint8_t sym[size] = {};
    uint32_t high = size - 1;
    for (int u = 1; u <= N; u++) {
      if (norm[u - 1] == -1) {
        cumul[u] = cumul[u - 1] + 1;
        sym[high--] = uint8_t(u - 1);
      } else {
        cumul[u] = cumul[u - 1] + uint32_t(norm[u - 1]);
      }
    }
    uint32_t pos = 0;
    for (int s = 0; s < N; s++)
      for (int k = 0; k < norm[s]; k++) {
        sym[pos] = uint8_t(s);
        pos = (pos + step) & mask;
        while (pos > high) pos = (pos + step) & mask;
      }
    for (uint32_t u = 0; u < size; u++) state[cumul[sym[u]]++] = uint16_t(size + u);
    uint32_t total = 0;
    for (int s = 0; s < N; s++) {
      const int c = norm[s];
      if (c == 0) {
        delta_nb[s] = ((LOG + 1) << 16) - size;
      } else if (c == -1 || c == 1) {
        delta_nb[s] = (LOG << 16) - size;
        delta_find[s] = int32_t(total) - 1;
        total++;
      } else {
        uint32_t hb = 31 - __builtin_clz(uint32_t(c - 1));
        const uint32_t max_bits = LOG - hb;
        const uint32_t min_plus = uint32_t(c) << max_bits;
        delta_nb[s] = (max_bits << 16) - min_plus;
        delta_find[s] = int32_t(total) - c;
        total += uint32_t(c);
      }
    }
  }
};
__device__ __constant__ FseCT<36, 6> kCtLL(kLLDef);
__device__ __constant__ FseCT<53, 6> kCtML(kMLDef);
__device__ __constant__ FseCT<29, 5> kCtOF(kOFDef);

// An FSE compression table in memory (the predefined ones above, or one built for a block).
struct FseRT {
  const uint16_t* state;
  const uint32_t* dnb;
  const int32_t* dfs;
  uint32_t L;
};
template <int N, int LOG>
__device__ inline FseRT fse_rt(const FseCT<N, LOG>& t) {
  return FseRT{t.state, t.delta_nb, reinterpret_cast<const int32_t*>(t.delta_find), uint32_t(LOG)};
}
struct FseStateR {
  uint32_t v;
  __device__ void init(const FseRT& t, uint32_t s) {
    const uint32_t nb_out = (t.dnb[s] + (1u << 15)) >> 16;
    const uint32_t v0 = (nb_out << 16) - t.dnb[s];
    v = t.state[(v0 >> nb_out) + t.dfs[s]];
  }
  __device__ void enc(Bits& b, BW& w, uint32_t lane, const FseRT& t, uint32_t s) {
    const uint32_t nb_out = (v + t.dnb[s]) >> 16;
    b.add(w, lane, v, nb_out);
    v = t.state[(v >> nb_out) + t.dfs[s]];
  }
  __device__ void flush(Bits& b, BW& w, uint32_t lane, const FseRT& t) { b.add(w, lane, v, t.L); }
};

__device__ inline uint32_t ll_code(uint32_t v) {
  if (v < 16) return v;
  uint32_t c = 16;
  while (c < 35 && kLLBase[c + 1] <= v) c++;
  return c;
}
__device__ inline uint32_t ml_code(uint32_t m) {  // m = match length
  if (m < 35) return m - 3;
  uint32_t c = 32;
  while (c < 52 && kMLBase[c + 1] <= m) c++;
  return c;
}

// The sequences' entropy stage (per wave, LDS): symbol counts, a normalized distribution, and the
// three compression tables built for the block.  Symbols of the three types side by side: LL codes
// at 0..35, OF at 36..67, ML at 68..120.
constexpr uint32_t kSymLL = 0, kSymOF = 36, kSymML = 68, kNSym = 121;
struct ZFse {
  uint32_t cnt[kNSym];
  uint32_t dnb[kNSym];
  int32_t dfs[kNSym];
  int16_t norm[kNSym + 1];
  uint32_t cumul[56];
  uint16_t state[512 + 256 + 512];  // LL (log <= 9), OF (<= 8), ML (<= 9)
  uint8_t sym[512];
};
constexpr uint32_t kZFseBytes = (sizeof(ZFse) + 15) & ~15u;
constexpr uint32_t kStOff[3] = {0, 512, 768};

// log2(x) * 256 for x >= 1, linear between powers of two (the mode choice's cost estimate)
__device__ inline uint32_t lg256(uint32_t x) {
  const uint32_t h = 31 - __builtin_clz(x);
  return 256 * h + (((x << 8) >> h) - 256);
}

// zstd's FSE_optimalTableLog for nseq sequences whose largest code is maxsym
__device__ inline uint32_t fse_table_log(uint32_t nseq, uint32_t maxsym, uint32_t maxlog) {
  const int hb_src = nseq > 1 ? 31 - __builtin_clz(nseq - 1) : 0;
  const uint32_t maxbits = hb_src >= 2 ? uint32_t(hb_src - 2) : 0u;
  const uint32_t minbits = min(uint32_t(31 - __builtin_clz(nseq)) + 1, (maxsym ? uint32_t(31 - __builtin_clz(maxsym)) : 0u) + 2);
  uint32_t L = maxlog;
  if (maxbits < L) L = maxbits;
  if (minbits > L) L = minbits;
  return max(5u, min(L, maxlog));
}

// counts -> a distribution over 2^L (every used symbol at least -1, the remainder on the most frequent);
// false if the remainder does not fit
__device__ bool fse_normalize(const uint32_t* cnt, uint32_t n, uint32_t tot, uint32_t L, int16_t* norm) {
  const uint32_t size = 1u << L;
  int32_t rest = int32_t(size);
  uint32_t big = 0;
  for (uint32_t s = 0; s < n; s++) {
    big = cnt[s] > cnt[big] ? s : big;
    int32_t v = 0;
    if (cnt[s]) {
      v = int32_t((uint64_t(cnt[s]) * size) / tot);
      v = v ? v : -1;
      rest -= v < 0 ? 1 : v;
    }
    norm[s] = int16_t(v);
  }
  const int32_t nb = int32_t(norm[big]) + rest;
  if (nb <= 0) return false;
  norm[big] = int16_t(nb);
  return true;
}

// FSE_writeNCount of norm[0..n) at accuracy L (dry: count the bits only); the bit count
__device__ uint32_t fse_ncount(Bits* b, BW* w, uint32_t lane, const int16_t* norm, uint32_t n, uint32_t L) {
  uint32_t bits = 4;
  if (b) b->add(*w, lane, L - 5, 4);
  int32_t rem = (1 << L) + 1, thr = 1 << L;
  uint32_t nbits = L + 1, s = 0;
  bool prev0 = false;
  while (s < n && rem > 1) {
    if (prev0) {
      uint32_t start = s;
      while (s < n && norm[s] == 0) s++;
      while (s >= start + 3) {
        start += 3;
        if (b) b->add(*w, lane, 3, 2);
        bits += 2;
      }
      if (b) b->add(*w, lane, s - start, 2);
      bits += 2;
    }
    int32_t c = norm[s++];
    const int32_t mx = 2 * thr - 1 - rem;
    rem -= c < 0 ? -c : c;
    c++;
    if (c >= thr) c += mx;
    const uint32_t k = nbits - (c < mx ? 1u : 0u);
    if (b) b->add(*w, lane, uint32_t(c), k);
    bits += k;
    prev0 = c == 1;
    while (rem < thr) {
      nbits--;
      thr >>= 1;
    }
  }
  return bits;
}

// FSE_buildCTable (the FseCT constructor at run time, on one lane): state[2^L], dnb / dfs per symbol
__device__ void fse_build_ct(const int16_t* norm, uint32_t n, uint32_t L, uint16_t* state, uint32_t* dnb, int32_t* dfs,
                             uint32_t* cumul, uint8_t* sym) {
  const uint32_t size = 1u << L, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  cumul[0] = 0;
  for (uint32_t u = 1; u <= n; u++) {
    if (norm[u - 1] == -1) {
      cumul[u] = cumul[u - 1] + 1;
      sym[high--] = uint8_t(u - 1);
    } else {
      cumul[u] = cumul[u - 1] + uint32_t(norm[u - 1]);
    }
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s < n; s++)
    for (int k = 0; k < norm[s]; k++) {
      sym[pos] = uint8_t(s);
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  for (uint32_t u = 0; u < size; u++) state[cumul[sym[u]]++] = uint16_t(size + u);
  uint32_t total = 0;
  for (uint32_t s = 0; s < n; s++) {
    const int c = norm[s];
    if (c == 0) {
      dnb[s] = ((L + 1) << 16) - size;
      dfs[s] = 0;
    } else if (c == -1 || c == 1) {
      dnb[s] = (L << 16) - size;
      dfs[s] = int32_t(total) - 1;
      total++;
    } else {
      const uint32_t hb = 31 - __builtin_clz(uint32_t(c - 1));
      const uint32_t max_bits = L - hb;
      dnb[s] = (max_bits << 16) - (uint32_t(c) << max_bits);
      dfs[s] = int32_t(total) - c;
      total += uint32_t(c);
    }
  }
}

// a compressed block body: raw literals section, then the sequences with repeat offsets (RFC 8878
// 3.1.2.5) and, per symbol type, the predefined, RLE or a block-built FSE table -- whichever the
// cost estimate prefers (Python model over configs[1] blocks: 1.097 -> 1.009 x libzstd level 3)
// first: the frame's first block.  A later block starts from the repeat offsets the previous
// block left (RFC 8878 3.1.2.5: they carry across a frame's blocks), which this piece, parsed on
// its own, does not know: its first three sequences use explicit offsets, after which the
// encoder's repeat offsets equal the decoder's whatever came before.
__device__ uint32_t zstd_body(const uint8_t* tags, uint32_t tn, const uint8_t* raw, uint32_t n, uint8_t* dst, uint32_t cap,
                              Seq* seqs, uint32_t seq_cap, ZFse* F, bool first, uint32_t lane, bool* over) {
  // pass 1: the sequences (literal run before each match) and the literal count
  uint32_t ns = 0, lit = 0, nlit = 0;
  bool too_many = false;
  {
    Parse P{Win{tags, tn}};
    uint32_t pos, len, off;
    while (P.next(lane, &pos, &len, &off)) {
      if (len < 3) continue;
      if (ns >= seq_cap) {
        too_many = true;
        break;
      }
      if (lane == 0) seqs[ns] = Seq{pos - lit, len, off};
      nlit += pos - lit;
      lit = pos + len;
      ns++;
    }
  }
  if (too_many) {  // cannot happen (a match is at least 4 bytes): the caller writes a raw block
    *over = true;
    return 0;
  }
  nlit += n - lit;
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  sync();
  auto rd = [&](uint32_t i) {
    const Seq q = seqs[i];
    return Seq{uint32_t(__builtin_amdgcn_readfirstlane(q.ll)), uint32_t(__builtin_amdgcn_readfirstlane(q.ml)),
               uint32_t(__builtin_amdgcn_readfirstlane(q.off))};
  };
  BW w{dst, 0, cap, false};
  // Literals_Section_Header, Raw_Literals_Block (RFC 8878 3.1.1.3.1.1)
  if (nlit < 32) {
    w.put(lane, nlit << 3);
  } else if (nlit < 4096) {
    w.put(lane, ((nlit & 0xf) << 4) | 0x4);
    w.put(lane, nlit >> 4);
  } else {
    w.put(lane, ((nlit & 0xf) << 4) | 0xc);
    w.put(lane, (nlit >> 4) & 0xff);
    w.put(lane, nlit >> 12);
  }
  {
    uint32_t a = 0;
    for (uint32_t i = 0; i <= ns; i++) {
      const Seq q = i < ns ? seqs[i] : Seq{n - a, 0, 0};
      const Seq qu{uint32_t(__builtin_amdgcn_readfirstlane(q.ll)), uint32_t(__builtin_amdgcn_readfirstlane(q.ml)),
                   uint32_t(__builtin_amdgcn_readfirstlane(q.off))};
      copy_bytes(dst, w.d, cap, raw, a, qu.ll, lane);
      w.over |= w.d + qu.ll > cap;
      w.d += qu.ll;
      a += qu.ll + qu.ml;
    }
  }
  // Sequences_Section_Header
  if (ns < 128) {
    w.put(lane, ns);
  } else if (ns < 0x7F00) {
    w.put(lane, (ns >> 8) + 128);
    w.put(lane, ns & 0xff);
  } else {
    w.put(lane, 255);
    w.put(lane, (ns - 0x7F00) & 0xff);
    w.put(lane, (ns - 0x7F00) >> 8);
  }
  if (ns) {
    // offsets as Offset_Values with the repeat offsets (the decoder's rules, zs_block): a repeat
    // when the offset equals one, else offset + 3; seqs[i].off becomes the value
    {
      uint32_t r0 = 1, r1 = 4, r2 = 8;
      for (uint32_t i = 0; i < ns; i++) {
        const Seq q = rd(i);
        const uint32_t o = q.off;
        uint32_t ov;
        if (!first && i < 3) ov = o + 3;
        else if (q.ll != 0) ov = o == r0 ? 1u : (o == r1 ? 2u : (o == r2 ? 3u : o + 3));
        else ov = o == r1 ? 1u : (o == r2 ? 2u : (o + 1 == r0 ? 3u : o + 3));
        if (ov > 3) {
          r2 = r1;
          r1 = r0;
          r0 = o;
        } else {
          const uint32_t idx = ov - 1 + (q.ll == 0 ? 1u : 0u);
          if (idx >= 2) r2 = r1;
          if (idx >= 1) {
            r1 = r0;
            r0 = o;
          }
        }
        if (lane == 0) seqs[i].off = ov;
      }
    }
    for (uint32_t s = lane; s < kNSym; s += 64) F->cnt[s] = 0;
    sync();
    for (uint32_t i = lane; i < ns; i += 64) {
      const Seq q = seqs[i];
      atomicAdd(&F->cnt[kSymLL + ll_code(q.ll)], 1u);
      atomicAdd(&F->cnt[kSymOF + (31 - __builtin_clz(q.off))], 1u);
      atomicAdd(&F->cnt[kSymML + ml_code(q.ml)], 1u);
    }
    sync();
    // per type (LL, OF, ML, in the modes byte's order): predefined, RLE or an FSE_Compressed table
    constexpr uint32_t kBase[3] = {kSymLL, kSymOF, kSymML}, kN[3] = {36, 32, 53}, kMaxLog[3] = {9, 8, 9},
                       kDefLog[3] = {6, 5, 6};
    uint32_t mode[3], L[3], nsym[3], rle[3];
    if (lane == 0) {
      for (int k = 0; k < 3; k++) {
        const uint32_t* c = F->cnt + kBase[k];
        const int16_t* def = k == 0 ? kLLDef : (k == 1 ? kOFDef : kMLDef);
        const uint32_t defs = k == 0 ? 36u : (k == 1 ? 29u : 53u);
        uint32_t used = 0, maxs = 0;
        for (uint32_t s = 0; s < kN[k]; s++)
          if (c[s]) {
            used++;
            maxs = s;
          }
        rle[k] = maxs;
        nsym[k] = maxs + 1;
        L[k] = kDefLog[k];
        mode[k] = 0;
        if (used == 1) {
          mode[k] = 1;
          continue;
        }
        // the predefined table's cost (x256 bits; a symbol it cannot code rules it out)
        uint64_t cp = 0;
        bool def_ok = maxs < defs;
        for (uint32_t s = 0; s < nsym[k] && def_ok; s++)
          if (c[s]) {
            const int d = def[s];
            if (d == 0) def_ok = false;
            cp += uint64_t(c[s]) * (256 * kDefLog[k] - lg256(uint32_t(d < 0 ? 1 : d)));
          }
        // a table built for this block
        const uint32_t Lb = fse_table_log(ns, maxs, kMaxLog[k]);
        int16_t* nrm = F->norm;
        if (fse_normalize(c, nsym[k], ns, Lb, nrm)) {
          uint64_t cc = 256ull * fse_ncount(nullptr, nullptr, lane, nrm, nsym[k], Lb);
          for (uint32_t s = 0; s < nsym[k]; s++)
            if (c[s]) cc += uint64_t(c[s]) * (256 * Lb - lg256(uint32_t(nrm[s] < 0 ? 1 : nrm[s])));
          if (!def_ok || cc < cp) {
            mode[k] = 2;
            L[k] = Lb;
            fse_build_ct(nrm, nsym[k], Lb, F->state + kStOff[k], F->dnb + kBase[k], F->dfs + kBase[k], F->cumul, F->sym);
          }
        }
        // (a distribution that does not normalize keeps the predefined table: every code used here
        // is below 29, which the predefined offsets cover)
      }
    }
    for (int k = 0; k < 3; k++) {
      mode[k] = uint32_t(__builtin_amdgcn_readfirstlane(mode[k]));
      L[k] = uint32_t(__builtin_amdgcn_readfirstlane(L[k]));
      nsym[k] = uint32_t(__builtin_amdgcn_readfirstlane(nsym[k]));
      rle[k] = uint32_t(__builtin_amdgcn_readfirstlane(rle[k]));
    }
    sync();
    w.put(lane, (mode[0] << 6) | (mode[1] << 4) | (mode[2] << 2));
    // the table descriptions: an FSE_Compressed table's counts (renormalized, as built), an RLE symbol
    for (int k = 0; k < 3; k++) {
      if (mode[k] == 1) {
        w.put(lane, rle[k]);
      } else if (mode[k] == 2) {
        const uint32_t* c = F->cnt + kBase[k];
        int16_t* nrm = F->norm;
        if (lane == 0) (void)fse_normalize(c, nsym[k], ns, L[k], nrm);
        sync();
        Bits hb;
        fse_ncount(&hb, &w, lane, nrm, nsym[k], L[k]);
        hb.pad(w, lane);
        sync();
      }
    }
    FseRT t[3];
    for (int k = 0; k < 3; k++) {
      if (mode[k] == 2) t[k] = FseRT{F->state + kStOff[k], F->dnb + kBase[k], F->dfs + kBase[k], L[k]};
      else if (k == 0) t[k] = fse_rt(kCtLL);
      else if (k == 1) t[k] = fse_rt(kCtOF);
      else t[k] = fse_rt(kCtML);
    }
    const bool act_ll = mode[0] != 1, act_of = mode[1] != 1, act_ml = mode[2] != 1;
    Bits b;
    FseStateR sll{0}, sml{0}, sof{0};
    // zstd's ZSTD_encodeSequences order: the last sequence first, states last (read first)
    {
      const Seq q = rd(ns - 1);
      const uint32_t lc = ll_code(q.ll), mc = ml_code(q.ml), ob = q.off, oc = 31 - __builtin_clz(ob);
      if (act_ml) sml.init(t[2], mc);
      if (act_of) sof.init(t[1], oc);
      if (act_ll) sll.init(t[0], lc);
      b.add(w, lane, q.ll - kLLBase[lc], kLLBits[lc]);
      b.add(w, lane, q.ml - kMLBase[mc], kMLBits[mc]);
      b.add(w, lane, ob, oc);
    }
    for (uint32_t i = ns - 1; i-- > 0;) {
      const Seq q = rd(i);
      const uint32_t lc = ll_code(q.ll), mc = ml_code(q.ml), ob = q.off, oc = 31 - __builtin_clz(ob);
      if (act_of) sof.enc(b, w, lane, t[1], oc);
      if (act_ml) sml.enc(b, w, lane, t[2], mc);
      if (act_ll) sll.enc(b, w, lane, t[0], lc);
      b.add(w, lane, q.ll - kLLBase[lc], kLLBits[lc]);
      b.add(w, lane, q.ml - kMLBase[mc], kMLBits[mc]);
      b.add(w, lane, ob, oc);
    }
    if (act_ml) sml.flush(b, w, lane, t[2]);
    if (act_of) sof.flush(b, w, lane, t[1]);
    if (act_ll) sll.flush(b, w, lane, t[0]);
    b.add(w, lane, 1, 1);  // end mark
    b.pad(w, lane);
  }
  *over = w.over;
  return w.d;
}

// ------------------------------------------------------------------ checksums of a raw payload
constexpr uint32_t kXP1 = 2654435761u, kXP2 = 2246822519u, kXP3 = 3266489917u, kXP4 = 668265263u, kXP5 = 374761393u;
__device__ inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ inline uint32_t ldu32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
__device__ inline uint64_t ldu64(const uint8_t* p) { return uint64_t(ldu32(p)) | uint64_t(ldu32(p + 4)) << 32; }

// XXH32 (seed 0): lanes 0..3 the four stripe accumulators; 64 stripes per round are loaded by the
// 64 lanes (one each) and handed to lanes 0..3 by shuffles, so the loads are not on the chain
__device__ uint32_t wxxh32(const uint8_t* p, uint32_t n, uint32_t lane) {
  uint32_t h;
  uint32_t i = 0;
  if (n >= 16) {
    uint32_t v = lane == 0 ? kXP1 + kXP2 : (lane == 1 ? kXP2 : (lane == 2 ? 0u : 0u - kXP1));
    const uint32_t stripes = n / 16;
    for (uint32_t s0 = 0; s0 < stripes; s0 += 64) {
      const uint32_t s = s0 + lane;
      uint32_t q[4] = {0, 0, 0, 0};
      if (s < stripes)
        for (int k = 0; k < 4; k++) q[k] = ldu32(p + 16 * s + 4 * k);
      const uint32_t m = min(64u, stripes - s0);
      for (uint32_t j = 0; j < m; j++) {
        uint32_t x = 0;
        for (int k = 0; k < 4; k++) {
          const uint32_t y = __shfl(q[k], int(j), 64);
          x = lane == uint32_t(k) ? y : x;
        }
        v = rotl32(v + x * kXP2, 13) * kXP1;
      }
    }
    const uint32_t v1 = __builtin_amdgcn_readlane(v, 0), v2 = __builtin_amdgcn_readlane(v, 1),
                   v3 = __builtin_amdgcn_readlane(v, 2), v4 = __builtin_amdgcn_readlane(v, 3);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    i = stripes * 16;
  } else {
    h = kXP5;
  }
  h += n;
  for (; i + 4 <= n; i += 4) h = rotl32(h + ldu32(p + i) * kXP3, 17) * kXP4;
  for (; i < n; i++) h = rotl32(h + uint32_t(p[i]) * kXP5, 11) * kXP1;
  h ^= h >> 15;
  h *= kXP2;
  h ^= h >> 13;
  h *= kXP3;
  h ^= h >> 16;
  return __builtin_amdgcn_readfirstlane(h);
}

constexpr uint64_t kX64P1 = 0x9E3779B185EBCA87ull, kX64P2 = 0xC2B2AE3D27D4EB4Full, kX64P3 = 0x165667B19E3779F9ull,
                   kX64P4 = 0x85EBCA77C2B2AE63ull, kX64P5 = 0x27D4EB2F165667C5ull;
__device__ inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ inline uint64_t x64round(uint64_t acc, uint64_t in) { return rotl64(acc + in * kX64P2, 31) * kX64P1; }
// XXH64 (seed 0): lanes 0..3 the four stripe accumulators, stripes loaded as in wxxh32
__device__ uint64_t wxxh64(const uint8_t* p, uint32_t n, uint32_t lane) {
  uint64_t h;
  uint32_t i = 0;
  if (n >= 32) {
    uint64_t v = lane == 0 ? kX64P1 + kX64P2 : (lane == 1 ? kX64P2 : (lane == 2 ? 0ull : 0ull - kX64P1));
    const uint32_t stripes = n / 32;
    for (uint32_t s0 = 0; s0 < stripes; s0 += 64) {
      const uint32_t s = s0 + lane;
      uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (s < stripes)
        for (int k = 0; k < 8; k++) q[k] = ldu32(p + 32 * s + 4 * k);
      const uint32_t m = min(64u, stripes - s0);
      for (uint32_t j = 0; j < m; j++) {
        uint32_t lo = 0, hi = 0;
        for (int k = 0; k < 4; k++) {
          const uint32_t a = __shfl(q[2 * k], int(j), 64), b = __shfl(q[2 * k + 1], int(j), 64);
          lo = lane == uint32_t(k) ? a : lo;
          hi = lane == uint32_t(k) ? b : hi;
        }
        v = x64round(v, uint64_t(lo) | (uint64_t(hi) << 32));
      }
    }
    uint64_t vv[4];
    for (int l = 0; l < 4; l++)
      vv[l] = uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v), l))) |
              (uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v >> 32), l))) << 32);
    h = rotl64(vv[0], 1) + rotl64(vv[1], 7) + rotl64(vv[2], 12) + rotl64(vv[3], 18);
    for (int l = 0; l < 4; l++) h = (h ^ x64round(0, vv[l])) * kX64P1 + kX64P4;
    i = stripes * 32;
  } else {
    h = kX64P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) h = rotl64(h ^ x64round(0, ldu64(p + i)), 27) * kX64P1 + kX64P4;
  if (i + 4 <= n) {
    h = rotl64(h ^ uint64_t(ldu32(p + i)) * kX64P1, 23) * kX64P2 + kX64P3;
    i += 4;
  }
  for (; i < n; i++) h = rotl64(h ^ uint64_t(p[i]) * kX64P5, 11) * kX64P1;
  h ^= h >> 33;
  h *= kX64P2;
  h ^= h >> 29;
  h *= kX64P3;
  h ^= h >> 32;
  return uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(h))) |
         (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(h >> 32))) << 32);
}

// Adler-32 (RFC 1950) of p[0, n): the sums over the lanes, 64-bit
__device__ uint32_t wadler(const uint8_t* p, uint32_t n, uint32_t lane) {
  uint64_t sa = 0, sb = 0;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint64_t x = p[i];
    sa += x;
    sb += uint64_t(n - i) * x;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sb += __shfl_xor(sb, o, 64);
  }
  const uint32_t a = uint32_t((1 + sa) % 65521u), b = uint32_t((uint64_t(n) + sb) % 65521u);
  return __builtin_amdgcn_readfirstlane((b << 16) | a);
}

}  // namespace

// ------------------------------------------------------------------ kernels
// pass 1: golang/snappy block encoding of each piece (tags only) into its tag slot
template <bool kBig>
__global__ __launch_bounds__(kBig ? 64 : 256) void pc_snappy_kernel(const uint8_t* __restrict__ raw,
                                                                     const CodecPiece* __restrict__ pieces,
                                                                     const uint32_t* __restrict__ list, uint32_t count,
                                                                     uint8_t* __restrict__ tags, uint32_t* __restrict__ tag_len) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr uint32_t cap = kBig ? kPieceMax : kSmallPiece;
  constexpr uint32_t ts = kBig ? kSnapMaxTable : kSmallPiece;
  constexpr uint32_t per_wave = ((cap + 16 + 3 * ts) + 15) & ~15u;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves_wg = blockDim.x >> 6;
  uint8_t* stage = smem + wave * per_wave;
  uint16_t* table = reinterpret_cast<uint16_t*>(stage + cap + 16);
  uint8_t* owner = reinterpret_cast<uint8_t*>(table + ts);
  for (uint32_t k = blockIdx.x * waves_wg + wave; k < count; k += gridDim.x * waves_wg) {
    const CodecPiece pc = pieces[list[k]];
    const uint8_t* p = raw + pc.raw;
    uint8_t* o = tags + pc.tags;
    snap_sync();
    for (uint32_t i = lane; i < pc.len; i += 64) stage[i] = p[i];
    if (lane < 16) stage[pc.len + lane] = 0;
    snap_sync();
    uint32_t d;
    if (pc.len < kSnapMinNonLiteral) d = pc.len ? snap_emit_literal(o, 0, stage, pc.len, int(lane)) : 0u;
    else d = snappy_encode_block_wave(stage, pc.len, o, table, owner, int(lane));
    if (lane == 0) tag_len[list[k]] = d;
  }
}

// per-wave LDS of pass 2 after the sequence lists: the entropy stage (Zstd, Zlib), and for Zlib's
// small pieces the staged piece and the chain parse's hash head and links
template <int kCodec, bool kBig>
constexpr uint32_t kTcWaveBytes =
    kCodec == SLATE_CODEC_ZSTD ? kZFseBytes
    : kCodec == SLATE_CODEC_ZLIB ? (kDFseBytes + (kBig ? 0u : kSmallPiece + 16 + 4u * (1u << kHashBits)))
                                 : 0u;

// pass 2: the tags of each piece transcoded into the codec's body (global slot); body_len
// gets the length, or kBodyRaw when the piece goes out in its raw / stored form
template <int kCodec, bool kBig>
__global__ __launch_bounds__(kBig ? 64 : 256) void pc_transcode_kernel(const uint8_t* __restrict__ raw,
                                                                        const CodecPiece* __restrict__ pieces,
                                                                        const uint32_t* __restrict__ list, uint32_t count,
                                                                        const uint8_t* __restrict__ tags,
                                                                        const uint32_t* __restrict__ tag_len,
                                                                        uint8_t* __restrict__ bodies,
                                                                        uint32_t* __restrict__ body_len,
                                                                        Seq* __restrict__ big_seqs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves_wg = blockDim.x >> 6;
  Seq* lds_seqs = reinterpret_cast<Seq*>(smem) + (kBig ? 0 : wave * kSmallSeqs);
  // the entropy stage's scratch per wave after the sequence lists (small pieces) or alone (big);
  // CodecZlib small pieces also stage the piece and the chain parse's hash head / links there
  uint8_t* wscr = smem + (kBig ? 0 : waves_wg * kSmallSeqs * sizeof(Seq)) + wave * kTcWaveBytes<kCodec, kBig>;
  ZFse* fse = reinterpret_cast<ZFse*>(wscr);
  for (uint32_t k = blockIdx.x * waves_wg + wave; k < count; k += gridDim.x * waves_wg) {
    const uint32_t id = list[k];
    const CodecPiece pc = pieces[id];
    const uint8_t* p = raw + pc.raw;
    const uint8_t* t = tags + pc.tags;
    const uint32_t tn = tag_len[id];
    uint8_t* o = bodies + pc.body;
    const uint32_t cap = codec_body_cap(pc.len);
    bool over = false;
    uint32_t d = 0;
    if (kCodec == SLATE_CODEC_LZ4) {
      d = lz4_body(t, tn, p, pc.len, o, cap, lane, &over);
      if (d >= pc.len) over = true;  // an uncompressed block is smaller
    } else if (kCodec == SLATE_CODEC_ZLIB) {
      DFse* F = reinterpret_cast<DFse*>(wscr);
      DSrc src{t, tn, nullptr, 0};
      const uint8_t* rp = p;
      if (!kBig && pc.len <= kSmallPiece) {
        // a block-sized piece: the hash-chain parse over the piece staged in LDS
        uint8_t* lraw = wscr + kDFseBytes;
        uint16_t* head = reinterpret_cast<uint16_t*>(lraw + kSmallPiece + 16);
        uint16_t* prev = head + (1u << kHashBits);
        for (uint32_t i = lane; i < pc.len; i += 64) lraw[i] = p[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nm = chain_parse(lraw, pc.len, head, prev, lds_seqs, kSmallSeqs, lane);
        if (nm != ~0u) {
          src.list = lds_seqs;
          src.nlist = nm;
        }
        rp = lraw;
      }
      d = deflate_body(src, rp, pc.len, (pc.flags & 2) != 0, o, cap, F, lane, &over);
    } else {
      Seq* seqs = kBig ? big_seqs + pc.seqs : lds_seqs;
      d = zstd_body(t, tn, p, pc.len, o, cap, seqs, kBig ? pc.len / 3 + 2 : kSmallSeqs, fse, (pc.flags & 1) != 0, lane,
                    &over);
      if (d >= pc.len) over = true;  // a raw block is smaller
    }
    if (lane == 0) body_len[id] = over ? kBodyRaw : d;
  }
}

// pass 3: one frame per payload at out_off[p]: header, pieces, trailer, and (with_crc) the BE32
// CRC32 of the frame
template <int kCodec>
__global__ __launch_bounds__(64) void pc_frame_kernel(const uint8_t* __restrict__ raw, const CodecPayload* __restrict__ pay,
                                                      uint32_t n, const CodecPiece* __restrict__ pieces,
                                                      const uint8_t* __restrict__ bodies,
                                                      const uint32_t* __restrict__ body_len,
                                                      const uint64_t* __restrict__ out_off, uint8_t* __restrict__ out,
                                                      uint32_t with_crc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
    const CodecPayload P = pay[q];
    uint8_t* o = out + out_off[q];
    const uint8_t* rp = raw + P.raw;
    BW w{o, 0, 0xFFFFFFFFu, false};
    // header
    if (kCodec == SLATE_CODEC_LZ4) {
      // magic, FLG (version 01, independent blocks, content checksum), BD (64 KiB blocks), HC
      const uint8_t hdr[6] = {0x04, 0x22, 0x4D, 0x18, 0x64, 0x40};
      for (int i = 0; i < 6; i++) w.put(lane, hdr[i]);
      w.put(lane, 0xA7);  // HC = (XXH32 of FLG, BD = 0x64 0x40) >> 8 & 0xff
    } else if (kCodec == SLATE_CODEC_ZLIB) {
      w.put(lane, 0x78);
      w.put(lane, 0x9C);
    } else {
      w.put(lane, 0x28);
      w.put(lane, 0xB5);
      w.put(lane, 0x2F);
      w.put(lane, 0xFD);
      // FHD: Single_Segment, Content_Checksum, FCS field 1 / 2 / 4 bytes
      const uint32_t L = P.len;
      const uint32_t fcs = L < 256 ? 0u : (L < 65536 + 256 ? 1u : 2u);
      w.put(lane, (fcs << 6) | 0x20 | 0x04);
      if (fcs == 0) {
        w.put(lane, L);
      } else if (fcs == 1) {
        w.put(lane, (L - 256) & 0xff);
        w.put(lane, (L - 256) >> 8);
      } else {
        for (int i = 0; i < 4; i++) w.put(lane, (L >> (8 * i)) & 0xff);
      }
    }
    // pieces
    for (uint32_t k = 0; k < P.npieces; k++) {
      const CodecPiece pc = pieces[P.first + k];
      const uint32_t bl = body_len[P.first + k];
      const bool rawform = bl == kBodyRaw;
      const uint32_t len = rawform ? pc.len : bl;
      if (kCodec == SLATE_CODEC_LZ4) {
        if (pc.len == 0) continue;  // a block of size 0 would read as the EndMark
        const uint32_t sz = rawform ? (pc.len | 0x80000000u) : bl;
        for (int i = 0; i < 4; i++) w.put(lane, (sz >> (8 * i)) & 0xff);
      } else if (kCodec == SLATE_CODEC_ZSTD) {
        const uint32_t last = (pc.flags & 2) ? 1u : 0u;
        const uint32_t bh = last | ((rawform ? 0u : 2u) << 1) | (len << 3);
        w.put(lane, bh & 0xff);
        w.put(lane, (bh >> 8) & 0xff);
        w.put(lane, bh >> 16);
      }
      // Zlib: a body is always written (stored blocks are one of its forms)
      const uint8_t* src = (rawform && kCodec != SLATE_CODEC_ZLIB) ? raw + pc.raw : bodies + pc.body;
      for (uint32_t i = lane; i < len; i += 64) o[w.d + i] = src[i];
      w.d += len;
    }
    // trailer
    if (kCodec == SLATE_CODEC_LZ4) {
      for (int i = 0; i < 4; i++) w.put(lane, 0);  // EndMark
      const uint32_t h = wxxh32(rp, P.len, lane);
      for (int i = 0; i < 4; i++) w.put(lane, (h >> (8 * i)) & 0xff);
    } else if (kCodec == SLATE_CODEC_ZLIB) {
      const uint32_t a = wadler(rp, P.len, lane);
      for (int i = 3; i >= 0; i--) w.put(lane, (a >> (8 * i)) & 0xff);
    } else {
      const uint32_t h = uint32_t(wxxh64(rp, P.len, lane));
      for (int i = 0; i < 4; i++) w.put(lane, (h >> (8 * i)) & 0xff);
    }
    if (with_crc) {
      __threadfence();  // the frame bytes this wave stored, read back by the CRC below
      // the CRC reads aligned dwords relative to its base: an aligned base, the frame at msg
      const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(o) & 3);
      const uint32_t crc = wave_crc32(tab, o - mis, int32_t(mis), w.d, int(lane));
      if (lane == 0) st_be32(o + w.d, crc);
    }
  }
}

size_t codec_piece_tags_bytes(uint32_t len) { return align16(snappy_max_encoded_len(len) + 16); }
size_t codec_piece_body_bytes(uint32_t len) { return align16(codec_body_cap(len) + 16); }

hipError_t launch_codec_encode(hipStream_t st, int codec, const uint8_t* raw, const CodecPiece* pieces,
                               const uint32_t* small_list, uint32_t n_small, const uint32_t* big_list, uint32_t n_big,
                               uint8_t* tags, uint32_t* tag_len, uint8_t* bodies, uint32_t* body_len, void* big_seqs,
                               int num_cus) {
  constexpr size_t lds_small = 4 * ((((kSmallPiece + 16 + 3 * kSmallPiece) + 15) & ~size_t(15)));
  constexpr size_t lds_big = ((kPieceMax + 16 + 3 * kSnapMaxTable) + 15) & ~size_t(15);
  static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&pc_snappy_kernel<true>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_big));
  if (a1 != hipSuccess) return a1;
  static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&pc_snappy_kernel<false>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_small));
  if (a2 != hipSuccess) return a2;
  if (n_small)
    pc_snappy_kernel<false><<<min((n_small + 3) / 4, uint32_t(num_cus) * 8), 256, lds_small, st>>>(
        raw, pieces, small_list, n_small, tags, tag_len);
  if (n_big) pc_snappy_kernel<true><<<min(n_big, uint32_t(num_cus)), 64, lds_big, st>>>(raw, pieces, big_list, n_big, tags, tag_len);
  Seq* bs = static_cast<Seq*>(big_seqs);
  // (+ the per-wave scratch of the entropy stage, kTcWaveBytes)
  const size_t lds_seq = 4 * kSmallSeqs * sizeof(Seq) + 4 * (codec == SLATE_CODEC_ZSTD   ? kTcWaveBytes<SLATE_CODEC_ZSTD, false>
                                                          : codec == SLATE_CODEC_ZLIB ? kTcWaveBytes<SLATE_CODEC_ZLIB, false>
                                                                                      : 0u);
  const size_t lds_big_tc = codec == SLATE_CODEC_ZSTD   ? kTcWaveBytes<SLATE_CODEC_ZSTD, true>
                            : codec == SLATE_CODEC_ZLIB ? kTcWaveBytes<SLATE_CODEC_ZLIB, true>
                                                        : 0u;
#define SLATE_PC_TRANSCODE(C)                                                                                       \
  do {                                                                                                            \
    if (n_small)                                                                                                  \
      pc_transcode_kernel<C, false><<<min((n_small + 3) / 4, uint32_t(num_cus) * 8), 256, lds_seq, st>>>(          \
          raw, pieces, small_list, n_small, tags, tag_len, bodies, body_len, bs);                                   \
    if (n_big)                                                                                                    \
      pc_transcode_kernel<C, true><<<min(n_big, uint32_t(num_cus) * 4), 64, lds_big_tc, st>>>(raw, pieces, big_list, n_big, \
                                                                                      tags, tag_len, bodies,       \
                                                                                      body_len, bs);              \
  } while (0)
  if (codec == SLATE_CODEC_LZ4) SLATE_PC_TRANSCODE(SLATE_CODEC_LZ4);
  else if (codec == SLATE_CODEC_ZLIB) {
    static const hipError_t a4 = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&pc_transcode_kernel<SLATE_CODEC_ZLIB, false>),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_seq));
    if (a4 != hipSuccess) return a4;
    SLATE_PC_TRANSCODE(SLATE_CODEC_ZLIB);
  }
  else if (codec == SLATE_CODEC_ZSTD) {
    static const hipError_t a3 = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&pc_transcode_kernel<SLATE_CODEC_ZSTD, false>),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_seq));
    if (a3 != hipSuccess) return a3;
    SLATE_PC_TRANSCODE(SLATE_CODEC_ZSTD);
  }
  else return hipErrorInvalidValue;
#undef SLATE_PC_TRANSCODE
  return hipGetLastError();
}

hipError_t launch_codec_frames(hipStream_t st, int codec, const uint8_t* raw, const CodecPayload* pay, uint32_t n,
                               const CodecPiece* pieces, const uint8_t* bodies, const uint32_t* body_len,
                               const uint64_t* out_off, uint8_t* out, bool with_crc, int num_cus) {
  if (n == 0) return hipGetLastError();
  const uint32_t grid = min(n, uint32_t(num_cus) * 16);
  if (codec == SLATE_CODEC_LZ4)
    pc_frame_kernel<SLATE_CODEC_LZ4><<<grid, 64, kTabBytes, st>>>(raw, pay, n, pieces, bodies, body_len, out_off, out, with_crc);
  else if (codec == SLATE_CODEC_ZLIB)
    pc_frame_kernel<SLATE_CODEC_ZLIB><<<grid, 64, kTabBytes, st>>>(raw, pay, n, pieces, bodies, body_len, out_off, out, with_crc);
  else if (codec == SLATE_CODEC_ZSTD)
    pc_frame_kernel<SLATE_CODEC_ZSTD><<<grid, 64, kTabBytes, st>>>(raw, pay, n, pieces, bodies, body_len, out_off, out, with_crc);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace slate
