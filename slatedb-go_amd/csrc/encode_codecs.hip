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

// ------------------------------------------------------------------ deflate (fixed Huffman)
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

// one piece as deflate blocks: fixed Huffman, or stored when that is not larger; a non-final
// piece ends with an empty stored block (byte alignment for the next piece)
__device__ uint32_t deflate_body(const uint8_t* tags, uint32_t tn, const uint8_t* raw, uint32_t n, bool final,
                                 uint8_t* dst, uint32_t cap, uint32_t lane, bool* over) {
  // size of the fixed-Huffman form, in bits
  uint64_t bits = 3 + 7;
  {
    Win r{raw, n};
    uint32_t lit = 0;
    auto lits = [&](uint32_t a, uint32_t e) {
      for (uint32_t p = a; p < e; p++) bits += fixed_bits(r.at(p, lane));
    };
    deflate_matches(tags, tn, lane, [&](uint32_t pos, uint32_t len, uint32_t off) {
      lits(lit, pos);
      const uint32_t lc = dcode_len(len), dc = dcode_dist(off);
      bits += fixed_bits(257 + lc) + kDLenExtra[lc] + 5 + kDDistExtra[dc];
      lit = pos + len;
    });
    lits(lit, n);
  }
  const uint64_t stored = 8ull * (n + 5 * ((n + 65534) / 65535 + (n == 0))) + 8;
  BW w{dst, 0, cap, false};
  Bits b;
  if (bits <= stored) {
    b.add(w, lane, final ? 1 : 0, 1);
    b.add(w, lane, 1, 2);  // BTYPE 01
    Win r{raw, n};
    uint32_t lit = 0;
    auto lits = [&](uint32_t a, uint32_t e) {
      for (uint32_t p = a; p < e; p++) fixed_sym(b, w, lane, r.at(p, lane));
    };
    deflate_matches(tags, tn, lane, [&](uint32_t pos, uint32_t len, uint32_t off) {
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

template <int N, int LOG>
struct FseState {
  uint32_t v;
  __device__ void init(const FseCT<N, LOG>& t, uint32_t s) {
    const uint32_t nb_out = (t.delta_nb[s] + (1u << 15)) >> 16;
    const uint32_t v0 = (nb_out << 16) - t.delta_nb[s];
    v = t.state[(v0 >> nb_out) + t.delta_find[s]];
  }
  __device__ void enc(Bits& b, BW& w, uint32_t lane, const FseCT<N, LOG>& t, uint32_t s) {
    const uint32_t nb_out = (v + t.delta_nb[s]) >> 16;
    b.add(w, lane, v, nb_out);
    v = t.state[(v >> nb_out) + t.delta_find[s]];
  }
  __device__ void flush(Bits& b, BW& w, uint32_t lane) { b.add(w, lane, v, LOG); }
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

struct Seq {
  uint32_t ll, ml, off;
};

// a compressed block body: raw literals section, then the sequences (predefined tables)
__device__ uint32_t zstd_body(const uint8_t* tags, uint32_t tn, const uint8_t* raw, uint32_t n, uint8_t* dst, uint32_t cap,
                              Seq* seqs, uint32_t seq_cap, uint32_t lane, bool* over) {
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
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
    w.put(lane, 0);  // Literals_Lengths_Mode, Offsets_Mode, Match_Lengths_Mode: predefined
    Bits b;
    FseState<36, 6> sll;
    FseState<53, 6> sml;
    FseState<29, 5> sof;
    auto rd = [&](uint32_t i) {
      const Seq q = seqs[i];
      return Seq{uint32_t(__builtin_amdgcn_readfirstlane(q.ll)), uint32_t(__builtin_amdgcn_readfirstlane(q.ml)),
                 uint32_t(__builtin_amdgcn_readfirstlane(q.off))};
    };
    // zstd's ZSTD_encodeSequences order: the last sequence first, states last (read first)
    {
      const Seq q = rd(ns - 1);
      const uint32_t lc = ll_code(q.ll), mc = ml_code(q.ml), ob = q.off + 3, oc = 31 - __builtin_clz(ob);
      sml.init(kCtML, mc);
      sof.init(kCtOF, oc);
      sll.init(kCtLL, lc);
      b.add(w, lane, q.ll - kLLBase[lc], kLLBits[lc]);
      b.add(w, lane, q.ml - kMLBase[mc], kMLBits[mc]);
      b.add(w, lane, ob, oc);
    }
    for (uint32_t i = ns - 1; i-- > 0;) {
      const Seq q = rd(i);
      const uint32_t lc = ll_code(q.ll), mc = ml_code(q.ml), ob = q.off + 3, oc = 31 - __builtin_clz(ob);
      sof.enc(b, w, lane, kCtOF, oc);
      sml.enc(b, w, lane, kCtML, mc);
      sll.enc(b, w, lane, kCtLL, lc);
      b.add(w, lane, q.ll - kLLBase[lc], kLLBits[lc]);
      b.add(w, lane, q.ml - kMLBase[mc], kMLBits[mc]);
      b.add(w, lane, ob, oc);
    }
    sml.flush(b, w, lane);
    sof.flush(b, w, lane);
    sll.flush(b, w, lane);
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
  Seq* lds_seqs = reinterpret_cast<Seq*>(smem) + wave * kSmallSeqs;
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
      d = deflate_body(t, tn, p, pc.len, (pc.flags & 2) != 0, o, cap, lane, &over);
    } else {
      Seq* seqs = kBig ? big_seqs + pc.seqs : lds_seqs;
      d = zstd_body(t, tn, p, pc.len, o, cap, seqs, kBig ? pc.len / 3 + 2 : kSmallSeqs, lane, &over);
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
  const size_t lds_seq = 4 * kSmallSeqs * sizeof(Seq);
#define SLATE_PC_TRANSCODE(C)                                                                                       \
  do {                                                                                                            \
    if (n_small)                                                                                                  \
      pc_transcode_kernel<C, false><<<min((n_small + 3) / 4, uint32_t(num_cus) * 8), 256, lds_seq, st>>>(          \
          raw, pieces, small_list, n_small, tags, tag_len, bodies, body_len, bs);                                   \
    if (n_big)                                                                                                    \
      pc_transcode_kernel<C, true><<<min(n_big, uint32_t(num_cus) * 4), 64, 0, st>>>(raw, pieces, big_list, n_big, \
                                                                                      tags, tag_len, bodies,       \
                                                                                      body_len, bs);              \
  } while (0)
  if (codec == SLATE_CODEC_LZ4) SLATE_PC_TRANSCODE(SLATE_CODEC_LZ4);
  else if (codec == SLATE_CODEC_ZLIB) SLATE_PC_TRANSCODE(SLATE_CODEC_ZLIB);
  else if (codec == SLATE_CODEC_ZSTD) SLATE_PC_TRANSCODE(SLATE_CODEC_ZSTD);
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
