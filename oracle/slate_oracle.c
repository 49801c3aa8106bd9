/*
 * slate_oracle.c — TEST INFRASTRUCTURE ONLY (see slate_oracle.h).
 *
 * Plain-C restatement of the slatedb-go SST block codec.  Every function cites
 * the reference file:line it follows (paths relative to /root/reference).
 * Never linked into the product library.
 */
#include "slate_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ statuses */
const char* or_status_string(int s) {
  switch (s) {
    case OR_OK: return "ok";
    case OR_E_BLOCK_TOO_SMALL: return "corrupted block: block is too small; must be at least 6 bytes";
    case OR_E_BLOCK_CHECKSUM: return "corrupted block: checksum mismatch";
    case OR_E_BLOCK_UNCOMP_SMALL: return "corrupted block: uncompressed block is too small; must be at least 2 bytes";
    case OR_E_BLOCK_INDEX_OFFSET: return "corrupted block: invalid index offset '%d'; cannot be negative";
    case OR_E_BLOCK_OFFSET_BOUNDS: return "corrupted block: block offset[%d] = %d exceeds key value bounds";
    case OR_E_BLOCK_NO_OFFSETS: return "corrupted block: Block.Offsets must be greater than 0";
    case OR_E_BLOCK_FIRSTKEY_PANIC: return "runtime error: slice bounds out of range (Block.FirstKey)";
    case OR_E_BLOCK_EMPTY: return "assertion failed; block cannot be empty";
    case OR_E_INVALID_CODEC: return "corrupted; invalid compression codec";
    case OR_E_SNAPPY_CORRUPT: return "snappy: corrupt input";
    case OR_E_SNAPPY_TOO_LARGE: return "snappy: decoded block is too large";
    case OR_E_CODEC_UNSUPPORTED: return "compression codec not supported by this backend";
    case OR_E_LZ4_MAGIC: return "lz4: bad magic number";
    case OR_E_LZ4_HEADER_CHECKSUM: return "lz4: invalid header checksum";
    case OR_E_LZ4_BLOCK_CHECKSUM: return "lz4: invalid block checksum";
    case OR_E_LZ4_FRAME_CHECKSUM: return "lz4: invalid frame checksum";
    case OR_E_LZ4_CORRUPT: return "lz4: invalid source or destination buffer too short";
    case OR_E_ZLIB_HEADER: return "zlib: invalid header";
    case OR_E_ZLIB_DICTIONARY: return "zlib: invalid dictionary";
    case OR_E_ZLIB_CHECKSUM: return "zlib: invalid checksum";
    case OR_E_FLATE_CORRUPT: return "flate: corrupt input before offset %d";
    case OR_E_UNEXPECTED_EOF: return "unexpected EOF";
    case OR_E_EOF: return "EOF";
    case OR_E_ZSTD_MAGIC: return "invalid input: magic number mismatch";
    case OR_E_ZSTD_CHECKSUM: return "CRC check failed";
    case OR_E_ZSTD_CORRUPT: return "zstd: corrupt input";
    case OR_E_ZSTD_FRAME_SIZE: return "frame size does not match size on stream";
    case OR_E_ZSTD_DICT: return "unknown dictionary";
    case OR_E_ZSTD_RESERVED_BLOCK: return "invalid input: reserved block type encountered";
    case OR_E_ROW_TOO_SHORT: return "corrupt v0 row: data length too short to decode a row";
    case OR_E_ROW_PREFIX: return "corrupt v0 row: key prefix length exceeds length of first key in block";
    case OR_E_ROW_SUFFIX: return "corrupt v0 row: key suffix length exceeds length of block";
    case OR_E_ROW_EXPIRE: return "corrupt v0 row: data length too short for expire";
    case OR_E_ROW_CREATE: return "corrupt v0 row: data length too short for create";
    case OR_E_ROW_VALUE_LEN: return "corrupt v0 row: data length too short for for value length";
    case OR_E_ROW_VALUE: return "corrupt v0 row: data length too short for for value";
    case OR_E_ROW_PANIC: return "runtime error: index out of range (v0 row seq/flags)";
    case OR_E_ROW_PEEK_SHORT: return "corrupt v0 row: data length too short to peek at row";
    case OR_E_SEEK_NO_OFFSETS: return "number of block.Offsets must be greater than zero";
    case OR_E_SEEK_NO_FULL_KEY: return "unable to locate uncorrupted first key in block; block is corrupt";
    case OR_E_SEEK_PANIC: return "runtime error: slice bounds out of range (block.NewIteratorAtKey)";
    case OR_E_ROW_OFFSET_RANGE: return "block.Offset[%d] = %d is out of bounds";
    case OR_E_FILTER_TOO_SMALL: return "corrupt filter: filter is too small; must be at least 2 bytes";
    case OR_E_FILTER_CHECKSUM: return "corrupt filter: invalid checksum";
    case OR_E_FILTER_PANIC: return "runtime error: slice bounds out of range (bloom.Decode)";
    case OR_E_INDEX_TOO_SHORT: return "corrupted index; too short";
    case OR_E_INDEX_CHECKSUM: return "corrupted index; checksum mismatch";
    case OR_E_INFO_TOO_SHORT: return "corrupted info; too short";
    case OR_E_INFO_CHECKSUM: return "corrupted info; checksum mismatch";
    case OR_E_SST_TOO_SHORT: return "corrupted SSTable; too short";
    case OR_E_BLOB_RANGE: return "corrupted; [%d:%d] is an invalid range";
    case OR_E_RANGE_START: return "block start '%d' range cannot be greater than end range '%d'";
    case OR_E_RANGE_END: return "block end '%d' range cannot be greater than size of block meta range '%d'";
    case OR_E_FLATBUF: return "runtime error: malformed flatbuffer";
    case OR_E_INVALID_ARG: return "invalid argument";
    case OR_E_CAPACITY: return "output buffer too small";
    case OR_E_OOM: return "out of memory";
    default: return "unknown status";
  }
}

/* ------------------------------------------------------------ byte helpers */
static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline void put_be16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static inline void put_be64(uint8_t* p, uint64_t v) { put_be32(p, (uint32_t)(v >> 32)); put_be32(p + 4, (uint32_t)v); }
static inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t le64(const uint8_t* p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

/* -------------------------------------------------- CRC32-IEEE (hash/crc32) */
/* Reflected polynomial 0xEDB88320, init/xorout 0xFFFFFFFF (crc32.ChecksumIEEE). */
static uint32_t g_crc_tab[256];
static pthread_once_t g_crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    g_crc_tab[i] = c;
  }
}
uint32_t or_crc32(const uint8_t* p, size_t n) {
  pthread_once(&g_crc_once, crc_init);
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = g_crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return ~c;
}

/* ------------------------------------------------------ FNV-1 64 (hash/fnv) */
/* bloom.go:141-145 filterHash: fnv.New64 is FNV-1 (multiply, then xor). */
uint64_t or_fnv1_64(const uint8_t* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; i++) { h *= 0x100000001b3ull; h ^= p[i]; }
  return h;
}

/* row.go:292-318 computePrefixLen/computePrefixChunks(…,128): the chunked compare
 * yields the plain common-prefix length; the result is truncated to uint16. */
uint16_t or_compute_prefix_len(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
  size_t m = an < bn ? an : bn, off = 0;
  size_t chunks = m / 128;
  for (size_t i = 0; i < chunks; i++) {
    if (memcmp(a + i * 128, b + i * 128, 128) != 0) break;
    off += 128;
  }
  while (off < m && a[off] == b[off]) off++;
  return (uint16_t)off;
}

/* =================================================== golang/snappy v0.0.4 */
/* encode.go: MaxEncodedLen */
size_t or_snappy_max_encoded_len(size_t n) { return 32 + n + n / 6; }

static size_t put_uvarint(uint8_t* dst, uint64_t v) {
  size_t i = 0;
  while (v >= 0x80) { dst[i++] = (uint8_t)v | 0x80; v >>= 7; }
  dst[i++] = (uint8_t)v;
  return i;
}

/* encode_other.go emitLiteral */
static size_t sn_emit_literal(uint8_t* dst, const uint8_t* lit, size_t len) {
  size_t i;
  uint32_t n = (uint32_t)(len - 1);
  if (n < 60) { dst[0] = (uint8_t)(n << 2); i = 1; }
  else if (n < (1u << 8)) { dst[0] = 60 << 2; dst[1] = (uint8_t)n; i = 2; }
  else { dst[0] = 61 << 2; dst[1] = (uint8_t)n; dst[2] = (uint8_t)(n >> 8); i = 3; }
  memcpy(dst + i, lit, len);
  return i + len;
}

/* encode_other.go emitCopy */
static size_t sn_emit_copy(uint8_t* dst, int offset, int length) {
  size_t i = 0;
  while (length >= 68) {
    dst[i + 0] = 63 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
    i += 3; length -= 64;
  }
  if (length > 64) {
    dst[i + 0] = 59 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
    i += 3; length -= 60;
  }
  if (length >= 12 || offset >= 2048) {
    dst[i + 0] = (uint8_t)((length - 1) << 2 | 2); dst[i + 1] = (uint8_t)offset;
    dst[i + 2] = (uint8_t)(offset >> 8);
    return i + 3;
  }
  dst[i + 0] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | 1);
  dst[i + 1] = (uint8_t)offset;
  return i + 2;
}

static inline uint32_t sn_hash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

/* encode_other.go encodeBlock (inputMargin = 15, table 1<<8 .. 1<<14) */
static size_t sn_encode_block(uint8_t* dst, const uint8_t* src, size_t n) {
  enum { maxTableSize = 1 << 14, tableMask = maxTableSize - 1, inputMargin = 15 };
  uint32_t shift = 32 - 8;
  for (size_t ts = 1 << 8; ts < maxTableSize && ts < n; ts *= 2) shift--;
  static __thread uint16_t table[maxTableSize];
  memset(table, 0, sizeof(table));
  int sLimit = (int)n - inputMargin;
  int nextEmit = 0, s = 1;
  size_t d = 0;
  uint32_t nextHash = sn_hash(le32(src + s), shift);
  for (;;) {
    int skip = 32, nextS = s, candidate = 0;
    for (;;) {
      s = nextS;
      int bytesBetween = skip >> 5;
      nextS = s + bytesBetween;
      skip += bytesBetween;
      if (nextS > sLimit) goto emit_remainder;
      candidate = table[nextHash & tableMask];
      table[nextHash & tableMask] = (uint16_t)s;
      nextHash = sn_hash(le32(src + nextS), shift);
      if (le32(src + s) == le32(src + candidate)) break;
    }
    d += sn_emit_literal(dst + d, src + nextEmit, (size_t)(s - nextEmit));
    for (;;) {
      int base = s;
      s += 4;
      for (int i = candidate + 4; s < (int)n && src[i] == src[s]; i++, s++) {}
      d += sn_emit_copy(dst + d, base - candidate, s - base);
      nextEmit = s;
      if (s >= sLimit) goto emit_remainder;
      uint64_t x = le64(src + s - 1);
      uint32_t prevHash = sn_hash((uint32_t)(x >> 0), shift);
      table[prevHash & tableMask] = (uint16_t)(s - 1);
      uint32_t currHash = sn_hash((uint32_t)(x >> 8), shift);
      candidate = table[currHash & tableMask];
      table[currHash & tableMask] = (uint16_t)s;
      if ((uint32_t)(x >> 8) != le32(src + candidate)) {
        nextHash = sn_hash((uint32_t)(x >> 16), shift);
        s++;
        break;
      }
    }
  }
emit_remainder:
  if ((size_t)nextEmit < n) d += sn_emit_literal(dst + d, src + nextEmit, n - (size_t)nextEmit);
  return d;
}

/* encode.go Encode: varint length, then 64 KiB blocks; < 17 bytes => literal only */
size_t or_snappy_encode(const uint8_t* src, size_t n, uint8_t* dst) {
  enum { maxBlockSize = 65536, minNonLiteralBlockSize = 1 + 1 + 15 };
  size_t d = put_uvarint(dst, (uint64_t)n);
  while (n > 0) {
    size_t pn = n > maxBlockSize ? maxBlockSize : n;
    if (pn < minNonLiteralBlockSize) d += sn_emit_literal(dst + d, src, pn);
    else d += sn_encode_block(dst + d, src, pn);
    src += pn; n -= pn;
  }
  return d;
}

/* decode.go decodedLen: binary.Uvarint; n <= 0 || v > 0xffffffff => ErrCorrupt */
int or_snappy_decoded_len(const uint8_t* src, size_t n, uint64_t* dlen, int* hdr) {
  uint64_t x = 0;
  unsigned s = 0;
  for (size_t i = 0; i < n; i++) {
    if (i == 10) return OR_E_SNAPPY_CORRUPT; /* overflow */
    uint8_t b = src[i];
    if (b < 0x80) {
      if (i == 9 && b > 1) return OR_E_SNAPPY_CORRUPT;
      x |= (uint64_t)b << s;
      if (x > 0xffffffffull) return OR_E_SNAPPY_CORRUPT;
      *dlen = x; *hdr = (int)i + 1;
      return OR_OK;
    }
    x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  return OR_E_SNAPPY_CORRUPT; /* n == 0: truncated */
}

/* decode_other.go decode (amd64 asm has the same accept/reject semantics) */
static int sn_decode(uint8_t* dst, size_t dn, const uint8_t* src, size_t sn) {
  size_t d = 0, s = 0;
  size_t offset = 0, length = 0;
  while (s < sn) {
    uint8_t tag = src[s] & 3;
    if (tag == 0) {
      uint32_t x = src[s] >> 2;
      if (x < 60) { s += 1; }
      else if (x == 60) { s += 2; if (s > sn) return 1; x = src[s - 1]; }
      else if (x == 61) { s += 3; if (s > sn) return 1; x = (uint32_t)src[s - 2] | (uint32_t)src[s - 1] << 8; }
      else if (x == 62) { s += 4; if (s > sn) return 1; x = (uint32_t)src[s - 3] | (uint32_t)src[s - 2] << 8 | (uint32_t)src[s - 1] << 16; }
      else { s += 5; if (s > sn) return 1; x = le32(src + s - 4); }
      length = (size_t)x + 1;
      if (length > dn - d || length > sn - s) return 1;
      memcpy(dst + d, src + s, length);
      d += length; s += length;
      continue;
    } else if (tag == 1) {
      s += 2; if (s > sn) return 1;
      length = 4 + ((src[s - 2] >> 2) & 7);
      offset = ((size_t)(src[s - 2] & 0xe0) << 3) | src[s - 1];
    } else if (tag == 2) {
      s += 3; if (s > sn) return 1;
      length = 1 + (src[s - 3] >> 2);
      offset = (size_t)src[s - 2] | (size_t)src[s - 1] << 8;
    } else {
      s += 5; if (s > sn) return 1;
      length = 1 + (src[s - 5] >> 2);
      offset = le32(src + s - 4);
    }
    if (offset == 0 || d < offset || length > dn - d) return 1;
    for (size_t i = 0; i < length; i++) dst[d + i] = dst[d - offset + i]; /* forward, overlap-safe */
    d += length;
  }
  return d != dn;
}

int or_snappy_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_len) {
  uint64_t dl; int hdr;
  int st = or_snappy_decoded_len(src, n, &dl, &hdr);
  if (st) return st;
  if (dl != dst_len) return OR_E_INVALID_ARG;
  return sn_decode(dst, (size_t)dl, src + hdr, n - (size_t)hdr) ? OR_E_SNAPPY_CORRUPT : OR_OK;
}

/* ============================================================ LZ4 frame decode
 * compress.Decode CodecLz4 = io.ReadAll(lz4.NewReader(buf)) (compression.go:143-144) with
 * github.com/pierrec/lz4/v4 v4.1.21 (go.mod:13), absent here: restated from the LZ4 frame
 * format (v1.6.x) and block format specifications, which that reader implements, plus
 * XXH32 (the frame's header / block / content checksums).  Parity is pinned by frames
 * from liblz4 1.9.3 (tests/golden/lz4_frames.json, tests/golden/make_lz4_fixtures.py);
 * pierrec's exact error strings and its handling of trailing data are unpinned: one frame
 * per buffer, anything after it is corrupt. */
static const uint32_t XP1 = 2654435761u, XP2 = 2246822519u, XP3 = 3266489917u, XP4 = 668265263u,
                      XP5 = 374761393u;
static uint32_t xrotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t or_xxh32(const uint8_t* p, size_t n, uint32_t seed) {
  size_t i = 0;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    for (; i + 16 <= n; i += 16) {
      v1 = xrotl(v1 + le32(p + i) * XP2, 13) * XP1;
      v2 = xrotl(v2 + le32(p + i + 4) * XP2, 13) * XP1;
      v3 = xrotl(v3 + le32(p + i + 8) * XP2, 13) * XP1;
      v4 = xrotl(v4 + le32(p + i + 12) * XP2, 13) * XP1;
    }
    h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
  } else {
    h = seed + XP5;
  }
  h += (uint32_t)n;
  for (; i + 4 <= n; i += 4) h = xrotl(h + le32(p + i) * XP3, 17) * XP4;
  for (; i < n; i++) h = xrotl(h + p[i] * XP5, 11) * XP1;
  h ^= h >> 15; h *= XP2; h ^= h >> 13; h *= XP3; h ^= h >> 16;
  return h;
}

/* One LZ4 block (sequences) into out[d0..): matches may reach back to out[lo].  `limit`
 * bounds the block's decoded size (the frame's max block size), `cap` the buffer.
 * out == NULL: sizes only. */
static int lz4_block(const uint8_t* src, size_t sn, uint8_t* out, size_t d0, size_t lo, size_t cap, size_t limit,
                     size_t* d_end) {
  size_t s = 0, d = d0;
  for (;;) {
    if (s >= sn) return OR_E_LZ4_CORRUPT;
    uint32_t token = src[s++];
    size_t ll = token >> 4;
    if (ll == 15) {
      uint32_t b;
      do {
        if (s >= sn) return OR_E_LZ4_CORRUPT;
        b = src[s++];
        ll += b;
      } while (b == 255);
    }
    if (ll > sn - s || ll > limit - (d - d0) || ll > cap - d) return OR_E_LZ4_CORRUPT;
    if (out) memcpy(out + d, src + s, ll);
    s += ll;
    d += ll;
    if (s == sn) break; /* the last sequence has literals only */
    if (sn - s < 2) return OR_E_LZ4_CORRUPT;
    size_t off = src[s] | (size_t)src[s + 1] << 8;
    s += 2;
    if (off == 0 || off > d - lo) return OR_E_LZ4_CORRUPT;
    size_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (s >= sn) return OR_E_LZ4_CORRUPT;
        b = src[s++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > limit - (d - d0) || ml > cap - d) return OR_E_LZ4_CORRUPT;
    if (out)
      for (size_t j = 0; j < ml; j++) out[d + j] = out[d - off + j]; /* overlapping copies repeat */
    d += ml;
  }
  *d_end = d;
  return OR_OK;
}

/* The frame, decoded in order.  out == NULL: structure only (no checksums), and *out_len is
 * the decoded size of the blocks before the first structural error (what a sequential
 * decoder writes before it can fail): the plan sizes buffers with it. */
static int lz4_frame(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  *out_len = 0;
  if (n < 4) return OR_E_LZ4_CORRUPT;
  if (le32(in) != 0x184D2204u) return OR_E_LZ4_MAGIC;
  if (n < 7) return OR_E_LZ4_CORRUPT;
  const uint32_t flg = in[4], bd = in[5];
  if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8F)) return OR_E_LZ4_CORRUPT;
  const uint32_t bsid = (bd >> 4) & 7;
  if (bsid < 4) return OR_E_LZ4_CORRUPT;
  const size_t bmax = (size_t)1 << (8 + 2 * bsid); /* 4: 64 KiB ... 7: 4 MiB */
  const int indep = (flg >> 5) & 1, bcheck = (flg >> 4) & 1, csize = (flg >> 3) & 1, ccheck = (flg >> 2) & 1,
            dict = flg & 1;
  const size_t hl = 2 + (csize ? 8 : 0) + (dict ? 4 : 0);
  if (n < 4 + hl + 1) return OR_E_LZ4_CORRUPT;
  if (out && in[4 + hl] != ((or_xxh32(in + 4, hl, 0) >> 8) & 0xFF)) return OR_E_LZ4_HEADER_CHECKSUM;
  if (dict) return OR_E_LZ4_CORRUPT; /* no dictionaries are configured */
  uint64_t content = 0;
  if (csize)
    for (int k = 7; k >= 0; k--) content = (content << 8) | in[6 + k];
  size_t pos = 4 + hl + 1, d = 0;
  for (;;) {
    if (n - pos < 4) return OR_E_LZ4_CORRUPT;
    const uint32_t bs = le32(in + pos);
    pos += 4;
    if (bs == 0) break;
    const size_t sz = bs & 0x7FFFFFFFu;
    if (sz > bmax || n - pos < sz + (bcheck ? 4 : 0)) return OR_E_LZ4_CORRUPT;
    if (out && bcheck && or_xxh32(in + pos, sz, 0) != le32(in + pos + sz)) return OR_E_LZ4_BLOCK_CHECKSUM;
    if (bs >> 31) {
      if (sz > cap - d) return OR_E_LZ4_CORRUPT;
      if (out) memcpy(out + d, in + pos, sz);
      d += sz;
    } else {
      size_t e;
      int st = lz4_block(in + pos, sz, out, d, indep ? d : 0, cap, bmax, &e);
      if (st) return st;
      d = e;
    }
    *out_len = d;
    pos += sz + (bcheck ? 4 : 0);
  }
  if (ccheck) {
    if (n - pos < 4) return OR_E_LZ4_CORRUPT;
    if (out && or_xxh32(out, d, 0) != le32(in + pos)) return OR_E_LZ4_FRAME_CHECKSUM;
    pos += 4;
  }
  if (csize && content != d) return OR_E_LZ4_CORRUPT;
  if (pos != n) return OR_E_LZ4_CORRUPT;
  return OR_OK;
}

int or_lz4_frame_len(const uint8_t* in, size_t n, uint64_t* dlen) {
  size_t l;
  int st = lz4_frame(in, n, NULL, (size_t)-1, &l);
  *dlen = l;
  return st;
}

int or_lz4_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  uint8_t dummy;
  return lz4_frame(in, n, out ? out : &dummy, out ? cap : 0, out_len);
}

/* ============================================================ Zlib (inflate)
 * compress.Decode CodecZlib = io.ReadAll(zlib.NewReader(buf)) (compression.go:134-140),
 * Go's compress/zlib + compress/flate, restated from RFC 1950 / RFC 1951 and the
 * behaviour of those readers: the 2-byte header check (CM 8, CINFO <= 7, FCHECK; FDICT
 * without a dictionary fails), blocks decoded in order, Huffman tables built as
 * flate's huffmanDecoder.init accepts them (complete codes, an empty tree, or one code
 * of length 1), then the big-endian Adler-32 of the output; bytes after it are not
 * read.  Running out of input is io.ErrUnexpectedEOF (io.EOF on an empty buffer).
 * Parity: decoded bytes pinned by zlib-written streams (tests/golden/zlib_streams.json);
 * error precedence on damaged streams follows the readers' structure but is unpinned
 * (no Go here), and flate's CorruptInputError offset is not reported. */
typedef struct { const uint8_t* in; size_t n, pos; uint32_t bits, nb; } zbits;
static int zneed(zbits* z, uint32_t k) { /* 0 ok, -1 out of input */
  while (z->nb < k) {
    if (z->pos >= z->n) return -1;
    z->bits |= (uint32_t)z->in[z->pos++] << z->nb;
    z->nb += 8;
  }
  return 0;
}
static uint32_t ztake(zbits* z, uint32_t k) {
  uint32_t v = z->bits & ((1u << k) - 1u);
  z->bits >>= k; z->nb -= k;
  return v;
}
typedef struct { uint16_t count[16], sym[288]; int max; } zhuff;
/* Canonical code from code lengths.  Returns 0 when flate's huffmanDecoder.init rejects
 * it: accepted are complete codes, the empty tree and one code of length 1. */
static int zhuff_build(zhuff* h, const uint8_t* len, int n) {
  memset(h->count, 0, sizeof h->count);
  int max = 0;
  for (int i = 0; i < n; i++) { h->count[len[i]]++; if (len[i] > max) max = len[i]; }
  h->count[0] = 0;
  h->max = max;
  int c = 0;
  for (int l = 1; l <= max; l++) { c <<= 1; c += h->count[l]; }
  uint16_t offs[17];
  offs[1] = 0;
  for (int l = 1; l < 16; l++) offs[l + 1] = (uint16_t)(offs[l] + h->count[l]);
  for (int i = 0; i < n; i++) if (len[i]) h->sym[offs[len[i]]++] = (uint16_t)i;
  if (max == 0) return 1;
  return c == (1 << max) || (c == 1 && max == 1);
}
/* One symbol, MSB-first code bits: -1 out of input, -2 no code matches (an empty tree, or
 * the unused half of a single-code tree) */
static int zdecode(zbits* z, const zhuff* h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l <= h->max; l++) {
    if (zneed(z, 1)) return -1;
    code |= (int)ztake(z, 1);
    const int cnt = h->count[l];
    if (code - first < cnt) return h->sym[index + (code - first)];
    index += cnt; first += cnt; first <<= 1; code <<= 1;
  }
  return -2;
}
static const uint16_t zlen_base[29] = {3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
static const uint8_t zlen_extra[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
static const uint16_t zdist_base[30] = {1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,
                                        4097,6145,8193,12289,16385,24577};
static const uint8_t zdist_extra[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};

/* out == NULL: sizes only (no Adler-32); *out_len = bytes the in-order decoder writes. */
static int zlib_stream(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  *out_len = 0;
  if (n == 0) return OR_E_EOF;
  if (n < 2) return OR_E_UNEXPECTED_EOF;
  const uint32_t h = ((uint32_t)in[0] << 8) | in[1];
  if ((in[0] & 0x0f) != 8 || (in[0] >> 4) > 7 || h % 31 != 0) return OR_E_ZLIB_HEADER;
  size_t start = 2;
  if (in[1] & 0x20) { /* FDICT: the dictionary id must be Adler-32 of the (empty) dictionary, 1 */
    if (n < 6) return OR_E_UNEXPECTED_EOF;
    if (be32(in + 2) != 1) return OR_E_ZLIB_DICTIONARY;
    start = 6;
  }
  zbits z = {in, n, start, 0, 0};
  size_t d = 0;
  zhuff fixed_l, fixed_d; /* RFC 1951 3.2.6 (built per call: the batch decoder is threaded) */
  {
    uint8_t l[288];
    for (int i = 0; i < 144; i++) l[i] = 8;
    for (int i = 144; i < 256; i++) l[i] = 9;
    for (int i = 256; i < 280; i++) l[i] = 7;
    for (int i = 280; i < 288; i++) l[i] = 8;
    zhuff_build(&fixed_l, l, 288);
    for (int i = 0; i < 30; i++) l[i] = 5;
    zhuff_build(&fixed_d, l, 30);
  }
  int final = 0;
  while (!final) {
    if (zneed(&z, 3)) return OR_E_UNEXPECTED_EOF;
    final = (int)ztake(&z, 1);
    const uint32_t type = ztake(&z, 2);
    if (type == 0) { /* stored */
      z.bits = 0; z.nb = 0; /* to a byte boundary */
      if (z.n - z.pos < 4) return OR_E_UNEXPECTED_EOF;
      const uint32_t len = z.in[z.pos] | (uint32_t)z.in[z.pos + 1] << 8;
      const uint32_t nlen = z.in[z.pos + 2] | (uint32_t)z.in[z.pos + 3] << 8;
      z.pos += 4;
      if (len != (~nlen & 0xffff)) return OR_E_FLATE_CORRUPT;
      if (len > cap - d) return OR_E_FLATE_CORRUPT;
      size_t avail = z.n - z.pos < len ? z.n - z.pos : len;
      if (out) memcpy(out + d, z.in + z.pos, avail);
      d += avail; z.pos += avail; *out_len = d;
      if (avail < len) return OR_E_UNEXPECTED_EOF;
      continue;
    }
    if (type == 3) return OR_E_FLATE_CORRUPT;
    zhuff dl, dd;
    const zhuff *hl = &fixed_l, *hd = &fixed_d;
    if (type == 2) {
      if (zneed(&z, 14)) return OR_E_UNEXPECTED_EOF;
      const uint32_t nlit = ztake(&z, 5) + 257, ndist = ztake(&z, 5) + 1, nclen = ztake(&z, 4) + 4;
      if (nlit > 286 || ndist > 30) return OR_E_FLATE_CORRUPT;
      static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      uint8_t cl[19] = {0};
      for (uint32_t i = 0; i < nclen; i++) {
        if (zneed(&z, 3)) return OR_E_UNEXPECTED_EOF;
        cl[order[i]] = (uint8_t)ztake(&z, 3);
      }
      zhuff hc;
      if (!zhuff_build(&hc, cl, 19)) return OR_E_FLATE_CORRUPT;
      uint8_t lens[316];
      uint32_t i = 0;
      while (i < nlit + ndist) {
        int sym = zdecode(&z, &hc);
        if (sym == -1) return OR_E_UNEXPECTED_EOF;
        if (sym < 0) return OR_E_FLATE_CORRUPT;
        if (sym < 16) { lens[i++] = (uint8_t)sym; continue; }
        uint32_t rep, val = 0;
        if (sym == 16) {
          if (i == 0) return OR_E_FLATE_CORRUPT;
          val = lens[i - 1];
          if (zneed(&z, 2)) return OR_E_UNEXPECTED_EOF;
          rep = 3 + ztake(&z, 2);
        } else if (sym == 17) {
          if (zneed(&z, 3)) return OR_E_UNEXPECTED_EOF;
          rep = 3 + ztake(&z, 3);
        } else {
          if (zneed(&z, 7)) return OR_E_UNEXPECTED_EOF;
          rep = 11 + ztake(&z, 7);
        }
        if (i + rep > nlit + ndist) return OR_E_FLATE_CORRUPT;
        while (rep--) lens[i++] = (uint8_t)val;
      }
      if (!zhuff_build(&dl, lens, (int)nlit) || !zhuff_build(&dd, lens + nlit, (int)ndist)) return OR_E_FLATE_CORRUPT;
      if (lens[256] == 0) return OR_E_FLATE_CORRUPT; /* every block ends with the end-of-block code */
      hl = &dl; hd = &dd;
    }
    for (;;) {
      int sym = zdecode(&z, hl);
      if (sym == -1) return OR_E_UNEXPECTED_EOF;
      if (sym < 0) return OR_E_FLATE_CORRUPT;
      if (sym < 256) {
        if (d >= cap) return OR_E_FLATE_CORRUPT;
        if (out) out[d] = (uint8_t)sym;
        d++; *out_len = d;
        continue;
      }
      if (sym == 256) break;
      sym -= 257;
      if (sym >= 29) return OR_E_FLATE_CORRUPT;
      if (zneed(&z, zlen_extra[sym])) return OR_E_UNEXPECTED_EOF;
      const uint32_t len = zlen_base[sym] + ztake(&z, zlen_extra[sym]);
      int ds = zdecode(&z, hd);
      if (ds == -1) return OR_E_UNEXPECTED_EOF;
      if (ds < 0 || ds >= 30) return OR_E_FLATE_CORRUPT;
      if (zneed(&z, zdist_extra[ds])) return OR_E_UNEXPECTED_EOF;
      const uint32_t dist = zdist_base[ds] + ztake(&z, zdist_extra[ds]);
      if (dist > d || dist > 32768) return OR_E_FLATE_CORRUPT;
      if (len > cap - d) return OR_E_FLATE_CORRUPT;
      if (out) for (uint32_t j = 0; j < len; j++) out[d + j] = out[d - dist + j];
      d += len; *out_len = d;
    }
  }
  /* the Adler-32 trailer starts at the next byte boundary */
  if (z.n - z.pos < 4) return OR_E_UNEXPECTED_EOF;
  if (out) {
    uint32_t a = 1, b = 0;
    for (size_t i = 0; i < d; i++) { a = (a + out[i]) % 65521u; b = (b + a) % 65521u; }
    const uint32_t want = ((uint32_t)z.in[z.pos] << 24) | ((uint32_t)z.in[z.pos + 1] << 16) |
                          ((uint32_t)z.in[z.pos + 2] << 8) | z.in[z.pos + 3];
    if (((b << 16) | a) != want) return OR_E_ZLIB_CHECKSUM;
  }
  return OR_OK;
}

int or_zlib_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  uint8_t dummy;
  return zlib_stream(in, n, out ? out : &dummy, out ? cap : 0, out_len);
}

/* ================================================ compress (compression.go) */
int or_compress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  if (codec == OR_CODEC_NONE) {
    if (cap < n) return OR_E_CAPACITY;
    memcpy(out, in, n); *out_len = n; return OR_OK;
  }
  if (codec == OR_CODEC_SNAPPY) {
    if (cap < or_snappy_max_encoded_len(n)) return OR_E_CAPACITY;
    *out_len = or_snappy_encode(in, n, out); return OR_OK;
  }
  if (codec >= OR_CODEC_ZLIB && codec <= OR_CODEC_ZSTD) return OR_E_CODEC_UNSUPPORTED;
  return OR_E_INVALID_CODEC;
}

int or_decompress_len(int codec, const uint8_t* in, size_t n, uint64_t* dlen) {
  if (codec == OR_CODEC_NONE) { *dlen = n; return OR_OK; }
  if (codec == OR_CODEC_SNAPPY) { int hdr; return or_snappy_decoded_len(in, n, dlen, &hdr); }
  if (codec == OR_CODEC_LZ4) return or_lz4_frame_len(in, n, dlen);
  if (codec == OR_CODEC_ZLIB) { size_t l; int st = zlib_stream(in, n, NULL, (size_t)-1, &l); *dlen = l; return st; }
  if (codec == OR_CODEC_ZSTD) return or_zstd_plan(in, n, dlen);
  return OR_E_INVALID_CODEC;
}

int or_decompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  if (codec == OR_CODEC_LZ4) return or_lz4_decode(in, n, out, cap, out_len); /* sequential: first error wins */
  if (codec == OR_CODEC_ZLIB) return or_zlib_decode(in, n, out, cap, out_len);
  if (codec == OR_CODEC_ZSTD) return or_zstd_decode(in, n, out, cap, out_len);
  uint64_t dl;
  int st = or_decompress_len(codec, in, n, &dl);
  if (st) return st;
  /* Snappy output is at most 64/3 bytes per input byte (copy2 tag): a larger
   * header length can only end in decode's d != len(dst) => ErrCorrupt. */
  if (codec == OR_CODEC_SNAPPY && dl > 22ull * n) return OR_E_SNAPPY_CORRUPT;
  if (dl > cap) return OR_E_CAPACITY;
  if (codec == OR_CODEC_NONE) { memcpy(out, in, n); *out_len = n; return OR_OK; }
  st = or_snappy_decode(in, n, out, (size_t)dl);
  *out_len = (size_t)dl;
  return st;
}

/* ============================================================ v0 row codec */
/* row.go:95-107 v0Size */
size_t or_v0_size(const or_row_value* r) {
  size_t size = 2 + 2 + r->key_suffix_len + 8 + 1;
  if (r->has_expire) size += 8;
  if (r->has_create) size += 8;
  if (!r->tombstone) size += 4 + r->value_len;
  return size;
}

/* row.go:149-189 Encode (flags from row.go:81-93) */
size_t or_v0_encode(const or_row_value* r, uint8_t* out) {
  size_t o = 0;
  put_be16(out + o, r->key_prefix_len); o += 2;
  put_be16(out + o, (uint16_t)r->key_suffix_len); o += 2;
  memcpy(out + o, r->key_suffix, r->key_suffix_len); o += r->key_suffix_len;
  put_be64(out + o, r->seq); o += 8;
  out[o++] = (uint8_t)((r->tombstone ? 1 : 0) | (r->has_expire ? 2 : 0) | (r->has_create ? 4 : 0));
  if (r->has_expire) { put_be64(out + o, (uint64_t)r->expire_ms); o += 8; }
  if (r->has_create) { put_be64(out + o, (uint64_t)r->create_ms); o += 8; }
  if (!r->tombstone) {
    put_be32(out + o, (uint32_t)r->value_len); o += 4;
    memcpy(out + o, r->value, r->value_len); o += r->value_len;
  }
  return o;
}

/* row.go:191-261 Decode.  first_key_len < 0 <=> firstKey == nil (length 0). */
int or_v0_decode(const uint8_t* data, size_t n, long first_key_len, or_row_value* r) {
  memset(r, 0, sizeof(*r));
  if (n < 13) return OR_E_ROW_TOO_SHORT;
  size_t o = 0;
  r->key_prefix_len = be16(data); o += 2;
  uint16_t sl = be16(data + 2); o += 2;
  uint16_t fk = (uint16_t)(first_key_len < 0 ? 0 : first_key_len); /* uint16(len(firstKey)) */
  if (r->key_prefix_len > fk) return OR_E_ROW_PREFIX;
  if (n - o < sl) return OR_E_ROW_SUFFIX;
  r->key_suffix = data + o; r->key_suffix_len = sl; o += sl;
  if (n - o < 8) return OR_E_ROW_PANIC; /* binary.BigEndian.Uint64 bounds panic */
  r->seq = be64(data + o); o += 8;
  if (n - o < 1) return OR_E_ROW_PANIC; /* data[offset] index panic */
  uint8_t flags = data[o++];
  if (flags & 2) {
    if (n - o < 8) return OR_E_ROW_EXPIRE;
    r->has_expire = 1; r->expire_ms = (int64_t)be64(data + o); o += 8;
  }
  if (flags & 4) {
    if (n - o < 8) return OR_E_ROW_CREATE;
    r->has_create = 1; r->create_ms = (int64_t)be64(data + o); o += 8;
  }
  if ((flags & 1) == 0) {
    if (n - o < 4) return OR_E_ROW_VALUE_LEN;
    uint32_t vl = be32(data + o); o += 4;
    if (n - o < vl) return OR_E_ROW_VALUE;
    r->value = data + o; r->value_len = vl;
  } else {
    r->tombstone = 1;
  }
  return OR_OK;
}

/* row.go:265-288 PeekAtKey */
int or_v0_peek(const uint8_t* data, size_t n, long first_key_len, uint16_t* pl, uint16_t* sl) {
  if (n < 4) return OR_E_ROW_PEEK_SHORT;
  *pl = be16(data); *sl = be16(data + 2);
  uint16_t fk = (uint16_t)(first_key_len < 0 ? 0 : first_key_len);
  if (*pl > fk) return OR_E_ROW_PREFIX;
  if (n - 4 < *sl) return OR_E_ROW_SUFFIX;
  return OR_OK;
}

/* bytes.Compare */
static int bytes_compare(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
  size_t m = an < bn ? an : bn;
  int c = m ? memcmp(a, b, m) : 0;
  if (c) return c < 0 ? -1 : 1;
  return an < bn ? -1 : (an > bn ? 1 : 0);
}

/* block/iterator.go:31-82 NewIteratorAtKey with firstFullKey (:117-132) and sort.Search
 * (Go's binary search: i, j = 0, n; h = (i + j) / 2; !f(h) -> i = h + 1 else j = h).
 * Every warning types.ErrWarn.Add receives is recorded, in order, as (kind, err, a, b) in
 * warn[4 * k ..] for the first cap of them: kind 1 "while peeking at key at offset %d: %v" (:121),
 * 2 "unable to locate uncorrupted first key in block; block is corrupt" (:130),
 * 3 "block.Offset[%d] = %d is out of bounds" (:65), 4 "while peeking at block.Offset[%d]: %s" (:70). */
static void seek_warn(uint32_t* warn, uint32_t cap, uint32_t* n_warn, uint32_t kind, int err, uint32_t a, uint32_t b) {
  if (warn && *n_warn < cap) {
    uint32_t* w = warn + 4 * (size_t)*n_warn;
    w[0] = kind; w[1] = (uint32_t)err; w[2] = a; w[3] = b;
  }
  (*n_warn)++;
}

int or_block_seek_w(const uint8_t* data, uint32_t data_len, const uint16_t* offsets, uint32_t n, const uint8_t* key,
                    size_t key_len, uint32_t* start, int32_t* first_idx, uint32_t* first_len, uint32_t* n_warn,
                    uint32_t* warn, uint32_t cap) {
  *start = 0; *first_idx = -1; *first_len = 0; *n_warn = 0;
  if (n == 0) return OR_E_SEEK_NO_OFFSETS;                         /* :32-34 */
  /* firstFullKey: PeekAtKey(block.Data[offset:], nil); a full key has keyPrefixLen 0 */
  int32_t idx = -1;
  uint32_t fk_off = 0, fk_len = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (offsets[i] > data_len) return OR_E_SEEK_PANIC;              /* block.Data[offset:] */
    uint16_t pl, sl;
    int st = or_v0_peek(data + offsets[i], data_len - offsets[i], -1, &pl, &sl);
    if (st) { seek_warn(warn, cap, n_warn, 1, st, offsets[i], 0); continue; }  /* :120-123 */
    if (pl == 0) { idx = (int32_t)i; fk_off = offsets[i] + 4; fk_len = sl; break; }
  }
  if (idx < 0) { seek_warn(warn, cap, n_warn, 2, OR_OK, 0, 0); return OR_E_SEEK_NO_FULL_KEY; }  /* :130-131, :41-47 */
  *first_idx = idx;
  *first_len = fk_len;
  const uint8_t* fk = data + fk_off;
  if (bytes_compare(fk, fk_len, key, key_len) == 0) { *start = 0; return OR_OK; }  /* :51-58 */
  uint32_t lo = 0, hi = n - (uint32_t)idx;
  while (lo < hi) {
    uint32_t h = (lo + hi) >> 1;
    uint32_t o = offsets[h + (uint32_t)idx];
    int ok = 0;
    if (o > (uint16_t)data_len) {                                   /* :65-68 */
      seek_warn(warn, cap, n_warn, 3, OR_OK, h + (uint32_t)idx, o);
    } else {
      uint16_t pl, sl;
      int st = or_v0_peek(data + o, data_len - o, (long)fk_len, &pl, &sl);
      if (st) {
        seek_warn(warn, cap, n_warn, 4, st, h + (uint32_t)idx, 0);  /* :70-73 */
      } else {
        /* v0FullKey(p, firstKey) = firstKey[:prefixLen] || suffix (row.go:72-79) */
        size_t kl = (size_t)pl + sl;
        size_t m = kl < key_len ? kl : key_len;
        int c = 0;
        for (size_t b = 0; b < m && !c; b++) {
          uint8_t x = b < pl ? fk[b] : data[o + 4 + (b - pl)];
          if (x != key[b]) c = x < key[b] ? -1 : 1;
        }
        if (!c) c = kl < key_len ? -1 : (kl > key_len ? 1 : 0);
        ok = c >= 0;
      }
    }
    if (!ok) lo = h + 1; else hi = h;
  }
  *start = lo + (uint32_t)idx;
  return OR_OK;
}

int or_block_seek(const uint8_t* data, uint32_t data_len, const uint16_t* offsets, uint32_t n, const uint8_t* key,
                  size_t key_len, uint32_t* start, int32_t* first_idx, uint32_t* first_len, uint32_t* n_warn) {
  return or_block_seek_w(data, data_len, offsets, n, key, key_len, start, first_idx, first_len, n_warn, NULL, 0);
}

/* sstable/iterator.go:123-153 firstBlockIncludingOrAfterKey */
uint64_t or_index_seek(const uint8_t* keys, const uint64_t* key_off, uint64_t n_blocks, const uint8_t* key,
                       size_t key_len) {
  int64_t low = 0, high = (int64_t)n_blocks - 1, found = 0;
  while (low <= high) {
    int64_t mid = low + (high - low) / 2;
    int c = bytes_compare(keys + key_off[mid], key_off[mid + 1] - key_off[mid], key, key_len);
    if (c < 0) { low = mid + 1; found = mid; }
    else if (c > 0) { if (mid > 0) high = mid - 1; else break; }
    else return (uint64_t)mid;
  }
  return (uint64_t)found;
}

/* row.go:50-65 V0EstimateBlockSize: 2 + Σ(v0Size(suffix=key) + 2) + 4 */
uint64_t or_v0_estimate_block_size(const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals,
                                   const uint64_t* val_off, size_t n) {
  (void)keys; (void)vals;
  uint64_t result = 2;
  for (size_t i = 0; i < n; i++) {
    or_row_value r; memset(&r, 0, sizeof(r));
    r.key_suffix_len = key_off[i + 1] - key_off[i];
    r.value_len = val_off[i + 1] - val_off[i];
    r.tombstone = 0; /* Value{Value: kv.Value} has Kind KeyValue */
    result += or_v0_size(&r) + 2;
  }
  return result + 4;
}

/* ======================================================== block.Builder */
struct or_block_builder {
  uint64_t block_size;
  uint8_t* data; size_t data_len, data_cap;
  uint16_t* offsets; size_t n, off_cap;
  uint8_t* first_key; size_t first_key_len; int has_first_key;
};

or_block_builder* or_block_builder_new(uint64_t block_size) {
  or_block_builder* b = (or_block_builder*)calloc(1, sizeof(*b));
  b->block_size = block_size;
  return b;
}
void or_block_builder_free(or_block_builder* b) {
  if (!b) return;
  free(b->data); free(b->offsets); free(b->first_key); free(b);
}
void or_block_builder_reset(or_block_builder* b) {
  b->data_len = 0; b->n = 0; b->has_first_key = 0; b->first_key_len = 0;
}
int or_block_builder_is_empty(const or_block_builder* b) { return b->n == 0; }

/* block.go:156-160 curBlockSize */
static uint64_t bb_cur_size(const or_block_builder* b) { return 2 + b->n * 2 + b->data_len; }

/* block.go:162-182 Add */
int or_block_builder_add(or_block_builder* b, const uint8_t* key, size_t klen, int tombstone,
                         const uint8_t* value, size_t vlen) {
  or_row_value r; memset(&r, 0, sizeof(r));
  uint16_t p = or_compute_prefix_len(b->has_first_key ? b->first_key : NULL,
                                     b->has_first_key ? b->first_key_len : 0, key, klen);
  r.key_prefix_len = p;
  r.key_suffix = key + p; r.key_suffix_len = klen - p;
  r.tombstone = tombstone; r.value = value; r.value_len = tombstone ? 0 : vlen;
  size_t rs = or_v0_size(&r);
  if (bb_cur_size(b) + 2 + rs > b->block_size && b->n != 0) return 0;
  if (b->n == b->off_cap) {
    b->off_cap = b->off_cap ? b->off_cap * 2 : 64;
    b->offsets = (uint16_t*)realloc(b->offsets, b->off_cap * sizeof(uint16_t));
  }
  if (b->data_len + rs > b->data_cap) {
    size_t nc = b->data_cap ? b->data_cap * 2 : 4096;
    while (nc < b->data_len + rs) nc *= 2;
    b->data = (uint8_t*)realloc(b->data, nc); b->data_cap = nc;
  }
  b->offsets[b->n++] = (uint16_t)b->data_len;
  b->data_len += or_v0_encode(&r, b->data + b->data_len);
  if (!b->has_first_key) {
    b->first_key = (uint8_t*)realloc(b->first_key, klen ? klen : 1);
    memcpy(b->first_key, key, klen); b->first_key_len = klen; b->has_first_key = 1;
  }
  return 1;
}

/* block.go:184-189 AddValue: empty value => tombstone */
int or_block_builder_add_value(or_block_builder* b, const uint8_t* key, size_t klen,
                               const uint8_t* value, size_t vlen) {
  return or_block_builder_add(b, key, klen, vlen == 0, value, vlen);
}
size_t or_block_builder_data(const or_block_builder* b, const uint8_t** d) { *d = b->data; return b->data_len; }
size_t or_block_builder_offsets(const or_block_builder* b, const uint16_t** o) { *o = b->offsets; return b->n; }
size_t or_block_builder_first_key(const or_block_builder* b, const uint8_t** k) { *k = b->first_key; return b->first_key_len; }

/* ================================================== block.Encode / Decode */
size_t or_block_encode_bound(size_t data_len, size_t n) {
  return or_snappy_max_encoded_len(data_len + 2 * n + 2) + 4;
}

/* block.go:54-75 */
int or_block_encode(const uint8_t* data, size_t data_len, const uint16_t* offsets, size_t n, int codec,
                    uint8_t* out, size_t cap, size_t* out_len) {
  size_t blen = data_len + 2 * n + 2;
  uint8_t* buf = (uint8_t*)malloc(blen ? blen : 1);
  if (!buf) return OR_E_OOM;
  memcpy(buf, data, data_len);
  for (size_t i = 0; i < n; i++) put_be16(buf + data_len + 2 * i, offsets[i]);
  put_be16(buf + data_len + 2 * n, (uint16_t)n);
  size_t clen = 0;
  int st = or_compress(codec, buf, blen, out, cap >= 4 ? cap - 4 : 0, &clen);
  free(buf);
  if (st) return st;
  put_be32(out + clen, or_crc32(out, clen));
  *out_len = clen + 4;
  return OR_OK;
}

/* Row-descriptor capacity used by both this oracle and the GPU plan kernel: a
 * valid v0 row is >= 13 bytes plus its 2-byte offset. */
uint64_t or_row_capacity(uint64_t decoded_len) { return (decoded_len + 13) / 15; }

/* v0 row decode as block.Iterator.Next does it (block/iterator.go:84-107). */
static void row_descriptor(const uint8_t* data, uint32_t data_len, uint32_t off, long fk,
                           or_row* d, or_row_value* rv) {
  memset(d, 0, sizeof(*d));
  d->row_off = off;
  const uint8_t* p = data + off;
  size_t n = data_len - off;
  if (n >= 4) { d->key_prefix_len = be16(p); d->key_suffix_len = be16(p + 2); }
  int st = or_v0_decode(p, n, fk, rv);
  d->status = (int16_t)st;
  if (st == OR_OK) {
    d->flags = (uint8_t)((rv->tombstone ? 1 : 0) | (rv->has_expire ? 2 : 0) | (rv->has_create ? 4 : 0));
    d->value_len = (uint32_t)rv->value_len;
    d->meta_len = (uint8_t)(9 + (rv->has_expire ? 8 : 0) + (rv->has_create ? 8 : 0) + (rv->tombstone ? 0 : 4));
  }
}

/* block.go:78-134 Decode + the Iterator's per-row decode. */
int or_block_decode(const uint8_t* in, size_t n, int codec, uint8_t* out, size_t cap, size_t* out_len,
                    or_block_meta* meta, or_row* rows, size_t rows_cap) {
  memset(meta, 0, sizeof(*meta));
  *out_len = 0;
#define FAIL(code) do { meta->status = (int16_t)(code); return (code); } while (0)
  if (n < 6) FAIL(OR_E_BLOCK_TOO_SMALL);
  size_t ci = n - 4;
  if (be32(in + ci) != or_crc32(in, ci)) FAIL(OR_E_BLOCK_CHECKSUM);
  size_t blen = 0;
  int st = or_decompress(codec, in, ci, out, cap, &blen);
  if (st) FAIL(st);
  *out_len = blen;
  const uint8_t* buf = out;
  if (blen < 2) FAIL(OR_E_BLOCK_UNCOMP_SMALL);
  size_t oci = blen - 2;
  uint16_t cnt = be16(buf + oci);
  long osi = (long)oci - (long)cnt * 2;
  if (osi <= 0) { meta->detail = (int32_t)osi; FAIL(OR_E_BLOCK_INDEX_OFFSET); }
  for (uint32_t i = 0; i < cnt; i++) {
    uint16_t off = be16(buf + osi + 2 * i);
    if (off > (uint16_t)osi) { /* uint16(offsetStartIndex) truncation, block.go:116 */
      meta->aux = (uint16_t)i; meta->detail = off; FAIL(OR_E_BLOCK_OFFSET_BOUNDS);
    }
  }
  meta->data_len = (uint32_t)osi;
  meta->n_rows = cnt;
  if (cnt == 0) FAIL(OR_E_BLOCK_NO_OFFSETS);
  /* block.go:130-131 FirstKey quirk: keyLen := BE16(Data[off0:]);
   * FirstKey = Data[off0+2 : off0+2+keyLen] with uint16 arithmetic.  Go panics
   * when fewer than 2 bytes remain, when lo > hi, or hi > cap(Data); we take cap
   * as the decoded buffer length (exact for Snappy). */
  uint16_t off0 = be16(buf + osi);
  if ((size_t)osi - off0 < 2) FAIL(OR_E_BLOCK_FIRSTKEY_PANIC);
  uint16_t kl = be16(buf + off0);
  uint16_t lo = (uint16_t)(off0 + 2), hi = (uint16_t)(off0 + 2 + kl);
  if (lo > hi || hi > blen) FAIL(OR_E_BLOCK_FIRSTKEY_PANIC);
  meta->aux = kl;
  /* rows */
  size_t nr = cnt;
  if (nr > rows_cap) { nr = rows_cap; meta->flags |= 1; }
  long fk = -1;
  for (size_t i = 0; i < nr; i++) {
    or_row_value rv;
    row_descriptor(buf, (uint32_t)osi, be16(buf + osi + 2 * i), i == 0 ? -1 : fk, &rows[i], &rv);
    if (i == 0 && rows[0].status == OR_OK) fk = (long)rv.key_suffix_len;
  }
  return OR_OK;
#undef FAIL
}

typedef struct {
  int codec; const uint8_t* in; const uint64_t* in_off; uint32_t lo, hi;
  uint8_t* out; const uint64_t* out_off; or_block_meta* meta; or_row* rows; const uint64_t* row_base;
} dec_job;

static void* dec_worker(void* arg) {
  dec_job* j = (dec_job*)arg;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    size_t olen;
    uint64_t cap = j->out_off[i + 1] - j->out_off[i];
    or_block_decode(j->in + j->in_off[i], j->in_off[i + 1] - j->in_off[i], j->codec, j->out + j->out_off[i],
                    cap, &olen, &j->meta[i], j->rows + j->row_base[i], j->row_base[i + 1] - j->row_base[i]);
  }
  return NULL;
}

/* Same two-step layout as slate_block_decode_plan_device + slate_block_decode_device. */
int or_block_decode_batch(int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n, uint8_t* out,
                          uint64_t out_cap, uint64_t* out_off, or_block_meta* meta, or_row* rows,
                          uint64_t rows_cap, uint64_t* row_base, int nthreads) {
  uint64_t o = 0, r = 0;
  for (uint32_t i = 0; i < n; i++) {
    size_t len = in_off[i + 1] - in_off[i];
    uint64_t dl = 0;
    if (len >= 6 && or_decompress_len(codec, in + in_off[i], len - 4, &dl) != OR_OK && codec != OR_CODEC_LZ4 &&
        codec != OR_CODEC_ZLIB && codec != OR_CODEC_ZSTD)
      dl = 0;
    if (codec == OR_CODEC_SNAPPY && dl > 22ull * (len - 4)) dl = 0; /* provably corrupt (> 64/3 expansion) */
    out_off[i] = o; row_base[i] = r;
    o += (dl + 15) & ~15ull; r += or_row_capacity(dl); /* 16-byte aligned blocks, as the GPU plan */
  }
  out_off[n] = o; row_base[n] = r;
  if (o > out_cap || r > rows_cap) return OR_E_CAPACITY;
  if (!meta) return OR_OK; /* plan only (no outputs given: a batch of empty plans fits zero capacity) */
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  dec_job* jobs = (dec_job*)malloc(sizeof(dec_job) * nthreads);
  for (int t = 0; t < nthreads; t++) {
    dec_job jb = {codec, in, in_off, (uint32_t)((uint64_t)n * t / nthreads),
                  (uint32_t)((uint64_t)n * (t + 1) / nthreads), out, out_off, meta, rows, row_base};
    jobs[t] = jb;
    if (nthreads == 1) dec_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, dec_worker, &jobs[t]);
  }
  if (nthreads > 1) for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th); free(jobs);
  return OR_OK;
}

/* ================================================================= bloom */
/* bloom.go:174-178: uint16(float32(bitsPerKey) * 0.69) */
uint16_t or_bloom_optimal_num_probes(uint32_t bpk) {
  volatile float f = (float)bpk * 0.69f;
  return (uint16_t)f;
}
/* bloom.go:135-139: uint32 arithmetic */
uint64_t or_bloom_filter_bytes(uint32_t nk, uint32_t bpk) {
  uint32_t bits = nk * bpk;
  return (uint64_t)((uint32_t)(bits + 7) / 8);
}
/* bloom.go:147-160 enhanced double hashing */
void or_bloom_probes(uint64_t hash, uint16_t np, uint32_t fbits, uint32_t* probes) {
  uint64_t m = fbits;
  uint64_t h = ((hash << 32) >> 32) % m;
  uint64_t delta = (hash >> 32) % m;
  for (uint32_t i = 0; i < np; i++) {
    delta = (delta + i) % m;
    probes[i] = (uint32_t)h;
    h = (h + delta) % m;
  }
}

/* bloom.go:112-133 Build */
int or_bloom_build(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t bpk, uint8_t* bits,
                   size_t cap, size_t* bits_len, uint16_t* num_probes) {
  if (n == 0) { *bits_len = 0; *num_probes = 0; return OR_OK; }
  uint16_t np = or_bloom_optimal_num_probes(bpk);
  uint64_t nb = or_bloom_filter_bytes((uint32_t)n, bpk);
  if (nb > cap) return OR_E_CAPACITY;
  memset(bits, 0, nb);
  uint32_t fbits = (uint32_t)(nb * 8);
  if (fbits == 0) return OR_E_INVALID_ARG; /* Go: integer divide by zero panic in probesForKey */
  uint32_t* pr = (uint32_t*)malloc(sizeof(uint32_t) * (np ? np : 1));
  for (uint64_t i = 0; i < n; i++) {
    uint64_t h = or_fnv1_64(keys + key_off[i], key_off[i + 1] - key_off[i]);
    or_bloom_probes(h, np, fbits, pr);
    for (uint32_t k = 0; k < np; k++) bits[pr[k] / 8] |= (uint8_t)(1u << (pr[k] % 8));
  }
  free(pr);
  *bits_len = nb; *num_probes = np;
  return OR_OK;
}

/* bloom.go:19-31 HasKey */
int or_bloom_has_key(uint16_t np, const uint8_t* bits, size_t bl, const uint8_t* key, size_t kl) {
  if (bl == 0) return 0;
  uint32_t pr[64];
  uint32_t* p = np <= 64 ? pr : (uint32_t*)malloc(sizeof(uint32_t) * np);
  or_bloom_probes(or_fnv1_64(key, kl), np, (uint32_t)(bl * 8), p);
  int ok = 1;
  for (uint32_t k = 0; k < np; k++)
    if (!(bits[p[k] / 8] & (1u << (p[k] % 8)))) { ok = 0; break; }
  if (p != pr) free(p);
  return ok;
}

/* bloom.go:52-67 Encode */
int or_bloom_encode(uint16_t np, const uint8_t* bits, size_t bl, int codec, uint8_t* out, size_t cap,
                    size_t* out_len) {
  uint8_t* buf = (uint8_t*)malloc(bl + 2);
  put_be16(buf, np);
  memcpy(buf + 2, bits, bl);
  size_t cl = 0;
  int st = or_compress(codec, buf, bl + 2, out, cap >= 4 ? cap - 4 : 0, &cl);
  free(buf);
  if (st) return st;
  put_be32(out + cl, or_crc32(out, cl));
  *out_len = cl + 4;
  return OR_OK;
}

/* bloom.go:70-91 Decode */
int or_bloom_decode(const uint8_t* data, size_t n, int codec, uint16_t* np, uint8_t* bits, size_t cap,
                    size_t* bl) {
  if (n < 2) return OR_E_FILTER_TOO_SMALL;
  if (n < 4) return OR_E_FILTER_PANIC; /* data[:len-4] with a negative index */
  size_t ci = n - 4;
  if (be32(data + ci) != or_crc32(data, ci)) return OR_E_FILTER_CHECKSUM;
  uint64_t dl;
  int st = or_decompress_len(codec, data, ci, &dl);
  if (st) return st;
  uint8_t* buf = (uint8_t*)malloc(dl ? dl : 1);
  size_t ol;
  st = or_decompress(codec, data, ci, buf, dl, &ol);
  if (st) { free(buf); return st; }
  if (ol < 2) { free(buf); return OR_E_FILTER_PANIC; }
  if (ol - 2 > cap) { free(buf); return OR_E_CAPACITY; }
  *np = be16(buf);
  memcpy(bits, buf + 2, ol - 2);
  *bl = ol - 2;
  free(buf);
  return OR_OK;
}

/* ============================================ flatbuffers Go builder (v24.3.25) */
/* A faithful simulation of github.com/google/flatbuffers/go Builder: the buffer
 * grows at the front; every alignment decision depends only on Offset() =
 * len(Bytes) - head, so the finished bytes equal Go's. */
typedef struct fb_builder {
  uint8_t* bytes; size_t len; size_t head; /* data is bytes[head:len] */
  int minalign;
  uint32_t* vtable; size_t vt_n, vt_cap;
  uint32_t object_end;
  uint32_t* vtables; size_t vts_n, vts_cap;
  int nested;
} fb_builder;

static void fb_init(fb_builder* b) { memset(b, 0, sizeof(*b)); b->minalign = 1; }
static void fb_free(fb_builder* b) { free(b->bytes); free(b->vtable); free(b->vtables); }
static uint32_t fb_offset(const fb_builder* b) { return (uint32_t)(b->len - b->head); }
static void fb_grow(fb_builder* b) {
  size_t nl = b->len ? b->len * 2 : 1;
  uint8_t* nb = (uint8_t*)calloc(nl, 1);
  memcpy(nb + (nl - b->len), b->bytes, b->len);
  free(b->bytes);
  b->bytes = nb; b->head += nl - b->len; b->len = nl;
}
static void fb_place_byte(fb_builder* b, uint8_t x) { b->bytes[--b->head] = x; }
static void fb_pad(fb_builder* b, int n) { for (int i = 0; i < n; i++) fb_place_byte(b, 0); }
static void fb_prep(fb_builder* b, int size, int additional) {
  if (size > b->minalign) b->minalign = size;
  int align = (int)((~((b->len - b->head) + (size_t)additional)) + 1) & (size - 1);
  while ((long)b->head <= (long)(align + size + additional)) fb_grow(b);
  fb_pad(b, align);
}
static void fb_place_u16(fb_builder* b, uint16_t x) { b->head -= 2; b->bytes[b->head] = (uint8_t)x; b->bytes[b->head + 1] = (uint8_t)(x >> 8); }
static void fb_place_u32(fb_builder* b, uint32_t x) { b->head -= 4; for (int i = 0; i < 4; i++) b->bytes[b->head + i] = (uint8_t)(x >> (8 * i)); }
static void fb_place_u64(fb_builder* b, uint64_t x) { b->head -= 8; for (int i = 0; i < 8; i++) b->bytes[b->head + i] = (uint8_t)(x >> (8 * i)); }
static void fb_prepend_u64(fb_builder* b, uint64_t x) { fb_prep(b, 8, 0); fb_place_u64(b, x); }
static void fb_prepend_i8(fb_builder* b, int8_t x) { fb_prep(b, 1, 0); fb_place_byte(b, (uint8_t)x); }
static void fb_prepend_voff(fb_builder* b, uint16_t x) { fb_prep(b, 2, 0); fb_place_u16(b, x); }
static void fb_prepend_soff(fb_builder* b, int32_t off) {
  fb_prep(b, 4, 0);
  int32_t off2 = (int32_t)fb_offset(b) - off + 4;
  fb_place_u32(b, (uint32_t)off2);
}
static void fb_prepend_uoff(fb_builder* b, uint32_t off) {
  fb_prep(b, 4, 0);
  uint32_t off2 = fb_offset(b) - off + 4;
  fb_place_u32(b, off2);
}
static void fb_start_object(fb_builder* b, int numfields) {
  if ((size_t)numfields > b->vt_cap) { b->vt_cap = numfields; b->vtable = (uint32_t*)realloc(b->vtable, sizeof(uint32_t) * numfields); }
  b->vt_n = numfields;
  for (int i = 0; i < numfields; i++) b->vtable[i] = 0;
  b->object_end = fb_offset(b);
  b->nested = 1;
}
static void fb_slot(fb_builder* b, int slot) { b->vtable[slot] = fb_offset(b); }
static uint32_t fb_end_object(fb_builder* b) {
  fb_prepend_soff(b, 0);
  uint32_t object_offset = fb_offset(b);
  uint32_t existing = 0;
  long i = (long)b->vt_n - 1;
  while (i >= 0 && b->vtable[i] == 0) i--;
  b->vt_n = (size_t)(i + 1);
  for (long k = (long)b->vts_n - 1; k >= 0; k--) {
    uint32_t vt2off = b->vtables[k];
    size_t vt2start = b->len - vt2off;
    uint16_t vt2len = (uint16_t)(b->bytes[vt2start] | (b->bytes[vt2start + 1] << 8));
    const uint8_t* vt2 = b->bytes + vt2start + 4;
    size_t vt2n = (size_t)vt2len - 4;
    /* vtableEqual: compares field entries only; both-zero entries match */
    int eq = (b->vt_n * 2 == vt2n);
    for (size_t f = 0; eq && f < b->vt_n; f++) {
      uint16_t x = (uint16_t)(vt2[2 * f] | (vt2[2 * f + 1] << 8));
      if (x == 0 && b->vtable[f] == 0) continue;
      int32_t y = (int32_t)object_offset - (int32_t)b->vtable[f];
      if ((int32_t)x != y) eq = 0;
    }
    if (eq) { existing = vt2off; break; }
  }
  if (existing == 0) {
    for (long f = (long)b->vt_n - 1; f >= 0; f--) {
      uint32_t off = b->vtable[f] ? object_offset - b->vtable[f] : 0;
      fb_prepend_voff(b, (uint16_t)off);
    }
    fb_prepend_voff(b, (uint16_t)(object_offset - b->object_end));
    fb_prepend_voff(b, (uint16_t)((b->vt_n + 2) * 2));
    size_t object_start = b->len - object_offset;
    int32_t v = (int32_t)fb_offset(b) - (int32_t)object_offset;
    for (int q = 0; q < 4; q++) b->bytes[object_start + q] = (uint8_t)((uint32_t)v >> (8 * q));
    if (b->vts_n == b->vts_cap) { b->vts_cap = b->vts_cap ? b->vts_cap * 2 : 16; b->vtables = (uint32_t*)realloc(b->vtables, sizeof(uint32_t) * b->vts_cap); }
    b->vtables[b->vts_n++] = fb_offset(b);
  } else {
    size_t object_start = b->len - object_offset;
    b->head = object_start;
    int32_t v = (int32_t)existing - (int32_t)object_offset;
    for (int q = 0; q < 4; q++) b->bytes[b->head + q] = (uint8_t)((uint32_t)v >> (8 * q));
  }
  b->vt_n = 0;
  b->nested = 0;
  return object_offset;
}
static uint32_t fb_end_vector(fb_builder* b, uint32_t n) { fb_place_u32(b, n); b->nested = 0; return fb_offset(b); }
static uint32_t fb_start_vector(fb_builder* b, int elem, int n, int align) {
  b->nested = 1;
  fb_prep(b, 4, elem * n);
  fb_prep(b, align, elem * n);
  return fb_offset(b);
}
/* CreateByteString: NUL-terminated */
static uint32_t fb_create_byte_string(fb_builder* b, const uint8_t* s, size_t n) {
  b->nested = 1;
  fb_prep(b, 4, (int)(n + 1));
  fb_place_byte(b, 0);
  b->head -= n;
  memcpy(b->bytes + b->head, s, n);
  return fb_end_vector(b, (uint32_t)n);
}
/* CreateByteVector: no terminator */
static uint32_t fb_create_byte_vector(fb_builder* b, const uint8_t* s, size_t n) {
  b->nested = 1;
  fb_prep(b, 4, (int)n);
  b->head -= n;
  if (n) memcpy(b->bytes + b->head, s, n);
  return fb_end_vector(b, (uint32_t)n);
}
static void fb_finish(fb_builder* b, uint32_t root) {
  fb_prep(b, b->minalign, 4);
  fb_prepend_uoff(b, root);
}

/* flatbuf.go:62-81 EncodeInfo */
int or_encode_info(const or_sst_info* info, const uint8_t* fk, uint8_t* out, size_t cap, size_t* out_len) {
  fb_builder b; fb_init(&b);
  uint32_t fko = fb_create_byte_vector(&b, fk, fk ? info->first_key_len : 0);
  fb_start_object(&b, 6);
  if (fko != 0) { fb_prepend_uoff(&b, fko); fb_slot(&b, 0); }
  if (info->index_offset) { fb_prepend_u64(&b, info->index_offset); fb_slot(&b, 1); }
  if (info->index_len) { fb_prepend_u64(&b, info->index_len); fb_slot(&b, 2); }
  if (info->filter_offset) { fb_prepend_u64(&b, info->filter_offset); fb_slot(&b, 3); }
  if (info->filter_len) { fb_prepend_u64(&b, info->filter_len); fb_slot(&b, 4); }
  if ((int8_t)info->codec != 0) { fb_prepend_i8(&b, (int8_t)info->codec); fb_slot(&b, 5); }
  uint32_t io = fb_end_object(&b);
  fb_finish(&b, io);
  size_t n = b.len - b.head;
  if (n + 4 > cap) { fb_free(&b); return OR_E_CAPACITY; }
  memcpy(out, b.bytes + b.head, n);
  put_be32(out + n, or_crc32(out, n));
  *out_len = n + 4;
  fb_free(&b);
  return OR_OK;
}

/* flatbuffers Go Table accessors (table.go) */
static int fb_field(const uint8_t* buf, size_t n, uint32_t pos, uint16_t vo, uint32_t* out) {
  if ((size_t)pos + 4 > n) return -1;
  int32_t so = (int32_t)le32(buf + pos);
  long vt = (long)pos - so;
  if (vt < 0 || (size_t)vt + 2 > n) return -1;
  uint16_t vtlen = (uint16_t)(buf[vt] | buf[vt + 1] << 8);
  if (vo < vtlen) {
    if ((size_t)vt + vo + 2 > n) return -1;
    *out = (uint16_t)(buf[vt + vo] | buf[vt + vo + 1] << 8);
  } else *out = 0;
  return 0;
}
static int fb_u64(const uint8_t* buf, size_t n, uint32_t pos, uint16_t vo, uint64_t* v) {
  uint32_t o; if (fb_field(buf, n, pos, vo, &o)) return -1;
  if (!o) { *v = 0; return 0; }
  if ((size_t)pos + o + 8 > n) return -1;
  *v = le64(buf + pos + o); return 0;
}
static int fb_bytes(const uint8_t* buf, size_t n, uint32_t pos, uint16_t vo, const uint8_t** p, size_t* len, int* present) {
  uint32_t o; if (fb_field(buf, n, pos, vo, &o)) return -1;
  *present = o != 0;
  if (!o) { *p = NULL; *len = 0; return 0; }
  size_t at = (size_t)pos + o;
  if (at + 4 > n) return -1;
  at += le32(buf + at);
  if (at + 4 > n) return -1;
  size_t l = le32(buf + at);
  if (at + 4 + l > n) return -1;
  *p = buf + at + 4; *len = l; return 0;
}

/* flatbuf.go:102-124 DecodeInfo */
int or_decode_info(const uint8_t* b, size_t n, or_sst_info* info, uint8_t* fk, size_t fk_cap) {
  memset(info, 0, sizeof(*info));
  if (n <= 4) return OR_E_INFO_TOO_SHORT;
  size_t ci = n - 4;
  if (be32(b + ci) != or_crc32(b, ci)) return OR_E_INFO_CHECKSUM;
  if (n < 4) return OR_E_FLATBUF;
  uint32_t root = le32(b);
  const uint8_t* p; size_t l; int present;
  if (fb_bytes(b, n, root, 4, &p, &l, &present)) return OR_E_FLATBUF;
  if (fb_u64(b, n, root, 6, &info->index_offset) || fb_u64(b, n, root, 8, &info->index_len) ||
      fb_u64(b, n, root, 10, &info->filter_offset) || fb_u64(b, n, root, 12, &info->filter_len))
    return OR_E_FLATBUF;
  uint32_t o;
  if (fb_field(b, n, root, 14, &o)) return OR_E_FLATBUF;
  info->codec = o ? (int8_t)b[root + o] : 0;
  if (l > fk_cap) return OR_E_CAPACITY;
  if (l) memcpy(fk, p, l);
  info->first_key_len = (uint32_t)l;
  return OR_OK;
}

/* flatbuf.go:126-139 encodeIndex = SsTableIndexT.Pack (manifest_generated.go:586-606)
 * with BlockMetaT.Pack (manifest_generated.go:457-469), then compress + CRC. */
int or_encode_index(const uint64_t* offsets, const uint8_t* keys, const uint64_t* key_off, size_t n,
                    int codec, uint8_t* out, size_t cap, size_t* out_len) {
  fb_builder b; fb_init(&b);
  uint32_t* mo = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  for (size_t j = 0; j < n; j++) {
    uint32_t fko = fb_create_byte_string(&b, keys + key_off[j], key_off[j + 1] - key_off[j]);
    fb_start_object(&b, 2);
    if (offsets[j]) { fb_prepend_u64(&b, offsets[j]); fb_slot(&b, 0); }
    if (fko) { fb_prepend_uoff(&b, fko); fb_slot(&b, 1); }
    mo[j] = fb_end_object(&b);
  }
  fb_start_vector(&b, 4, (int)n, 4);
  for (long j = (long)n - 1; j >= 0; j--) fb_prepend_uoff(&b, mo[j]);
  uint32_t vec = fb_end_vector(&b, (uint32_t)n);
  free(mo);
  fb_start_object(&b, 1);
  if (vec) { fb_prepend_uoff(&b, vec); fb_slot(&b, 0); }
  uint32_t root = fb_end_object(&b);
  fb_finish(&b, root);
  size_t fl = b.len - b.head, cl = 0;
  int st = or_compress(codec, b.bytes + b.head, fl, out, cap >= 4 ? cap - 4 : 0, &cl);
  fb_free(&b);
  if (st) return st;
  put_be32(out + cl, or_crc32(out, cl));
  *out_len = cl + 4;
  return OR_OK;
}

/* flatbuf.go:83-100 DecodeIndex + Index.BlockMeta() (flatbuf.go:22-31) */
int or_decode_index(const uint8_t* buf, size_t len, int codec, uint64_t* offsets, uint8_t* keys,
                    uint64_t* key_off, size_t metas_cap, size_t keys_cap, size_t* n_out) {
  if (len <= 4) return OR_E_INDEX_TOO_SHORT;
  size_t ci = len - 4;
  if (be32(buf + ci) != or_crc32(buf, ci)) return OR_E_INDEX_CHECKSUM;
  uint64_t dl;
  int st = or_decompress_len(codec, buf, ci, &dl);
  if (st) return st;
  uint8_t* d = (uint8_t*)malloc(dl ? dl : 1);
  size_t ol;
  st = or_decompress(codec, buf, ci, d, dl, &ol);
  if (st) { free(d); return st; }
  st = OR_E_FLATBUF;
  if (ol < 4) goto out;
  uint32_t root = le32(d);
  uint32_t o;
  if (fb_field(d, ol, root, 4, &o) || !o) goto out;
  size_t vec = (size_t)root + o;
  if (vec + 4 > ol) goto out;
  vec += le32(d + vec);
  if (vec + 4 > ol) goto out;
  uint32_t nm = le32(d + vec);
  if (nm > metas_cap) { st = OR_E_CAPACITY; goto out; }
  size_t ko = 0;
  key_off[0] = 0;
  for (uint32_t j = 0; j < nm; j++) {
    size_t ep = vec + 4 + 4 * (size_t)j;
    if (ep + 4 > ol) goto out;
    uint32_t tp = (uint32_t)(ep + le32(d + ep));
    const uint8_t* kp; size_t kl; int present;
    if (fb_u64(d, ol, tp, 4, &offsets[j]) || fb_bytes(d, ol, tp, 6, &kp, &kl, &present)) goto out;
    if (ko + kl > keys_cap) { st = OR_E_CAPACITY; goto out; }
    memcpy(keys + ko, kp, kl); ko += kl; key_off[j + 1] = ko;
  }
  *n_out = nm;
  st = OR_OK;
out:
  free(d);
  return st;
}

/* ====================================================== sstable.Builder */
typedef struct { uint8_t* p; size_t n; } chunk_t;

struct or_sst_builder {
  uint64_t block_size; uint32_t min_filter_keys, bpk; int codec;
  or_block_builder* bb;
  /* bloom keys (all keys, duplicates included) */
  uint8_t* fkeys; size_t fkeys_len, fkeys_cap; uint64_t* fkey_off; size_t nkeys_cap;
  /* block metas */
  uint64_t* meta_off; uint8_t* meta_keys; uint64_t* meta_key_off; size_t nmeta, meta_cap, mkeys_len, mkeys_cap;
  uint8_t* first_key; size_t first_key_len; int has_first_key;
  chunk_t* chunks; size_t head, nchunks, chunks_cap; /* deque */
  uint8_t* popped; /* last NextBlock result */
  uint64_t current_len;
  uint32_t num_keys;
  /* Build results */
  int built; or_sst_info info; uint8_t* bloom_bits; size_t bloom_len; uint16_t bloom_np; int has_bloom;
};

or_sst_builder* or_sst_builder_new(uint64_t block_size, uint32_t mfk, uint32_t bpk, int codec) {
  or_sst_builder* b = (or_sst_builder*)calloc(1, sizeof(*b));
  b->block_size = block_size; b->min_filter_keys = mfk; b->bpk = bpk; b->codec = codec;
  b->bb = or_block_builder_new(block_size);
  b->nkeys_cap = 1024; b->fkey_off = (uint64_t*)malloc(sizeof(uint64_t) * (b->nkeys_cap + 1)); b->fkey_off[0] = 0;
  b->meta_cap = 64; b->meta_off = (uint64_t*)malloc(sizeof(uint64_t) * 64);
  b->meta_key_off = (uint64_t*)malloc(sizeof(uint64_t) * 65); b->meta_key_off[0] = 0;
  return b;
}
void or_sst_builder_free(or_sst_builder* b) {
  if (!b) return;
  or_block_builder_free(b->bb);
  free(b->fkeys); free(b->fkey_off); free(b->meta_off); free(b->meta_keys); free(b->meta_key_off);
  free(b->first_key);
  for (size_t i = b->head; i < b->head + b->nchunks; i++) free(b->chunks[i].p);
  free(b->chunks); free(b->popped); free(b->bloom_bits); free(b);
}
static void push_chunk(or_sst_builder* b, uint8_t* p, size_t n) {
  if (b->head + b->nchunks == b->chunks_cap) {
    if (b->head > 0) { memmove(b->chunks, b->chunks + b->head, sizeof(chunk_t) * b->nchunks); b->head = 0; }
    if (b->nchunks == b->chunks_cap) { b->chunks_cap = b->chunks_cap ? b->chunks_cap * 2 : 64; b->chunks = (chunk_t*)realloc(b->chunks, sizeof(chunk_t) * b->chunks_cap); }
  }
  b->chunks[b->head + b->nchunks].p = p; b->chunks[b->head + b->nchunks].n = n; b->nchunks++;
}

/* builder.go:192-213 finishBlock: returns NULL when the block builder is empty */
static int finish_block(or_sst_builder* b, uint8_t** out, size_t* out_len) {
  *out = NULL; *out_len = 0;
  if (or_block_builder_is_empty(b->bb)) return OR_OK;
  const uint8_t* data; const uint16_t* offs; const uint8_t* fk;
  size_t dl = or_block_builder_data(b->bb, &data), n = or_block_builder_offsets(b->bb, &offs);
  size_t fkl = or_block_builder_first_key(b->bb, &fk);
  size_t cap = or_block_encode_bound(dl, n);
  uint8_t* buf = (uint8_t*)malloc(cap);
  int st = or_block_encode(data, dl, offs, n, b->codec, buf, cap, out_len);
  if (st) { free(buf); return st; }
  *out = buf;
  if (b->nmeta == b->meta_cap) {
    b->meta_cap *= 2;
    b->meta_off = (uint64_t*)realloc(b->meta_off, sizeof(uint64_t) * b->meta_cap);
    b->meta_key_off = (uint64_t*)realloc(b->meta_key_off, sizeof(uint64_t) * (b->meta_cap + 1));
  }
  if (b->mkeys_len + fkl > b->mkeys_cap) {
    b->mkeys_cap = (b->mkeys_cap + fkl) * 2;
    b->meta_keys = (uint8_t*)realloc(b->meta_keys, b->mkeys_cap);
  }
  b->meta_off[b->nmeta] = b->current_len;
  memcpy(b->meta_keys + b->mkeys_len, fk, fkl); b->mkeys_len += fkl;
  b->meta_key_off[++b->nmeta] = b->mkeys_len;
  or_block_builder_reset(b->bb);
  return OR_OK;
}

/* builder.go:160-183 Add */
int or_sst_builder_add(or_sst_builder* b, const uint8_t* key, size_t klen, const uint8_t* value,
                       size_t vlen, int tombstone) {
  if (klen == 0) return OR_E_INVALID_ARG; /* block.go:163 assert panics */
  b->num_keys += 1;
  if (!or_block_builder_add(b->bb, key, klen, tombstone, value, vlen)) {
    uint8_t* buf; size_t bl;
    int st = finish_block(b, &buf, &bl);
    if (st) return st;
    b->current_len += bl;
    push_chunk(b, buf, bl);
    or_block_builder_add(b->bb, key, klen, tombstone, value, vlen);
  }
  if (!b->has_first_key) {
    b->first_key = (uint8_t*)malloc(klen); memcpy(b->first_key, key, klen);
    b->first_key_len = klen; b->has_first_key = 1;
  }
  /* filterBuilder.Add(key) */
  size_t nk = b->num_keys; /* keys so far, this one included */
  if (nk > b->nkeys_cap) { b->nkeys_cap *= 2; b->fkey_off = (uint64_t*)realloc(b->fkey_off, sizeof(uint64_t) * (b->nkeys_cap + 1)); }
  if (b->fkeys_len + klen > b->fkeys_cap) { b->fkeys_cap = (b->fkeys_cap + klen) * 2; b->fkeys = (uint8_t*)realloc(b->fkeys, b->fkeys_cap); }
  memcpy(b->fkeys + b->fkeys_len, key, klen); b->fkeys_len += klen;
  b->fkey_off[nk] = b->fkeys_len;
  return OR_OK;
}

/* builder.go:149-158 AddValue */
int or_sst_builder_add_value(or_sst_builder* b, const uint8_t* key, size_t klen, const uint8_t* value,
                             size_t vlen) {
  return or_sst_builder_add(b, key, klen, value, vlen, vlen == 0);
}

int or_sst_builder_add_batch(or_sst_builder* b, const uint8_t* keys, const uint64_t* key_off,
                             const uint8_t* vals, const uint64_t* val_off, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) {
    int st = or_sst_builder_add_value(b, keys + key_off[i], key_off[i + 1] - key_off[i], vals + val_off[i],
                                      val_off[i + 1] - val_off[i]);
    if (st) return st;
  }
  return OR_OK;
}

/* builder.go:185-190 NextBlock */
int or_sst_builder_next_block(or_sst_builder* b, const uint8_t** data, size_t* len) {
  if (b->nchunks == 0) return 0;
  free(b->popped);
  b->popped = b->chunks[b->head].p;
  *data = b->popped; *len = b->chunks[b->head].n;
  b->head++; b->nchunks--;
  return 1;
}

/* builder.go:215-268 Build */
int or_sst_builder_build(or_sst_builder* b) {
  uint8_t* buf; size_t bl;
  int st = finish_block(b, &buf, &bl);
  if (st) return st;
  size_t cap = bl + 64, len = bl;
  uint8_t* out = (uint8_t*)malloc(cap);
  if (bl) memcpy(out, buf, bl);
  free(buf);
  uint64_t filter_off = b->current_len + len;
  size_t filter_len = 0;
  if (b->num_keys >= b->min_filter_keys) {
    uint64_t nb = or_bloom_filter_bytes(b->num_keys, b->bpk);
    b->bloom_bits = (uint8_t*)malloc(nb ? nb : 1);
    or_bloom_build(b->fkeys, b->fkey_off, b->num_keys, b->bpk, b->bloom_bits, nb, &b->bloom_len, &b->bloom_np);
    size_t ecap = or_snappy_max_encoded_len(b->bloom_len + 2) + 4;
    if (len + ecap > cap) { cap = len + ecap + 64; out = (uint8_t*)realloc(out, cap); }
    st = or_bloom_encode(b->bloom_np, b->bloom_bits, b->bloom_len, b->codec, out + len, ecap, &filter_len);
    if (st) { free(out); return st; }
    len += filter_len;
    b->has_bloom = 1;
  }
  /* index */
  size_t icap = or_snappy_max_encoded_len(64 + b->nmeta * 32 + b->mkeys_len + 4 * b->nmeta) + 4;
  if (len + icap > cap) { cap = len + icap + 64; out = (uint8_t*)realloc(out, cap); }
  size_t ilen;
  st = or_encode_index(b->meta_off, b->meta_keys, b->meta_key_off, b->nmeta, b->codec, out + len, icap, &ilen);
  if (st) { free(out); return st; }
  uint64_t index_off = b->current_len + len;
  len += ilen;
  uint64_t meta_off = b->current_len + len;
  or_sst_info info;
  info.index_offset = index_off; info.index_len = ilen; info.filter_offset = filter_off;
  info.filter_len = filter_len; info.codec = b->codec; info.first_key_len = (uint32_t)b->first_key_len;
  size_t infcap = 128 + b->first_key_len;
  if (len + infcap + 4 > cap) { cap = len + infcap + 64; out = (uint8_t*)realloc(out, cap); }
  size_t inflen;
  st = or_encode_info(&info, b->has_first_key ? b->first_key : NULL, out + len, infcap, &inflen);
  if (st) { free(out); return st; }
  len += inflen;
  put_be32(out + len, (uint32_t)meta_off); len += 4;
  push_chunk(b, out, len);
  b->info = info;
  b->built = 1;
  return OR_OK;
}

size_t or_sst_table_num_chunks(const or_sst_builder* b) { return b->nchunks; }
int or_sst_table_chunk(const or_sst_builder* b, size_t i, const uint8_t** d, size_t* len) {
  if (i >= b->nchunks) return OR_E_INVALID_ARG;
  *d = b->chunks[b->head + i].p; *len = b->chunks[b->head + i].n; return OR_OK;
}
size_t or_sst_table_encoded_len(const or_sst_builder* b) {
  size_t n = 0;
  for (size_t i = 0; i < b->nchunks; i++) n += b->chunks[b->head + i].n;
  return n;
}
int or_sst_table_encode(const or_sst_builder* b, uint8_t* out, size_t cap) {
  size_t o = 0;
  for (size_t i = 0; i < b->nchunks; i++) {
    const chunk_t* c = &b->chunks[b->head + i];
    if (o + c->n > cap) return OR_E_CAPACITY;
    memcpy(out + o, c->p, c->n); o += c->n;
  }
  return OR_OK;
}
int or_sst_table_info(const or_sst_builder* b, or_sst_info* info, uint8_t* fk, size_t fk_cap) {
  if (!b->built) return OR_E_INVALID_ARG;
  *info = b->info;
  if (b->first_key_len > fk_cap) return OR_E_CAPACITY;
  if (b->first_key_len) memcpy(fk, b->first_key, b->first_key_len);
  return OR_OK;
}
int or_sst_table_bloom(const or_sst_builder* b, int* present, uint16_t* np, uint8_t* bits, size_t cap,
                       size_t* bl) {
  *present = b->has_bloom; *np = b->bloom_np; *bl = b->bloom_len;
  if (!b->has_bloom) return OR_OK;
  if (b->bloom_len > cap) return OR_E_CAPACITY;
  memcpy(bits, b->bloom_bits, b->bloom_len);
  return OR_OK;
}

/* decode.go:25-48 ReadInfo */
int or_sst_read_info(const uint8_t* sst, size_t n, or_sst_info* info, uint8_t* fk, size_t fk_cap) {
  if (n <= 4) return OR_E_SST_TOO_SHORT;
  uint64_t oi = n - 4;
  uint32_t mo = be32(sst + oi);
  if (mo > oi) return OR_E_BLOB_RANGE; /* bytesBlob.ReadRange bounds (blob.go:24) */
  return or_decode_info(sst + mo, (size_t)(oi - mo), info, fk, fk_cap);
}

/* ------------------------------------------------------------------ iter.MergeSort */
/* merge.go:84-95 heapItem.Compare: bytes.Compare on keys, then the iterator index. */
static int merge_item_cmp(const uint8_t* keys, const uint64_t* key_off, uint64_t ea, uint32_t ia, uint64_t eb,
                          uint32_t ib) {
  const uint64_t la = key_off[ea + 1] - key_off[ea], lb = key_off[eb + 1] - key_off[eb];
  const uint64_t m = la < lb ? la : lb;
  int c = m ? memcmp(keys + key_off[ea], keys + key_off[eb], m) : 0;
  if (c == 0) c = la < lb ? -1 : (la > lb ? 1 : 0);
  if (c == 0) c = ia < ib ? -1 : (ia > ib ? 1 : 0);
  return c;
}

typedef struct {
  uint64_t e;  /* element (global index) */
  uint32_t it; /* iterator index */
} or_heap_item;

static void merge_sift_down(or_heap_item* h, size_t n, size_t i, const uint8_t* keys, const uint64_t* key_off) {
  for (;;) {
    size_t l = 2 * i + 1, s = i;
    if (l < n && merge_item_cmp(keys, key_off, h[l].e, h[l].it, h[s].e, h[s].it) < 0) s = l;
    if (l + 1 < n && merge_item_cmp(keys, key_off, h[l + 1].e, h[l + 1].it, h[s].e, h[s].it) < 0) s = l + 1;
    if (s == i) return;
    or_heap_item t = h[i];
    h[i] = h[s];
    h[s] = t;
    i = s;
  }
}

static void merge_sift_up(or_heap_item* h, size_t i, const uint8_t* keys, const uint64_t* key_off) {
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (merge_item_cmp(keys, key_off, h[i].e, h[i].it, h[p].e, h[p].it) >= 0) return;
    or_heap_item t = h[i];
    h[i] = h[p];
    h[p] = t;
    i = p;
  }
}

int or_merge_sort(uint32_t k, const uint8_t* keys, const uint64_t* key_off, const uint64_t* src_start,
                  uint32_t* out_idx, uint64_t* n_out) {
  *n_out = 0;
  if (k == 0) return OR_OK;
  or_heap_item* h = (or_heap_item*)malloc(sizeof(or_heap_item) * k);
  uint64_t* next = (uint64_t*)malloc(sizeof(uint64_t) * k);
  if (!h || !next) {
    free(h);
    free(next);
    return OR_E_INVALID_ARG;
  }
  size_t hn = 0;
  /* NewMergeSort (merge.go:30-50): the first entry of every iterator */
  for (uint32_t i = 0; i < k; i++) {
    next[i] = src_start[i];
    if (next[i] < src_start[i + 1]) {
      h[hn].e = next[i]++;
      h[hn].it = i;
      merge_sift_up(h, hn++, keys, key_off);
    }
  }
  /* Next (merge.go:54-76) */
  int have_last = 0; /* lastKey == nil */
  uint64_t last = 0;
  uint64_t n = 0;
  while (hn > 0) {
    or_heap_item it = h[0];
    h[0] = h[--hn];
    merge_sift_down(h, hn, 0, keys, key_off);
    if (next[it.it] < src_start[it.it + 1]) {
      h[hn].e = next[it.it]++;
      h[hn].it = it.it;
      merge_sift_up(h, hn++, keys, key_off);
    }
    const uint64_t len = key_off[it.e + 1] - key_off[it.e];
    int equal;
    if (!have_last) {
      equal = len == 0; /* bytes.Equal(key, nil) */
    } else {
      const uint64_t ll = key_off[last + 1] - key_off[last];
      equal = ll == len && (len == 0 || memcmp(keys + key_off[last], keys + key_off[it.e], len) == 0);
    }
    if (!equal) {
      last = it.e;
      have_last = 1;
      out_idx[n++] = (uint32_t)it.e;
    }
  }
  free(h);
  free(next);
  *n_out = n;
  return OR_OK;
}
