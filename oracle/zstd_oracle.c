/* Zstandard frame decode for the CPU oracle (TEST INFRASTRUCTURE ONLY: never linked into
 * the product library).
 *
 * compress.Decode CodecZstd = io.ReadAll(zstd.NewReader(bytes.NewReader(buf)))
 * (internal/compress/compression.go:146-153) with github.com/klauspost/compress v1.17.11
 * (go.mod:10), which is absent here.  This restates its decoder from the format it
 * implements, RFC 8878: concatenated frames and skippable frames read in order; the frame
 * header (reserved bit, window descriptor, dictionary id, content size); raw / RLE /
 * compressed blocks (Block_Maximum_Size = min(window, 128 KiB)); literals (raw, RLE,
 * Huffman with 1 or 4 streams, treeless = the frame's previous table; weights direct or
 * FSE-compressed); sequences (predefined / RLE / FSE / repeat tables per LL, OF, ML;
 * three repeat offsets starting 1, 4, 8; no state update after the last sequence; every
 * backward bitstream consumed exactly); then Frame_Content_Size and the XXH64 content
 * checksum (low 32 bits).
 *
 * Parity: decoded bytes are pinned by frames written by libzstd 1.4.9 (/opt/conda) over
 * every level/strategy the tests use (tests/test_zstd_oracle.py, fixtures in
 * tests/golden/zstd_frames.json).  klauspost's error strings and its choice between
 * errors on damaged input are PARITY UNPINNED (no Go here); this file maps them to the
 * status codes 54 and 56-61.
 *
 * Plan size (what the block decoder sizes its output by): per frame, the content size
 * when the header carries one (clamped by the blocks' own bounds), otherwise the bytes an
 * in-order decode of that frame produces.  csrc/zstd.h follows the same rule. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "slate_oracle.h"

#define ZS_BLOCK_MAX (128u * 1024u)
#define ZS_MAX_WINDOW (1ull << 29) /* klauspost MaxWindowSize (64-bit) */

static inline uint32_t zs_le16(const uint8_t* p) { return p[0] | (uint32_t)p[1] << 8; }
static inline uint32_t zs_le24(const uint8_t* p) { return zs_le16(p) | (uint32_t)p[2] << 16; }
static inline uint32_t zs_le32(const uint8_t* p) { return zs_le16(p) | zs_le16(p + 2) << 16; }
static inline uint64_t zs_le64(const uint8_t* p) { return zs_le32(p) | (uint64_t)zs_le32(p + 4) << 32; }
static inline int zs_highbit(uint32_t v) { return 31 - __builtin_clz(v); } /* v > 0 */

/* ------------------------------------------------------------------ XXH64 */
#define XP1 0x9E3779B185EBCA87ull
#define XP2 0xC2B2AE3D27D4EB4Full
#define XP3 0x165667B19E3779F9ull
#define XP4 0x85EBCA77C2B2AE63ull
#define XP5 0x27D4EB2F165667C5ull
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * XP2, 31) * XP1; }
static inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * XP1 + XP4; }
uint64_t or_xxh64(const uint8_t* p, size_t n, uint64_t seed) {
  const uint8_t* e = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    while (e - p >= 32) {
      v1 = xround(v1, zs_le64(p)); v2 = xround(v2, zs_le64(p + 8));
      v3 = xround(v3, zs_le64(p + 16)); v4 = xround(v4, zs_le64(p + 24));
      p += 32;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += n;
  for (; e - p >= 8; p += 8) h = rotl64(h ^ xround(0, zs_le64(p)), 27) * XP1 + XP4;
  if (e - p >= 4) { h = rotl64(h ^ (uint64_t)zs_le32(p) * XP1, 23) * XP2 + XP3; p += 4; }
  for (; p < e; p++) h = rotl64(h ^ *p * XP5, 11) * XP1;
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

/* --------------------------------------------------- backward bitstream (RFC 8878 4.1) */
typedef struct { const uint8_t* p; int64_t pos; } zsbr; /* pos: bits left; < 0 after an overread */
static int zsbr_init(zsbr* b, const uint8_t* p, size_t n) {
  if (n == 0 || p[n - 1] == 0) return -1;
  b->p = p;
  b->pos = 8 * (int64_t)(n - 1) + zs_highbit(p[n - 1]);
  return 0;
}
static uint64_t zsbr_peek(const zsbr* b, unsigned k) { /* k <= 56: bits [pos-k, pos), zeros below 0 */
  if (k == 0 || b->pos <= 0) return 0;
  const int64_t lo = b->pos - (int64_t)k, s = lo > 0 ? lo : 0;
  uint64_t v = 0;
  for (int64_t i = (b->pos - 1) >> 3; i >= (s >> 3); i--) v = (v << 8) | b->p[i];
  v >>= s & 7;
  v &= (1ull << (b->pos - s)) - 1;
  return v << (s - lo);
}
static uint64_t zsbr_read(zsbr* b, unsigned k) {
  uint64_t v = zsbr_peek(b, k);
  b->pos -= k;
  return v;
}

/* ----------------------------------------------------------------------- FSE */
typedef struct { uint8_t sym, nb; uint16_t base; } zsfse;
typedef struct { zsfse t[512]; int al, valid; } zstab;

/* FSE_readNCount (RFC 8878 4.1.1): the forward bitstream at p[0, n) (zero padded; reading
 * past n is corruption).  Returns the bytes used or -1. */
static long zs_ncount(const uint8_t* p, size_t n, int16_t* norm, int maxs, int maxal, int* al_out, int* last) {
  uint64_t bp = 0;
  if (n == 0) return -1;
  const int al = (p[0] & 15) + 5;
  bp = 4;
  if (al > maxal) return -1;
  int remaining = (1 << al) + 1, threshold = 1 << al, nb = al + 1, s = 0, prev0 = 0;
  memset(norm, 0, sizeof(int16_t) * (size_t)(maxs + 1));
  while (remaining > 1 && s <= maxs) {
    if (prev0) {
      int n0 = s;
      for (;;) {
        uint32_t r = 0;
        for (int i = 0; i < 2; i++, bp++) if ((bp >> 3) < n) r |= (uint32_t)((p[bp >> 3] >> (bp & 7)) & 1) << i;
        n0 += (int)r;
        if (r != 3) break;
      }
      if (n0 > maxs) return -1;
      while (s < n0) norm[s++] = 0;
      prev0 = 0;
    }
    uint32_t v = 0;
    for (int i = 0; i < nb; i++) {
      uint64_t q = bp + (uint64_t)i;
      if ((q >> 3) < n) v |= (uint32_t)((p[q >> 3] >> (q & 7)) & 1) << i;
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    if ((int)(v & (uint32_t)(threshold - 1)) < max) {
      count = (int)(v & (uint32_t)(threshold - 1));
      bp += (uint64_t)(nb - 1);
    } else {
      count = (int)(v & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bp += (uint64_t)nb;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[s++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold && nb > 1) { nb--; threshold >>= 1; }
  }
  if (remaining != 1) return -1;
  if ((bp + 7) / 8 > n) return -1;
  *al_out = al;
  *last = s - 1;
  return (long)((bp + 7) / 8);
}

/* FSE decoding table (RFC 8878 4.1.1): -1 cells at the top, the spread step, states. */
static int zs_fse_build(zstab* t, const int16_t* norm, int last, int al) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t hi = size - 1, next[256];
  for (int s = 0; s <= last; s++) {
    if (norm[s] == -1) { t->t[hi--].sym = (uint8_t)s; next[s] = 1; }
    else next[s] = (uint32_t)(norm[s] > 0 ? norm[s] : 0);
  }
  uint32_t pos = 0;
  for (int s = 0; s <= last; s++)
    for (int i = 0; i < norm[s]; i++) {
      t->t[pos].sym = (uint8_t)s;
      do pos = (pos + step) & mask; while (pos > hi);
    }
  if (pos != 0) return -1;
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t x = next[t->t[u].sym]++;
    const int nb = al - zs_highbit(x);
    t->t[u].nb = (uint8_t)nb;
    t->t[u].base = (uint16_t)((x << nb) - size);
  }
  t->al = al;
  t->valid = 1;
  return 0;
}

/* ------------------------------------------------------------------- Huffman */
typedef struct { uint8_t sym[2048], nb[2048]; int tl, valid; } zshuf;

/* Huffman_Tree_Description at p[0, n): returns bytes used or -1 (RFC 8878 4.2.1). */
static long zs_huf_read(const uint8_t* p, size_t n, zshuf* h) {
  if (n < 1) return -1;
  const uint32_t hb = p[0];
  uint8_t w[256];
  int nw = 0;
  long used;
  if (hb >= 128) {
    nw = (int)hb - 127;
    const size_t nbytes = ((size_t)nw + 1) / 2;
    if (1 + nbytes > n) return -1;
    for (int i = 0; i < nw; i++) w[i] = (i & 1) ? (p[1 + i / 2] & 15) : (p[1 + i / 2] >> 4);
    used = (long)(1 + nbytes);
  } else {
    if (1 + (size_t)hb > n) return -1;
    int16_t norm[256];
    int al, last;
    const long hs = zs_ncount(p + 1, hb, norm, 255, 6, &al, &last);
    if (hs < 0) return -1;
    static __thread zstab t;
    if (zs_fse_build(&t, norm, last, al)) return -1;
    zsbr b;
    if (zsbr_init(&b, p + 1 + hs, hb - (size_t)hs)) return -1;
    uint32_t s1 = (uint32_t)zsbr_read(&b, (unsigned)al), s2 = (uint32_t)zsbr_read(&b, (unsigned)al);
    for (;;) { /* two interleaved states until the stream overreads (FSE_decompress tail) */
      if (nw > 253) return -1;
      w[nw++] = t.t[s1].sym;
      s1 = t.t[s1].base + (uint32_t)zsbr_read(&b, t.t[s1].nb);
      if (b.pos < 0) { w[nw++] = t.t[s2].sym; break; }
      if (nw > 253) return -1;
      w[nw++] = t.t[s2].sym;
      s2 = t.t[s2].base + (uint32_t)zsbr_read(&b, t.t[s2].nb);
      if (b.pos < 0) { w[nw++] = t.t[s1].sym; break; }
    }
    used = (long)(1 + hb);
  }
  uint32_t rank[13] = {0}, total = 0;
  for (int i = 0; i < nw; i++) {
    if (w[i] > 11) return -1;
    rank[w[i]]++;
    total += (1u << w[i]) >> 1;
  }
  if (total == 0) return -1;
  const int tl = zs_highbit(total) + 1;
  if (tl > 11) return -1;
  const uint32_t rest = (1u << tl) - total;
  if (rest == 0 || (rest & (rest - 1))) return -1;
  w[nw] = (uint8_t)(zs_highbit(rest) + 1);
  rank[w[nw]]++;
  if (rank[1] < 2 || (rank[1] & 1)) return -1;
  uint32_t start[13], acc = 0;
  for (int k = 1; k <= tl; k++) { start[k] = acc; acc += rank[k] << (k - 1); }
  for (int s = 0; s <= nw; s++) {
    const int k = w[s];
    if (!k) continue;
    const uint32_t len = 1u << (k - 1);
    for (uint32_t i = 0; i < len; i++) { h->sym[start[k] + i] = (uint8_t)s; h->nb[start[k] + i] = (uint8_t)(tl + 1 - k); }
    start[k] += len;
  }
  h->tl = tl;
  h->valid = 1;
  return used;
}

/* One Huffman stream p[0, n) -> exactly m literals, the stream consumed exactly. */
static int zs_huf_stream(const zshuf* h, const uint8_t* p, size_t n, uint8_t* out, size_t m) {
  zsbr b;
  if (zsbr_init(&b, p, n)) return -1;
  for (size_t i = 0; i < m; i++) {
    const uint32_t v = (uint32_t)zsbr_peek(&b, (unsigned)h->tl);
    out[i] = h->sym[v];
    b.pos -= h->nb[v];
  }
  return b.pos == 0 ? 0 : -1;
}

/* -------------------------------------------------------------- sequences */
static const int16_t zs_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                      2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t zs_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t zs_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t zs_ll_base[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,   14,    15,    16,    18,
                                        20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t zs_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,
                                       1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t zs_ml_base[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                        21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                        43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t zs_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                       0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

typedef struct {
  zshuf huf;
  zstab ll, of, ml;
  uint32_t rep[3];
  uint8_t lit[ZS_BLOCK_MAX];
} zsframe;

/* Symbol_Compression_Mode for one table type; returns bytes used or -1. */
static long zs_table(int mode, const uint8_t* p, size_t n, zstab* t, const int16_t* def, int deflast, int defal,
                     int maxs, int maxal) {
  if (mode == 0) { zs_fse_build(t, def, deflast, defal); return 0; }
  if (mode == 1) {
    if (n < 1 || p[0] > maxs) return -1;
    t->t[0].sym = p[0]; t->t[0].nb = 0; t->t[0].base = 0;
    t->al = 0; t->valid = 1;
    return 1;
  }
  if (mode == 2) {
    int16_t norm[64];
    int al, last;
    long hs = zs_ncount(p, n, norm, maxs, maxal, &al, &last);
    if (hs < 0 || zs_fse_build(t, norm, last, al)) return -1;
    return hs;
  }
  return t->valid ? 0 : -1; /* repeat */
}

/* Copy helper: out == NULL sizes only. */
static void zs_put(uint8_t* out, size_t d, const uint8_t* src, size_t n) { if (out) memcpy(out + d, src, n); }

/* A compressed block p[0, n) appended at out[*d]; fstart = the frame's first output byte. */
static int zs_block(zsframe* f, const uint8_t* p, size_t n, uint8_t* out, size_t cap, size_t* d, size_t fstart,
                    uint32_t bmax) {
  /* Literals_Section (RFC 8878 3.1.1.3.1) */
  if (n < 1) return OR_E_ZSTD_CORRUPT;
  const uint32_t type = p[0] & 3, sf = (p[0] >> 2) & 3;
  size_t pos, nlit;
  if (type <= 1) {
    size_t hs;
    if (sf == 1) { hs = 2; if (n < 2) return OR_E_ZSTD_CORRUPT; nlit = (p[0] >> 4) + ((size_t)p[1] << 4); }
    else if (sf == 3) { hs = 3; if (n < 3) return OR_E_ZSTD_CORRUPT; nlit = (p[0] >> 4) + ((size_t)p[1] << 4) + ((size_t)p[2] << 12); }
    else { hs = 1; nlit = p[0] >> 3; }
    if (nlit > bmax) return OR_E_ZSTD_CORRUPT;
    if (type == 0) {
      if (n - hs < nlit) return OR_E_ZSTD_CORRUPT;
      memcpy(f->lit, p + hs, nlit);
      pos = hs + nlit;
    } else {
      if (n - hs < 1) return OR_E_ZSTD_CORRUPT;
      memset(f->lit, p[hs], nlit);
      pos = hs + 1;
    }
  } else {
    size_t hs, cs;
    int streams = sf == 0 ? 1 : 4;
    if (sf <= 1) {
      hs = 3; if (n < 3) return OR_E_ZSTD_CORRUPT;
      const uint32_t h = zs_le24(p);
      nlit = (h >> 4) & 0x3FF; cs = (h >> 14) & 0x3FF;
    } else if (sf == 2) {
      hs = 4; if (n < 4) return OR_E_ZSTD_CORRUPT;
      const uint32_t h = zs_le32(p);
      nlit = (h >> 4) & 0x3FFF; cs = (h >> 18) & 0x3FFF;
    } else {
      hs = 5; if (n < 5) return OR_E_ZSTD_CORRUPT;
      const uint64_t h = zs_le32(p) | (uint64_t)p[4] << 32;
      nlit = (size_t)((h >> 4) & 0x3FFFF); cs = (size_t)((h >> 22) & 0x3FFFF);
    }
    if (nlit > bmax || n - hs < cs) return OR_E_ZSTD_CORRUPT;
    const uint8_t* q = p + hs;
    size_t qn = cs;
    if (type == 2) {
      long t = zs_huf_read(q, qn, &f->huf);
      if (t < 0) return OR_E_ZSTD_CORRUPT;
      q += t; qn -= (size_t)t;
    } else if (!f->huf.valid) {
      return OR_E_ZSTD_CORRUPT;
    }
    if (streams == 1) {
      if (zs_huf_stream(&f->huf, q, qn, f->lit, nlit)) return OR_E_ZSTD_CORRUPT;
    } else {
      if (qn < 10) return OR_E_ZSTD_CORRUPT;
      const size_t l1 = zs_le16(q), l2 = zs_le16(q + 2), l3 = zs_le16(q + 4);
      if (l1 + l2 + l3 + 6 > qn) return OR_E_ZSTD_CORRUPT;
      const size_t l4 = qn - 6 - l1 - l2 - l3, seg = (nlit + 3) / 4;
      if (3 * seg > nlit) return OR_E_ZSTD_CORRUPT;
      const uint8_t* s = q + 6;
      if (zs_huf_stream(&f->huf, s, l1, f->lit, seg) || zs_huf_stream(&f->huf, s + l1, l2, f->lit + seg, seg) ||
          zs_huf_stream(&f->huf, s + l1 + l2, l3, f->lit + 2 * seg, seg) ||
          zs_huf_stream(&f->huf, s + l1 + l2 + l3, l4, f->lit + 3 * seg, nlit - 3 * seg))
        return OR_E_ZSTD_CORRUPT;
    }
    pos = hs + cs;
  }
  /* Sequences_Section (RFC 8878 3.1.1.3.2) */
  if (pos >= n) return OR_E_ZSTD_CORRUPT;
  const uint8_t* s = p + pos;
  size_t sn = n - pos, sp;
  uint32_t nseq;
  if (s[0] < 128) { nseq = s[0]; sp = 1; }
  else if (s[0] < 255) { if (sn < 2) return OR_E_ZSTD_CORRUPT; nseq = ((uint32_t)(s[0] - 128) << 8) + s[1]; sp = 2; }
  else { if (sn < 3) return OR_E_ZSTD_CORRUPT; nseq = s[1] + ((uint32_t)s[2] << 8) + 0x7F00; sp = 3; }
  const size_t d0 = *d;
  size_t lp = 0, o = d0;
  if (nseq == 0) {
    if (sp != sn) return OR_E_ZSTD_CORRUPT;
  } else {
    if (sp >= sn) return OR_E_ZSTD_CORRUPT;
    const uint32_t modes = s[sp++];
    if (modes & 3) return OR_E_ZSTD_CORRUPT;
    long t;
    if ((t = zs_table((int)(modes >> 6), s + sp, sn - sp, &f->ll, zs_ll_def, 35, 6, 35, 9)) < 0) return OR_E_ZSTD_CORRUPT;
    sp += (size_t)t;
    if ((t = zs_table((int)((modes >> 4) & 3), s + sp, sn - sp, &f->of, zs_of_def, 28, 5, 31, 8)) < 0)
      return OR_E_ZSTD_CORRUPT;
    sp += (size_t)t;
    if ((t = zs_table((int)((modes >> 2) & 3), s + sp, sn - sp, &f->ml, zs_ml_def, 52, 6, 52, 9)) < 0)
      return OR_E_ZSTD_CORRUPT;
    sp += (size_t)t;
    zsbr b;
    if (zsbr_init(&b, s + sp, sn - sp)) return OR_E_ZSTD_CORRUPT;
    uint32_t sll = (uint32_t)zsbr_read(&b, (unsigned)f->ll.al), sof = (uint32_t)zsbr_read(&b, (unsigned)f->of.al),
             sml = (uint32_t)zsbr_read(&b, (unsigned)f->ml.al);
    for (uint32_t i = 0; i < nseq; i++) {
      const uint32_t ofc = f->of.t[sof].sym, llc = f->ll.t[sll].sym, mlc = f->ml.t[sml].sym;
      if (ofc > 31) return OR_E_ZSTD_CORRUPT;
      const uint64_t ofv = (1ull << ofc) + zsbr_read(&b, ofc);
      const uint32_t ml = zs_ml_base[mlc] + (uint32_t)zsbr_read(&b, zs_ml_bits[mlc]);
      const uint32_t ll = zs_ll_base[llc] + (uint32_t)zsbr_read(&b, zs_ll_bits[llc]);
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        f->rep[2] = f->rep[1]; f->rep[1] = f->rep[0]; f->rep[0] = (uint32_t)off;
      } else {
        const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0);
        off = idx == 3 ? (uint64_t)f->rep[0] - 1 : f->rep[idx];
        if (off == 0) off = 1; /* corrupt input; klauspost and libzstd force 1 */
        if (idx >= 2) f->rep[2] = f->rep[1];
        if (idx >= 1) { f->rep[1] = f->rep[0]; f->rep[0] = (uint32_t)off; }
      }
      if (i + 1 < nseq) {
        sll = f->ll.t[sll].base + (uint32_t)zsbr_read(&b, f->ll.t[sll].nb);
        sml = f->ml.t[sml].base + (uint32_t)zsbr_read(&b, f->ml.t[sml].nb);
        sof = f->of.t[sof].base + (uint32_t)zsbr_read(&b, f->of.t[sof].nb);
      }
      if (b.pos < 0) return OR_E_ZSTD_CORRUPT;
      /* execute: literals, then the match */
      if (ll > nlit - lp) return OR_E_ZSTD_CORRUPT;
      if ((uint64_t)(o - d0) + ll + ml > bmax || (uint64_t)o + ll + ml > cap) return OR_E_ZSTD_CORRUPT;
      zs_put(out, o, f->lit + lp, ll);
      lp += ll; o += ll;
      if (off > o - fstart) return OR_E_ZSTD_CORRUPT;
      if (out) for (uint32_t j = 0; j < ml; j++) out[o + j] = out[o - off + j];
      o += ml;
    }
    if (b.pos != 0) return OR_E_ZSTD_CORRUPT;
  }
  if ((uint64_t)(o - d0) + (nlit - lp) > bmax || (uint64_t)o + (nlit - lp) > cap) return OR_E_ZSTD_CORRUPT;
  zs_put(out, o, f->lit + lp, nlit - lp);
  *d = o + (nlit - lp);
  return OR_OK;
}

typedef struct { size_t hsize; uint64_t window, fcs; int has_fcs, checksum; } zshdr;

/* Frame header after the magic at p[0, n): 0, or a status. */
static int zs_header(const uint8_t* p, size_t n, zshdr* h) {
  if (n < 1) return OR_E_UNEXPECTED_EOF;
  const uint32_t fhd = p[0], fcsf = fhd >> 6, ss = (fhd >> 5) & 1, dif = fhd & 3;
  if (fhd & 8) return OR_E_ZSTD_CORRUPT; /* reserved bit */
  static const uint8_t dsz[4] = {0, 1, 2, 4}, fsz[4] = {0, 2, 4, 8};
  const size_t fl = fcsf == 0 ? (ss ? 1 : 0) : fsz[fcsf];
  h->hsize = 1 + (ss ? 0 : 1) + dsz[dif] + fl;
  if (n < h->hsize) return OR_E_UNEXPECTED_EOF;
  size_t q = 1;
  if (!ss) {
    const uint32_t wd = p[q++], wl = 10 + (wd >> 3);
    h->window = (1ull << wl) + ((1ull << wl) >> 3) * (wd & 7);
  }
  uint32_t dict = 0;
  for (uint32_t i = 0; i < dsz[dif]; i++) dict |= (uint32_t)p[q++] << (8 * i);
  if (dict != 0) return OR_E_ZSTD_DICT;
  h->has_fcs = fl != 0;
  h->fcs = 0;
  if (fl == 1) h->fcs = p[q];
  else if (fl == 2) h->fcs = zs_le16(p + q) + 256;
  else if (fl == 4) h->fcs = zs_le32(p + q);
  else if (fl == 8) h->fcs = zs_le64(p + q);
  if (ss) h->window = h->fcs;
  if (h->window > ZS_MAX_WINDOW) return OR_E_ZSTD_CORRUPT;
  h->checksum = (fhd >> 2) & 1;
  return 0;
}

/* One frame at in[*pos] (magic included) into out[*d]; out == NULL sizes only. */
static int zs_frame(zsframe* f, const uint8_t* in, size_t n, size_t* pos, uint8_t* out, size_t cap, size_t* d) {
  size_t p = *pos + 4;
  zshdr h;
  int st = zs_header(in + p, n - p, &h);
  if (st) return st;
  p += h.hsize;
  const uint32_t bmax = (uint32_t)(h.window < ZS_BLOCK_MAX ? h.window : ZS_BLOCK_MAX);
  f->huf.valid = f->ll.valid = f->of.valid = f->ml.valid = 0;
  f->rep[0] = 1; f->rep[1] = 4; f->rep[2] = 8;
  const size_t fstart = *d;
  for (;;) {
    if (n - p < 3) return OR_E_UNEXPECTED_EOF;
    const uint32_t bh = zs_le24(in + p), last = bh & 1, bt = (bh >> 1) & 3, bs = bh >> 3;
    p += 3;
    if (bt == 3) return OR_E_ZSTD_RESERVED_BLOCK;
    if (bs > bmax) return OR_E_ZSTD_CORRUPT;
    if (bt == 0) {
      if (n - p < bs) return OR_E_UNEXPECTED_EOF;
      if (bs > cap - *d) return OR_E_ZSTD_CORRUPT;
      zs_put(out, *d, in + p, bs);
      *d += bs; p += bs;
    } else if (bt == 1) {
      if (n - p < 1) return OR_E_UNEXPECTED_EOF;
      if (bs > cap - *d) return OR_E_ZSTD_CORRUPT;
      if (out) memset(out + *d, in[p], bs);
      *d += bs; p += 1;
    } else {
      if (n - p < bs) return OR_E_UNEXPECTED_EOF;
      st = zs_block(f, in + p, bs, out, cap, d, fstart, bmax);
      if (st) return st;
      p += bs;
    }
    if (last) break;
  }
  if (h.has_fcs && *d - fstart != h.fcs) return OR_E_ZSTD_FRAME_SIZE;
  if (h.checksum) {
    if (n - p < 4) return OR_E_UNEXPECTED_EOF;
    if (out && (uint32_t)or_xxh64(out + fstart, *d - fstart, 0) != zs_le32(in + p)) return OR_E_ZSTD_CHECKSUM;
    p += 4;
  }
  *pos = p;
  return OR_OK;
}

static int zs_frames(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  zsframe* f = (zsframe*)malloc(sizeof(zsframe));
  size_t pos = 0, d = 0;
  int st = OR_OK;
  while (pos < n) {
    if (n - pos < 4) { st = OR_E_UNEXPECTED_EOF; break; }
    const uint32_t magic = zs_le32(in + pos);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* skippable frame */
      if (n - pos < 8) { st = OR_E_UNEXPECTED_EOF; break; }
      const uint32_t sz = zs_le32(in + pos + 4);
      if (sz > n - pos - 8) { st = OR_E_UNEXPECTED_EOF; break; }
      pos += 8 + (size_t)sz;
      continue;
    }
    if (magic != 0xFD2FB528u) { st = OR_E_ZSTD_MAGIC; break; }
    if ((st = zs_frame(f, in, n, &pos, out, cap, &d)) != OR_OK) break;
  }
  free(f);
  *out_len = d;
  return st;
}

/* The plan size (header comment): stops at the first structural error. */
int or_zstd_plan(const uint8_t* in, size_t n, uint64_t* dlen) {
  size_t pos = 0, d = 0;
  zsframe* f = NULL;
  while (pos < n && n - pos >= 4) {
    const uint32_t magic = zs_le32(in + pos);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (n - pos < 8 || zs_le32(in + pos + 4) > n - pos - 8) break;
      pos += 8 + (size_t)zs_le32(in + pos + 4);
      continue;
    }
    if (magic != 0xFD2FB528u) break;
    zshdr h;
    if (zs_header(in + pos + 4, n - pos - 4, &h)) break;
    if (!h.has_fcs) { /* exact: decode the frame, sizes only */
      if (!f) f = (zsframe*)malloc(sizeof(zsframe));
      if (zs_frame(f, in, n, &pos, NULL, (size_t)-1, &d) != OR_OK) break;
      continue;
    }
    const uint32_t bmax = (uint32_t)(h.window < ZS_BLOCK_MAX ? h.window : ZS_BLOCK_MAX);
    size_t p = pos + 4 + h.hsize;
    uint64_t bound = 0;
    int ok = 1;
    for (;;) {
      if (n - p < 3) { ok = 0; break; }
      const uint32_t bh = zs_le24(in + p), bt = (bh >> 1) & 3, bs = bh >> 3;
      p += 3;
      if (bt == 3 || bs > bmax) { ok = 0; break; }
      const size_t adv = bt == 1 ? 1 : bs;
      if (n - p < adv) { ok = 0; break; }
      bound += bt == 2 ? bmax : bs;
      p += adv;
      if (bh & 1) break;
    }
    d += (size_t)(h.fcs < bound ? h.fcs : bound);
    if (!ok) break;
    if (h.checksum) { if (n - p < 4) break; p += 4; }
    pos = p;
  }
  free(f);
  *dlen = d;
  return OR_OK;
}

int or_zstd_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  return zs_frames(in, n, out, cap, out_len);
}

