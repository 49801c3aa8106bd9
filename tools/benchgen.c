/* Bench input tooling (not product, not oracle): compress a batch of decoded
 * blocks with the C++ snappy library or liblz4's frame API in /opt/conda (dlopen)
 * and append the block CRC32 trailer (block.go:54-75 layout), in parallel.  Used
 * only to synthesise encoded blocks for bench.py's and tools/ablate.py's workloads. */
#define _GNU_SOURCE 1 /* RTLD_DEEPBIND */
#include <dlfcn.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

typedef int (*compress_fn)(const char*, size_t, char*, size_t*);
static compress_fn g_compress;
/* LZ4F_preferences_t of lz4frame.h 1.9.x */
typedef struct {
  int blockSizeID, blockMode, contentChecksumFlag, frameType;
  unsigned long long contentSize;
  unsigned dictID;
  int blockChecksumFlag, compressionLevel;
  unsigned autoFlush, favorDecSpeed, reserved[3];
} lz4f_prefs;
typedef size_t (*lz4f_fn)(void*, size_t, const void*, size_t, const lz4f_prefs*);
typedef unsigned (*lz4f_err_fn)(size_t);
static lz4f_fn g_lz4f;
static lz4f_err_fn g_lz4f_err;

/* pierrec/lz4 v4 writer defaults: 4 MiB max blocks, independent blocks, content checksum */
int bg_init_lz4(const char* liblz4) {
  void* h = dlopen(liblz4, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
  if (!h) return -1;
  g_lz4f = (lz4f_fn)dlsym(h, "LZ4F_compressFrame");
  g_lz4f_err = (lz4f_err_fn)dlsym(h, "LZ4F_isError");
  return (g_lz4f && g_lz4f_err) ? 0 : -2;
}
/* libzstd 1.4.9 (dlopen): level 3 + content checksum + content size, one CCtx per call */
typedef void* (*zcreate_fn)(void);
typedef size_t (*zfree_fn)(void*);
typedef size_t (*zsetp_fn)(void*, int, int);
typedef size_t (*zc2_fn)(void*, void*, size_t, const void*, size_t);
typedef unsigned (*zerr_fn)(size_t);
static zcreate_fn g_zcreate;
static zfree_fn g_zfree;
static zsetp_fn g_zsetp;
static zc2_fn g_zc2;
static zerr_fn g_zerr;
int bg_init_zstd(const char* libzstd) {
  void* h = dlopen(libzstd, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
  if (!h) return -1;
  g_zcreate = (zcreate_fn)dlsym(h, "ZSTD_createCCtx");
  g_zfree = (zfree_fn)dlsym(h, "ZSTD_freeCCtx");
  g_zsetp = (zsetp_fn)dlsym(h, "ZSTD_CCtx_setParameter");
  g_zc2 = (zc2_fn)dlsym(h, "ZSTD_compress2");
  g_zerr = (zerr_fn)dlsym(h, "ZSTD_isError");
  return (g_zcreate && g_zfree && g_zsetp && g_zc2 && g_zerr) ? 0 : -2;
}
static uint32_t g_tab[256];

static uint32_t bg_crc32(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = g_tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

int bg_init(const char* libsnappy) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    g_tab[i] = c;
  }
  void* h = dlopen(libsnappy, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
  if (!h) return -1;
  g_compress = (compress_fn)dlsym(h, "snappy_compress");
  return g_compress ? 0 : -2;
}

/* CodecZlib (codec 2): zlib level 6, in the shape Go's compress/zlib writer closes a stream with --
 * the data's non-final deflate blocks, an empty FINAL stored block, the Adler-32 (tests/sstgen.py
 * go_zlib): zlib's sync flush ends with an empty non-final stored block, whose BFINAL bit is set
 * (the bit found by trial: the one flip after which inflate ends there with the same bytes). */
static long go_zlib6(const uint8_t* s, size_t n, uint8_t* d, size_t cap) {
  if (cap < 16) return -1;
  z_stream z;
  memset(&z, 0, sizeof z);
  if (deflateInit2(&z, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
  z.next_in = (Bytef*)s;
  z.avail_in = (uInt)n;
  z.next_out = d + 2;
  z.avail_out = (uInt)(cap - 6);
  int r = deflate(&z, Z_SYNC_FLUSH);
  size_t bl = (cap - 6) - z.avail_out;
  deflateEnd(&z);
  if (r != Z_OK || z.avail_in != 0 || bl < 5) return -1;
  uint8_t* body = d + 2;
  static __thread uint8_t chk[1 << 17];
  int found = 0;
  for (size_t pos = bl - 5; !found && pos + 6 >= bl && pos < bl; pos--) {
    for (int bit = 0; bit < 8 && !found; bit++) {
      body[pos] ^= (uint8_t)(1u << bit);
      z_stream t;
      memset(&t, 0, sizeof t);
      if (inflateInit2(&t, -15) == Z_OK) {
        t.next_in = body;
        t.avail_in = (uInt)bl;
        t.next_out = chk;
        t.avail_out = sizeof chk;
        const int e = inflate(&t, Z_FINISH);
        found = e == Z_STREAM_END && t.avail_in == 0 && t.total_out == n && memcmp(chk, s, n) == 0;
        inflateEnd(&t);
      }
      if (!found) body[pos] ^= (uint8_t)(1u << bit);
    }
    if (pos == 0) break;
  }
  if (!found) return -1;
  d[0] = 0x78;
  d[1] = 0x9c;
  const uint32_t a = (uint32_t)adler32(adler32(0L, Z_NULL, 0), s, (uInt)n);
  d[2 + bl] = (uint8_t)(a >> 24); d[3 + bl] = (uint8_t)(a >> 16); d[4 + bl] = (uint8_t)(a >> 8); d[5 + bl] = (uint8_t)a;
  return (long)(bl + 6);
}

typedef struct {
  int codec; const uint8_t* src; const uint64_t* src_off; uint8_t* dst; uint64_t stride; uint64_t* dst_len;
  uint64_t lo, hi; int rc;
} job_t;

static void* work(void* arg) {
  job_t* j = (job_t*)arg;
  void* zc = NULL;
  if (j->codec == 4) {
    zc = g_zcreate();
    g_zsetp(zc, 100, 3);  /* ZSTD_c_compressionLevel */
    g_zsetp(zc, 201, 1);  /* ZSTD_c_checksumFlag */
    g_zsetp(zc, 200, 1);  /* ZSTD_c_contentSizeFlag */
  }
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint8_t* s = j->src + j->src_off[i];
    size_t n = j->src_off[i + 1] - j->src_off[i];
    uint8_t* d = j->dst + i * j->stride;
    size_t cl = j->stride - 4;
    if (j->codec == 0) { memcpy(d, s, n); cl = n; }
    else if (j->codec == 3) {
      lz4f_prefs p;
      memset(&p, 0, sizeof p);
      p.blockSizeID = 7;
      p.contentChecksumFlag = 1;
      size_t r = g_lz4f(d, j->stride - 4, s, n, &p);
      if (g_lz4f_err(r)) { j->rc = -4; return NULL; }
      cl = r;
    }
    else if (j->codec == 2) {
      const long r = go_zlib6(s, n, d, j->stride - 4);
      if (r < 0) { j->rc = -6; return NULL; }
      cl = (size_t)r;
    }
    else if (j->codec == 4) {
      size_t r = g_zc2(zc, d, j->stride - 4, s, n);
      if (g_zerr(r)) { j->rc = -5; g_zfree(zc); return NULL; }
      cl = r;
    }
    else if (g_compress((const char*)s, n, (char*)d, &cl) != 0) { j->rc = -3; return NULL; }
    uint32_t c = bg_crc32(d, cl);
    d[cl] = (uint8_t)(c >> 24); d[cl + 1] = (uint8_t)(c >> 16); d[cl + 2] = (uint8_t)(c >> 8); d[cl + 3] = (uint8_t)c;
    j->dst_len[i] = cl + 4;
  }
  if (zc) g_zfree(zc);
  return NULL;
}

/* dst has n slots of `stride` bytes; dst_len receives each encoded length. */
int bg_encode_blocks(int codec, const uint8_t* src, const uint64_t* src_off, uint64_t n, uint8_t* dst,
                     uint64_t stride, uint64_t* dst_len, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pthread_t th[64];
  job_t jobs[64];
  for (int t = 0; t < nthreads; t++) {
    job_t jb = {codec, src, src_off, dst, stride, dst_len, n * t / nthreads, n * (t + 1) / nthreads, 0};
    jobs[t] = jb;
    pthread_create(&th[t], NULL, work, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
  return rc;
}

/* Decoded v0 blocks for the SURVEY 8d synthetic KVs: key i = "k%015d", value =
 * r_i || r_i (half) or r_i (84 random bytes), greedy block fill of
 * block.Builder.Add (block.go:162-182) with prefix compression against each
 * block's first key.  out receives blocks back to back (rows || BE16 offsets ||
 * BE16 count); returns the number of blocks. */
static void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

uint64_t bg_build_blocks(uint64_t kv_begin, uint64_t n_kv, const uint8_t* rv, uint32_t rv_len, int half,
                         uint64_t block_size, uint8_t* out, uint64_t* out_off, uint64_t max_blocks) {
  char first[17], key[17];
  uint32_t vlen = half ? 2 * rv_len : rv_len;
  uint64_t nb = 0, pos = 0;
  uint64_t i = 0;
  uint16_t offs[65536];
  while (i < n_kv && nb < max_blocks) {
    out_off[nb] = pos;
    uint8_t* blk = out + pos;
    uint32_t n = 0, dlen = 0;
    for (; i < n_kv; i++) {
      snprintf(key, sizeof key, "k%015llu", (unsigned long long)(kv_begin + i));
      uint32_t p = 0;
      if (n) while (p < 16 && first[p] == key[p]) p++;
      uint32_t row = 4 + (16 - p) + 9 + 4 + vlen;
      if ((uint64_t)2 + 2 * n + dlen + 2 + row > block_size && n) break;
      uint8_t* r = blk + dlen;
      put16(r, p); put16(r + 2, 16 - p);
      memcpy(r + 4, key + p, 16 - p);
      memset(r + 4 + 16 - p, 0, 9);
      uint8_t* v = r + 4 + 16 - p + 9;
      v[0] = (uint8_t)(vlen >> 24); v[1] = (uint8_t)(vlen >> 16); v[2] = (uint8_t)(vlen >> 8); v[3] = (uint8_t)vlen;
      memcpy(v + 4, rv + i * rv_len, rv_len);
      if (half) memcpy(v + 4 + rv_len, rv + i * rv_len, rv_len);
      offs[n++] = (uint16_t)dlen;
      dlen += row;
      if (n == 1) memcpy(first, key, 17);
    }
    for (uint32_t k = 0; k < n; k++) put16(blk + dlen + 2 * k, offs[k]);
    put16(blk + dlen + 2 * n, n);
    pos += dlen + 2 * n + 2;
    nb++;
  }
  out_off[nb] = pos;
  return nb;
}

/* Pack fixed-stride slots into a contiguous blob; blob_off[n] = total. */
void bg_compact(const uint8_t* slots, uint64_t stride, const uint64_t* len, uint64_t n, uint8_t* blob,
                uint64_t* blob_off) {
  uint64_t p = 0;
  for (uint64_t i = 0; i < n; i++) {
    blob_off[i] = p;
    memcpy(blob + p, slots + i * stride, len[i]);
    p += len[i];
  }
  blob_off[n] = p;
}

/* BASELINE configs[4] ("mixed") decoded blocks: ascending keys of 8-256 bytes sharing
 * 3 + (Zipf(s=1.2) - 1) bytes with the previous key (the 3-byte head absorbs carries; same
 * rule as tests/blockgen.py kv_mixed, with a splitmix64 stream and the Zipf law truncated at
 * 256), 1 KiB V-half values (r||r, 512 B halves), greedy block fill (block.go:162-182). */
static uint64_t sm64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t bg_build_mixed(uint64_t seed, uint64_t n_kv, uint64_t block_size, uint8_t* out, uint64_t* out_off,
                        uint64_t max_blocks) {
  static double cdf[257];
  double acc = 0;
  for (int k = 1; k <= 256; k++) { acc += 1.0 / __builtin_pow(k, 1.2); cdf[k] = acc; }
  uint64_t st = seed;
  uint8_t prev[256], key[256], first[256], r[512];
  uint32_t plen = 0, flen = 0;
  uint64_t nb = 0, pos = 0, i = 0;
  uint16_t offs[4096];
  uint32_t n = 0, dlen = 0;
  uint8_t* blk = out;
  out_off[0] = 0;
  while (i < n_kv && nb < max_blocks) {
    /* next key */
    uint32_t ln = 8 + (uint32_t)(sm64(&st) % 249), klen;
    if (plen == 0) {
      memcpy(key, "aaaa", 4); klen = 4;
    } else {
      double u = (double)(sm64(&st) >> 11) / 9007199254740992.0 * acc;
      int z = 1;
      while (z < 256 && cdf[z] < u) z++;
      int p = 3 + z - 1;
      if (p > (int)plen - 1) p = (int)plen - 1;
      if (p > (int)ln - 1) p = (int)ln - 1;
      memcpy(key, prev, (size_t)p + 1);
      while (key[p] >= 0xFE) p--;  /* carry left (the head starts at "aaaa") */
      key[p] = (uint8_t)(key[p] + 1 + (sm64(&st) & 1));
      klen = (uint32_t)p + 1;
    }
    while (klen < ln) key[klen++] = (uint8_t)('a' + sm64(&st) % 26);
    for (int b = 0; b < 512; b += 8) { uint64_t x = sm64(&st); memcpy(r + b, &x, 8); }
    /* block.Builder.Add */
    uint32_t p = 0;
    if (n) while (p < flen && p < klen && first[p] == key[p]) p++;
    uint32_t row = 4 + (klen - p) + 9 + 4 + 1024;
    if ((uint64_t)2 + 2 * n + dlen + 2 + row > block_size && n) {  /* finish the block, retry the key */
      for (uint32_t k = 0; k < n; k++) put16(blk + dlen + 2 * k, offs[k]);
      put16(blk + dlen + 2 * n, n);
      pos += dlen + 2 * n + 2;
      out_off[++nb] = pos;
      blk = out + pos;
      n = 0; dlen = 0;
      if (nb == max_blocks) break;
      p = 0;
      row = 4 + klen + 9 + 4 + 1024;
    }
    uint8_t* w = blk + dlen;
    put16(w, p); put16(w + 2, klen - p);
    memcpy(w + 4, key + p, klen - p);
    memset(w + 4 + klen - p, 0, 9);
    uint8_t* v = w + 4 + klen - p + 9;
    v[0] = 0; v[1] = 0; v[2] = 4; v[3] = 0;  /* BE32 1024 */
    memcpy(v + 4, r, 512); memcpy(v + 4 + 512, r, 512);
    offs[n++] = (uint16_t)dlen;
    dlen += row;
    if (n == 1) { memcpy(first, key, klen); flen = klen; }
    memcpy(prev, key, klen); plen = klen;
    i++;
  }
  if (n && nb < max_blocks) {
    for (uint32_t k = 0; k < n; k++) put16(blk + dlen + 2 * k, offs[k]);
    put16(blk + dlen + 2 * n, n);
    pos += dlen + 2 * n + 2;
    out_off[++nb] = pos;
  }
  return nb;
}

/* ---- block sets for the round-robin multi-GPU bench (BASELINE configs[1] / configs[3]) ----
 * Block i of a set is generated on its own: keys "k%015d" % (40 i + j), values r || r with r
 * 42 bytes from a splitmix64 stream seeded by (seed, i) (V-half; or 84 random bytes), greedy
 * fill of block.Builder.Add (block.go:162-182).  So a rank can build exactly its shard
 * (blocks i = i_begin + k * stride) and check its decoded output block by block. */
static uint32_t set_block(uint64_t seed, int half, uint64_t block_size, uint64_t i, uint8_t* blk, uint16_t* offs,
                          uint32_t* nrows, uint32_t* pls) {
  char first[17], key[17];
  uint64_t st = seed * 0x9E3779B97F4A7C15ull ^ (i + 1) * 0xD1B54A32D192ED03ull;
  const uint32_t rv_len = half ? 42 : 84, vlen = 84;
  uint32_t n = 0, dlen = 0;
  for (uint64_t j = 0;; j++) {
    { /* "k%015llu" */
      uint64_t x = 40 * i + j;
      key[0] = 'k';
      for (int d = 15; d >= 1; d--) { key[d] = (char)('0' + x % 10); x /= 10; }
      key[16] = 0;
    }
    uint32_t p = 0;
    if (n) while (p < 16 && first[p] == key[p]) p++;
    uint32_t row = 4 + (16 - p) + 9 + 4 + vlen;
    if ((uint64_t)2 + 2 * n + dlen + 2 + row > block_size && n) break;
    uint8_t* r = blk + dlen;
    put16(r, p); put16(r + 2, 16 - p);
    memcpy(r + 4, key + p, 16 - p);
    memset(r + 4 + 16 - p, 0, 9);
    uint8_t* v = r + 4 + 16 - p + 9;
    v[0] = 0; v[1] = 0; v[2] = 0; v[3] = (uint8_t)vlen;
    uint8_t rv[88];
    for (uint32_t b = 0; b < rv_len; b += 8) { uint64_t x = sm64(&st); memcpy(rv + b, &x, 8); }
    memcpy(v + 4, rv, rv_len);
    if (half) memcpy(v + 4 + rv_len, rv, rv_len);
    if (pls) pls[n] = p;
    offs[n++] = (uint16_t)dlen;
    dlen += row;
    if (n == 1) memcpy(first, key, 17);
  }
  for (uint32_t k = 0; k < n; k++) put16(blk + dlen + 2 * k, offs[k]);
  put16(blk + dlen + 2 * n, n);
  *nrows = n;
  return dlen + 2 * n + 2;
}

typedef struct {
  uint64_t seed; int half; uint64_t block_size, i_begin, stride, lo, hi; int codec;
  uint8_t* enc; uint64_t enc_stride; uint64_t* enc_len;
  const uint8_t* out; const uint64_t* out_off; const uint8_t* rows; const uint64_t* row_base; const uint8_t* meta;
  int64_t bad; int rc;
} set_job_t;

static void* set_build_work(void* arg) {
  set_job_t* j = (set_job_t*)arg;
  uint8_t blk[8192];
  uint16_t offs[4096];
  void* zc = NULL;
  if (j->codec == 4) {
    zc = g_zcreate();
    g_zsetp(zc, 100, 3);
    g_zsetp(zc, 201, 1);
    g_zsetp(zc, 200, 1);
  }
  for (uint64_t k = j->lo; k < j->hi; k++) {
    uint32_t nr;
    const uint32_t n = set_block(j->seed, j->half, j->block_size, j->i_begin + k * j->stride, blk, offs, &nr, NULL);
    uint8_t* d = j->enc + k * j->enc_stride;
    size_t cl = j->enc_stride - 4;
    if (j->codec == 0) { memcpy(d, blk, n); cl = n; }
    else if (j->codec == 3) {  /* pierrec/lz4 v4 writer defaults: 4 MiB blocks, content checksum */
      lz4f_prefs p;
      memset(&p, 0, sizeof p);
      p.blockSizeID = 7;
      p.contentChecksumFlag = 1;
      size_t r = g_lz4f(d, j->enc_stride - 4, blk, n, &p);
      if (g_lz4f_err(r)) { j->rc = -4; break; }
      cl = r;
    }
    else if (j->codec == 4) {
      size_t r = g_zc2(zc, d, j->enc_stride - 4, blk, n);
      if (g_zerr(r)) { j->rc = -5; break; }
      cl = r;
    } else if (g_compress((const char*)blk, n, (char*)d, &cl) != 0) { j->rc = -3; break; }
    uint32_t c = bg_crc32(d, cl);
    d[cl] = (uint8_t)(c >> 24); d[cl + 1] = (uint8_t)(c >> 16); d[cl + 2] = (uint8_t)(c >> 8); d[cl + 3] = (uint8_t)c;
    j->enc_len[k] = cl + 4;
  }
  if (zc) g_zfree(zc);
  return NULL;
}

/* Encoded blocks k = 0..count-1 of the set (global index i_begin + k * stride) into fixed slots
 * of enc_stride bytes (codec 0 None, 1 Snappy via libsnappy, 3 LZ4 frames via liblz4, 4 Zstd), lengths in enc_len. */
int bg_build_set(uint64_t seed, int half, uint64_t block_size, uint64_t i_begin, uint64_t stride, uint64_t count,
                 int codec, uint8_t* enc, uint64_t enc_stride, uint64_t* enc_len, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  if (block_size > 8000) return -6;
  pthread_t th[64];
  set_job_t jobs[64];
  for (int t = 0; t < nthreads; t++) {
    set_job_t jb = {seed, half, block_size, i_begin, stride, count * t / nthreads, count * (t + 1) / nthreads, codec,
                    enc, enc_stride, enc_len, NULL, NULL, NULL, NULL, NULL, 0, 0};
    jobs[t] = jb;
    pthread_create(&th[t], NULL, set_build_work, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
  return rc;
}

static void* set_verify_work(void* arg) {
  set_job_t* j = (set_job_t*)arg;
  uint8_t blk[8192];
  uint16_t offs[4096];
  uint32_t pls[4096];
  for (uint64_t k = j->lo; k < j->hi; k++) {
    uint32_t nr;
    const uint32_t n = set_block(j->seed, j->half, j->block_size, j->i_begin + k * j->stride, blk, offs, &nr, pls);
    const uint32_t data_len = n - 2 * nr - 2;
    int ok = j->out_off[k + 1] - j->out_off[k] >= n && memcmp(j->out + j->out_off[k], blk, n) == 0;
    /* slate_block_meta {i16 status, u16 flags, i32 detail, u32 data_len, u16 n_rows, u16 aux} */
    const uint8_t* m = j->meta + 16 * k;
    uint32_t dl; uint16_t nrow, st, fl, aux; int32_t det;
    memcpy(&st, m, 2); memcpy(&fl, m + 2, 2); memcpy(&det, m + 4, 4); memcpy(&dl, m + 8, 4);
    memcpy(&nrow, m + 12, 2); memcpy(&aux, m + 14, 2);
    ok = ok && st == 0 && fl == 0 && dl == data_len && nrow == nr && aux == 0;
    /* slate_row {u32 row_off, u16 prefix, u16 suffix, u32 value_len, u8 flags, u8 meta_len, i16 status} */
    ok = ok && j->row_base[k + 1] - j->row_base[k] >= nr;
    for (uint32_t r = 0; ok && r < nr; r++) {
      const uint8_t* d = j->rows + 16 * (j->row_base[k] + r);
      uint32_t ro, vl; uint16_t pl, sl, rst;
      memcpy(&ro, d, 4); memcpy(&pl, d + 4, 2); memcpy(&sl, d + 6, 2); memcpy(&vl, d + 8, 4); memcpy(&rst, d + 14, 2);
      ok = ro == offs[r] && pl == pls[r] && sl == 16 - pls[r] && vl == 84 && d[12] == 0 && d[13] == 13 && rst == 0;
    }
    if (!ok) j->bad++;
  }
  return NULL;
}

/* Decoded outputs of blocks k = 0..count-1 (decode kernel layout: bytes at out + out_off[k],
 * row descriptors at rows + 16 row_base[k], meta 16 B each) against the generator: returns
 * the number of blocks whose bytes, meta or rows differ. */
int64_t bg_verify_set(uint64_t seed, int half, uint64_t block_size, uint64_t i_begin, uint64_t stride, uint64_t count,
                      const uint8_t* out, const uint64_t* out_off, const uint8_t* rows, const uint64_t* row_base,
                      const uint8_t* meta, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  if (block_size > 8000) return -1;
  pthread_t th[64];
  set_job_t jobs[64];
  for (int t = 0; t < nthreads; t++) {
    set_job_t jb = {seed, half, block_size, i_begin, stride, count * t / nthreads, count * (t + 1) / nthreads, 0,
                    NULL, 0, NULL, out, out_off, rows, row_base, meta, 0, 0};
    jobs[t] = jb;
    pthread_create(&th[t], NULL, set_verify_work, &jobs[t]);
  }
  int64_t bad = 0;
  for (int t = 0; t < nthreads; t++) { pthread_join(th[t], NULL); bad += jobs[t].bad; }
  return bad;
}

/* Blocks whose decoded bytes (out[out_off[i] ..], dec_off[i+1] - dec_off[i] bytes) differ from the
 * blocks before encoding (dec[dec_off[i] ..]): bench.py's configs[4] check. */
int64_t bg_compare_blocks(const uint8_t* out, const uint64_t* out_off, const uint8_t* dec, const uint64_t* dec_off,
                          uint64_t n) {
  int64_t bad = 0;
  for (uint64_t i = 0; i < n; i++)
    if (memcmp(out + out_off[i], dec + dec_off[i], dec_off[i + 1] - dec_off[i]) != 0) bad++;
  return bad;
}
