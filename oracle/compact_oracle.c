/*
 * compact_oracle.c — TEST INFRASTRUCTURE ONLY (see slate_oracle.h).
 *
 * executeCompaction's codec path (slatedb/compaction/executor.go:92-151) restated in C over clean
 * inputs, for bench.py's compaction leg (CPU baseline) and tests/test_compaction_gpu.py:
 *   - loadIterators (executor.go:49-90): one sstable.Iterator per input SST, sources in precedence
 *     order; each reads ReadInfo / ReadIndex (decode.go:25-83) and every data block through
 *     block.Decode (block.go:78-134), walking rows as block.Iterator does (block/iterator.go:84-107:
 *     row 0's suffix is the first key, later rows are firstKey[:prefixLen] || suffix, row.go:72-79);
 *   - iter.MergeSort over the sources (internal/iter/merge.go:12-111: or_merge_sort);
 *   - the writer loop: EncodedSSTableWriter.Add = Builder.AddValue (store/table_store.go:221-223,
 *     builder.go:149), a new output after the entry that takes the running key + value size past
 *     MaxSSTSize (executor.go:119-139), the last one when any size is left (:141-148).
 * nthreads > 1 decodes the blocks and builds the output SSTs on that many threads (the merge stays
 * serial, as Go's heap is); the cut points depend only on the merged sizes, so the outputs are the
 * same bytes either way.  Corrupt inputs are not handled here (tests/compactgen.py has Go's
 * warning semantics): a failing block or row returns its status.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "slate_oracle.h"

typedef struct {
  const uint8_t* blk;  /* encoded block */
  size_t len;
  int codec;
  uint64_t kv0;        /* index of the block's first row among all rows */
  uint32_t n_rows;
  uint8_t* out;        /* pass 0 -> 1: the decoded block and its row descriptors */
  or_row* rows;
} cblock;

typedef struct {
  cblock* b;
  uint32_t n;
  uint8_t* keys;       /* full keys, all rows */
  uint64_t* key_off;
  uint8_t* vals;       /* values, all rows (value_len bytes; tombstones: none) */
  uint64_t* val_off;
  uint8_t* tomb;
  uint64_t* kvoff;     /* per block: its first key byte / value byte (prefix sums of the sizes) */
  uint64_t* vvoff;
  int status;
  uint32_t next;       /* work queue */
  pthread_mutex_t mu;
} cdecode;

/* pass 0: one block decoded (kept for pass 1), its row count and key / value bytes;
 * pass 1: its rows' full keys and values at their places */
static int decode_one(cdecode* D, uint32_t i, int pass) {
  cblock* c = &D->b[i];
  int st = OR_OK;
  if (pass == 0) {
    uint64_t dl = 0;
    if (c->len < 6 || or_decompress_len(c->codec, c->blk, c->len - 4, &dl)) dl = c->len;
    c->out = (uint8_t*)malloc(dl + 16);
    const size_t rc = or_row_capacity(dl) + 1;
    c->rows = (or_row*)malloc(sizeof(or_row) * rc);
    size_t ol = 0;
    or_block_meta m;
    st = or_block_decode(c->blk, c->len, c->codec, c->out, dl + 16, &ol, &m, c->rows, rc);
    if (!st) st = m.status;
    uint64_t kb = 0, vb = 0;
    for (uint32_t r = 0; !st && r < m.n_rows; r++) {
      if (c->rows[r].status) st = c->rows[r].status;
      kb += r == 0 ? c->rows[r].key_suffix_len : (uint64_t)c->rows[r].key_prefix_len + c->rows[r].key_suffix_len;
      vb += (c->rows[r].flags & 1) ? 0 : c->rows[r].value_len;
    }
    c->n_rows = st ? 0 : m.n_rows;
    D->kvoff[i] = kb;
    D->vvoff[i] = vb;
    return st;
  }
  uint64_t kv = c->kv0, ko = D->kvoff[i], vo = D->vvoff[i];
  const uint8_t* fk = NULL;
  size_t fkl = 0;
  for (uint32_t r = 0; r < c->n_rows; r++) {
    const or_row* w = &c->rows[r];
    const uint8_t* sfx = c->out + w->row_off + 4;
    D->key_off[kv] = ko;
    if (r == 0) {
      memcpy(D->keys + ko, sfx, w->key_suffix_len);
      fk = D->keys + ko;
      fkl = w->key_suffix_len;
      ko += w->key_suffix_len;
    } else {
      if (w->key_prefix_len > fkl) {
        st = OR_E_ROW_PREFIX;
        break;
      }
      memcpy(D->keys + ko, fk, w->key_prefix_len);
      memcpy(D->keys + ko + w->key_prefix_len, sfx, w->key_suffix_len);
      ko += (uint64_t)w->key_prefix_len + w->key_suffix_len;
    }
    D->val_off[kv] = vo;
    D->tomb[kv] = w->flags & 1;
    if (!(w->flags & 1)) {
      memcpy(D->vals + vo, c->out + w->row_off + 4 + w->key_suffix_len + w->meta_len, w->value_len);
      vo += w->value_len;
    }
    kv++;
  }
  free(c->out);
  free(c->rows);
  c->out = NULL;
  c->rows = NULL;
  return st;
}

typedef struct { cdecode* D; int pass; } cjob;

static void* decode_worker(void* arg) {
  cjob* j = (cjob*)arg;
  cdecode* D = j->D;
  for (;;) {
    pthread_mutex_lock(&D->mu);
    uint32_t i = D->next < D->n ? D->next++ : D->n;
    pthread_mutex_unlock(&D->mu);
    if (i >= D->n) break;
    int st = decode_one(D, i, j->pass);
    if (st) {
      pthread_mutex_lock(&D->mu);
      if (!D->status) D->status = st;
      pthread_mutex_unlock(&D->mu);
    }
  }
  return NULL;
}

static int run_pass(cdecode* D, int pass, int nthreads) {
  D->next = 0;
  cjob j = {D, pass};
  if (nthreads <= 1) {
    decode_worker(&j);
    return D->status;
  }
  pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int k = 0; k < nthreads; k++) pthread_create(&t[k], NULL, decode_worker, &j);
  for (int k = 0; k < nthreads; k++) pthread_join(t[k], NULL);
  free(t);
  return D->status;
}

typedef struct {
  const cdecode* D;
  const uint32_t* idx;  /* merged order */
  const uint64_t* cut;  /* output o = merged entries [cut[o], cut[o+1]) */
  uint32_t n_out, next;
  uint64_t block_size;
  int codec;
  uint8_t** enc;        /* per output: its encoded bytes */
  size_t* enc_len;
  int status;
  pthread_mutex_t mu;
} cbuild;

static int build_one(cbuild* B, uint32_t o) {
  const cdecode* D = B->D;
  or_sst_builder* w = or_sst_builder_new(B->block_size, 0, 10, B->codec);
  int st = OR_OK;
  for (uint64_t e = B->cut[o]; e < B->cut[o + 1] && !st; e++) {
    const uint32_t i = B->idx[e];
    const uint8_t* k = D->keys + D->key_off[i];
    const size_t kl = D->key_off[i + 1] - D->key_off[i];
    const size_t vl = D->val_off[i + 1] - D->val_off[i];
    st = or_sst_builder_add_value(w, k, kl, D->vals + D->val_off[i], D->tomb[i] ? 0 : vl);
  }
  if (!st) st = or_sst_builder_build(w);
  if (!st) {
    size_t n = or_sst_table_encoded_len(w);
    B->enc[o] = (uint8_t*)malloc(n ? n : 1);
    B->enc_len[o] = n;
    st = or_sst_table_encode(w, B->enc[o], n);
  }
  or_sst_builder_free(w);
  return st;
}

static void* build_worker(void* arg) {
  cbuild* B = (cbuild*)arg;
  for (;;) {
    pthread_mutex_lock(&B->mu);
    uint32_t o = B->next < B->n_out ? B->next++ : B->n_out;
    pthread_mutex_unlock(&B->mu);
    if (o >= B->n_out) break;
    int st = build_one(B, o);
    if (st) {
      pthread_mutex_lock(&B->mu);
      if (!B->status) B->status = st;
      pthread_mutex_unlock(&B->mu);
    }
  }
  return NULL;
}

int or_compact(const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst, const uint32_t* src_sst, uint32_t n_src,
               uint64_t block_size, int codec, uint64_t max_sst_size, int nthreads, uint8_t* out, uint64_t cap,
               uint64_t* out_off, uint32_t out_off_cap, uint32_t* n_out) {
  *n_out = 0;
  if (nthreads < 1) nthreads = 1;
  /* the blocks of every SST (ReadInfo, ReadIndex, getBlockRange) */
  uint32_t nb = 0, bcap = 1024;
  cblock* b = (cblock*)malloc(sizeof(cblock) * bcap);
  uint64_t* blocks_src = NULL;  /* per source: its first block */
  blocks_src = (uint64_t*)calloc(n_src + 1, sizeof(uint64_t));
  int st = OR_OK;
  for (uint32_t s = 0; s < n_src && !st; s++) {
    blocks_src[s] = nb;
    for (uint32_t t = src_sst[s]; t < src_sst[s + 1] && !st; t++) {
      const uint8_t* sst = ssts + sst_off[t];
      const size_t len = sst_off[t + 1] - sst_off[t];
      or_sst_info info;
      uint8_t* fk = (uint8_t*)malloc(len + 1);  /* Info.FirstKey (not needed here, but decoded) */
      st = or_sst_read_info(sst, len, &info, fk, len);
      free(fk);
      if (st) break;
      size_t mcap = len / 6 + 2, kcap = 1 << 16, n = 0;
      uint64_t *offs = NULL, *koff = NULL;
      uint8_t* keys = NULL;
      for (;;) {
        offs = (uint64_t*)realloc(offs, sizeof(uint64_t) * (mcap + 1));
        koff = (uint64_t*)realloc(koff, sizeof(uint64_t) * (mcap + 1));
        keys = (uint8_t*)realloc(keys, kcap);
        st = or_decode_index(sst + info.index_offset, info.index_len, info.codec, offs, keys, koff, mcap, kcap, &n);
        if (st != OR_E_CAPACITY) break;
        kcap *= 4;
      }
      if (!st) {
        for (size_t i = 0; i < n; i++) {
          if (nb == bcap) b = (cblock*)realloc(b, sizeof(cblock) * (bcap *= 2));
          const uint64_t e = i + 1 < n ? offs[i + 1] : info.filter_offset;
          b[nb].blk = sst + offs[i];
          b[nb].len = e - offs[i];
          b[nb].codec = info.codec;
          b[nb].n_rows = 0;
          b[nb].out = NULL;
          b[nb].rows = NULL;
          nb++;
        }
      }
      free(offs);
      free(koff);
      free(keys);
    }
  }
  blocks_src[n_src] = nb;
  cdecode D;
  memset(&D, 0, sizeof(D));
  pthread_mutex_init(&D.mu, NULL);
  D.b = b;
  D.n = nb;
  D.kvoff = (uint64_t*)calloc(nb + 1, sizeof(uint64_t));
  D.vvoff = (uint64_t*)calloc(nb + 1, sizeof(uint64_t));
  if (!st) st = run_pass(&D, 0, nthreads);  /* row counts and key / value sizes per block */
  uint64_t nkv = 0, kb = 0, vb = 0;
  if (!st) {
    for (uint32_t i = 0; i < nb; i++) {  /* exclusive scans */
      const uint64_t k = D.kvoff[i], v = D.vvoff[i];
      b[i].kv0 = nkv;
      D.kvoff[i] = kb;
      D.vvoff[i] = vb;
      nkv += b[i].n_rows;
      kb += k;
      vb += v;
    }
    D.keys = (uint8_t*)malloc(kb + 1);
    D.vals = (uint8_t*)malloc(vb + 1);
    D.key_off = (uint64_t*)malloc(sizeof(uint64_t) * (nkv + 1));
    D.val_off = (uint64_t*)malloc(sizeof(uint64_t) * (nkv + 1));
    D.tomb = (uint8_t*)malloc(nkv + 1);
    st = run_pass(&D, 1, nthreads);
    D.key_off[nkv] = kb;
    D.val_off[nkv] = vb;
  }
  uint32_t* idx = NULL;
  uint64_t nm = 0;
  if (!st) {
    uint64_t* src_start = (uint64_t*)malloc(sizeof(uint64_t) * (n_src + 1));
    for (uint32_t s = 0; s <= n_src; s++) src_start[s] = blocks_src[s] < nb ? b[blocks_src[s]].kv0 : nkv;
    idx = (uint32_t*)malloc(sizeof(uint32_t) * (nkv + 1));
    st = or_merge_sort(n_src, D.keys, D.key_off, src_start, idx, &nm);
    free(src_start);
  }
  /* the writer loop's cuts (executor.go:119-148) */
  uint64_t* cut = NULL;
  uint32_t no = 0;
  if (!st) {
    cut = (uint64_t*)malloc(sizeof(uint64_t) * (nm + 2));
    cut[0] = 0;
    uint64_t size = 0;
    for (uint64_t e = 0; e < nm; e++) {
      const uint32_t i = idx[e];
      size += (D.key_off[i + 1] - D.key_off[i]) + (D.tomb[i] ? 0 : D.val_off[i + 1] - D.val_off[i]);
      if (size > max_sst_size) {
        size = 0;
        cut[++no] = e + 1;
      }
    }
    if (size > 0) cut[++no] = nm;
  }
  if (!st) {
    cbuild B;
    memset(&B, 0, sizeof(B));
    pthread_mutex_init(&B.mu, NULL);
    B.D = &D;
    B.idx = idx;
    B.cut = cut;
    B.n_out = no;
    B.block_size = block_size;
    B.codec = codec;
    B.enc = (uint8_t**)calloc(no + 1, sizeof(uint8_t*));
    B.enc_len = (size_t*)calloc(no + 1, sizeof(size_t));
    if (nthreads <= 1 || no <= 1) {
      build_worker(&B);
    } else {
      const int nt = nthreads < (int)no ? nthreads : (int)no;
      pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * nt);
      for (int k = 0; k < nt; k++) pthread_create(&t[k], NULL, build_worker, &B);
      for (int k = 0; k < nt; k++) pthread_join(t[k], NULL);
      free(t);
    }
    st = B.status;
    uint64_t at = 0;
    if (!st && no + 1 > out_off_cap) st = OR_E_CAPACITY;
    for (uint32_t o = 0; o < no && !st; o++) {
      out_off[o] = at;
      if (at + B.enc_len[o] > cap) st = OR_E_CAPACITY;
      else memcpy(out + at, B.enc[o], B.enc_len[o]);
      at += B.enc_len[o];
    }
    if (!st) {
      out_off[no] = at;
      *n_out = no;
    }
    for (uint32_t o = 0; o < no; o++) free(B.enc[o]);
    free(B.enc);
    free(B.enc_len);
    pthread_mutex_destroy(&B.mu);
  }
  free(cut);
  free(idx);
  free(D.keys);
  free(D.vals);
  free(D.key_off);
  free(D.val_off);
  free(D.tomb);
  free(D.kvoff);
  free(D.vvoff);
  pthread_mutex_destroy(&D.mu);
  for (uint32_t i = 0; i < nb; i++) {
    free(b[i].out);
    free(b[i].rows);
  }
  free(b);
  free(blocks_src);
  return st;
}
