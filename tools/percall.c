/* Per-call latency of the single-block entry points from C, the way a cgo shim calls them
 * (tooling for bench.py's per_call leg; tools/percall_bench.py writes the input file):
 *   slate_block_decode  (block.Decode, internal/sstable/block/block.go:78) against the oracle's
 *                       or_block_decode (CPU baseline, one thread), same blocks, same order;
 *   slate_block_seek    (block.NewIteratorAtKey) over one decoded block against or_block_seek;
 *   slate_block_reader  (sstable.Iterator.nextBlockIter, iterator.go:92-118, with read-ahead) over
 *                       every block of one Snappy SST: us per block, the caller's loop as a cgo shim
 *                       runs it (next; on NEED_DATA want + the range's bytes + feed), the object
 *                       store's GetRange standing in as a pointer into the SST in memory.
 * Input file: u32 n, n x (u32 len, bytes) Snappy blocks, then u32 klen, key bytes (a key of block 0),
 * then (optional) u64 sst_len, the SST's bytes, u32 read_ahead.
 * usage: percall FILE CALLS   -> one JSON object on stdout */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "slatecodec.h"
#include "slate_oracle.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static uint32_t rd32(FILE* f) {
  uint32_t v = 0;
  if (fread(&v, 4, 1, f) != 1) exit(2);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int calls = atoi(argv[2]);
  const uint32_t n = rd32(f);
  uint8_t** blk = malloc(n * sizeof(uint8_t*));
  uint32_t* len = malloc(n * 4);
  for (uint32_t i = 0; i < n; i++) {
    len[i] = rd32(f);
    blk[i] = malloc(len[i] + 16);
    if (fread(blk[i], 1, len[i], f) != len[i]) return 2;
  }
  const uint32_t klen = rd32(f);
  uint8_t* key = malloc(klen + 1);
  if (fread(key, 1, klen, f) != klen) return 2;
  uint64_t sst_len = 0;
  uint8_t* sst = NULL;
  uint32_t ahead = 64;
  if (fread(&sst_len, 8, 1, f) == 1 && sst_len) {
    sst = malloc(sst_len);
    if (fread(sst, 1, sst_len, f) != sst_len) return 2;
    ahead = rd32(f);
  }
  fclose(f);

  int st = 0;
  slate_ctx* ctx = slate_ctx_create(0, &st);
  if (!ctx) return 3;
  const size_t cap = 1 << 20;
  uint8_t* out = malloc(cap);
  uint16_t* offs = malloc(cap);
  or_row* rows = malloc(sizeof(or_row) * 70000);
  slate_block_meta m;
  or_block_meta om;
  size_t ol = 0;

  /* block.Decode, one block per call */
  for (int w = 0; w < 20; w++) slate_block_decode(ctx, 1, blk[w % n], len[w % n], out, cap, &ol, &m, offs, cap / 2);
  double t0 = now_us();
  for (int c = 0; c < calls; c++) {
    st = slate_block_decode(ctx, 1, blk[c % n], len[c % n], out, cap, &ol, &m, offs, cap / 2);
    if (st) return 4;
  }
  const double gpu_dec = (now_us() - t0) / calls;
  if (getenv("PERCALL_DECODE_ONLY")) { /* tools/onestop.sh: profiling library, phases cut short */
    printf("{\"calls\": %d, \"slate_block_decode_us\": %.2f}\n", calls, gpu_dec);
    return 0;
  }
  t0 = now_us();
  for (int c = 0; c < calls; c++) {
    st = or_block_decode(blk[c % n], len[c % n], 1, out, cap, &ol, &om, rows, 70000);
    if (st) return 5;
  }
  const double cpu_dec = (now_us() - t0) / calls;

  /* block.NewIteratorAtKey over block 0 */
  st = slate_block_decode(ctx, 1, blk[0], len[0], out, cap, &ol, &m, offs, cap / 2);
  if (st) return 6;
  uint64_t out_off[2] = {0, (ol + 15) & ~(uint64_t)15};
  uint32_t qb = 0;
  uint64_t key_off[2] = {0, klen};
  slate_seek res;
  for (int w = 0; w < 20; w++) slate_block_seek(ctx, out, out_off, &m, 1, &qb, key, key_off, 1, &res);
  t0 = now_us();
  for (int c = 0; c < calls; c++) {
    st = slate_block_seek(ctx, out, out_off, &m, 1, &qb, key, key_off, 1, &res);
    if (st || res.status) return 7;
  }
  const double gpu_seek = (now_us() - t0) / calls;
  uint32_t s0, fl, nw;
  int32_t fi;
  t0 = now_us();
  for (int c = 0; c < calls; c++) {
    st = or_block_seek(out, m.data_len, offs, m.n_rows, key, klen, &s0, &fi, &fl, &nw);
    if (st) return 8;
  }
  const double cpu_seek = (now_us() - t0) / calls;
  if (s0 != res.start || fi != res.first_idx) return 9;
  /* sstable.Iterator over one SST through the read-ahead reader: every block, in order */
  double reader_us = -1.0, reader_oracle_us = -1.0;
  uint64_t reader_blocks = 0, reader_rows = 0;
  if (sst) {
    slate_sst_info info;
    slate_index* index = NULL;
    uint8_t* fk = malloc(sst_len);
    if (slate_sst_read_info(sst, sst_len, &info, fk, sst_len)) return 10;
    free(fk);
    if (slate_decode_index(ctx, sst + info.index_offset, info.index_len, info.codec, &index)) return 11;
    const uint64_t nb = slate_index_num_blocks(index);
    double best = 1e30;
    for (int pass = 0; pass < 6; pass++) { /* pass 0 warms up (staging allocations, code objects) */
      slate_block_reader* r = NULL;
      if (slate_block_reader_create(ctx, &info, index, 0, ahead, &r)) return 12;
      uint64_t got = 0, rows = 0;
      const double t = now_us();
      for (;;) {
        slate_block_view v;
        st = slate_block_reader_next(r, &v);
        if (st == SLATE_E_READER_END) break;
        if (st == SLATE_E_READER_NEED_DATA) {
          uint64_t rs, re;
          if (slate_block_reader_want(r, &rs, &re)) return 13;
          if (slate_block_reader_feed(r, sst + rs, re - rs)) return 14;
          continue;
        }
        if (st || v.block != got) return 15;
        rows += v.meta.n_rows; /* the caller reads the block: its meta and rows */
        got++;
      }
      const double us = (now_us() - t) / (double)nb;
      slate_block_reader_free(r);
      if (got != nb) return 16;
      if (pass && us < best) best = us;
      reader_rows = rows;
    }
    reader_us = best;
    reader_blocks = nb;
    /* the oracle: the same blocks, one thread, block.Decode per block (what nextBlockIter calls) */
    uint64_t* offs = malloc(8 * (nb + 1));
    if (slate_index_block_offsets(index, offs, nb)) return 17;
    offs[nb] = info.filter_offset;
    t0 = now_us();
    for (uint64_t b = 0; b < nb; b++) {
      st = or_block_decode(sst + offs[b], offs[b + 1] - offs[b], info.codec, out, cap, &ol, &om, rows, 70000);
      if (st || om.status) return 18;
    }
    reader_oracle_us = (now_us() - t0) / (double)nb;
    free(offs);
    slate_index_free(index);
  }
  printf("{\"calls\": %d, \"slate_block_decode_us\": %.2f, \"oracle_block_decode_us_1thread\": %.2f, "
         "\"slate_block_seek_us\": %.2f, \"oracle_block_seek_us_1thread\": %.2f, "
         "\"reader_blocks\": %llu, \"reader_rows\": %llu, \"reader_read_ahead\": %u, "
         "\"slate_block_reader_us_per_block\": %.3f, \"oracle_block_decode_us_per_block_1thread\": %.3f}\n",
         calls, gpu_dec, cpu_dec, gpu_seek, cpu_seek, (unsigned long long)reader_blocks,
         (unsigned long long)reader_rows, ahead, reader_us, reader_oracle_us);
  slate_ctx_destroy(ctx);
  return 0;
}
