/*
 * slate_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the slatedb-go SST block-codec path (plain C), used as the
 * parity checker for the HIP product library and as bench.py's cpu_baseline.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product (slatedb-go_amd/, include/) never links or calls it.
 *
 * Pinning: the Go reference cannot be built here (no Go toolchain, module cache or
 * network), so this restatement is pinned by the reference's own known-answer
 * tests (tests/golden/reference_vectors.json) and cross-checked against an
 * independent Python restatement (oracle/pyoracle.py).  Third-party arithmetic it
 * restates: golang/snappy v0.0.4 (go.mod:7) block format encoder/decoder,
 * google/flatbuffers v24.3.25 Go builder (go.mod:8), Go stdlib hash/crc32 (IEEE)
 * and hash/fnv (FNV-1 64).  Snappy *encoded* bytes and flatbuffer index/info bytes
 * are "parity unpinned" with respect to Go itself (reference tests only round-trip
 * them); see DESIGN.md §Oracle.
 *
 * Status codes deliberately duplicate include/slatecodec.h's values (checked by
 * tests/test_oracle.py::test_status_strings_match).
 */
#ifndef SLATE_ORACLE_H
#define SLATE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OR_OK = 0,
  OR_E_BLOCK_TOO_SMALL = 1, OR_E_BLOCK_CHECKSUM = 2, OR_E_BLOCK_UNCOMP_SMALL = 3,
  OR_E_BLOCK_INDEX_OFFSET = 4, OR_E_BLOCK_OFFSET_BOUNDS = 5, OR_E_BLOCK_NO_OFFSETS = 6,
  OR_E_BLOCK_FIRSTKEY_PANIC = 7, OR_E_BLOCK_EMPTY = 8,
  OR_E_INVALID_CODEC = 10, OR_E_SNAPPY_CORRUPT = 11, OR_E_SNAPPY_TOO_LARGE = 12,
  OR_E_CODEC_UNSUPPORTED = 13,
  OR_E_LZ4_MAGIC = 14, OR_E_LZ4_HEADER_CHECKSUM = 15, OR_E_LZ4_BLOCK_CHECKSUM = 16,
  OR_E_LZ4_FRAME_CHECKSUM = 17, OR_E_LZ4_CORRUPT = 18,
  OR_E_ROW_TOO_SHORT = 20, OR_E_ROW_PREFIX = 21, OR_E_ROW_SUFFIX = 22, OR_E_ROW_EXPIRE = 23,
  OR_E_ROW_CREATE = 24, OR_E_ROW_VALUE_LEN = 25, OR_E_ROW_VALUE = 26, OR_E_ROW_PANIC = 27,
  OR_E_ROW_PEEK_SHORT = 28, OR_E_ROW_OFFSET_RANGE = 29,
  OR_E_FILTER_TOO_SMALL = 30, OR_E_FILTER_CHECKSUM = 31, OR_E_FILTER_PANIC = 32,
  OR_E_INDEX_TOO_SHORT = 40, OR_E_INDEX_CHECKSUM = 41, OR_E_INFO_TOO_SHORT = 42,
  OR_E_INFO_CHECKSUM = 43, OR_E_SST_TOO_SHORT = 44, OR_E_BLOB_RANGE = 45,
  OR_E_RANGE_START = 46, OR_E_RANGE_END = 47, OR_E_FLATBUF = 48,
  OR_E_ZLIB_HEADER = 50, OR_E_ZLIB_DICTIONARY = 51, OR_E_ZLIB_CHECKSUM = 52, OR_E_FLATE_CORRUPT = 53,
  OR_E_UNEXPECTED_EOF = 54, OR_E_EOF = 55,
  OR_E_ZSTD_MAGIC = 56, OR_E_ZSTD_CHECKSUM = 57, OR_E_ZSTD_CORRUPT = 58, OR_E_ZSTD_FRAME_SIZE = 59,
  OR_E_ZSTD_DICT = 60, OR_E_ZSTD_RESERVED_BLOCK = 61,
  OR_E_SEEK_NO_OFFSETS = 62, OR_E_SEEK_NO_FULL_KEY = 63, OR_E_SEEK_PANIC = 64,
  OR_E_INVALID_ARG = 102, OR_E_CAPACITY = 103, OR_E_OOM = 104,
};

enum { OR_CODEC_NONE = 0, OR_CODEC_SNAPPY = 1, OR_CODEC_ZLIB = 2, OR_CODEC_LZ4 = 3, OR_CODEC_ZSTD = 4 };

/* Same layouts as slate_block_meta / slate_row (16 bytes each). */
typedef struct or_block_meta {
  int16_t status; uint16_t flags; int32_t detail; uint32_t data_len; uint16_t n_rows; uint16_t aux;
} or_block_meta;
typedef struct or_row {
  uint32_t row_off; uint16_t key_prefix_len; uint16_t key_suffix_len; uint32_t value_len;
  uint8_t flags; uint8_t meta_len; int16_t status;
} or_row;

const char* or_status_string(int status);

/* hashes */
uint32_t or_crc32(const uint8_t* p, size_t n);            /* hash/crc32.ChecksumIEEE */
uint64_t or_fnv1_64(const uint8_t* p, size_t n);          /* bloom.go:141 filterHash */
uint16_t or_compute_prefix_len(const uint8_t* a, size_t an, const uint8_t* b, size_t bn); /* row.go:292 */

/* golang/snappy v0.0.4 block format */
size_t or_snappy_max_encoded_len(size_t n);
size_t or_snappy_encode(const uint8_t* src, size_t n, uint8_t* dst);
int or_snappy_decoded_len(const uint8_t* src, size_t n, uint64_t* dlen, int* hdr);
int or_snappy_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_len);

/* compress.Encode/Decode (compression.go:80,126); out must hold the result.
 * Decode writes *out_len; for NONE it copies. */
int or_compress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
uint32_t or_xxh32(const uint8_t* p, size_t n, uint32_t seed);
int or_lz4_frame_len(const uint8_t* in, size_t n, uint64_t* dlen);
int or_lz4_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
int or_zlib_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
uint64_t or_xxh64(const uint8_t* p, size_t n, uint64_t seed);
int or_zstd_plan(const uint8_t* in, size_t n, uint64_t* dlen);   /* zstd_oracle.c */
int or_zstd_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
int or_decompress_len(int codec, const uint8_t* in, size_t n, uint64_t* dlen);
int or_decompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* v0 row codec (row.go) */
typedef struct or_row_value {
  uint16_t key_prefix_len; const uint8_t* key_suffix; size_t key_suffix_len; uint64_t seq;
  int tombstone; int has_expire; int64_t expire_ms; int has_create; int64_t create_ms;
  const uint8_t* value; size_t value_len;
} or_row_value;
size_t or_v0_size(const or_row_value* r);                                 /* row.go:95 */
size_t or_v0_encode(const or_row_value* r, uint8_t* out);                 /* row.go:149 */
/* row.go:191 Decode.  first_key_len < 0 means firstKey == nil.  On success fills r
 * (pointers into data). */
int or_v0_decode(const uint8_t* data, size_t n, long first_key_len, or_row_value* r);
int or_v0_peek(const uint8_t* data, size_t n, long first_key_len, uint16_t* prefix_len,
               uint16_t* suffix_len);                                     /* row.go:265 */
uint64_t or_v0_estimate_block_size(const uint8_t* keys, const uint64_t* key_off,
                                   const uint8_t* vals, const uint64_t* val_off, size_t n); /* row.go:50 */

/* block.Builder (block.go:136-204) */
typedef struct or_block_builder or_block_builder;
or_block_builder* or_block_builder_new(uint64_t block_size);
void or_block_builder_free(or_block_builder* b);
int or_block_builder_add(or_block_builder* b, const uint8_t* key, size_t klen, int tombstone,
                         const uint8_t* value, size_t vlen);                  /* block.go:162 */
int or_block_builder_add_value(or_block_builder* b, const uint8_t* key, size_t klen,
                               const uint8_t* value, size_t vlen);            /* block.go:184 */
int or_block_builder_is_empty(const or_block_builder* b);
size_t or_block_builder_data(const or_block_builder* b, const uint8_t** data);
size_t or_block_builder_offsets(const or_block_builder* b, const uint16_t** offsets);
size_t or_block_builder_first_key(const or_block_builder* b, const uint8_t** key);
void or_block_builder_reset(or_block_builder* b);

/* block.Encode (block.go:54): *out_len = bytes written (cap must be >= bound). */
size_t or_block_encode_bound(size_t data_len, size_t n_offsets);
int or_block_encode(const uint8_t* data, size_t data_len, const uint16_t* offsets, size_t n,
                    int codec, uint8_t* out, size_t cap, size_t* out_len);
/* block.Decode (block.go:78) + per-row v0 decode the way block.Iterator walks the
 * block.  out receives the decoded buffer (rows||offsets||count), *out_len its
 * length; rows[] receives min(n_rows, rows_cap) descriptors. */
int or_block_decode(const uint8_t* in, size_t n, int codec, uint8_t* out, size_t cap,
                    size_t* out_len, or_block_meta* meta, or_row* rows, size_t rows_cap);
/* Batch helper for the cpu baseline: nthreads workers over n blocks, same layout as
 * slate_block_decode_batch (out_off/row_base are outputs). */
int or_block_decode_batch(int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                          uint8_t* out, uint64_t out_cap, uint64_t* out_off, or_block_meta* meta,
                          or_row* rows, uint64_t rows_cap, uint64_t* row_base, int nthreads);
uint64_t or_row_capacity(uint64_t decoded_len);

/* bloom (bloom.go) */
uint16_t or_bloom_optimal_num_probes(uint32_t bits_per_key);             /* bloom.go:174 */
uint64_t or_bloom_filter_bytes(uint32_t num_keys, uint32_t bits_per_key); /* bloom.go:135 */
void or_bloom_probes(uint64_t hash, uint16_t num_probes, uint32_t filter_bits, uint32_t* probes);
/* Build from keys; bits must hold or_bloom_filter_bytes(n, bpk).  n == 0 => empty. */
int or_bloom_build(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t bits_per_key,
                   uint8_t* bits, size_t cap, size_t* bits_len, uint16_t* num_probes);
int or_bloom_has_key(uint16_t num_probes, const uint8_t* bits, size_t bits_len, const uint8_t* key,
                     size_t klen);
int or_bloom_encode(uint16_t num_probes, const uint8_t* bits, size_t bits_len, int codec,
                    uint8_t* out, size_t cap, size_t* out_len);
int or_bloom_decode(const uint8_t* buf, size_t n, int codec, uint16_t* num_probes, uint8_t* bits,
                    size_t cap, size_t* bits_len);

/* flatbuffers (flatbuf.go, manifest_generated.go) */
typedef struct or_sst_info {
  uint64_t index_offset, index_len, filter_offset, filter_len; int32_t codec; uint32_t first_key_len;
} or_sst_info;
/* EncodeInfo (flatbuf.go:62): first_key NULL => nil. */
int or_encode_info(const or_sst_info* info, const uint8_t* first_key, uint8_t* out, size_t cap,
                   size_t* out_len);
int or_decode_info(const uint8_t* buf, size_t n, or_sst_info* info, uint8_t* first_key,
                   size_t fk_cap);
/* encodeIndex (flatbuf.go:126): metas = (offset, first key) list. */
int or_encode_index(const uint64_t* offsets, const uint8_t* keys, const uint64_t* key_off,
                    size_t n, int codec, uint8_t* out, size_t cap, size_t* out_len);
/* DecodeIndex + BlockMeta() unpack: returns number of metas via *n (needs caps). */
int or_decode_index(const uint8_t* buf, size_t len, int codec, uint64_t* offsets, uint8_t* keys,
                    uint64_t* key_off, size_t metas_cap, size_t keys_cap, size_t* n);

/* sstable.Builder (builder.go) */
typedef struct or_sst_builder or_sst_builder;
or_sst_builder* or_sst_builder_new(uint64_t block_size, uint32_t min_filter_keys,
                                   uint32_t filter_bits_per_key, int codec);
void or_sst_builder_free(or_sst_builder* b);
int or_sst_builder_add(or_sst_builder* b, const uint8_t* key, size_t klen, const uint8_t* value,
                       size_t vlen, int tombstone);                            /* builder.go:160 */
int or_sst_builder_add_value(or_sst_builder* b, const uint8_t* key, size_t klen,
                             const uint8_t* value, size_t vlen);               /* builder.go:149 */
int or_sst_builder_add_batch(or_sst_builder* b, const uint8_t* keys, const uint64_t* key_off,
                             const uint8_t* vals, const uint64_t* val_off, uint64_t n);
/* NextBlock (builder.go:185): returns 1 and a pointer valid until the next call. */
int or_sst_builder_next_block(or_sst_builder* b, const uint8_t** data, size_t* len);
/* Build (builder.go:215): after this, chunks()/info()/bloom() describe Table. */
int or_sst_builder_build(or_sst_builder* b);
size_t or_sst_table_num_chunks(const or_sst_builder* b);
int or_sst_table_chunk(const or_sst_builder* b, size_t i, const uint8_t** data, size_t* len);
size_t or_sst_table_encoded_len(const or_sst_builder* b);
int or_sst_table_encode(const or_sst_builder* b, uint8_t* out, size_t cap);
int or_sst_table_info(const or_sst_builder* b, or_sst_info* info, uint8_t* fk, size_t fk_cap);
int or_sst_table_bloom(const or_sst_builder* b, int* present, uint16_t* num_probes, uint8_t* bits,
                       size_t cap, size_t* bits_len);

/* ReadInfo (decode.go:25) */
int or_sst_read_info(const uint8_t* sst, size_t n, or_sst_info* info, uint8_t* fk, size_t fk_cap);

/* iter.MergeSort (internal/iter/merge.go:12-111): k sorted iterators, concatenated.
 * keys/key_off: n = src_start[k] keys (key i = keys[key_off[i]..key_off[i+1])); iterator j holds
 * elements [src_start[j], src_start[j+1]).  out_idx receives the element index of every entry Next()
 * returns, in order; *n_out their count.  Heap order is (bytes.Compare(key), iterator index)
 * (merge.go:88-95); an entry is returned only when its key differs from the last returned key
 * (merge.go:67-72), and lastKey starts nil, so empty keys are never returned. */
int or_merge_sort(uint32_t k, const uint8_t* keys, const uint64_t* key_off, const uint64_t* src_start,
                  uint32_t* out_idx, uint64_t* n_out);

/* executeCompaction's codec path (slatedb/compaction/executor.go:92-151) over clean inputs
 * (compact_oracle.c): n_sst encoded SSTs, sst i = ssts[sst_off[i] .. sst_off[i+1]); n_src sources
 * in precedence order, source j = SSTs [src_sst[j], src_sst[j+1]).  Outputs built with
 * (block_size, MinFilterKeys 0, 10 bits per key, codec), cut at max_sst_size as executor.go:119-148,
 * concatenated into out with out_off[*n_out + 1].  nthreads workers decode blocks and build outputs
 * (the merge is serial). */
int or_compact(const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst, const uint32_t* src_sst, uint32_t n_src,
               uint64_t block_size, int codec, uint64_t max_sst_size, int nthreads, uint8_t* out, uint64_t cap,
               uint64_t* out_off, uint32_t out_off_cap, uint32_t* n_out);

/* block.NewIteratorAtKey (block/iterator.go:31-82) over a decoded block (Data, Offsets):
 * *start = the iterator's offsetIndex, *first_idx = the row firstFullKey returned (its suffix
 * is the iterator's firstKey, *first_len bytes), *n_warn = warnings added.  Returns OR_OK,
 * OR_E_SEEK_NO_OFFSETS, OR_E_SEEK_NO_FULL_KEY or OR_E_SEEK_PANIC (Go slice panic). */
int or_block_seek(const uint8_t* data, uint32_t data_len, const uint16_t* offsets, uint32_t n, const uint8_t* key,
                  size_t key_len, uint32_t* start, int32_t* first_idx, uint32_t* first_len, uint32_t* n_warn);
int or_block_seek_w(const uint8_t* data, uint32_t data_len, const uint16_t* offsets, uint32_t n, const uint8_t* key,
                    size_t key_len, uint32_t* start, int32_t* first_idx, uint32_t* first_len, uint32_t* n_warn,
                    uint32_t* warn, uint32_t cap);
/* sstable.Iterator.firstBlockIncludingOrAfterKey (iterator.go:123-153) over the index's first keys. */
uint64_t or_index_seek(const uint8_t* keys, const uint64_t* key_off, uint64_t n_blocks, const uint8_t* key,
                       size_t key_len);

#ifdef __cplusplus
}
#endif
#endif
