/*
 * slatecodec.h — C-ABI of the MI355X-native SST block codec (drop-in for the
 * slatedb-go `internal/sstable` block/bloom/builder/reader hot path).
 *
 * Every function here is `extern "C"`, takes plain pointers and sizes, never
 * retains a caller pointer after it returns (cgo rule), and never aborts: Go
 * `error` returns and Go `panic`s on corrupt input both become status codes.
 * All compute (CRC32, Snappy, row packing/unpacking, bloom) runs in HIP kernels
 * on the context's GPU; there is no CPU fallback — without a usable GPU every
 * compute entry point returns SLATE_E_NO_DEVICE.
 *
 * Reference interface each group replaces (paths relative to slatedb-go):
 *   block codec     internal/sstable/block/block.go:54 Encode, :78 Decode
 *   row codec       internal/sstable/block/row.go:149 Encode, :191 Decode
 *   bloom           internal/sstable/bloom/bloom.go:19 HasKey, :52 Encode, :70 Decode, :112 Build
 *   compression     internal/compress/compression.go:80 Encode, :126 Decode
 *   SST builder     internal/sstable/builder.go:136 NewBuilder, :149 AddValue, :160 Add,
 *                   :185 NextBlock, :215 Build; flatbuf.go:143 EncodeTable
 *   SST reader      internal/sstable/decode.go:25 ReadInfo, :50 ReadFilter, :73 ReadIndex,
 *                   :86 ReadIndexRaw, :107 ReadBlocks, :151 ReadBlockRaw;
 *                   flatbuf.go:62 EncodeInfo, :83 DecodeIndex, :102 DecodeInfo
 */
#ifndef SLATECODEC_H
#define SLATECODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLATECODEC_ABI_VERSION 1

/* ---- compression codec (internal/compress/compression.go:15-21) ---------------- */
enum slate_codec {
  SLATE_CODEC_NONE = 0,
  SLATE_CODEC_SNAPPY = 1,
  SLATE_CODEC_ZLIB = 2,
  SLATE_CODEC_LZ4 = 3,
  SLATE_CODEC_ZSTD = 4,
};

/* ---- status codes ---------------------------------------------------------------
 * Each code maps 1:1 onto the reference's error string (slate_status_string) with
 * the %d fields carried in slate_block_meta.detail / .aux.  Codes >= 100 are
 * C-ABI conditions that have no Go counterpart. */
enum slate_status {
  SLATE_OK = 0,
  /* block.Decode (block.go:79-131) */
  SLATE_E_BLOCK_TOO_SMALL = 1,      /* "corrupted block: block is too small; must be at least 6 bytes" */
  SLATE_E_BLOCK_CHECKSUM = 2,       /* "corrupted block: checksum mismatch" */
  SLATE_E_BLOCK_UNCOMP_SMALL = 3,   /* "corrupted block: uncompressed block is too small; must be at least 2 bytes" */
  SLATE_E_BLOCK_INDEX_OFFSET = 4,   /* "corrupted block: invalid index offset '%d'; cannot be negative" (detail) */
  SLATE_E_BLOCK_OFFSET_BOUNDS = 5,  /* "corrupted block: block offset[%d] = %d exceeds key value bounds" (aux, detail) */
  SLATE_E_BLOCK_NO_OFFSETS = 6,     /* "corrupted block: Block.Offsets must be greater than 0" */
  SLATE_E_BLOCK_FIRSTKEY_PANIC = 7, /* Go panics slicing FirstKey (block.go:130-131) */
  SLATE_E_BLOCK_EMPTY = 8,          /* "assertion failed; block cannot be empty" (block.go:197) */
  /* compress (compression.go) and golang/snappy v0.0.4 */
  SLATE_E_INVALID_CODEC = 10,       /* "corrupted; invalid compression codec" */
  SLATE_E_SNAPPY_CORRUPT = 11,      /* "snappy: corrupt input" */
  SLATE_E_SNAPPY_TOO_LARGE = 12,    /* "snappy: decoded block is too large" */
  SLATE_E_CODEC_UNSUPPORTED = 13,   /* reserved: every codec decodes and encodes, no entry point returns it */
  /* CodecLz4 (compression.go:143-144, github.com/pierrec/lz4/v4 v4.1.21 errors; strings unpinned) */
  SLATE_E_LZ4_MAGIC = 14,           /* "lz4: bad magic number" */
  SLATE_E_LZ4_HEADER_CHECKSUM = 15, /* "lz4: invalid header checksum" */
  SLATE_E_LZ4_BLOCK_CHECKSUM = 16,  /* "lz4: invalid block checksum" */
  SLATE_E_LZ4_FRAME_CHECKSUM = 17,  /* "lz4: invalid frame checksum" */
  SLATE_E_LZ4_CORRUPT = 18,         /* "lz4: invalid source or destination buffer too short" */
  /* CodecZlib (compression.go:134-140, Go compress/zlib + compress/flate errors) */
  SLATE_E_ZLIB_HEADER = 50,         /* "zlib: invalid header" */
  SLATE_E_ZLIB_DICTIONARY = 51,     /* "zlib: invalid dictionary" */
  SLATE_E_ZLIB_CHECKSUM = 52,       /* "zlib: invalid checksum" */
  SLATE_E_FLATE_CORRUPT = 53,       /* "flate: corrupt input before offset %d" (offset not reported) */
  SLATE_E_UNEXPECTED_EOF = 54,      /* "unexpected EOF" (io.ErrUnexpectedEOF) */
  SLATE_E_EOF = 55,                 /* "EOF" (io.EOF: empty zlib stream) */
  /* CodecZstd (compression.go:146-153, github.com/klauspost/compress v1.17.11 errors; strings unpinned) */
  SLATE_E_ZSTD_MAGIC = 56,          /* "invalid input: magic number mismatch" */
  SLATE_E_ZSTD_CHECKSUM = 57,       /* "CRC check failed" (XXH64 content checksum) */
  SLATE_E_ZSTD_CORRUPT = 58,        /* malformed literals / sequences / tables / sizes */
  SLATE_E_ZSTD_FRAME_SIZE = 59,     /* "frame size does not match size on stream" */
  SLATE_E_ZSTD_DICT = 60,           /* "unknown dictionary" (no dictionaries are configured) */
  SLATE_E_ZSTD_RESERVED_BLOCK = 61, /* "invalid input: reserved block type encountered" */
  /* block.NewIteratorAtKey (block/iterator.go:31-82) */
  SLATE_E_SEEK_NO_OFFSETS = 62,     /* "number of block.Offsets must be greater than zero" */
  SLATE_E_SEEK_NO_FULL_KEY = 63,    /* "unable to locate uncorrupted first key in block; block is corrupt" */
  SLATE_E_SEEK_PANIC = 64,          /* Go panics slicing block.Data[offset:] in firstFullKey */
  /* v0 row codec (row.go:191-288) — per-row status in slate_row.status */
  SLATE_E_ROW_TOO_SHORT = 20,       /* "corrupt v0 row: data length too short to decode a row" */
  SLATE_E_ROW_PREFIX = 21,          /* "corrupt v0 row: key prefix length exceeds length of first key in block" */
  SLATE_E_ROW_SUFFIX = 22,          /* "corrupt v0 row: key suffix length exceeds length of block" */
  SLATE_E_ROW_EXPIRE = 23,          /* "corrupt v0 row: data length too short for expire" */
  SLATE_E_ROW_CREATE = 24,          /* "corrupt v0 row: data length too short for create" */
  SLATE_E_ROW_VALUE_LEN = 25,       /* "corrupt v0 row: data length too short for for value length" */
  SLATE_E_ROW_VALUE = 26,           /* "corrupt v0 row: data length too short for for value" */
  SLATE_E_ROW_PANIC = 27,           /* Go panics reading seq/flags (row.go:218-223) */
  SLATE_E_ROW_PEEK_SHORT = 28,      /* "corrupt v0 row: data length too short to peek at row" */
  SLATE_E_ROW_OFFSET_RANGE = 29,    /* offset beyond Block.Data (block/iterator.go:59-62 warns) */
  /* bloom (bloom.go:70-91) */
  SLATE_E_FILTER_TOO_SMALL = 30,    /* "corrupt filter: filter is too small; must be at least 2 bytes" */
  SLATE_E_FILTER_CHECKSUM = 31,     /* "corrupt filter: invalid checksum" */
  SLATE_E_FILTER_PANIC = 32,        /* Go panics on a 2..3 byte filter / short payload */
  /* sstable (decode.go, flatbuf.go, blob.go) */
  SLATE_E_INDEX_TOO_SHORT = 40,     /* "corrupted index; too short" */
  SLATE_E_INDEX_CHECKSUM = 41,      /* "corrupted index; checksum mismatch" */
  SLATE_E_INFO_TOO_SHORT = 42,      /* "corrupted info; too short" */
  SLATE_E_INFO_CHECKSUM = 43,       /* "corrupted info; checksum mismatch" */
  SLATE_E_SST_TOO_SHORT = 44,       /* "corrupted SSTable; too short" */
  SLATE_E_BLOB_RANGE = 45,          /* "corrupted; [%d:%d] is an invalid range" */
  SLATE_E_RANGE_START = 46,         /* "block start '%d' range cannot be greater than end range '%d'" */
  SLATE_E_RANGE_END = 47,           /* "block end '%d' range cannot be greater than size of block meta range '%d'" */
  SLATE_E_FLATBUF = 48,             /* malformed flatbuffer (Go would panic in GetRootAs / accessors) */
  /* C-ABI / runtime conditions */
  SLATE_E_NO_DEVICE = 100,          /* no usable HIP device / kernels not loadable */
  SLATE_E_HIP = 101,                /* HIP runtime error */
  SLATE_E_INVALID_ARG = 102,
  SLATE_E_CAPACITY = 103,           /* caller-provided output buffer too small */
  SLATE_E_OOM = 104,
  SLATE_E_MERGE_UNSORTED = 105,     /* an iterator handed to the merge is not sorted (merge.go's precondition) */
  SLATE_E_LIMIT = 106,              /* an internal limit of this library (e.g. >= 2^32 rows in one call) */
  SLATE_E_WARNINGS = 107,           /* slate_compact_ex: done, with types.ErrWarn warnings (see there) */
  SLATE_E_READER_NEED_DATA = 108,   /* slate_block_reader_next: fetch the range slate_block_reader_want gives */
  SLATE_E_READER_END = 109,         /* slate_block_reader_next: no block left (or the iteration ended on an error) */
};

/* ---- layouts ----------------------------------------------------------------- */

/* Per-block result of block.Decode (block.go:78-134).  16 bytes. */
typedef struct slate_block_meta {
  int16_t status;     /* slate_status */
  uint16_t flags;     /* SLATE_BLKF_* */
  int32_t detail;     /* E_BLOCK_INDEX_OFFSET: offsetStartIndex; E_BLOCK_OFFSET_BOUNDS: offset value */
  uint32_t data_len;  /* len(Block.Data) == offsetStartIndex */
  uint16_t n_rows;    /* len(Block.Offsets) */
  uint16_t aux;       /* E_BLOCK_OFFSET_BOUNDS: offending index; OK: len(Block.FirstKey) (quirk, block.go:130) */
} slate_block_meta;

#define SLATE_BLKF_ROWS_TRUNCATED 0x1u /* more offsets than row-descriptor capacity */

/* Per-row descriptor emitted by the decode kernel: what v0Codec.Decode
 * (row.go:191-261) extracts, against the block iterator's firstKey
 * (block/iterator.go:84-107: row 0 is decoded with firstKey = nil).  16 bytes.
 *   key suffix = Data[row_off + 4 .. + key_suffix_len]
 *   seq (BE u64) at row_off + 4 + key_suffix_len, flags byte right after it
 *   value = Data[row_off + 4 + key_suffix_len + meta_len .. + value_len]          */
typedef struct slate_row {
  uint32_t row_off;         /* Block.Offsets[i] */
  uint16_t key_prefix_len;  /* bytes shared with the block's first key */
  uint16_t key_suffix_len;
  uint32_t value_len;       /* 0 for tombstones */
  uint8_t flags;            /* v0 flags: 1 tombstone, 2 hasExpire, 4 hasCreate */
  uint8_t meta_len;         /* seq(8)+flags(1)+[expire 8]+[create 8]+[value_len 4] */
  int16_t status;           /* SLATE_OK or SLATE_E_ROW_* */
} slate_row;

/* Result of block.NewIteratorAtKey (block/iterator.go:31-82) for one (block, key) query.
 * The iterator starts at row `start` (its offsetIndex); its firstKey is the suffix of row
 * `first_idx` (first_len bytes: firstFullKey's choice, row 0 unless that row is corrupt), and
 * iterator.Next decodes row i >= start against it: key = firstKey[:prefixLen] || suffix.
 * n_warn = warnings NewIteratorAtKey added (types.ErrWarn).  16 bytes. */
typedef struct slate_seek {
  uint32_t start;
  int32_t first_idx;  /* -1 when no full key was found */
  uint32_t n_warn;
  int16_t status;     /* SLATE_OK, SLATE_E_SEEK_*, or the block's own decode status */
  uint16_t first_len;
} slate_seek;

/* One warning NewIteratorAtKey added to its types.ErrWarn, in the order Go adds them, so a shim can
 * rebuild the ErrWarn text (err: a SLATE_E_ROW_* status, slate_status_string gives its text).  16 bytes.
 *   SLATE_WARN_PEEK_FIRST_KEY  "while peeking at key at offset %d: %v"  (a = offset, err)  iterator.go:121
 *   SLATE_WARN_NO_FULL_KEY     "unable to locate uncorrupted first key in block; block is corrupt"  :130
 *   SLATE_WARN_OFFSET_BOUNDS   "block.Offset[%d] = %d is out of bounds"  (a = index, b = offset)  :65
 *   SLATE_WARN_PEEK_ROW        "while peeking at block.Offset[%d]: %s"   (a = index, err)  :70        */
enum slate_seek_warn_kind {
  SLATE_WARN_PEEK_FIRST_KEY = 1,
  SLATE_WARN_NO_FULL_KEY = 2,
  SLATE_WARN_OFFSET_BOUNDS = 3,
  SLATE_WARN_PEEK_ROW = 4,
};
typedef struct slate_seek_warn {
  uint16_t kind;
  int16_t err;
  uint32_t a;
  uint32_t b;
  uint32_t reserved;
} slate_seek_warn;

/* sstable.Config (builder.go:118-133); defaults in decode.go:16-23. */
typedef struct slate_sst_config {
  uint64_t block_size;
  uint32_t min_filter_keys;
  uint32_t filter_bits_per_key;
  int32_t codec; /* slate_codec */
} slate_sst_config;

/* sstable.Info (sstable.go:12-31); first_key bytes returned separately. */
typedef struct slate_sst_info {
  uint64_t index_offset;
  uint64_t index_len;
  uint64_t filter_offset;
  uint64_t filter_len;
  int32_t codec;
  uint32_t first_key_len;
} slate_sst_info;

typedef struct slate_ctx slate_ctx;
typedef struct slate_devbuf slate_devbuf;
typedef struct slate_hostbuf slate_hostbuf;
typedef struct slate_sst_builder slate_sst_builder;
typedef struct slate_sst_table slate_sst_table;
typedef struct slate_index slate_index;

/* ---- library / context --------------------------------------------------------- */
int slate_abi_version(void);
const char* slate_status_string(int status); /* reference error text ("%d" left verbatim) */
/* One context = one device + one HIP stream; contexts are independent and the
 * library keeps no global mutable state, so one context per calling goroutine/
 * thread is reentrant (SURVEY 8b "Threading"). */
slate_ctx* slate_ctx_create(int device, int* status);
void slate_ctx_destroy(slate_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream) for device-resident
 * calls; NULL restores the context's own stream. */
int slate_ctx_set_stream(slate_ctx* ctx, void* hip_stream);
int slate_ctx_synchronize(slate_ctx* ctx);
/* Host threads this context copies with in the host-buffer pipelines (slate_block_decode_batch,
 * slate_read_blocks, devbuf upload/download; default 16 or SLATE_COPY_THREADS, 1..256).  Each
 * context has its own: slate_block_decode_sharded over G contexts uses G x threads. */
int slate_ctx_set_copy_threads(slate_ctx* ctx, uint32_t threads);
/* Measurement aid (no Go counterpart): with timing on, the SST builder's GPU passes (segmentation,
 * pack, Snappy, bloom, CRC kernels) are bracketed by HIP events and their device time summed;
 * slate_ctx_gpu_time returns the sum in milliseconds (and zeroes it when reset != 0).  Kernel
 * groups on the filter's side stream overlap the flush, so the sum can exceed the wall time. */
int slate_ctx_set_timing(slate_ctx* ctx, int on);
/* Observability (no Go counterpart): the number of blocks this context's decodes handed from a fast
 * path (CodecZstd, CodecZlib, CodecLz4) to the exact wave-per-block decoder since the context was
 * made or the count last reset (reset != 0 zeroes it).  Waits for every stream of the context
 * (its stream, side stream, pipeline lanes).  The results are the same either way; a hand-back
 * only costs time. */
int slate_ctx_handbacks(slate_ctx* ctx, uint64_t* n, int reset);
int slate_ctx_gpu_time(slate_ctx* ctx, double* ms, int reset);
/* The same spans' union (*busy_ms: device time with overlapping spans of the side streams counted
 * once) and sum (*sum_ms, may be null) since timing was switched on or last reset.  Every device
 * pass of slate_sst_builder_add_batch_device and slate_sst_builder_build is inside a span
 * (device copies, rebases, scans and memsets included); host-to-device uploads of host batches
 * and the blocks' device-to-host copies are not. */
int slate_ctx_gpu_busy(slate_ctx* ctx, double* busy_ms, double* sum_ms, int reset);

/* ---- library-owned memory (SURVEY 8b "Ownership": device-resident mode uses opaque handles
 * owned by the C side) ----------------------------------------------------------------------
 * cgo lets C keep no Go pointer once a call returns, and the *_device entry points only enqueue
 * work on the context's stream.  So a Go caller gives them memory the library owns:
 *   slate_devbuf   HBM of the context's GPU; every *_device entry point takes
 *                  slate_devbuf_ptr(b) (plus a byte offset) wherever it takes a device pointer;
 *   slate_hostbuf  page-locked host memory, the endpoint of the asynchronous copies (the DMA may
 *                  run after the call returns, so it must not be Go memory).
 * upload / download are synchronous (any host memory, large copies through the context's
 * page-locked staging); copy, memset and the _async copies are ordered on the context's stream
 * (slate_ctx_synchronize waits for them).  A buffer is used with contexts of its own device only. */
slate_devbuf* slate_devbuf_alloc(slate_ctx* ctx, uint64_t bytes, int* status);
void slate_devbuf_free(slate_devbuf* b); /* waits for the device first */
void* slate_devbuf_ptr(const slate_devbuf* b);
uint64_t slate_devbuf_size(const slate_devbuf* b);
int slate_devbuf_upload(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const void* src, uint64_t n);
int slate_devbuf_download(slate_ctx* ctx, void* dst, const slate_devbuf* src, uint64_t src_off, uint64_t n);
int slate_devbuf_copy(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const slate_devbuf* src, uint64_t src_off,
                      uint64_t n);
int slate_devbuf_memset(slate_ctx* ctx, slate_devbuf* b, uint64_t off, int value, uint64_t n);
slate_hostbuf* slate_hostbuf_alloc(slate_ctx* ctx, uint64_t bytes, int* status);
void slate_hostbuf_free(slate_hostbuf* b);
void* slate_hostbuf_ptr(const slate_hostbuf* b);
uint64_t slate_hostbuf_size(const slate_hostbuf* b);
int slate_devbuf_upload_async(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const slate_hostbuf* src,
                              uint64_t src_off, uint64_t n);
int slate_devbuf_download_async(slate_ctx* ctx, slate_hostbuf* dst, uint64_t dst_off, const slate_devbuf* src,
                                uint64_t src_off, uint64_t n);

/* ---- block decode: block.Decode (block.go:78) ----------------------------------
 * Device-resident batch.  Block i's encoded bytes are d_in[d_in_off[i] .. d_in_off[i+1]).
 * Step 1 (plan): decoded lengths and row capacities -> exclusive scans into
 *   d_out_off[n+1] (bytes) and d_row_base[n+1] (slate_row slots); the totals are
 *   d_out_off[n] and d_row_base[n].  d_scratch must hold slate_decode_scratch_bytes(n).
 * Step 2 (decode): writes the decoded buffer (rows || BE16 offsets || BE16 count)
 *   of block i at d_out + d_out_off[i], its meta and its row descriptors.  CodecNone with
 *   d_out == NULL decodes as Go does, without a copy (block.go:122 aliases the input): block i's
 *   data is d_in + d_in_off[i] itself, d_out_off may be NULL, metas and rows as always.
 * Both enqueue on the context stream and return without synchronising.
 * CodecZlib (n >= 64): a zlib stream carries no decoded size, so the plan inflates every block
 * (lane per block) and keeps what it parsed -- literals, matches, the Adler-32 -- in the context;
 * the next decode call on the context with the same d_in, d_in_off, d_out_off and n, on the same
 * stream, builds the blocks from it instead of inflating again (each stream inflated once per
 * plan + decode).  As for every codec, the input must not change between the two calls (the
 * plan's sizes depend on it).  Any other decode call inflates by itself. */
size_t slate_decode_scratch_bytes(uint32_t n_blocks);
/* The scratch one codec needs (<= slate_decode_scratch_bytes): CodecNone / CodecSnappy batches
 * skip the Zstd / Zlib / LZ4 fast paths' records and sequence slots (~8 B per block instead of
 * ~560).  Scratch sized this way may be used only with that codec. */
size_t slate_decode_scratch_bytes_codec(uint32_t n_blocks, int codec);
int slate_block_decode_plan_device(slate_ctx* ctx, int codec, const uint8_t* d_in,
                                   const uint64_t* d_in_off, uint32_t n_blocks,
                                   uint64_t* d_out_off, uint64_t* d_row_base, void* d_scratch);
int slate_block_decode_device(slate_ctx* ctx, int codec, const uint8_t* d_in,
                              const uint64_t* d_in_off, uint32_t n_blocks, uint8_t* d_out,
                              const uint64_t* d_out_off, slate_block_meta* d_meta,
                              slate_row* d_rows, const uint64_t* d_row_base);

/* Host-buffer batch (object-store GET buffers in, caller buffers out; sstable.ReadBlocks,
 * decode.go:107-149, and the compaction reads, compaction/executor.go:92-151): chunks of up to
 * 64 K blocks go through page-locked staging on two stream lanes of the context (upload and plan
 * of chunk c+1 overlap decode and download of chunk c); synchronous for the caller.
 * out_off/row_base are outputs (n+1 each, always filled); out_cap/rows_cap are capacities:
 * when the outputs do not fit (or out/meta are NULL) the call only plans and returns
 * SLATE_E_CAPACITY with out_off[n] / row_base[n] the sizes needed. */
int slate_block_decode_batch(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off,
                             uint32_t n_blocks, uint8_t* out, uint64_t out_cap, uint64_t* out_off,
                             slate_block_meta* meta, slate_row* rows, uint64_t rows_cap,
                             uint64_t* row_base);
/* Single block: block.Decode(&b, input, codec) (block.go:78), the one-block-per-call pattern of
 * sstable.Iterator.nextBlockIter (iterator.go:92-118).  Data = out[0 .. meta.data_len);
 * offsets[] receives Block.Offsets (meta.n_rows entries, capacity offsets_cap). */
int slate_block_decode(slate_ctx* ctx, int codec, const uint8_t* in, size_t in_len, uint8_t* out,
                       size_t out_cap, size_t* out_len, slate_block_meta* meta, uint16_t* offsets,
                       size_t offsets_cap);

/* ---- round-robin sharding of one block set (BASELINE configs[3]) -------------
 * Blocks are independent, so block i of a batch goes to shard i mod n_shards (one shard per
 * GPU) with no collective.  slate_shard_blocks = blocks of one shard; slate_shard_pack copies
 * them back to back (out_off: shard-local offsets, blocks+1 entries).  Host code: needs no GPU. */
uint32_t slate_shard_blocks(uint32_t n_blocks, uint32_t n_shards, uint32_t shard);
int slate_shard_pack(const uint8_t* in, const uint64_t* in_off, uint32_t n_blocks, uint32_t n_shards,
                     uint32_t shard, uint8_t* out, uint64_t out_cap, uint64_t* out_off);
/* One batch decoded by n_ctx contexts at once (one host thread each; contexts on different
 * GPUs, or several on one): context g decodes shard g through the host pipeline, and the
 * results come back in the original block order, laid out exactly as slate_block_decode_batch
 * lays them out.  What a compactor process holding one slate_ctx per GPU calls. */
int slate_block_decode_sharded(slate_ctx* const* ctxs, uint32_t n_ctx, int codec, const uint8_t* in,
                               const uint64_t* in_off, uint32_t n_blocks, uint8_t* out,
                               uint64_t out_cap, uint64_t* out_off, slate_block_meta* meta,
                               slate_row* rows, uint64_t rows_cap, uint64_t* row_base);

/* ---- seeks for the point-read path (slatedb/db.go:291-315) ---------------------------
 * block.NewIteratorAtKey (block/iterator.go:31-82, firstFullKey :117-132) for n queries at
 * once: query i seeks key i (keys[key_off[i]..key_off[i+1])) in block qblock[i] of a batch
 * decoded by slate_block_decode_device / _batch (data, out_off, meta as those produce them).
 * Device variant: device pointers, on the context stream.  Host variant: host buffers
 * (the decode_batch layout, n_blocks blocks), synchronous. */
int slate_block_seek_device(slate_ctx* ctx, const uint8_t* d_data, const uint64_t* d_out_off,
                            const slate_block_meta* d_meta, const uint32_t* d_qblock, const uint8_t* d_keys,
                            const uint64_t* d_key_off, uint64_t n, slate_seek* d_res);
int slate_block_seek(slate_ctx* ctx, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                     uint32_t n_blocks, const uint32_t* qblock, const uint8_t* keys, const uint64_t* key_off,
                     uint64_t n, slate_seek* res);
/* The same, also returning the warnings: query i's first warn_cap warnings at warn[i * warn_cap ..]
 * (res[i].n_warn counts all of them; firstFullKey adds one per corrupt row before the first full key,
 * the binary search at most log2(n_rows) + 1). */
int slate_block_seek_warn_device(slate_ctx* ctx, const uint8_t* d_data, const uint64_t* d_out_off,
                                 const slate_block_meta* d_meta, const uint32_t* d_qblock, const uint8_t* d_keys,
                                 const uint64_t* d_key_off, uint64_t n, slate_seek* d_res, slate_seek_warn* d_warn,
                                 uint32_t warn_cap);
int slate_block_seek_warn(slate_ctx* ctx, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                          uint32_t n_blocks, const uint32_t* qblock, const uint8_t* keys, const uint64_t* key_off,
                          uint64_t n, slate_seek* res, slate_seek_warn* warn, uint32_t warn_cap);

/* ---- block encode: block.Encode (block.go:54) ----------------------------------
 * Encodes one block (Data + Offsets) with codec: compress(Data || BE16 offsets ||
 * BE16 n) || BE32 CRC32-IEEE. */
int slate_block_encode(slate_ctx* ctx, int codec, const uint8_t* data, size_t data_len,
                       const uint16_t* offsets, size_t n_offsets, uint8_t* out, size_t out_cap,
                       size_t* out_len);

/* ---- SST builder: sstable.Builder (builder.go:92-268) ----------------------------
 * Keys/values are copied on Add.  Blocks are cut on the GPU (greedy fill of
 * block.Builder.Add, block.go:162-182) when NextBlock/Build needs them. */
slate_sst_builder* slate_sst_builder_new(slate_ctx* ctx, const slate_sst_config* cfg, int* status);
void slate_sst_builder_free(slate_sst_builder* b);
/* Add (builder.go:160): kind 0 = KindKeyValue, 1 = KindTombStone. */
int slate_sst_builder_add(slate_sst_builder* b, const uint8_t* key, size_t key_len,
                          const uint8_t* value, size_t value_len, int kind);
/* AddValue (builder.go:149): empty value => tombstone. */
int slate_sst_builder_add_value(slate_sst_builder* b, const uint8_t* key, size_t key_len,
                                const uint8_t* value, size_t value_len);
/* Bulk AddValue of n sorted KVs: key i = keys[key_off[i]..key_off[i+1]), same for
 * values; is_tomb may be NULL (then empty value => tombstone as AddValue). */
int slate_sst_builder_add_batch(slate_sst_builder* b, const uint8_t* keys, const uint64_t* key_off,
                                const uint8_t* values, const uint64_t* value_off,
                                const uint8_t* is_tomb, uint64_t n);
/* NextBlock (builder.go:185): *present = 0 when no finished block is queued.
 * The block is copied into out (capacity out_cap); *len receives its size
 * (also when it does not fit, with SLATE_E_CAPACITY). */
/* The same as slate_sst_builder_add_batch for KVs already in device memory of the builder's
 * context (compaction's merged output, slatedb/compaction/executor.go:100-146 writing through
 * table_store.go:221-266): device pointers; d_is_tomb may be NULL (empty value = tombstone). */
int slate_sst_builder_add_batch_device(slate_sst_builder* b, const uint8_t* d_keys, const uint64_t* d_key_off,
                                       const uint8_t* d_values, const uint64_t* d_value_off,
                                       const uint8_t* d_is_tomb, uint64_t n);
int slate_sst_builder_next_block(slate_sst_builder* b, uint8_t* out, size_t out_cap, size_t* len,
                                 int* present);
/* Build (builder.go:215): consumes the builder's pending KVs; the table owns the
 * remaining block queue (last element = last block || filter || index || info || BE32 offset). */
int slate_sst_builder_build(slate_sst_builder* b, slate_sst_table** table);
void slate_sst_table_free(slate_sst_table* t);
int slate_sst_table_info(const slate_sst_table* t, slate_sst_info* info, uint8_t* first_key,
                         size_t first_key_cap);
size_t slate_sst_table_num_chunks(const slate_sst_table* t); /* Table.Blocks.Len() */
int slate_sst_table_chunk(const slate_sst_table* t, size_t i, const uint8_t** data, size_t* len);
/* EncodeTable (flatbuf.go:143): concatenation of the remaining chunks. */
size_t slate_sst_table_encoded_len(const slate_sst_table* t);
int slate_sst_table_encode(const slate_sst_table* t, uint8_t* out, size_t out_cap);
/* Table.Bloom: *present = 0 when absent; filter bits copied into bits. */
int slate_sst_table_bloom(const slate_sst_table* t, int* present, uint16_t* num_probes,
                          uint8_t* bits, size_t bits_cap, size_t* bits_len);

/* crc32.ChecksumIEEE of n device bytes at any alignment (the checksum every block, filter, index
 * and info payload carries: block.go:73, bloom.go:61, flatbuf.go:53-60), computed on the GPU. */
int slate_crc32_device(slate_ctx* ctx, const uint8_t* d_data, size_t n, uint32_t* crc);

/* ---- SST reader (decode.go / flatbuf.go) ------------------------------------------
 * The caller performs the object-store reads (ReadOnlyBlob.ReadRange) and hands
 * the byte ranges in; nothing is retained. */
/* ReadInfo (decode.go:25) over the whole SST object (only its tail is touched). */
int slate_sst_read_info(const uint8_t* sst, size_t sst_len, slate_sst_info* info,
                        uint8_t* first_key, size_t first_key_cap);
/* DecodeInfo (flatbuf.go:102) on info||crc bytes; EncodeInfo (flatbuf.go:62). */
int slate_decode_info(const uint8_t* buf, size_t len, slate_sst_info* info, uint8_t* first_key,
                      size_t first_key_cap);
int slate_encode_info(const slate_sst_info* info, const uint8_t* first_key, uint8_t* out,
                      size_t out_cap, size_t* out_len);
/* DecodeIndex (flatbuf.go:83): CRC verify + decompress (every codec: Snappy by the streaming
 * decoder, LZ4 / Zlib / Zstd by one wave per payload in HBM); index handle owns the bytes. */
int slate_decode_index(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec, slate_index** index);
void slate_index_free(slate_index* index);
size_t slate_index_num_blocks(const slate_index* index); /* BlockMetaLength() */
int slate_index_block_meta(const slate_index* index, size_t i, uint64_t* offset,
                           const uint8_t** first_key, size_t* first_key_len);
/* sstable.Iterator.firstBlockIncludingOrAfterKey (iterator.go:123-153) for n keys: the block
 * each NewIteratorAtKey (iterator.go:43-57) starts reading at, on the GPU. */
int slate_index_seek(slate_ctx* ctx, const slate_index* index, const uint8_t* keys, const uint64_t* key_off,
                     uint64_t n, uint64_t* block_out);
/* Every BlockMeta's Offset at once (cap >= slate_index_num_blocks): what a batched reader or the
 * compaction path needs to slice an SST's data blocks without per-block calls. */
int slate_index_block_offsets(const slate_index* index, uint64_t* offsets, size_t cap);
/* ReadBlocks (decode.go:107): data = the object's bytes [meta[start].Offset, end offset)
 * (slate_read_blocks_range gives that range).  Blocks are decoded as one GPU batch;
 * outputs as slate_block_decode_batch.  *failed_block receives the first failing
 * block index (the reference wraps its error with that index and range). */
int slate_read_blocks_range(const slate_sst_info* info, const slate_index* index, uint64_t start,
                            uint64_t end, uint64_t* range_start, uint64_t* range_end);
int slate_read_blocks(slate_ctx* ctx, const slate_sst_info* info, const slate_index* index,
                      uint64_t start, uint64_t end, const uint8_t* data, size_t data_len,
                      uint8_t* out, uint64_t out_cap, uint64_t* out_off, slate_block_meta* meta,
                      slate_row* rows, uint64_t rows_cap, uint64_t* row_base,
                      uint64_t* failed_block);

/* Read-ahead block reader: sstable.Iterator's nextBlockIter (internal/sstable/iterator.go:92-118)
 * asks ReadBlocksUsingIndex for one block per call; this reader keeps that contract -- the blocks
 * in order from first_block, one at a time, an iteration that ends at the first failing block
 * with that block's status -- but fetches and decodes read_ahead blocks per GPU call (one object-
 * store range read and one batch), up to three batches held: next asks for the following batch as
 * soon as a slot is free, before serving the current one, so fetch and decode run ahead of the
 * walk (feed queues the decode and returns).  The caller's loop:
 *   st = slate_block_reader_next(r, &view):
 *     SLATE_OK                 view is the next block (pointers valid until the next feed);
 *     SLATE_E_READER_NEED_DATA slate_block_reader_want(r, &rs, &re) gives the SST byte range to
 *                              read [rs, re); hand it to slate_block_reader_feed, then call next;
 *     SLATE_E_READER_END       no block left;
 *     any other status         view.block failed block.Decode with it: the SST iterator adds its
 *                              warning and ends (iterator.go:59-68); later calls return END.
 * feed returns the decode call's status (a range / length error of the data handed in). */
typedef struct slate_block_reader slate_block_reader;
typedef struct slate_block_view {
  uint64_t block;          /* index of the block in the SST */
  slate_block_meta meta;   /* block.Decode's result (status, data_len, n_rows, FirstKey length) */
  const uint8_t* data;     /* Block.Data: meta.data_len bytes, then the BE16 offsets (n_rows) */
  const slate_row* rows;   /* the row descriptors (n_rows, or the capacity when truncated) */
} slate_block_view;
int slate_block_reader_create(slate_ctx* ctx, const slate_sst_info* info, const slate_index* index,
                              uint64_t first_block, uint32_t read_ahead, slate_block_reader** reader);
void slate_block_reader_free(slate_block_reader* reader);
int slate_block_reader_next(slate_block_reader* reader, slate_block_view* view);
int slate_block_reader_want(const slate_block_reader* reader, uint64_t* range_start, uint64_t* range_end);
int slate_block_reader_feed(slate_block_reader* reader, const uint8_t* data, size_t data_len);

/* ---- bloom filter (bloom.go) -------------------------------------------------------- */
/* Build (bloom.go:112) over n keys (key i = keys[key_off[i]..key_off[i+1])) on the GPU. */
int slate_bloom_build(slate_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                      uint32_t bits_per_key, uint8_t* bits, size_t bits_cap, size_t* bits_len,
                      uint16_t* num_probes);
/* Encode (bloom.go:52) / Decode (bloom.go:70), every codec.  Decode's bits alias nothing: copied out.
 * When bits_cap is too small, Decode returns SLATE_E_CAPACITY with *bits_len set (the retry with a
 * buffer of that length decodes the payload again; the context keeps nothing in between). */
int slate_bloom_encode(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len,
                       int codec, uint8_t* out, size_t out_cap, size_t* out_len);
int slate_bloom_decode(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec,
                       uint16_t* num_probes, uint8_t* bits, size_t bits_cap, size_t* bits_len);
/* Filter.HasKey (bloom.go:19), batched on the GPU: out[i] = 1 if key i may be present. */
int slate_bloom_has_keys(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len,
                         const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint8_t* out);

/* ---- compaction merge (iter.MergeSort, internal/iter/merge.go:12-111) ----------------- */
/* k sorted iterators, concatenated: key i = keys[key_off[i]..key_off[i+1]), iterator j holds
 * elements [src_start[j], src_start[j+1]) (src_start: k+1 host values, src_start[0] = 0,
 * n = src_start[k] < 2^32 - 1).  out_idx[0..*n_out) receives the element index of every entry
 * MergeSort.Next (merge.go:54-76) returns, in order: keys ascending, on equal keys the entry of
 * the lowest iterator index, later duplicates dropped, empty keys never returned (lastKey starts
 * nil).  An unsorted iterator returns SLATE_E_MERGE_UNSORTED (Go does not check; its heap
 * output for such input is unspecified).  Replaces NewMergeSort + the Next loop of
 * executeCompaction (compaction/executor.go:92-151). */
int slate_merge_sorted(slate_ctx* ctx, uint32_t k, const uint8_t* keys, const uint64_t* key_off,
                       const uint64_t* src_start, uint32_t* out_idx, uint64_t* n_out);
/* Device-resident variant on the context's stream: d_keys/d_key_off/d_out_idx/d_n_out/d_flags/
 * d_scratch are device pointers, d_scratch holds slate_merge_scratch_bytes(n, k) bytes, and
 * *d_flags bit 0 is set when an iterator is not sorted.  src_start stays a host array. */
size_t slate_merge_scratch_bytes(uint64_t n, uint32_t k);
int slate_merge_sorted_device(slate_ctx* ctx, uint32_t k, const uint8_t* d_keys, const uint64_t* d_key_off,
                              const uint64_t* src_start, uint32_t* d_out_idx, uint64_t* d_n_out,
                              uint32_t* d_flags, void* d_scratch);

/* ---- compaction KV views (executeCompaction's iterators, compaction/executor.go:92-151) --
 * Device-resident, on the context's stream, two phases each (lengths, then copy into buffers
 * the caller sizes from the offsets' last element):
 * rows -> KV: for decoded blocks (slate_block_decode_device outputs; n_rows = the row-slot
 * count d_row_base[n_blocks]), the rows in block order (*d_n_kv of them), each with its full key
 * (block.Iterator, block/iterator.go:84-107: row 0's key is its suffix and is the block's
 * firstKey; row i's key = firstKey[:prefixLen] || suffix, row.go:72-79), value bytes (empty for
 * tombstones) and tombstone flag.  *d_flags bit 1 = a block or row failed to decode: a failed block
 * contributes no KV, a failed row neither it nor the rows after it in its block (block.Iterator
 * stops there, block/iterator.go:92-96).  d_key_off/d_val_off hold n_rows+1 entries (entries past *d_n_kv repeat the
 * total).  d_scratch holds slate_kv_scratch_bytes(n_rows) and must be kept, unchanged, from the
 * lengths call to the copy call (it carries the row-slot map).
 * gather: the KV of every merge result index (slate_merge_sorted_device's d_out_idx), in order,
 * ready for the SST builder (EncodedSSTableWriter.Add, table_store.go:221-266). */
size_t slate_kv_scratch_bytes(uint64_t n);
int slate_rows_kv_lengths_device(slate_ctx* ctx, uint32_t n_blocks, const uint64_t* d_row_base,
                                 const slate_block_meta* d_meta, const slate_row* d_rows, uint64_t n_rows,
                                 uint64_t* d_key_off, uint64_t* d_val_off, uint8_t* d_tomb, uint64_t* d_n_kv,
                                 uint32_t* d_flags, void* d_scratch);
int slate_rows_kv_copy_device(slate_ctx* ctx, uint32_t n_blocks, const uint8_t* d_data, const uint64_t* d_out_off,
                              const uint64_t* d_row_base, const slate_row* d_rows, uint64_t n_rows,
                              const uint64_t* d_n_kv, const void* d_scratch, const uint64_t* d_key_off,
                              uint8_t* d_keys, const uint64_t* d_val_off, uint8_t* d_vals);
int slate_kv_gather_lengths_device(slate_ctx* ctx, const uint32_t* d_idx, uint64_t n, const uint64_t* d_key_off,
                                   const uint64_t* d_val_off, const uint8_t* d_tomb, uint64_t* d_okey_off,
                                   uint64_t* d_oval_off, uint8_t* d_otomb, void* d_scratch);
int slate_kv_gather_copy_device(slate_ctx* ctx, const uint32_t* d_idx, uint64_t n, const uint8_t* d_keys,
                                const uint64_t* d_key_off, const uint8_t* d_vals, const uint64_t* d_val_off,
                                uint8_t* d_okeys, const uint64_t* d_okey_off, uint8_t* d_ovals,
                                const uint64_t* d_oval_off);

/* ---- executeCompaction's codec path (slatedb/compaction/executor.go:92-151) ----------------
 * One call for what executeCompaction does between reading its input SSTs and uploading its
 * outputs: every data block of every input SST decoded on the GPU (block.Decode as
 * sstable.Iterator applies it, internal/sstable/iterator.go:92-118), each row's full key and
 * value (block.Iterator, block/iterator.go:84-107), iter.MergeSort over the sources
 * (internal/iter/merge.go:12-111: keys ascending, the lowest source wins a duplicate key), and the
 * merged entries written through one SST builder per output (EncodedSSTableWriter.Add,
 * table_store.go:221-266: AddValue, an empty value is a tombstone), a new output starting after
 * the entry that takes the running key + value size past max_sst_size (executor.go:119-139).
 * Inputs: n_sst encoded SSTs in HOST memory (the object-store GET buffers), sst i =
 * ssts[sst_off[i] .. sst_off[i+1]); n_src sources in precedence order (executor.go:55-90: L0 SSTs,
 * then sorted runs), source j = SSTs [src_sst[j], src_sst[j+1]) read in order (src_sst: n_src + 1
 * entries, 0 .. n_sst).  The library uploads the data blocks itself; every intermediate stays in
 * library-owned HBM.
 * Outputs: *n_out tables in out_tables (the caller frees them with slate_sst_table_free).
 * out_cap too small (including out_cap = 0 to ask): SLATE_E_CAPACITY with *n_out = the number
 * needed (> out_cap); the merged entries are recomputed by the retry.
 *
 * Corrupt inputs end iterators the way Go's do, and the compaction goes on:
 *  - a data block that fails block.Decode ends its SST's iterator: the SST contributes the rows of
 *    the blocks before it (sstable.Iterator.Next, iterator.go:59-68 + nextBlockIter :92-118);
 *  - a row that fails v0RowCodec.Decode ends its block's iterator: the block contributes the rows
 *    before it, and the SST goes on with its next block (block/iterator.go:84-99);
 * the outputs are built from what is left, and the warnings Go collects in types.ErrWarn are
 * reported as records (below).  executeCompaction then returns warn.If() beside the sorted run
 * (executor.go:150) and startCompaction turns that into a failed Result (:166-173).
 * Internal limits (more than 2^32 - 1 rows or slots in one call, a block with more rows than its
 * planned slots) return SLATE_E_LIMIT with *n_out = 0.  A row that is not sorted within its source
 * returns SLATE_E_MERGE_UNSORTED. */
typedef struct slate_compact_warning {
  uint32_t src;       /* source index (0 .. n_src-1) */
  uint32_t sst;       /* input SST index (0 .. n_sst-1) */
  uint32_t block;     /* data block index within that SST */
  int32_t row;        /* block.Offsets index of the failing row; -1: the block failed block.Decode */
  int32_t status;     /* the block's SLATE_E_* (block.Decode) or the row's SLATE_E_ROW_* */
  uint32_t block_len; /* encoded bytes of the block: "data[0:block_len]" in the message */
} slate_compact_warning;
/* One record per warning, in the order types.ErrWarn receives them (iter.MergeSort merges a
 * source's warnings up to its first row when it is created, and the rest when the source ends;
 * sources end in the order their last keys leave the merge heap).  The texts, with the SST id the
 * caller knows (slate_status_string gives err):
 *   row = -1: "while fetching blocks for SST '%s': while reading block range [%d:%d]: while decoding
 *              block '%d' data[0:%d]: %s"   (sst id, block, block + 1, block, block_len, err)
 *   row >= 0: "while decoding block.Offset[%d]: %s"   (row, err)
 * ErrWarn.Merge drops a text equal to one already kept (types/errors.go:41-52), and so does the
 * library: a row record whose (row, status) pair an earlier record has is not returned (the row
 * text depends on nothing else; a block record names its SST, so it never repeats). */
int slate_compact(slate_ctx* ctx, const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst, const uint32_t* src_sst,
                  uint32_t n_src, const slate_sst_config* out_cfg, uint64_t max_sst_size, slate_sst_table** out_tables,
                  uint32_t out_cap, uint32_t* n_out);
/* slate_compact with the warning records: up to warn_cap records in warns, *n_warn = the number Go
 * collects (may exceed warn_cap).  Returns SLATE_E_WARNINGS, with the outputs built, when there is at
 * least one warning.  slate_compact returns the first record's status instead and frees the outputs
 * (*n_out = 0), as startCompaction drops the sorted run of a compaction that returned an error. */
int slate_compact_ex(slate_ctx* ctx, const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst,
                     const uint32_t* src_sst, uint32_t n_src, const slate_sst_config* out_cfg, uint64_t max_sst_size,
                     slate_sst_table** out_tables, uint32_t out_cap, uint32_t* n_out, slate_compact_warning* warns,
                     uint32_t warn_cap, uint32_t* n_warn);

#ifdef __cplusplus
}
#endif
#endif /* SLATECODEC_H */
