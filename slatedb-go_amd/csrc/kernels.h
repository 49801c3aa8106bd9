// Kernel launch interfaces shared between the HIP translation units and the
// C-ABI host code.
#pragma once
#include "common.h"

namespace slate {

// ---------------------------------------------------------------- decode
constexpr int kDecodeThreads = 256;          // 4 wavefronts, one block each at a time
constexpr uint32_t kDecodeWgPerCu = 4;       // LDS-limited residency (4 x 40 KiB)
constexpr uint32_t kFastInCap = 4608;        // staged encoded block (incl. 16-byte misalignment)
constexpr uint32_t kFastOutCap = 4608;       // decoded block
constexpr uint32_t kZsFastInCap = 4224;      // CodecZstd fast-kernel staging: 2 x (4 waves + tables) per CU
constexpr uint32_t kZsFastOutCap = 4112;
constexpr uint32_t kLargeInCap = 65552;      // large-block kernel, one wave per workgroup
constexpr uint32_t kLargeOutCap = 90112;
// lane-per-block Snappy decode v2 (decode_lpb2.hip): 136 B output ring + 136 B input ring
// per lane + 4 KiB CRC tables -> one 8-wave workgroup per CU.  (12 waves with a 4-slot
// input ring fit LDS and 168 VGPRs but ran slower: the smaller ring costs 15 % more
// iterations, and 3 waves per SIMD gained only 15 % per iteration.)  SLATE_LPB_THREADS /
// SLATE_LPB_NS override them for experiments (tools/variant.sh).
#ifndef SLATE_LPB_THREADS
#define SLATE_LPB_THREADS 384
#endif
constexpr int kLpb2Threads = SLATE_LPB_THREADS;

// A second stream with its fork / join events, owned by the caller's context (slate_ctx, or a
// pipeline lane of it) and destroyed with it: the CodecZstd fast path runs its Huffman-literal phase
// on it beside the build phase.  Created on first use; a failed creation leaves the launch serial.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  bool tried = false;
  hipStream_t get() {
    if (!tried) {
      tried = true;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&join, hipEventDisableTiming) != hipSuccess)
        release();
    }
    return s;
  }
  void release() {
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    if (s) (void)hipStreamDestroy(s);
    s = nullptr;
    fork = join = nullptr;
  }
};

struct DecodeArgs {
  int codec;
  const uint8_t* in;
  const uint64_t* in_off;
  uint32_t n;
  uint8_t* out;
  const uint64_t* out_off;
  slate_block_meta* meta;
  slate_row* rows;
  const uint64_t* row_base;
  uint32_t* large_list;   // filled by the launcher from scratch
  uint32_t* large_count;
  uint32_t debug;         // ablation switches (SLATE_DEBUG_MODE), read only by SLATE_PROFILING_BUILD variants
  uint32_t raw = 0;       // LPB only: payload is not a block (index/filter buffer): CRC + decompress, no block checks
  uint32_t rt_zero = 0;   // always 0: a value the compiler cannot fold (see decode_lpb2.hip rd128)
  uint32_t* round_counter = nullptr;  // decode_lpb2: rounds handed out so far (launcher zeroes it)
  SideStream* side = nullptr;         // host only: the caller's side stream (nullptr: one stream)
  uint64_t* handbacks = nullptr;      // device counter: blocks a fast path handed to the exact path
  // CodecNone only: the decoded bytes are not written -- out / out_off alias in / in_off, as
  // block.Decode aliases the input for CodecNone (block.go:122, compression.go:128-129); meta and
  // rows as always (slate_compact's row views read the uploaded SSTs)
  uint32_t no_data = 0;
};

// Ablation bits.  The shipped library is built without SLATE_PROFILING_BUILD, so every
// ablation branch folds away at compile time; tools/variant.sh builds profiling variants.
__host__ __device__ inline uint32_t dbg_bits(const DecodeArgs& a) {
#ifdef SLATE_PROFILING_BUILD
  return a.debug;
#else
  (void)a;
  return 0u;
#endif
}

// CodecZstd fast path (zstd_fast.hip): per block, what the lane-per-block parse found
constexpr uint32_t kZsFastSeqs = 16;  // sequences per block on the predefined-table parse (8-byte records)
// the FSE parse (FSE_Compressed tables, or more sequences): 4-byte records (kZfSeq4), up to 128
constexpr uint32_t kZsFseSeqs = 128;
constexpr uint32_t kZfSeqSlot = 128;  // dwords of z.seq per block (16 x 8 or 128 x 4 bytes)
constexpr uint32_t kZfFast = 1, kZfRle = 2, kZfSum = 4, kZfHuf = 8, kZfHuf4 = 16,
                   kZfSeq4 = 32;  // kZfHuf: Huffman literals; kZfSeq4: 4-byte sequence records
// CodecZlib blocks through the same build phase (zlib_fast.hip): the literal bytes are at the start
// of the block's output slot, not in the frame; want is the stream's Adler-32, checked in phase B
constexpr uint32_t kZfOutLit = 64, kZfAdler = 128;
// set with kZfHuf by phase A and never cleared (H2 clears kZfHuf once it has placed the literals):
// the main stream's phase B skips these blocks whatever H2 has done so far
constexpr uint32_t kZfHufOrig = 256;
struct ZsFastRec {
  uint32_t lit;       // frame offset of the raw literals, or the RLE literal byte
  uint32_t nlit;      // literal bytes
  uint32_t produced;  // decoded bytes
  uint32_t info;      // sequences | kZf* flags << 16 (kZfFast clear: the exact path decodes it)
  uint32_t want;      // the frame's checksum (low 32 bits of XXH64) when kZfSum
  uint32_t cs;        // kZfHuf: compressed literals bytes (tree description + streams) at lit
  uint32_t pad[2];
};
struct ZsFastArgs {
  ZsFastRec* rec;   // n
  uint32_t* seq;    // n * kZfSeqSlot dwords: uint2 (ll | ml << 16, offset) records, or (kZfSeq4) u32
                    // records ll | (ml - 3) << 10 | (offset - 1) << 20
  uint32_t* list;   // blocks for the exact path
  uint32_t* count;  // count[0]: list, count[1]: hlist, count[2]: flist entries
  uint32_t* hlist;  // kZfHuf blocks (phase B': Huffman literals)
  uint32_t* flist;  // blocks for the FSE parse (phase A')
  // CodecZlib after a staged plan: the literal bytes of block b at lit + kZlStageStride b (phase
  // B reads them there instead of the start of the output slot); nullptr otherwise
  const uint8_t* lit = nullptr;
  // CodecZstd Huffman-literal blocks (phases H1 / H2): hlist entries k < hcap get their decoding
  // table at htab + kZhTab k and four stream records at hdesc + 16 k (dwords); the rest phase B'
  uint8_t* htab = nullptr;
  uint32_t* hdesc = nullptr;
  uint32_t hcap = 0;
  // phase B: blist != nullptr builds only blist[k] for k < min(count[1], hcap) (the Huffman-literal
  // blocks phase H2 prepared); skip_hufo skips every kZfHufOrig block (they are the list's)
  const uint32_t* blist = nullptr;
  uint32_t skip_hufo = 0;
  // phase B draws its blocks `draw` at a time from count[3] (zeroed with the others) instead of a
  // static stride: workgroups that start late (CUs held by H1 / H2) take fewer
  uint32_t draw = 0;
  uint32_t out_nt = 0;  // phase B's output stores non-temporal
};
constexpr uint32_t kZhTab = 4096;  // a Huffman decoding table: 2^11 16-bit entries
// hlist entries with an H1 / H2 slot: every one for small batches, ~6 % of the blocks beyond
// (configs[4]: 1.1 % of blocks have Huffman literals); the rest take phase B'
__host__ __device__ inline uint32_t zf_huf_cap(uint32_t n) { return n <= 1024 ? n : min(n, n / 16 + 64); }
// The staged CodecZlib plan (zlib_fast.hip kZlStage): phase Z's records, sequences, literals and
// the hand-back list of n blocks, written by the plan and consumed by the decode that follows it
constexpr uint32_t kZlStageStride = kZsFastOutCap;  // literal bytes <= decoded bytes <= the fast path's cap
static_assert(kZlStageStride % 16 == 0, "stage slots stay 16-byte aligned");
struct ZlStage {
  ZsFastRec* rec;
  uint32_t* seq;    // n * kZfSeqSlot dwords
  uint32_t* list;   // n: the blocks phase Z left to the exact path (and the plan's wave plan)
  uint32_t* count;  // list entries (then two unused counters)
  uint8_t* lit;     // n * kZlStageStride bytes
};
size_t zl_stage_bytes(uint32_t n);
ZlStage zl_stage_carve(void* p, uint32_t n);

struct DecodeScratch {
  uint64_t* pa;
  uint64_t* pb;
  uint32_t* large_count;
  uint32_t* large_list;
  uint32_t* round_counter;
  uint32_t tiles;
  ZsFastArgs zf;
};

size_t decode_scratch_bytes(uint32_t n);
size_t decode_scratch_bytes_codec(uint32_t n, int codec);
// stage (CodecZlib, n >= 64 only; nullptr elsewhere): the plan parses each stream once into it
hipError_t launch_decode_plan(hipStream_t st, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                              uint64_t* out_off, uint64_t* row_base, void* scratch, const ZlStage* stage = nullptr,
                              int num_cus = 0);
// stage: a staged plan's (the same inputs, the same stream, nothing written to it since): the
// CodecZlib decode builds from it without phase Z
hipError_t launch_decode(hipStream_t st, const DecodeArgs& a, void* scratch, int num_cus,
                         const ZlStage* stage = nullptr);
hipError_t launch_decode_lpb2(hipStream_t st, const DecodeArgs& a, int num_cus);
// CodecNone blocks (not raw payloads): one wave per block, streaming (decode_none.hip); blocks with
// more than 5104 or fewer than 4 data bytes are appended to a.large_list for decode_large_kernel<0>.
hipError_t launch_decode_none(hipStream_t st, const DecodeArgs& a, int num_cus);
// CodecLz4 blocks: the lane-per-block decoder for one-block frames (XXH32 content checksum in its
// loop); every other shape and any failed check is appended to z.list for the exact path.
hipError_t launch_lz4_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus);
// CodecLz4 plan sizes lane per block for frames of one data block (out_sz[n] = row_sz[n] = 0 too);
// the rest appended to list (*count) for the serial plan.
hipError_t launch_lz4_plan(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n, uint64_t* out_sz,
                           uint64_t* row_sz, uint32_t* list, uint32_t* count);
// CodecZstd fast path (zstd_fast.hip): plan sizes of single-frame blocks (the rest appended to
// list for the wave plan); decode phases A-C (blocks for the exact path appended to z.list).
hipError_t launch_zstd_plan_fast(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n, uint64_t* out_sz,
                                 uint64_t* row_sz, uint32_t* list, uint32_t* count);
hipError_t launch_zstd_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus);
// CodecZlib fast path (zlib_fast.hip): plan sizes lane per block (the rest appended to list for the
// wave plan); decode: phase Z (lane per block: literals + sequences), then zstd_fast.hip's phases A2
// and B (launch_zlib_fast), hand-backs to z.list for the exact path.
hipError_t launch_zlib_plan_fast(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                                 uint64_t* out_sz, uint64_t* row_sz, uint32_t* list, uint32_t* count, int num_cus,
                                 const ZlStage* stage = nullptr);
hipError_t launch_zlib_fast_parse(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus);
// parsed: phase Z already ran (a staged plan; z points into the stage)
hipError_t launch_zlib_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus, bool parsed = false);
// The rows of a decoded batch, densely in block order, written to `dense` (device memory or
// page-locked host memory mapped for the device): block i's min(n_rows, capacity) rows when it
// decoded (status OK), none otherwise; dense_off (n+1 u64) gets the exclusive scan of those
// counts.  For host transfers: the plan's row capacity is an upper bound several times the rows
// a block holds.  scratch: rows_pack_scratch_bytes(n).
size_t rows_pack_scratch_bytes(uint32_t n);
// decoded bytes and rows of n blocks into mapped page-locked caller memory (decode.hip)
hipError_t launch_blocks_to_host(hipStream_t st, const uint8_t* out, const uint64_t* out_off, const uint64_t* row_base,
                                 const slate_block_meta* meta, const slate_row* rows, uint32_t n, uint8_t* dst_out,
                                 slate_row* dst_rows, const uint64_t* g_out, const uint64_t* g_row, uint64_t out_base,
                                 uint64_t row_base0);
// One CodecNone / CodecSnappy block, one launch (slate_block_decode): host_in / host_out are device
// addresses of page-locked host memory; out_sz = align16(decoded length), row_sz = its row capacity
// (the plan the host computed with decoded_len's rules); a.in / a.out / a.rows: device scratch.
// One small-batch block (launch_decode_small): offsets into the host-mapped staging (in_off: 16-byte
// aligned input; out_off: decoded bytes), its row slots, and for the one-wave decoder the device
// scratch offset of its decoded bytes (dev_out; its input goes at in_off, as in the staging).
struct SmallDesc {
  uint32_t block, in_len;
  uint64_t in_off, out_off, out_sz, row_base, row_sz, dev_out;
};
hipError_t launch_decode_small(hipStream_t st, const DecodeArgs& a, const SmallDesc* descs, uint32_t n_par, uint32_t n,
                               const uint8_t* hin, uint8_t* hout, uint8_t* dscr);
bool small_par_fits(int codec, uint64_t in_len, uint64_t out_sz);
bool small_wave_fits(uint64_t in_len, uint64_t out_sz);
hipError_t launch_decode_one(hipStream_t st, const DecodeArgs& a, const uint8_t* host_in, uint64_t in_len,
                             uint64_t out_sz, uint64_t row_sz, uint8_t* host_out);
hipError_t launch_rows_pack(hipStream_t st, const slate_block_meta* meta, const uint64_t* row_base, uint32_t n,
                            const slate_row* rows, uint64_t* dense_off, void* scratch, slate_row* dense);
// Index / filter payloads (`payload || BE32 CRC`) of any size for LZ4 / Zlib / Zstd (raw mode;
// out_off from launch_decode_plan): meta[i].status, meta[i].data_len = decoded length.
hipError_t launch_decode_payload(hipStream_t st, const DecodeArgs& a, int num_cus);
// ---------------------------------------------------------------- merge (merge.hip)
// iter.MergeSort over k concatenated sorted iterators (h_src_start: k+1 host element indices).
// out_idx[0..*n_out) = element indices in return order; *d_flags bit 0 = some iterator unsorted.
size_t merge_scratch_bytes(uint32_t n, uint32_t k);
hipError_t launch_merge(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint32_t n,
                        const uint32_t* h_src_start, uint32_t k, void* scratch, uint32_t* out_idx, uint64_t* n_out,
                        uint32_t* d_flags);

// Compaction KV views (merge.hip): full keys / values of decoded rows, and the merged gather.
size_t kv_scratch_bytes(uint64_t n);
hipError_t launch_rows_lengths(hipStream_t st, const uint64_t* row_base, uint32_t n_blocks,
                               const slate_block_meta* meta, const slate_row* rows, uint64_t n_slots,
                               uint64_t* key_off, uint64_t* val_off, uint8_t* tomb, uint64_t* n_kv, uint32_t* flags,
                               void* scratch);
hipError_t launch_rows_copy(hipStream_t st, const uint8_t* data, const uint64_t* out_off, const uint64_t* row_base,
                            uint32_t n_blocks, const slate_row* rows, uint64_t n_slots, const uint64_t* n_kv,
                            const void* scratch, const uint64_t* key_off, uint8_t* keys, const uint64_t* val_off,
                            uint8_t* vals);
hipError_t launch_gather_lengths(hipStream_t st, const uint32_t* idx, uint64_t n, const uint64_t* key_off,
                                 const uint64_t* val_off, const uint8_t* tomb, uint64_t* okey_off, uint64_t* oval_off,
                                 uint8_t* otomb, void* scratch);
// dst[i] = src[i] + delta (rebasing concatenated offset arrays; merge.hip)
hipError_t launch_u64_add(hipStream_t st, const uint64_t* src, uint64_t* dst, uint64_t n, uint64_t delta);
hipError_t launch_gather_copy(hipStream_t st, const uint32_t* idx, uint64_t n, const uint8_t* keys,
                              const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off, uint8_t* okeys,
                              const uint64_t* okey_off, uint8_t* ovals, const uint64_t* oval_off);

// Streaming one-wave Snappy decode of one large payload (snappy_stream.hip); *status = SLATE_OK or
// SLATE_E_SNAPPY_CORRUPT.  hdr = varint header bytes, dn = decoded length from the header.
hipError_t launch_snappy_stream(hipStream_t st, const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                uint32_t dn, int32_t* status);
// The same result through the tag-parallel path (snappy_stream.hip: chain strides, per-byte
// pointer doubling), falling back to launch_snappy_stream's kernel on the device for a stream
// that fails a check (so errors and their order are always the serial decoder's).
size_t snappy_par_scratch_bytes(uint32_t sn, uint32_t dn);
hipError_t launch_snappy_decode_par(hipStream_t st, const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                    uint32_t dn, void* scratch, int32_t* status);

// One independent LZ4 data block (sz bytes, decoding to at most cap) through the same passes:
// the chain pass, then (the host having read lz4_par_result's words: [0] != 0 = hand the
// payload to the exact decoder, [4] = decoded length) the bytes pass into out; [0] is checked
// again after it.  prior: how far before out a match may reach (0: independent blocks; linked
// blocks: the frame's bytes already decoded there).
size_t lz4_par_scratch_bytes(uint32_t sz, uint32_t cap);
const uint32_t* lz4_par_result(const void* scratch, uint32_t sz, uint32_t cap);
hipError_t launch_lz4_par_chain(hipStream_t st, const uint8_t* in, uint32_t sz, uint32_t cap, void* scratch);
hipError_t launch_lz4_par_bytes(hipStream_t st, const uint8_t* in, uint32_t sz, uint32_t cap, uint32_t dn,
                                uint32_t prior, void* scratch, uint8_t* out);

// A Zlib payload (zlib stream || BE32 CRC, clen = stream bytes) without flush points inflated in
// parallel (zlib_par.hip): the chain pass (block-start candidates, their speculative decode, the
// walk from bit p0 whose final block must end at byte dend), then -- the host having read
// zlib_par_result's words: [0] != 0 = hand the payload to the exact decoder, [4] = decoded length
// -- the bytes pass into out (val: total bytes, pa / pb: total + 1 words, changed: 64 words);
// [0] is checked again after it.
size_t zlib_par_scratch_bytes(uint32_t clen);
// Bytes from per-byte pointers (zlib_par.hip): pa[x] = x for a byte whose value is val[x], else the
// earlier byte it repeats; pointer doubling (pb, changed: 64 words of scratch) then
// out[x] = val[root].  Skipped when flag[0] is set (a pointer out of range sets it).
hipError_t launch_ptr_gather(hipStream_t st, uint32_t total, const uint8_t* val, uint32_t* pa, uint32_t* pb,
                             uint32_t* changed, uint32_t* flag, uint8_t* out);
const uint32_t* zlib_par_result(const void* scratch);
hipError_t launch_zlib_par_chain(hipStream_t st, const uint8_t* in, uint32_t clen, uint32_t p0, uint32_t dend,
                                 void* scratch, int num_cus);
hipError_t launch_zlib_par_bytes(hipStream_t st, const uint8_t* in, uint32_t clen, uint32_t total, void* scratch,
                                 uint8_t* val, uint32_t* pa, uint32_t* pb, uint32_t* changed, uint8_t* out,
                                 int num_cus);

// A Zstd payload's single frame whose blocks depend on each other (repeat offsets, treeless
// literals, repeat tables) decoded block-parallel (zstd_par.hip), blk = nblk x (block body offset,
// block header word) as the host parsed them, bmax = the frame's block maximum.  Three steps, the
// host reading zstd_par_result's words between them ([0] != 0 = hand the payload to the exact
// decoder): headers ([1] sequences, [2] literals: the sizes of lit / sll / sml / sof), body ([3] =
// decoded length), bytes into out (val: total bytes, pa / pb: total + 1 words, changed: 64 words).
size_t zstd_par_scratch_bytes(uint32_t nblk);
const uint32_t* zstd_par_result(const void* scratch);
hipError_t launch_zstd_par_headers(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                   uint32_t bmax, void* scratch, int num_cus);
hipError_t launch_zstd_par_body(hipStream_t st, const uint8_t* in, uint32_t nblk, uint32_t bmax, void* scratch,
                                uint8_t* lit, uint32_t* sll, uint32_t* sml, uint32_t* sof, int num_cus);
hipError_t launch_zstd_par_bytes(hipStream_t st, const uint8_t* in, uint32_t nblk, uint32_t total, void* scratch,
                                 const uint8_t* lit, const uint32_t* sll, const uint32_t* sml, const uint32_t* sof,
                                 uint8_t* val, uint32_t* pa, uint32_t* pb, uint32_t* changed, uint8_t* out,
                                 int num_cus);

// Seeks (seek.hip): block.NewIteratorAtKey per query over decoded blocks; the SST index seek.
hipError_t launch_block_seek_staged(hipStream_t st, const void* hsrc_dev, size_t bytes, void* base, size_t o_data,
                                    size_t o_off, size_t o_meta, size_t o_q, size_t o_keys, size_t o_koff, uint64_t nq,
                                    slate_seek* res, slate_seek_warn* warn, uint32_t warn_cap);
hipError_t launch_block_seek(hipStream_t st, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                             const uint32_t* qblock, const uint8_t* qkeys, const uint64_t* qkey_off, uint64_t nq,
                             slate_seek* res, slate_seek_warn* warn = nullptr, uint32_t warn_cap = 0);
hipError_t launch_index_seek(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint64_t n_blocks,
                             const uint8_t* qkeys, const uint64_t* qkey_off, uint64_t nq, uint64_t* out);

// CodecLz4 index / filter payloads split by (independent) data block: blk = nblk x (frame offset,
// block size word); one wave per block in LDS; sizes[k] = decoded bytes at slots + k * 64 KiB, or
// ~0u for a block the serial path must decode (decode.hip).
constexpr uint32_t kLz4PayloadSlot = 65536;
hipError_t launch_lz4_payload_blocks(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                     uint32_t bmax, uint8_t* slots, uint32_t* sizes, int num_cus);
// CodecZstd index / filter payloads split by block (blk = nblk x (frame offset, block header)),
// the same contract for blocks that decode on their own (decode.hip).
hipError_t launch_zstd_payload_blocks(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                      uint32_t bmax, uint8_t* slots, uint32_t* sizes, int num_cus);
// CodecZlib index / filter payloads split at this builder's piece ends (seg = nseg x (stream
// offset, length) of raw deflate segments), the same contract (decode.hip); Adler-32 partial sums
// per 4 KiB slice (part = 2 u64 per slice: sum x, sum (slice end - j) x).
hipError_t launch_zlib_payload_segs(hipStream_t st, const uint8_t* in, const uint32_t* seg, uint32_t nseg,
                                    uint8_t* slots, uint32_t* sizes, int num_cus);
hipError_t launch_adler_slices(hipStream_t st, const uint8_t* p, uint32_t n, uint64_t* part);
// The low 32 bits of XXH64 (seed 0) of a 16-byte aligned device buffer into *out (one wave).
hipError_t launch_xxh64_lo(hipStream_t st, const uint8_t* p, uint32_t n, uint32_t* out);
// XXH32 (seed 0) of n bytes of a 16-byte aligned device buffer into *out (one wave).
hipError_t launch_xxh32(hipStream_t st, const uint8_t* p, uint32_t n, uint32_t* out);

// Validates that the code object loads on the current device.
hipError_t decode_kernels_available();

}  // namespace slate
