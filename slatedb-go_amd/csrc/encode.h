// Encode-side kernel interfaces (SST builder, bloom, large-buffer CRC).
#pragma once
#include "common.h"

namespace slate {

constexpr int kPackThreads = 256;        // 4 wavefronts, one block each
constexpr uint32_t kPackCap = 8192;      // LDS bytes per wavefront for one encoded block
constexpr uint32_t kPackBigCap = 155648; // one wavefront per workgroup
#ifndef SLATE_SNAP_THREADS
#define SLATE_SNAP_THREADS 768
#endif
#ifndef SLATE_SNAP_OWNER
#define SLATE_SNAP_OWNER 512
#endif
// Snappy pack: one 12-wave workgroup per CU.  Per wave the raw block, its 4096-slot table and a
// 512-byte owner array for the duplicate-slot check (4 KiB before: nine waves per CU; 512 B
// aliases slots, which only makes the exact check run more often): 72 vs 79 ms of GPU time per
// 10 M-KV build, bit-exact (profiles/round3/enc_ab/occupancy.txt)
constexpr int kSnapThreads = SLATE_SNAP_THREADS;
constexpr uint32_t kSnapOwner = SLATE_SNAP_OWNER;
constexpr uint32_t kSnapRaw = 4096;      // raw block bytes handled in LDS (BlockSize 4096)
constexpr uint64_t kSnapChunkSlot = 76544;  // >= MaxEncodedLen(64 KiB), 16-aligned
constexpr uint64_t kSnapMaxChunk = 65536;   // golang/snappy maxBlockSize

struct EncodeArgs {
  const uint8_t* keys;
  const uint64_t* key_off;
  const uint8_t* vals;
  const uint64_t* val_off;
  const uint8_t* tomb;  // 1 = KindTombStone
  uint32_t n;
  uint64_t block_size;
  int codec;
};

// Device work buffers for one encode batch (sized by the host for n KVs).
struct EncodeBufs {
  uint64_t* hashes;      // [n] FNV-1 64 of every key (bloom input), appended per batch
  uint32_t* adj;         // [n]
  uint32_t* next;        // [n]
  uint64_t* bytes;       // [n]
  uint32_t* exit_pos;    // [n]
  uint32_t* entry;       // [chunks]
  uint32_t* starts_tmp;  // [n]
  uint64_t* counts;      // [chunks + 1] -> exclusive scan = chunk_base
  uint64_t* chunk_base;  // alias of counts after the scan
  uint32_t* block_start; // [n]
  uint64_t* block_size;  // [n + 1] -> exclusive scan = out_off
  uint32_t* big_list;    // [n]
  uint32_t* flags;       // 4 words: flags, maxlen, big_count, status
  uint32_t* maxlen;      // (not written: enc_next_kernel reduces the longest block per workgroup)
  uint32_t* big_count;
  uint32_t* status;
};

hipError_t launch_kv_hashes(hipStream_t st, const EncodeArgs& a, uint64_t* hashes, uint32_t* adj, uint32_t* flags);
hipError_t launch_encode(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, int num_cus);
hipError_t launch_encode_blocks(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w);
hipError_t launch_pack(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, uint32_t nblocks,
                       const uint64_t* out_off, uint8_t* out, int num_cus);
hipError_t launch_bloom_build(hipStream_t st, const uint64_t* hashes, uint64_t n, uint32_t num_probes,
                              uint32_t filter_bits, uint32_t* words);
// The same bits (words zeroed beforehand) without global atomics: probes bucketed per 64 KiB slice of
// the filter, each slice OR-ed in LDS.  Scratch bytes from bloom_bucket_scratch_bytes; 0 there means
// the shape is outside the bucketed path's bounds, and the call runs launch_bloom_build.
size_t bloom_bucket_scratch_bytes(uint64_t n, uint32_t num_probes, uint32_t filter_bits);
hipError_t launch_bloom_build_bucketed(hipStream_t st, const uint64_t* hashes, uint64_t n, uint32_t num_probes,
                                       uint32_t filter_bits, uint32_t* words, void* scratch);
hipError_t launch_bloom_check(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                              const uint8_t* bits, uint64_t bits_len, uint32_t num_probes, uint8_t* out);
// Snappy (golang/snappy byte-exact) block and buffer encode
size_t snappy_slots_bytes(uint64_t raw_total, uint64_t nblocks);
hipError_t launch_pack_snappy(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, uint32_t nblocks,
                              const uint64_t* raw_off, uint8_t* slots, uint64_t* csize, int num_cus);
hipError_t launch_pack_snappy_big(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, const uint64_t* raw_off,
                                  uint8_t* rawbuf, uint8_t* slots, uint64_t* csize, uint32_t big_count, int num_cus);
hipError_t launch_compact(hipStream_t st, const uint8_t* slots, const uint64_t* raw_off, const uint64_t* final_off,
                          uint32_t nblocks, uint8_t* out, int num_cus);
// chunk c's encoding (slots + c * kSnapChunkSlot, len[c] bytes) to dst + off[c], one launch
hipError_t launch_snappy_gather(hipStream_t st, const uint8_t* slots, const uint32_t* len, const uint64_t* off,
                                uint64_t nch, uint8_t* dst);
hipError_t launch_snappy_chunks(hipStream_t st, const uint8_t* src, uint64_t n, uint8_t* dst, uint32_t* len,
                                int num_cus);
size_t crc_scratch_bytes(uint64_t n);
hipError_t launch_crc32(hipStream_t st, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out, int num_cus);
// In-place exclusive scan of one u64 array of n+1 entries (the last becomes the total).
hipError_t launch_scan_u64(hipStream_t st, uint64_t* a, uint32_t n_plus_1, void* scratch);
size_t scan_scratch_bytes(uint32_t n_plus_1);

// SST builder KV staging: dst[0..n] = base + (src[i] - src[0]); tomb[i] = empty value;
// *out = index of the first empty key or ~0 (block.go:163); the keys at idx[0..m) gathered
// back to back (out_off: m+1 u64, exclusive scan of their lengths; scratch kv_pick_scratch_bytes).
hipError_t launch_kv_rebase(hipStream_t st, const uint64_t* src, uint64_t n, uint64_t* dst, uint64_t base);
hipError_t launch_kv_tomb_from_values(hipStream_t st, const uint64_t* val_off, uint64_t n, uint8_t* tomb);
hipError_t launch_kv_first_empty(hipStream_t st, const uint64_t* key_off, uint64_t n, uint64_t* out);
size_t kv_pick_scratch_bytes(uint64_t m);
hipError_t launch_kv_pick_keys(hipStream_t st, const uint32_t* idx, uint64_t m, const uint8_t* keys,
                               const uint64_t* key_off, uint64_t* out_off, void* scratch, uint8_t* out);

// compress.Encode for LZ4 / Zlib / Zstd (encode_codecs.hip).  A payload (a block, the filter, the
// index) is cut into pieces of at most 64 KiB; pass 1 parses each piece with the golang/snappy
// block encoder (tags into its slot), pass 2 transcodes the tags into the codec's body, pass 3
// writes each payload's frame (+ BE32 CRC32 of the frame when asked).
struct CodecPiece {
  uint64_t raw;    // offset of the piece's bytes in the raw buffer
  uint64_t tags;   // offset of its tag slot (codec_piece_tags_bytes(len))
  uint64_t body;   // offset of its body slot (codec_piece_body_bytes(len))
  uint64_t seqs;   // Zstd, pieces above 4 KiB: first Seq slot (len / 3 + 2 slots of 12 bytes)
  uint32_t len;
  uint32_t flags;  // bit 0: first piece of its payload, bit 1: last
};
struct CodecPayload {
  uint64_t raw;     // offset of the payload in the raw buffer
  uint32_t len;
  uint32_t first;   // its first piece
  uint32_t npieces;
  uint32_t pad;
};
constexpr uint32_t kBodyRaw = 0xFFFFFFFFu;  // body_len: the piece goes out raw (LZ4 / Zstd) instead
constexpr uint32_t kCodecPieceMax = 65536;
constexpr uint32_t kCodecSmallPiece = 4096;
__host__ __device__ inline uint32_t codec_body_cap(uint32_t len) { return len + len / 8 + 64; }
size_t codec_piece_tags_bytes(uint32_t len);
size_t codec_piece_body_bytes(uint32_t len);
constexpr size_t kCodecSeqBytes = 12;
hipError_t launch_codec_encode(hipStream_t st, int codec, const uint8_t* raw, const CodecPiece* pieces,
                               const uint32_t* small_list, uint32_t n_small, const uint32_t* big_list, uint32_t n_big,
                               uint8_t* tags, uint32_t* tag_len, uint8_t* bodies, uint32_t* body_len, void* big_seqs,
                               int num_cus);
// Frame sizes for out_off: header + pieces + trailer (+ 4 CRC), from the host's body_len copy.
hipError_t launch_codec_frames(hipStream_t st, int codec, const uint8_t* raw, const CodecPayload* pay, uint32_t n,
                               const CodecPiece* pieces, const uint8_t* bodies, const uint32_t* body_len,
                               const uint64_t* out_off, uint8_t* out, bool with_crc, int num_cus);

}  // namespace slate
