// C-ABI: library, context and block decode (block.go:78 Decode; decode.go:107
// ReadBlocks batches go through slate_block_decode_batch).
#include <algorithm>
#include <cstring>

#include "host_ctx.h"

using namespace slate;

extern "C" {

int slate_abi_version(void) { return SLATECODEC_ABI_VERSION; }

const char* slate_status_string(int s) {
  switch (s) {
    case SLATE_OK: return "ok";
    case SLATE_E_BLOCK_TOO_SMALL: return "corrupted block: block is too small; must be at least 6 bytes";
    case SLATE_E_BLOCK_CHECKSUM: return "corrupted block: checksum mismatch";
    case SLATE_E_BLOCK_UNCOMP_SMALL:
      return "corrupted block: uncompressed block is too small; must be at least 2 bytes";
    case SLATE_E_BLOCK_INDEX_OFFSET: return "corrupted block: invalid index offset '%d'; cannot be negative";
    case SLATE_E_BLOCK_OFFSET_BOUNDS: return "corrupted block: block offset[%d] = %d exceeds key value bounds";
    case SLATE_E_BLOCK_NO_OFFSETS: return "corrupted block: Block.Offsets must be greater than 0";
    case SLATE_E_BLOCK_FIRSTKEY_PANIC: return "runtime error: slice bounds out of range (Block.FirstKey)";
    case SLATE_E_BLOCK_EMPTY: return "assertion failed; block cannot be empty";
    case SLATE_E_INVALID_CODEC: return "corrupted; invalid compression codec";
    case SLATE_E_SNAPPY_CORRUPT: return "snappy: corrupt input";
    case SLATE_E_SNAPPY_TOO_LARGE: return "snappy: decoded block is too large";
    case SLATE_E_CODEC_UNSUPPORTED: return "compression codec not supported by this backend";
    case SLATE_E_LZ4_MAGIC: return "lz4: bad magic number";
    case SLATE_E_LZ4_HEADER_CHECKSUM: return "lz4: invalid header checksum";
    case SLATE_E_LZ4_BLOCK_CHECKSUM: return "lz4: invalid block checksum";
    case SLATE_E_LZ4_FRAME_CHECKSUM: return "lz4: invalid frame checksum";
    case SLATE_E_LZ4_CORRUPT: return "lz4: invalid source or destination buffer too short";
    case SLATE_E_ZLIB_HEADER: return "zlib: invalid header";
    case SLATE_E_ZLIB_DICTIONARY: return "zlib: invalid dictionary";
    case SLATE_E_ZLIB_CHECKSUM: return "zlib: invalid checksum";
    case SLATE_E_FLATE_CORRUPT: return "flate: corrupt input before offset %d";
    case SLATE_E_UNEXPECTED_EOF: return "unexpected EOF";
    case SLATE_E_EOF: return "EOF";
    case SLATE_E_ZSTD_MAGIC: return "invalid input: magic number mismatch";
    case SLATE_E_ZSTD_CHECKSUM: return "CRC check failed";
    case SLATE_E_ZSTD_CORRUPT: return "zstd: corrupt input";
    case SLATE_E_ZSTD_FRAME_SIZE: return "frame size does not match size on stream";
    case SLATE_E_ZSTD_DICT: return "unknown dictionary";
    case SLATE_E_ZSTD_RESERVED_BLOCK: return "invalid input: reserved block type encountered";
    case SLATE_E_ROW_TOO_SHORT: return "corrupt v0 row: data length too short to decode a row";
    case SLATE_E_ROW_PREFIX: return "corrupt v0 row: key prefix length exceeds length of first key in block";
    case SLATE_E_ROW_SUFFIX: return "corrupt v0 row: key suffix length exceeds length of block";
    case SLATE_E_ROW_EXPIRE: return "corrupt v0 row: data length too short for expire";
    case SLATE_E_ROW_CREATE: return "corrupt v0 row: data length too short for create";
    case SLATE_E_ROW_VALUE_LEN: return "corrupt v0 row: data length too short for for value length";
    case SLATE_E_ROW_VALUE: return "corrupt v0 row: data length too short for for value";
    case SLATE_E_ROW_PANIC: return "runtime error: index out of range (v0 row seq/flags)";
    case SLATE_E_ROW_PEEK_SHORT: return "corrupt v0 row: data length too short to peek at row";
    case SLATE_E_ROW_OFFSET_RANGE: return "block.Offset[%d] = %d is out of bounds";
    case SLATE_E_FILTER_TOO_SMALL: return "corrupt filter: filter is too small; must be at least 2 bytes";
    case SLATE_E_FILTER_CHECKSUM: return "corrupt filter: invalid checksum";
    case SLATE_E_FILTER_PANIC: return "runtime error: slice bounds out of range (bloom.Decode)";
    case SLATE_E_INDEX_TOO_SHORT: return "corrupted index; too short";
    case SLATE_E_INDEX_CHECKSUM: return "corrupted index; checksum mismatch";
    case SLATE_E_INFO_TOO_SHORT: return "corrupted info; too short";
    case SLATE_E_INFO_CHECKSUM: return "corrupted info; checksum mismatch";
    case SLATE_E_SST_TOO_SHORT: return "corrupted SSTable; too short";
    case SLATE_E_BLOB_RANGE: return "corrupted; [%d:%d] is an invalid range";
    case SLATE_E_RANGE_START: return "block start '%d' range cannot be greater than end range '%d'";
    case SLATE_E_RANGE_END: return "block end '%d' range cannot be greater than size of block meta range '%d'";
    case SLATE_E_FLATBUF: return "runtime error: malformed flatbuffer";
    case SLATE_E_NO_DEVICE: return "no usable HIP device (gfx950 code object not loadable)";
    case SLATE_E_HIP: return "HIP runtime error";
    case SLATE_E_INVALID_ARG: return "invalid argument";
    case SLATE_E_CAPACITY: return "output buffer too small";
    case SLATE_E_OOM: return "out of memory";
    case SLATE_E_MERGE_UNSORTED: return "merge input iterator is not sorted";
    default: return "unknown status";
  }
}

slate_ctx* slate_ctx_create(int device, int* status) {
  int st_dummy;
  if (!status) status = &st_dummy;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count) {
    *status = SLATE_E_NO_DEVICE;
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess || decode_kernels_available() != hipSuccess) {
    *status = SLATE_E_NO_DEVICE;
    return nullptr;
  }
  slate_ctx* ctx = new slate_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    *status = SLATE_E_HIP;
    return nullptr;
  }
  ctx->stream = ctx->own;
  *status = SLATE_OK;
  return ctx;
}

void slate_ctx_destroy(slate_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  ctx->release_all();
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
}

int slate_ctx_set_stream(slate_ctx* ctx, void* s) {
  if (!ctx) return SLATE_E_INVALID_ARG;
  ctx->stream = s ? static_cast<hipStream_t>(s) : ctx->own;
  return SLATE_OK;
}

int slate_ctx_synchronize(slate_ctx* ctx) {
  if (!ctx) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  return SLATE_OK;
}

size_t slate_decode_scratch_bytes(uint32_t n_blocks) { return decode_scratch_bytes(n_blocks); }

int slate_block_decode_plan_device(slate_ctx* ctx, int codec, const uint8_t* d_in, const uint64_t* d_in_off,
                                   uint32_t n, uint64_t* d_out_off, uint64_t* d_row_base, void* d_scratch) {
  if (!ctx || !d_in_off || !d_out_off || !d_row_base || !d_scratch) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_decode_plan(ctx->stream, codec, d_in, d_in_off, n, d_out_off, d_row_base, d_scratch));
  return SLATE_OK;
}

int slate_block_decode_device(slate_ctx* ctx, int codec, const uint8_t* d_in, const uint64_t* d_in_off, uint32_t n,
                              uint8_t* d_out, const uint64_t* d_out_off, slate_block_meta* d_meta, slate_row* d_rows,
                              const uint64_t* d_row_base) {
  if (!ctx || !d_in_off || !d_out_off || !d_meta || !d_row_base) return SLATE_E_INVALID_ARG;
  if ((reinterpret_cast<uintptr_t>(d_out) & 15) != 0) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  // the scratch is owned by the context for the device-resident call
  SLATE_HIP(ctx->d_scratch.ensure(decode_scratch_bytes(n)));
  DecodeArgs a{codec, d_in, d_in_off, n, d_out, d_out_off, d_meta, d_rows, d_row_base, nullptr, nullptr, 0};
  SLATE_HIP(launch_decode(ctx->stream, a, ctx->d_scratch.p, ctx->num_cus));
  return SLATE_OK;
}

// slate_block_decode_batch / slate_block_decode / the sharded decode: api_host.cpp.

}  // extern "C"
