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

// Host-buffer batch: H2D, plan, (sync to size the outputs), decode, D2H.
int slate_block_decode_batch(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_off, slate_block_meta* meta,
                             slate_row* rows, uint64_t rows_cap, uint64_t* row_base) {
  if (!ctx || !in_off || !out_off || !row_base || (n && (!meta || !in))) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  const uint64_t total_in = in_off[n] - in_off[0];
  // keep the device copy 16-byte aligned relative to the host layout
  SLATE_HIP(ctx->d_in.ensure(total_in + 32));
  SLATE_HIP(ctx->d_in_off.ensure((size_t(n) + 1) * 8));
  SLATE_HIP(ctx->d_out_off.ensure((size_t(n) + 1) * 8));
  SLATE_HIP(ctx->d_row_base.ensure((size_t(n) + 1) * 8));
  SLATE_HIP(ctx->d_scratch.ensure(decode_scratch_bytes(n) + 64));
  std::vector<uint64_t> rel(size_t(n) + 1);
  for (uint32_t i = 0; i <= n; i++) rel[i] = in_off[i] - in_off[0];
  if (total_in) SLATE_HIP(hipMemcpyAsync(ctx->d_in.p, in + in_off[0], total_in, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(ctx->d_in_off.p, rel.data(), (size_t(n) + 1) * 8, hipMemcpyHostToDevice, st));
  SLATE_HIP(launch_decode_plan(st, codec, ctx->d_in.as<uint8_t>(), ctx->d_in_off.as<uint64_t>(), n,
                               ctx->d_out_off.as<uint64_t>(), ctx->d_row_base.as<uint64_t>(), ctx->d_scratch.p));
  SLATE_HIP(hipMemcpyAsync(out_off, ctx->d_out_off.p, (size_t(n) + 1) * 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(row_base, ctx->d_row_base.p, (size_t(n) + 1) * 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const uint64_t total_out = out_off[n], total_rows = row_base[n];
  if (total_out > out_cap || total_rows > rows_cap || (total_out && !out) || (total_rows && !rows))
    return SLATE_E_CAPACITY;
  if (n == 0) return SLATE_OK;
  SLATE_HIP(ctx->d_out.ensure(total_out + 16));
  SLATE_HIP(ctx->d_meta.ensure(size_t(n) * sizeof(slate_block_meta)));
  SLATE_HIP(ctx->d_rows.ensure((total_rows + 1) * sizeof(slate_row)));
  DecodeArgs a{codec, ctx->d_in.as<uint8_t>(), ctx->d_in_off.as<uint64_t>(), n, ctx->d_out.as<uint8_t>(),
               ctx->d_out_off.as<uint64_t>(), ctx->d_meta.as<slate_block_meta>(), ctx->d_rows.as<slate_row>(),
               ctx->d_row_base.as<uint64_t>(), nullptr, nullptr, 0};
  SLATE_HIP(launch_decode(st, a, ctx->d_scratch.p, ctx->num_cus));
  if (total_out) SLATE_HIP(hipMemcpyAsync(out, ctx->d_out.p, total_out, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(meta, ctx->d_meta.p, size_t(n) * sizeof(slate_block_meta), hipMemcpyDeviceToHost, st));
  if (total_rows)
    SLATE_HIP(hipMemcpyAsync(rows, ctx->d_rows.p, total_rows * sizeof(slate_row), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

int slate_block_decode(slate_ctx* ctx, int codec, const uint8_t* in, size_t in_len, uint8_t* out, size_t out_cap,
                       size_t* out_len, slate_block_meta* meta, uint16_t* offsets, size_t offsets_cap) {
  if (!ctx || !meta || (in_len && !in)) return SLATE_E_INVALID_ARG;
  uint64_t in_off[2] = {0, in_len}, out_off[2], row_base[2];
  // decode into a scratch host vector (the batch output is 16-byte padded)
  std::vector<uint8_t> tmp;
  std::vector<slate_row> rows;
  // size pass
  int st = slate_block_decode_batch(ctx, codec, in, in_off, 1, nullptr, 0, out_off, meta, nullptr, 0, row_base);
  if (st == SLATE_E_CAPACITY) {
    tmp.resize(out_off[1] + 16);
    rows.resize(row_base[1] + 1);
    st = slate_block_decode_batch(ctx, codec, in, in_off, 1, tmp.data(), tmp.size(), out_off, meta, rows.data(),
                                  rows.size(), row_base);
  }
  if (st != SLATE_OK) return st;
  if (meta->status != SLATE_OK) return meta->status;
  // Decoded length = data_len + 2 * n_rows + 2 for a successfully decoded block.
  size_t dl = size_t(meta->data_len) + 2 * size_t(meta->n_rows) + 2;
  if (out_len) *out_len = dl;
  if (dl > out_cap || (offsets && meta->n_rows > offsets_cap)) return SLATE_E_CAPACITY;
  if (out && dl) memcpy(out, tmp.data(), dl);
  if (offsets)
    for (uint32_t i = 0; i < meta->n_rows; i++) offsets[i] = ld_be16(tmp.data() + meta->data_len + 2 * i);
  return SLATE_OK;
}

}  // extern "C"
