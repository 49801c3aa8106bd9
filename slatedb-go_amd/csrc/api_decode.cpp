// C-ABI: library, context and block decode (block.go:78 Decode; decode.go:107
// ReadBlocks batches go through slate_block_decode_batch).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host_ctx.h"

using namespace slate;

namespace {
constexpr size_t kSeekStageMax = size_t(1) << 20;  // slate_block_seek calls up to this many device bytes: one upload
}  // namespace

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
    case SLATE_E_SEEK_NO_OFFSETS: return "number of block.Offsets must be greater than zero";
    case SLATE_E_SEEK_NO_FULL_KEY: return "unable to locate uncorrupted first key in block; block is corrupt";
    case SLATE_E_SEEK_PANIC: return "runtime error: slice bounds out of range (block.NewIteratorAtKey)";
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
  if (const char* e = getenv("SLATE_COPY_THREADS")) {
    const unsigned long v = strtoul(e, nullptr, 0);
    if (v >= 1 && v <= 256) {
      ctx->copy_threads = v;
      ctx->copy_threads_set = true;
    }
  }
  *status = SLATE_OK;
  return ctx;
}

int slate_ctx_set_copy_threads(slate_ctx* ctx, uint32_t threads) {
  if (!ctx || threads == 0 || threads > 256) return SLATE_E_INVALID_ARG;
  ctx->copy_threads = threads;
  ctx->copy_threads_set = true;
  ctx->copy_pool.reset();  // joins the old workers; the next large copy starts the new count
  return SLATE_OK;
}

int slate_ctx_set_timing(slate_ctx* ctx, int on) {
  if (!ctx) return SLATE_E_INVALID_ARG;
  ctx->timing = on != 0;
  if (ctx->timing) {
    SLATE_HIP(ctx_bind(ctx));
    if (!ctx->t_ref) SLATE_HIP(hipEventCreate(&ctx->t_ref));
    SLATE_HIP(hipEventRecord(ctx->t_ref, ctx->stream));
    std::lock_guard<std::mutex> lk(ctx->span_mu);
    ctx->spans.clear();
  }
  return SLATE_OK;
}

int slate_ctx_gpu_busy(slate_ctx* ctx, double* busy_ms, double* sum_ms, int reset) {
  if (!ctx || !busy_ms) return SLATE_E_INVALID_ARG;
  *busy_ms = ctx->span_union_ms();
  const uint64_t ns = reset ? ctx->gpu_ns.exchange(0) : ctx->gpu_ns.load();
  if (sum_ms) *sum_ms = double(ns) * 1e-6;
  if (reset) {
    std::lock_guard<std::mutex> lk(ctx->span_mu);
    ctx->spans.clear();
  }
  return SLATE_OK;
}

int slate_ctx_handbacks(slate_ctx* ctx, uint64_t* n, int reset) {
  if (!ctx || !n) return SLATE_E_INVALID_ARG;
  *n = 0;
  SLATE_HIP(ctx_bind(ctx));
  // every stream that can add to the counter: the context stream, its side stream, the pipeline
  // lanes (host-buffer decodes) and the filter's aux stream; the single-block and compaction
  // paths run on the context stream or a lane
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->side.s) SLATE_HIP(hipStreamSynchronize(ctx->side.s));
  if (ctx->aux) SLATE_HIP(hipStreamSynchronize(ctx->aux));
  for (auto& L : ctx->lanes)
    if (L.stream) SLATE_HIP(hipStreamSynchronize(L.stream));
  if (!ctx->d_handbacks.p) return SLATE_OK;
  SLATE_HIP(hipMemcpy(n, ctx->d_handbacks.p, 8, hipMemcpyDeviceToHost));
  if (reset) SLATE_HIP(hipMemset(ctx->d_handbacks.p, 0, 8));
  return SLATE_OK;
}

int slate_ctx_gpu_time(slate_ctx* ctx, double* ms, int reset) {
  if (!ctx || !ms) return SLATE_E_INVALID_ARG;
  *ms = double(reset ? ctx->gpu_ns.exchange(0) : ctx->gpu_ns.load()) * 1e-6;
  return SLATE_OK;
}

}  // extern "C"

uint64_t* ctx_handbacks(slate_ctx* ctx) {
  if (!ctx->d_handbacks.p) {
    if (ctx->d_handbacks.ensure(16) != hipSuccess || hipMemset(ctx->d_handbacks.p, 0, 16) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  return ctx->d_handbacks.as<uint64_t>();
}

extern "C" {

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
size_t slate_decode_scratch_bytes_codec(uint32_t n_blocks, int codec) {
  return decode_scratch_bytes_codec(n_blocks, codec);
}

int slate_block_decode_plan_device(slate_ctx* ctx, int codec, const uint8_t* d_in, const uint64_t* d_in_off,
                                   uint32_t n, uint64_t* d_out_off, uint64_t* d_row_base, void* d_scratch) {
  if (!ctx || !d_in_off || !d_out_off || !d_row_base || !d_scratch) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  ctx->zl_armed = false;
  // CodecZlib: the plan is phase Z itself (the stream has no decoded size to read off), its output
  // kept in the context for the decode call that follows (each stream inflated once, not twice)
  // (SLATE_ZL_NO_STAGE, read per call: same-process A/B runs, tools/zlib_ab.py)
  if (codec == SLATE_CODEC_ZLIB && n >= 64 && d_in && !getenv("SLATE_ZL_NO_STAGE")) {
    SLATE_HIP(ctx->zl_stage.ensure(zl_stage_bytes(n)));
    const ZlStage g = zl_stage_carve(ctx->zl_stage.p, n);
    SLATE_HIP(launch_decode_plan(ctx->stream, codec, d_in, d_in_off, n, d_out_off, d_row_base, d_scratch, &g,
                                 ctx->num_cus));
    ctx->zl_plan.in = d_in;
    ctx->zl_plan.in_off = d_in_off;
    ctx->zl_plan.out_off = d_out_off;
    ctx->zl_plan.n = n;
    ctx->zl_plan.stream = ctx->stream;
    ctx->zl_armed = true;
    return SLATE_OK;
  }
  SLATE_HIP(launch_decode_plan(ctx->stream, codec, d_in, d_in_off, n, d_out_off, d_row_base, d_scratch));
  return SLATE_OK;
}

int slate_block_decode_device(slate_ctx* ctx, int codec, const uint8_t* d_in, const uint64_t* d_in_off, uint32_t n,
                              uint8_t* d_out, const uint64_t* d_out_off, slate_block_meta* d_meta, slate_row* d_rows,
                              const uint64_t* d_row_base) {
  // CodecNone with d_out == NULL: block.Decode's aliasing (block.go:122, compression.go:128-129) --
  // block i's Data is the input itself, d_in + d_in_off[i] (meta.data_len bytes; the offsets after
  // it), so nothing is copied and d_out_off is not used; metas and rows as always
  const bool alias = codec == SLATE_CODEC_NONE && d_out == nullptr && d_in != nullptr;
  if (!ctx || !d_in_off || (!d_out_off && !alias) || !d_meta || !d_row_base) return SLATE_E_INVALID_ARG;
  if ((reinterpret_cast<uintptr_t>(d_out) & 15) != 0 || (!d_out && !alias && n)) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  // the scratch is owned by the context for the device-resident call
  SLATE_HIP(ctx->d_scratch.ensure(decode_scratch_bytes_codec(n, codec)));
  DecodeArgs a{codec, d_in, d_in_off, n, alias ? const_cast<uint8_t*>(d_in) : d_out, alias ? d_in_off : d_out_off,
               d_meta, d_rows, d_row_base, nullptr, nullptr, 0};
  a.no_data = alias ? 1u : 0u;
  a.side = &ctx->side;
  a.handbacks = ctx_handbacks(ctx);
  // the staged plan of exactly these inputs and plan outputs, on this stream, not yet used
  const bool staged = ctx->zl_armed && codec == SLATE_CODEC_ZLIB && ctx->zl_plan.in == d_in &&
                      ctx->zl_plan.in_off == d_in_off && ctx->zl_plan.out_off == d_out_off &&
                      ctx->zl_plan.n == n && ctx->zl_plan.stream == ctx->stream;
  ctx->zl_armed = false;
  ZlStage g{};
  if (staged) g = zl_stage_carve(ctx->zl_stage.p, n);
  SLATE_HIP(launch_decode(ctx->stream, a, ctx->d_scratch.p, ctx->num_cus, staged ? &g : nullptr));
  return SLATE_OK;
}

// slate_block_decode_batch / slate_block_decode / the sharded decode: api_host.cpp.

int slate_block_seek_warn_device(slate_ctx* ctx, const uint8_t* d_data, const uint64_t* d_out_off,
                                 const slate_block_meta* d_meta, const uint32_t* d_qblock, const uint8_t* d_keys,
                                 const uint64_t* d_key_off, uint64_t n, slate_seek* d_res, slate_seek_warn* d_warn,
                                 uint32_t warn_cap) {
  if (!ctx || (n && (!d_out_off || !d_meta || !d_qblock || !d_key_off || !d_res))) return SLATE_E_INVALID_ARG;
  if (warn_cap && !d_warn) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_block_seek(ctx->stream, d_data, d_out_off, d_meta, d_qblock, d_keys, d_key_off, n, d_res,
                              warn_cap ? d_warn : nullptr, warn_cap));
  return SLATE_OK;
}

int slate_block_seek_device(slate_ctx* ctx, const uint8_t* d_data, const uint64_t* d_out_off,
                            const slate_block_meta* d_meta, const uint32_t* d_qblock, const uint8_t* d_keys,
                            const uint64_t* d_key_off, uint64_t n, slate_seek* d_res) {
  return slate_block_seek_warn_device(ctx, d_data, d_out_off, d_meta, d_qblock, d_keys, d_key_off, n, d_res, nullptr,
                                      0);
}

int slate_block_seek_warn(slate_ctx* ctx, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                          uint32_t n_blocks, const uint32_t* qblock, const uint8_t* keys, const uint64_t* key_off,
                          uint64_t n, slate_seek* res, slate_seek_warn* warn, uint32_t warn_cap) {
  if (!ctx || !out_off || (n_blocks && !meta) || (n && (!qblock || !key_off || !res))) return SLATE_E_INVALID_ARG;
  if (warn_cap && !warn) return SLATE_E_INVALID_ARG;
  if (n == 0) return SLATE_OK;
  for (uint64_t i = 0; i < n; i++)
    if (qblock[i] >= n_blocks) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  const uint64_t db = out_off[n_blocks], kb = key_off[n] - key_off[0];
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t wbytes = size_t(n) * warn_cap * sizeof(slate_seek_warn);
  const size_t o_data = carve(db + 16), o_off = carve((size_t(n_blocks) + 1) * 8),
               o_meta = carve(size_t(n_blocks) * sizeof(slate_block_meta) + 16), o_q = carve(n * 4),
               o_keys = carve(kb + 16), o_koff = carve((n + 1) * 8), o_res = carve(n * sizeof(slate_seek)),
               o_warn = carve(wbytes + 16);
  SLATE_HIP(ctx->e_g.ensure(off));
  uint8_t* base = ctx->e_g.as<uint8_t>();
  // Small calls (a point read: one block, one key): every input packed into page-locked staging
  // in the device layout and uploaded by one copy; the kernel writes the results into that
  // staging through its device address; one wait.  Pageable copies cost ~10 us each.
  if (off <= kSeekStageMax) {
    SLATE_HIP(ctx->h_seek.ensure(off));
    uint8_t* h = ctx->h_seek.as<uint8_t>();
    if (db) memcpy(h + o_data, data, db);
    memcpy(h + o_off, out_off, (size_t(n_blocks) + 1) * 8);
    if (n_blocks) memcpy(h + o_meta, meta, size_t(n_blocks) * sizeof(slate_block_meta));
    memcpy(h + o_q, qblock, n * 4);
    if (kb) memcpy(h + o_keys, keys + key_off[0], kb);
    uint64_t* hk = reinterpret_cast<uint64_t*>(h + o_koff);
    for (uint64_t i = 0; i <= n; i++) hk[i] = key_off[i] - key_off[0];
    uint8_t* hdev = static_cast<uint8_t*>(mapped_ptr(h));
    if (hdev && n <= 256) {  // one launch: the kernel pulls the staging over the link itself
      SLATE_HIP(launch_block_seek_staged(st, hdev, o_res, base, o_data, o_off, o_meta, o_q, o_keys, o_koff, n,
                                         reinterpret_cast<slate_seek*>(hdev + o_res),
                                         warn_cap ? reinterpret_cast<slate_seek_warn*>(hdev + o_warn) : nullptr,
                                         warn_cap));
      SLATE_HIP(hipStreamSynchronize(st));
      memcpy(res, h + o_res, n * sizeof(slate_seek));
      if (wbytes) memcpy(warn, h + o_warn, wbytes);
      return SLATE_OK;
    }
    if (hdev) {
      SLATE_HIP(hipMemcpyAsync(base, h, o_res, hipMemcpyHostToDevice, st));
      SLATE_HIP(launch_block_seek(st, base + o_data, reinterpret_cast<const uint64_t*>(base + o_off),
                                  reinterpret_cast<const slate_block_meta*>(base + o_meta),
                                  reinterpret_cast<const uint32_t*>(base + o_q), base + o_keys,
                                  reinterpret_cast<const uint64_t*>(base + o_koff), n,
                                  reinterpret_cast<slate_seek*>(hdev + o_res),
                                  warn_cap ? reinterpret_cast<slate_seek_warn*>(hdev + o_warn) : nullptr, warn_cap));
      SLATE_HIP(hipStreamSynchronize(st));
      memcpy(res, h + o_res, n * sizeof(slate_seek));
      if (wbytes) memcpy(warn, h + o_warn, wbytes);
      return SLATE_OK;
    }
  }
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = key_off[i] - key_off[0];
  if (db) SLATE_HIP(hipMemcpyAsync(base + o_data, data, db, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(base + o_off, out_off, (size_t(n_blocks) + 1) * 8, hipMemcpyHostToDevice, st));
  if (n_blocks)
    SLATE_HIP(hipMemcpyAsync(base + o_meta, meta, size_t(n_blocks) * sizeof(slate_block_meta), hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(base + o_q, qblock, n * 4, hipMemcpyHostToDevice, st));
  if (kb) SLATE_HIP(hipMemcpyAsync(base + o_keys, keys + key_off[0], kb, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(base + o_koff, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  slate_seek_warn* dw = warn_cap ? reinterpret_cast<slate_seek_warn*>(base + o_warn) : nullptr;
  SLATE_HIP(launch_block_seek(st, base + o_data, reinterpret_cast<const uint64_t*>(base + o_off),
                              reinterpret_cast<const slate_block_meta*>(base + o_meta),
                              reinterpret_cast<const uint32_t*>(base + o_q), base + o_keys,
                              reinterpret_cast<const uint64_t*>(base + o_koff), n,
                              reinterpret_cast<slate_seek*>(base + o_res), dw, warn_cap));
  SLATE_HIP(hipMemcpyAsync(res, base + o_res, n * sizeof(slate_seek), hipMemcpyDeviceToHost, st));
  if (wbytes) SLATE_HIP(hipMemcpyAsync(warn, dw, wbytes, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

int slate_block_seek(slate_ctx* ctx, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                     uint32_t n_blocks, const uint32_t* qblock, const uint8_t* keys, const uint64_t* key_off,
                     uint64_t n, slate_seek* res) {
  return slate_block_seek_warn(ctx, data, out_off, meta, n_blocks, qblock, keys, key_off, n, res, nullptr, 0);
}

}  // extern "C"
