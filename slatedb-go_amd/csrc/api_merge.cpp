// C-ABI for the compaction merge: iter.MergeSort (internal/iter/merge.go:12-111) over k sorted
// iterators, as executeCompaction (compaction/executor.go:92-151) feeds it.  Kernels: merge.hip.
#include <vector>

#include "../../include/slatecodec.h"
#include "host_ctx.h"

using namespace slate;

namespace {

int check_sources(uint32_t k, const uint64_t* src_start, uint64_t* n, std::vector<uint32_t>* s32) {
  if (k == 0 || !src_start || src_start[0] != 0) return SLATE_E_INVALID_ARG;
  s32->resize(size_t(k) + 1);
  for (uint32_t j = 0; j <= k; j++) {
    if (j && src_start[j] < src_start[j - 1]) return SLATE_E_INVALID_ARG;
    if (src_start[j] >= 0xFFFFFFFFull) return SLATE_E_INVALID_ARG;
    (*s32)[j] = uint32_t(src_start[j]);
  }
  *n = src_start[k];
  return SLATE_OK;
}

}  // namespace

extern "C" {

size_t slate_merge_scratch_bytes(uint64_t n, uint32_t k) {
  return n >= 0xFFFFFFFFull ? 0 : merge_scratch_bytes(uint32_t(n), k);
}

int slate_merge_sorted_device(slate_ctx* ctx, uint32_t k, const uint8_t* d_keys, const uint64_t* d_key_off,
                              const uint64_t* src_start, uint32_t* d_out_idx, uint64_t* d_n_out,
                              uint32_t* d_flags, void* d_scratch) {
  if (!ctx || !d_key_off || !d_out_idx || !d_n_out || !d_flags || !d_scratch) return SLATE_E_INVALID_ARG;
  uint64_t n = 0;
  std::vector<uint32_t> s32;
  int st = check_sources(k, src_start, &n, &s32);
  if (st != SLATE_OK) return st;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_merge(ctx->stream, d_keys, d_key_off, uint32_t(n), s32.data(), k, d_scratch, d_out_idx, d_n_out,
                         d_flags));
  // the k+1 source starts are copied from pageable host memory: make sure the copy has been
  // taken before the caller's vector can go away (cgo rule: no pointer kept after return)
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  return SLATE_OK;
}

int slate_merge_sorted(slate_ctx* ctx, uint32_t k, const uint8_t* keys, const uint64_t* key_off,
                       const uint64_t* src_start, uint32_t* out_idx, uint64_t* n_out) {
  if (!ctx || !key_off || !n_out) return SLATE_E_INVALID_ARG;
  *n_out = 0;
  uint64_t n = 0;
  std::vector<uint32_t> s32;
  int st = check_sources(k, src_start, &n, &s32);
  if (st != SLATE_OK) return st;
  if (n && (!out_idx || !keys)) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t s = ctx->stream;
  const uint64_t kb = key_off[n] - key_off[0];
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = key_off[i] - key_off[0];
  SLATE_HIP(ctx->e_a.ensure(kb + 16));
  SLATE_HIP(ctx->e_b.ensure((n + 1) * 8 + 4 * n + 64));
  SLATE_HIP(ctx->e_c.ensure(merge_scratch_bytes(uint32_t(n), k)));
  uint64_t* d_off = ctx->e_b.as<uint64_t>();
  uint64_t* d_n = d_off + n + 1;
  uint32_t* d_flags = reinterpret_cast<uint32_t*>(d_n + 1);
  uint32_t* d_out = d_flags + 2;
  if (kb) SLATE_HIP(hipMemcpyAsync(ctx->e_a.p, keys + key_off[0], kb, hipMemcpyHostToDevice, s));
  SLATE_HIP(hipMemcpyAsync(d_off, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
  SLATE_HIP(launch_merge(s, ctx->e_a.as<uint8_t>(), d_off, uint32_t(n), s32.data(), k, ctx->e_c.p, d_out, d_n,
                         d_flags));
  uint64_t hn = 0;
  uint32_t flags = 0;
  SLATE_HIP(hipMemcpyAsync(&hn, d_n, 8, hipMemcpyDeviceToHost, s));
  SLATE_HIP(hipMemcpyAsync(&flags, d_flags, 4, hipMemcpyDeviceToHost, s));
  SLATE_HIP(hipStreamSynchronize(s));
  if (flags & 1) return SLATE_E_MERGE_UNSORTED;
  if (hn) {
    SLATE_HIP(hipMemcpyAsync(out_idx, d_out, 4 * hn, hipMemcpyDeviceToHost, s));
    SLATE_HIP(hipStreamSynchronize(s));
  }
  *n_out = hn;
  return SLATE_OK;
}

size_t slate_kv_scratch_bytes(uint64_t n) { return kv_scratch_bytes(n); }

int slate_rows_kv_lengths_device(slate_ctx* ctx, uint32_t n_blocks, const uint64_t* d_row_base,
                                 const slate_block_meta* d_meta, const slate_row* d_rows, uint64_t n_rows,
                                 uint64_t* d_key_off, uint64_t* d_val_off, uint8_t* d_tomb, uint64_t* d_n_kv,
                                 uint32_t* d_flags, void* d_scratch) {
  if (!ctx || !d_row_base || !d_meta || !d_key_off || !d_val_off || !d_n_kv || !d_flags || !d_scratch ||
      n_blocks == 0 || n_rows >= 0xFFFFFFFFull)
    return SLATE_E_INVALID_ARG;
  if (n_rows && (!d_rows || !d_tomb)) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_rows_lengths(ctx->stream, d_row_base, n_blocks, d_meta, d_rows, n_rows, d_key_off, d_val_off,
                                d_tomb, d_n_kv, d_flags, d_scratch));
  return SLATE_OK;
}

int slate_rows_kv_copy_device(slate_ctx* ctx, uint32_t n_blocks, const uint8_t* d_data, const uint64_t* d_out_off,
                              const uint64_t* d_row_base, const slate_row* d_rows, uint64_t n_rows,
                              const uint64_t* d_n_kv, const void* d_scratch, const uint64_t* d_key_off,
                              uint8_t* d_keys, const uint64_t* d_val_off, uint8_t* d_vals) {
  if (!ctx || !d_out_off || !d_row_base || !d_key_off || !d_val_off || !d_n_kv || !d_scratch || n_blocks == 0)
    return SLATE_E_INVALID_ARG;
  if (n_rows && (!d_data || !d_rows)) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_rows_copy(ctx->stream, d_data, d_out_off, d_row_base, n_blocks, d_rows, n_rows, d_n_kv, d_scratch,
                             d_key_off, d_keys, d_val_off, d_vals));
  return SLATE_OK;
}

int slate_kv_gather_lengths_device(slate_ctx* ctx, const uint32_t* d_idx, uint64_t n, const uint64_t* d_key_off,
                                   const uint64_t* d_val_off, const uint8_t* d_tomb, uint64_t* d_okey_off,
                                   uint64_t* d_oval_off, uint8_t* d_otomb, void* d_scratch) {
  if (!ctx || !d_key_off || !d_val_off || !d_okey_off || !d_oval_off || !d_scratch) return SLATE_E_INVALID_ARG;
  if (n && (!d_idx || !d_tomb || !d_otomb)) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_gather_lengths(ctx->stream, d_idx, n, d_key_off, d_val_off, d_tomb, d_okey_off, d_oval_off, d_otomb,
                                  d_scratch));
  return SLATE_OK;
}

int slate_kv_gather_copy_device(slate_ctx* ctx, const uint32_t* d_idx, uint64_t n, const uint8_t* d_keys,
                                const uint64_t* d_key_off, const uint8_t* d_vals, const uint64_t* d_val_off,
                                uint8_t* d_okeys, const uint64_t* d_okey_off, uint8_t* d_ovals,
                                const uint64_t* d_oval_off) {
  if (!ctx || (n && (!d_idx || !d_key_off || !d_val_off || !d_okey_off || !d_oval_off))) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(launch_gather_copy(ctx->stream, d_idx, n, d_keys, d_key_off, d_vals, d_val_off, d_okeys, d_okey_off,
                               d_ovals, d_oval_off));
  return SLATE_OK;
}

}  // extern "C"
