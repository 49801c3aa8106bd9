// C-ABI: library-owned memory for the device-resident entry points (SURVEY 8b "Ownership":
// "Device-resident mode uses opaque handles (slate_ctx*, slate_devbuf*) owned by the C side"),
// and executeCompaction's codec path as one call over them (slate_compact).
//
// cgo forbids C from keeping Go pointers after a call returns, so a Go caller cannot hand Go
// memory to the stream-ordered device entries.  slate_devbuf is HBM of the context's GPU and
// slate_hostbuf page-locked host memory, both allocated and freed by the library; the *_device
// entry points take slate_devbuf_ptr(b) (+ a byte offset), and the asynchronous copies take
// hostbufs, so nothing the GPU touches after a call returns belongs to Go.
#include <algorithm>
#include <cstring>
#include <vector>

#include "host_ctx.h"

struct slate_devbuf {
  int device = 0;
  void* p = nullptr;     // base + kDevGuard (readable bytes in front, as DevBuf)
  void* base = nullptr;
  uint64_t size = 0;
};

struct slate_hostbuf {
  void* p = nullptr;
  uint64_t size = 0;
};

namespace {

bool in_range(uint64_t off, uint64_t n, uint64_t size) { return off <= size && n <= size - off; }

}  // namespace

extern "C" {

slate_devbuf* slate_devbuf_alloc(slate_ctx* ctx, uint64_t bytes, int* status) {
  int dummy;
  if (!status) status = &dummy;
  if (!ctx) {
    *status = SLATE_E_INVALID_ARG;
    return nullptr;
  }
  if (ctx_bind(ctx) != hipSuccess) {
    *status = SLATE_E_NO_DEVICE;
    return nullptr;
  }
  slate_devbuf* b = new slate_devbuf();
  b->device = ctx->device;
  b->size = bytes;
  // a zero-byte buffer still has a valid, distinct address (16 bytes: the decode kernels' alignment)
  const hipError_t e = hipMalloc(&b->base, std::max<uint64_t>(bytes, 16) + kDevGuard);
  if (e != hipSuccess) {
    delete b;
    *status = hip_status(e);
    return nullptr;
  }
  b->p = static_cast<uint8_t*>(b->base) + kDevGuard;
  *status = SLATE_OK;
  return b;
}

void slate_devbuf_free(slate_devbuf* b) {
  if (!b) return;
  (void)hipSetDevice(b->device);
  // hipFree synchronises the device: no kernel still reads or writes the buffer afterwards
  if (b->base) (void)hipFree(b->base);
  delete b;
}

void* slate_devbuf_ptr(const slate_devbuf* b) { return b ? b->p : nullptr; }
uint64_t slate_devbuf_size(const slate_devbuf* b) { return b ? b->size : 0; }

int slate_devbuf_upload(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const void* src, uint64_t n) {
  if (!ctx || !dst || (n && !src) || !in_range(dst_off, n, dst->size) || dst->device != ctx->device)
    return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  // large copies go through the context's page-locked staging (ctx_h2d), synchronous either way
  return ctx_h2d(ctx, static_cast<uint8_t*>(dst->p) + dst_off, src, n, ctx->stream);
}

int slate_devbuf_download(slate_ctx* ctx, void* dst, const slate_devbuf* src, uint64_t src_off, uint64_t n) {
  if (!ctx || !src || (n && !dst) || !in_range(src_off, n, src->size) || src->device != ctx->device)
    return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  return ctx_d2h(ctx, dst, static_cast<const uint8_t*>(src->p) + src_off, n, ctx->stream);
}

int slate_devbuf_copy(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const slate_devbuf* src, uint64_t src_off,
                      uint64_t n) {
  if (!ctx || !dst || !src || !in_range(dst_off, n, dst->size) || !in_range(src_off, n, src->size) ||
      dst->device != ctx->device || src->device != ctx->device)
    return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  if (n)
    SLATE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(dst->p) + dst_off, static_cast<const uint8_t*>(src->p) + src_off, n,
                             hipMemcpyDeviceToDevice, ctx->stream));
  return SLATE_OK;
}

int slate_devbuf_memset(slate_ctx* ctx, slate_devbuf* b, uint64_t off, int value, uint64_t n) {
  if (!ctx || !b || !in_range(off, n, b->size) || b->device != ctx->device) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  if (n) SLATE_HIP(hipMemsetAsync(static_cast<uint8_t*>(b->p) + off, value, n, ctx->stream));
  return SLATE_OK;
}

slate_hostbuf* slate_hostbuf_alloc(slate_ctx* ctx, uint64_t bytes, int* status) {
  int dummy;
  if (!status) status = &dummy;
  if (!ctx) {
    *status = SLATE_E_INVALID_ARG;
    return nullptr;
  }
  if (ctx_bind(ctx) != hipSuccess) {
    *status = SLATE_E_NO_DEVICE;
    return nullptr;
  }
  slate_hostbuf* b = new slate_hostbuf();
  b->size = bytes;
  const hipError_t e = hipHostMalloc(&b->p, std::max<uint64_t>(bytes, 16), hipHostMallocDefault);
  if (e != hipSuccess) {
    delete b;
    *status = hip_status(e);
    return nullptr;
  }
  *status = SLATE_OK;
  return b;
}

void slate_hostbuf_free(slate_hostbuf* b) {
  if (!b) return;
  if (b->p) (void)hipHostFree(b->p);
  delete b;
}

void* slate_hostbuf_ptr(const slate_hostbuf* b) { return b ? b->p : nullptr; }
uint64_t slate_hostbuf_size(const slate_hostbuf* b) { return b ? b->size : 0; }

int slate_devbuf_upload_async(slate_ctx* ctx, slate_devbuf* dst, uint64_t dst_off, const slate_hostbuf* src,
                              uint64_t src_off, uint64_t n) {
  if (!ctx || !dst || !src || !in_range(dst_off, n, dst->size) || !in_range(src_off, n, src->size) ||
      dst->device != ctx->device)
    return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  if (n)
    SLATE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(dst->p) + dst_off, static_cast<const uint8_t*>(src->p) + src_off, n,
                             hipMemcpyHostToDevice, ctx->stream));
  return SLATE_OK;
}

int slate_devbuf_download_async(slate_ctx* ctx, slate_hostbuf* dst, uint64_t dst_off, const slate_devbuf* src,
                                uint64_t src_off, uint64_t n) {
  if (!ctx || !dst || !src || !in_range(dst_off, n, dst->size) || !in_range(src_off, n, src->size) ||
      src->device != ctx->device)
    return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  if (n)
    SLATE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(dst->p) + dst_off, static_cast<const uint8_t*>(src->p) + src_off, n,
                             hipMemcpyDeviceToHost, ctx->stream));
  return SLATE_OK;
}

}  // extern "C"
