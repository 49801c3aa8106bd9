// Microbenchmark probe (tooling, not product): LDS behaviours that decide the
// Snappy decode design on gfx950.
//  1. correctness of unaligned ds_read_b32 / ds_write_b32 (byte offsets 0..3)
//  2. cost of per-lane byte rings: 64 lanes each streaming through their own
//     LDS region with ds_read_u8/ds_write_b8 vs dword ops
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void unaligned_rw(uint32_t* out, int shift) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = uint8_t(i * 7 + 3);
  __syncthreads();
  // unaligned read
  uint32_t off = threadIdx.x * 5 + shift;
  uint32_t v;
  __builtin_memcpy(&v, buf + off, 4);  // lets the compiler emit an unaligned ds_read_b32 if legal
  uint32_t w = *reinterpret_cast<const uint32_t*>(buf + off);  // explicit unaligned dword access
  out[threadIdx.x * 4 + 0] = v;
  out[threadIdx.x * 4 + 1] = w;
  __syncthreads();
  // unaligned write (lanes write disjoint 4-byte windows at byte offsets)
  *reinterpret_cast<uint32_t*>(buf + 2048 + threadIdx.x * 5 + shift) = 0xA1B2C3D4u + threadIdx.x;
  __syncthreads();
  uint32_t r = 0;
  for (int b = 0; b < 4; b++) r |= uint32_t(buf[2048 + threadIdx.x * 5 + shift + b]) << (8 * b);
  out[threadIdx.x * 4 + 2] = r;
  out[threadIdx.x * 4 + 3] = 0;
}

// Each lane owns a ring of RING bytes (lane stride STRIDE bytes); moves N bytes
// from position p - off to p, byte by byte (mode 0) or 4 at a time via
// unaligned dword ops (mode 1).
template <int MODE>
__global__ void ring_pump(uint32_t* sink, int iters, int off_base) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int STRIDE = 324, RING = 256;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* ring = smem + (wave * 64 + lane) * STRIDE;
  for (int i = 0; i < RING; i++) ring[i] = uint8_t(lane + i);
  uint32_t p = 128 + lane * 3, acc = 0;
  int off = off_base + (lane & 7);
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {
      for (int b = 0; b < 4; b++) {
        uint8_t x = ring[(p - off + b) & (RING - 1)];
        ring[(p + b) & (RING - 1)] = x;
        acc += x;
      }
    } else {
      uint32_t x = *reinterpret_cast<const uint32_t*>(ring + ((p - off) & (RING - 1 - 3)));
      *reinterpret_cast<uint32_t*>(ring + (p & (RING - 1 - 3))) = x;
      acc += x;
    }
    p += 4;
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 1 << 24);
  std::vector<uint32_t> h(256 * 4);
  int ok_read = 1, ok_write = 1;
  for (int shift = 0; shift < 4; shift++) {
    unaligned_rw<<<1, 256>>>(d, shift);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    for (int t = 0; t < 256; t++) {
      uint32_t off = t * 5 + shift, want = 0;
      for (int b = 0; b < 4; b++) want |= uint32_t(uint8_t((off + b) * 7 + 3)) << (8 * b);
      if (h[t * 4] != want || h[t * 4 + 1] != want) ok_read = 0;
      if (h[t * 4 + 2] != 0xA1B2C3D4u + t) ok_write = 0;
    }
  }
  printf("{\"unaligned_ds_read_b32_ok\": %d, \"unaligned_ds_write_b32_ok\": %d", ok_read, ok_write);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  size_t lds = size_t(threads) * 324;
  for (int mode = 0; mode < 2; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(a);
      if (mode == 0) ring_pump<0><<<blocks, threads, lds>>>(d, iters, 42);
      else ring_pump<1><<<blocks, threads, lds>>>(d, iters, 42);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        double bytes = double(blocks) * threads * iters * 4;
        printf(", \"ring_mode%d_ms\": %.3f, \"ring_mode%d_GBps_moved\": %.1f", mode, ms, mode, bytes / ms / 1e6);
      }
    }
  }
  printf("}\n");
  return 0;
}
