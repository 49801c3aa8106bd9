// Microbenchmark probe (tooling, not product): are unaligned ds_read_b64/b128 and
// ds_write_b64/b128 correct on gfx950 (unaligned access mode), and are
// unaligned 16-B global stores correct?
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef v4u v4u_a4 __attribute__((aligned(4)));
typedef v2u v2u_a4 __attribute__((aligned(4)));
typedef v4u v4u_a1 __attribute__((aligned(1)));

__global__ void probe(uint32_t* out, uint8_t* gbuf, int shift) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) buf[i] = uint8_t(i * 7 + 3);
  __syncthreads();
  const uint32_t off = threadIdx.x * 23 + shift;  // arbitrary byte alignment
  // --- read b128 at a 4-aligned-typed but byte-misaligned address
  v4u r = *reinterpret_cast<const v4u_a4*>(buf + off);
  v2u r2 = *reinterpret_cast<const v2u_a4*>(buf + off + 1);
  out[threadIdx.x * 8 + 0] = r.x;
  out[threadIdx.x * 8 + 1] = r.y;
  out[threadIdx.x * 8 + 2] = r.z;
  out[threadIdx.x * 8 + 3] = r.w;
  out[threadIdx.x * 8 + 4] = r2.x;
  out[threadIdx.x * 8 + 5] = r2.y;
  __syncthreads();
  // --- write b128 at misaligned addresses (disjoint 23-byte strides)
  v4u w = {0x03020100u + threadIdx.x, 0x07060504u, 0x0b0a0908u, 0x0f0e0d0cu};
  *reinterpret_cast<v4u_a4*>(buf + 4096 + off) = w;
  __syncthreads();
  uint32_t ok = 1;
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(&w);
  for (int b = 0; b < 16; b++) ok &= buf[4096 + off + b] == wb[b];
  out[threadIdx.x * 8 + 6] = ok;
  // --- unaligned 16-B global store
  *reinterpret_cast<v4u_a4*>(gbuf + off) = w;
}

int main() {
  uint32_t* d;
  uint8_t* g;
  if (hipMalloc(&d, 64 * 8 * 4) != hipSuccess || hipMalloc(&g, 8192) != hipSuccess) return 1;
  int bad = 0;
  for (int shift = 0; shift < 4; shift++) {
    if (hipMemset(g, 0, 8192) != hipSuccess) return 1;
    probe<<<1, 64>>>(d, g, shift);
    std::vector<uint32_t> h(64 * 8);
    std::vector<uint8_t> gh(8192);
    if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    if (hipMemcpy(gh.data(), g, 8192, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int t = 0; t < 64; t++) {
      const uint32_t off = t * 23 + shift;
      for (int j = 0; j < 4; j++) {
        uint32_t e = 0;
        for (int b = 0; b < 4; b++) e |= uint32_t(uint8_t((off + 4 * j + b) * 7 + 3)) << (8 * b);
        if (h[t * 8 + j] != e) bad |= 1;
      }
      for (int j = 0; j < 2; j++) {
        uint32_t e = 0;
        for (int b = 0; b < 4; b++) e |= uint32_t(uint8_t((off + 1 + 4 * j + b) * 7 + 3)) << (8 * b);
        if (h[t * 8 + 4 + j] != e) bad |= 2;
      }
      if (h[t * 8 + 6] != 1) bad |= 4;
      uint32_t w0 = 0x03020100u + t;
      if (gh[off] != (w0 & 0xff) || gh[off + 15] != 0x0f) bad |= 8;
    }
  }
  printf("unaligned ds_read_b128 %s, ds_read_b64 %s, ds_write_b128 %s, global store x4 %s\n",
         (bad & 1) ? "WRONG" : "ok", (bad & 2) ? "WRONG" : "ok", (bad & 4) ? "WRONG" : "ok",
         (bad & 8) ? "WRONG" : "ok");
  return 0;
}
