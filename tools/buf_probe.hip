// Microbenchmark probe (tooling, not product): raw buffer ops on gfx950 as the
// decode kernel uses them: unaligned buffer_load_dwordx4 (nt), out-of-range
// loads returning zero, out-of-range stores dropped.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void probe(uint8_t* buf, uint32_t* out, uint32_t nrec) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, nrec, 0x00020000);
  const uint32_t t = threadIdx.x;
  // unaligned loads
  v4u a = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, t * 23 + 1, 0, 2));
  // fully out-of-range load
  v4u b = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, 0xFFFFFFF0u, 0, 2));
  out[t * 8 + 0] = a.x;
  out[t * 8 + 1] = a.y;
  out[t * 8 + 2] = a.z;
  out[t * 8 + 3] = a.w;
  out[t * 8 + 4] = b.x | b.y | b.z | b.w;
  // stores: even lanes write in range, odd lanes out of range (dropped)
  v4u w = {0xA0A0A0A0u + t, 0xB0B0B0B0u, 0xC0C0C0C0u, 0xD0D0D0D0u};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, w), r,
                                         (t & 1) ? 0xFFFFFFF0u : 2048 + t * 16, 0, 0);
}

int main() {
  uint8_t* d;
  uint32_t* o;
  if (hipMalloc(&d, 8192) != hipSuccess || hipMalloc(&o, 64 * 32) != hipSuccess) return 1;
  std::vector<uint8_t> h(8192);
  for (int i = 0; i < 8192; i++) h[i] = uint8_t(i * 13 + 5);
  if (hipMemcpy(d, h.data(), 8192, hipMemcpyHostToDevice) != hipSuccess) return 1;
  probe<<<1, 64>>>(d, o, 4096);
  std::vector<uint32_t> ho(64 * 8);
  std::vector<uint8_t> hb(8192);
  if (hipMemcpy(ho.data(), o, 64 * 32, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(hb.data(), d, 8192, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad_ld = 0, bad_oob = 0, bad_st = 0;
  for (int t = 0; t < 64; t++) {
    for (int j = 0; j < 4; j++) {
      uint32_t e = 0;
      for (int k = 0; k < 4; k++) e |= uint32_t(h[t * 23 + 1 + 4 * j + k]) << (8 * k);
      bad_ld += ho[t * 8 + j] != e;
    }
    bad_oob += ho[t * 8 + 4] != 0;
    uint32_t first = 0;
    for (int k = 0; k < 4; k++) first |= uint32_t(hb[2048 + t * 16 + k]) << (8 * k);
    if (t & 1) bad_st += first != (uint32_t(h[2048 + t * 16]) | uint32_t(h[2049 + t * 16]) << 8 |
                                   uint32_t(h[2050 + t * 16]) << 16 | uint32_t(h[2051 + t * 16]) << 24);
    else bad_st += first != 0xA0A0A0A0u + t;
  }
  printf("unaligned buffer_load_dwordx4: %s; OOB load zero: %s; OOB store dropped / in-range written: %s\n",
         bad_ld ? "WRONG" : "ok", bad_oob ? "WRONG" : "ok", bad_st ? "WRONG" : "ok");
  return 0;
}
