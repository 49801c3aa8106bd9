// Microbenchmark probe (tooling, not product): cost of per-lane scattered 16-byte
// accesses vs grouped and coalesced shapes, and of out-of-range (dropped) lanes,
// for buffer loads and stores on gfx950.  Each variant moves the same number of
// wave-instructions; the time per wave-instruction is reported.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0xFFFFFFF0u;

// G = lanes per contiguous segment (1 = every lane its own stream, 64 = fully coalesced);
// OOBPCT = percentage of lanes given an out-of-range offset.
template <int G, int OOBPCT, bool STORE>
__global__ __launch_bounds__(256) void pattern(uint8_t* buf, uint64_t bytes, uint32_t iters, uint32_t* sink) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, int(uint32_t(bytes)), 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  // each segment (G lanes) streams through its own region of iters * 16 * G bytes
  const uint32_t seg = lane / G, in_seg = lane % G;
  const uint64_t seg_bytes = uint64_t(iters) * 16 * G;
  const uint64_t region = (uint64_t(gw) * (64 / G) + seg) * seg_bytes;
  const bool oob = (lane * 100 / 64) < OOBPCT;
  v4u acc = {0, 0, 0, 0};
  for (uint32_t i = 0; i < iters; i++) {
    const uint64_t off = (region + uint64_t(i) * 16 * G + in_seg * 16) % (bytes - 16);
    const uint32_t o = oob ? kOOB : uint32_t(off);
    if (STORE) {
      v4u v = {i, lane, gw, 0};
      __builtin_amdgcn_raw_buffer_store_b128(v, r, o, 0, 0);
    } else {
      acc ^= __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 2);
    }
  }
  if (!STORE && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[gw] = 1;
  (void)nw;
}

template <int G, int OOB, bool ST>
void run(const char* name, uint8_t* buf, uint64_t bytes, uint32_t* sink) {
  const uint32_t waves = 256 * 24, iters = 256;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  pattern<G, OOB, ST><<<waves / 4, 256>>>(buf, bytes, iters, sink);
  (void)hipDeviceSynchronize();
  float best = 1e9f;
  for (int k = 0; k < 3; k++) {
    (void)hipEventRecord(a);
    pattern<G, OOB, ST><<<waves / 4, 256>>>(buf, bytes, iters, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  const double instrs = double(waves) * iters;
  const double real_bytes = instrs * 64 * 16 * (100 - OOB) / 100.0;
  printf("%-34s %7.3f ms  %6.1f cyc/wave-instr/CU  %7.0f GB/s of real lanes\n", name, best,
         best * 1e-3 * 2.4e9 / (instrs / 256), real_bytes / (best * 1e-3) / 1e9);
}

int main() {
  const uint64_t bytes = 3ull << 30;
  uint8_t* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  run<1, 0, false>("load  G=1  (64 streams)", buf, bytes, sink);
  run<1, 50, false>("load  G=1  50% OOB", buf, bytes, sink);
  run<1, 94, false>("load  G=1  94% OOB", buf, bytes, sink);
  run<1, 100, false>("load  G=1  100% OOB", buf, bytes, sink);
  run<4, 0, false>("load  G=4  (16 x 64 B)", buf, bytes, sink);
  run<8, 0, false>("load  G=8  (8 x 128 B)", buf, bytes, sink);
  run<64, 0, false>("load  G=64 (coalesced 1 KiB)", buf, bytes, sink);
  run<1, 0, true>("store G=1  (64 streams)", buf, bytes, sink);
  run<1, 50, true>("store G=1  50% OOB", buf, bytes, sink);
  run<1, 100, true>("store G=1  100% OOB", buf, bytes, sink);
  run<4, 0, true>("store G=4  (16 x 64 B)", buf, bytes, sink);
  run<8, 0, true>("store G=8  (8 x 128 B)", buf, bytes, sink);
  run<64, 0, true>("store G=64 (coalesced 1 KiB)", buf, bytes, sink);
  return 0;
}
