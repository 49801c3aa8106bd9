// Microbenchmark probe (tooling, not product): cost per wave-instruction of the LDS
// operations the lane-per-block decoder issues, with its layout (one 8-wave workgroup per
// CU, per-lane records of 160 B), all 8 waves issuing: aligned vs unaligned b128
// reads/writes, partially-active (exec-masked) writes, random b32 table lookups.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kStride = 160;
constexpr int kIters = 2048;

enum Mode { kWrAligned, kWrUnaligned, kWrQuarter, kWrNone, kRdAligned, kRdUnaligned, kRdB32Rand, kRdB64Unaligned,
            kWrB64Unaligned, kWrB32Unaligned, kRdB128Al4, kRdB128Al8, kRdB64Al4, kWrB128Al4, kWrB128Al8, kWrB64Al4,
            kRd2B64Al8, kRdB32Al4, kWrB32Al4, kRdB96Al4, kRdB64Al8, kWrB64Al8, kRd2B32Al4, kRd2B64Al16 };

template <int M>
__global__ __launch_bounds__(kThreads) void probe(uint32_t* sink, uint32_t seed) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t t = threadIdx.x;
  const uint32_t rec = t * kStride + 16;
  uint32_t x = (t * 2654435761u) ^ seed;
  v4u acc = {t, t, t, t};
  for (int i = 0; i < kIters; i++) {
    x = x * 1664525u + 1013904223u;
    const uint32_t u = (x >> 8) & 127;  // unaligned offset in the 128-byte ring
    uint32_t a;
    if (M == kWrAligned || M == kRdAligned) a = rec + (u & ~15u);
    else if (M == kRdB32Rand) a = kThreads * kStride + 32 + ((x >> 4) & 1023) * 4;
    else if (M == kRdB128Al4 || M == kRdB64Al4 || M == kWrB128Al4 || M == kWrB64Al4 || M == kRdB32Al4 ||
             M == kWrB32Al4 || M == kRdB96Al4)
      a = rec + (u & ~3u);
    else if (M == kRdB128Al8 || M == kWrB128Al8 || M == kRd2B64Al8 || M == kRdB64Al8 || M == kWrB64Al8)
      a = rec + (u & ~7u);
    else if (M == kRd2B32Al4) a = rec + (u & ~3u);
    else if (M == kRd2B64Al16) a = rec + (u & ~15u);
    else a = rec + u;
    if (M == kWrAligned || M == kWrUnaligned || M == kWrB128Al4 || M == kWrB128Al8) {
      asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(acc) : "memory");
    } else if (M == kWrQuarter) {
      if ((x >> 20) & 3) asm volatile("s_nop 0");
      else asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(acc) : "memory");
    } else if (M == kWrNone) {
      if (x == 0x12345u && t == 999) asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(acc) : "memory");
    } else if (M == kWrB64Unaligned || M == kWrB64Al4 || M == kWrB64Al8) {
      asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(acc.xy) : "memory");
    } else if (M == kWrB32Unaligned || M == kWrB32Al4) {
      asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(acc.x) : "memory");
    } else if (M == kRdAligned || M == kRdUnaligned || M == kRdB128Al4 || M == kRdB128Al8) {
      v4u r;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
      acc ^= r;
    } else if (M == kRd2B32Al4) {
      uint64_t r;
      asm volatile("ds_read2_b32 %0, %1 offset1:1" : "=v"(r) : "v"(a) : "memory");
      acc.x ^= uint32_t(r) ^ uint32_t(r >> 32);
    } else if (M == kRd2B64Al8 || M == kRd2B64Al16) {
      v4u r;
      asm volatile("ds_read2_b64 %0, %1 offset1:1" : "=v"(r) : "v"(a) : "memory");
      acc ^= r;
    } else if (M == kRdB96Al4) {
      uint32_t r0, r1, r2;
      typedef uint32_t v3u __attribute__((ext_vector_type(3)));
      v3u r;
      asm volatile("ds_read_b96 %0, %1" : "=v"(r) : "v"(a) : "memory");
      acc.x ^= r.x ^ r.y ^ r.z;
      (void)r0; (void)r1; (void)r2;
    } else if (M == kRdB64Unaligned || M == kRdB64Al4 || M == kRdB64Al8) {
      uint64_t r;
      asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(a) : "memory");
      acc.x ^= uint32_t(r);
    } else {
      uint32_t r;
      asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a) : "memory");
      acc.x ^= r;
    }
    if ((i & 15) == 15) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0xdeadbeefu) sink[t] = acc.x;
}

template <int M>
void run(const char* name, uint32_t* sink, int n_cu) {
  const size_t lds = kThreads * kStride + 32 + 4096;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&probe<M>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(lds));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  probe<M><<<n_cu, kThreads, lds>>>(sink, 1);
  (void)hipDeviceSynchronize();
  float best = 1e9f;
  for (int k = 0; k < 5; k++) {
    (void)hipEventRecord(a);
    probe<M><<<n_cu * 4, kThreads, lds>>>(sink, 7 + k);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  // 4 workgroups per CU back to back, 8 waves each, kIters instructions per wave
  const double cyc = best * 1e-3 * 2.4e9;
  const double wave_instrs_per_cu = 4.0 * 8 * kIters;
  printf("%-28s %8.3f ms  %6.2f CU-cycles per wave-instruction\n", name, best, cyc / wave_instrs_per_cu);
}

int main() {
  int n_cu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) n_cu = p.multiProcessorCount;
  uint32_t* sink;
  if (hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
  printf("CUs %d, %d threads/WG, record stride %d B\n", n_cu, kThreads, kStride);
  run<kWrNone>("loop only (no LDS op)", sink, n_cu);
  run<kWrAligned>("ds_write_b128 aligned", sink, n_cu);
  run<kWrUnaligned>("ds_write_b128 unaligned", sink, n_cu);
  run<kWrQuarter>("ds_write_b128 unal 25% exec", sink, n_cu);
  run<kWrB64Unaligned>("ds_write_b64 unaligned", sink, n_cu);
  run<kWrB32Unaligned>("ds_write_b32 unaligned", sink, n_cu);
  run<kRdAligned>("ds_read_b128 aligned", sink, n_cu);
  run<kRdUnaligned>("ds_read_b128 unaligned", sink, n_cu);
  run<kRdB64Unaligned>("ds_read_b64 unaligned", sink, n_cu);
  run<kRdB32Rand>("ds_read_b32 random 4 KiB", sink, n_cu);
  run<kRdB128Al4>("ds_read_b128 4-aligned", sink, n_cu);
  run<kRdB128Al8>("ds_read_b128 8-aligned", sink, n_cu);
  run<kRdB96Al4>("ds_read_b96 4-aligned", sink, n_cu);
  run<kRdB64Al4>("ds_read_b64 4-aligned", sink, n_cu);
  run<kRd2B64Al8>("ds_read2_b64 8-aligned", sink, n_cu);
  run<kRdB32Al4>("ds_read_b32 4-aligned ring", sink, n_cu);
  run<kWrB128Al4>("ds_write_b128 4-aligned", sink, n_cu);
  run<kWrB128Al8>("ds_write_b128 8-aligned", sink, n_cu);
  run<kWrB64Al4>("ds_write_b64 4-aligned", sink, n_cu);
  run<kWrB32Al4>("ds_write_b32 4-aligned ring", sink, n_cu);
  run<kRdB64Al8>("ds_read_b64 8-aligned", sink, n_cu);
  run<kWrB64Al8>("ds_write_b64 8-aligned", sink, n_cu);
  run<kRd2B32Al4>("ds_read2_b32 4-aligned", sink, n_cu);
  run<kRd2B64Al16>("ds_read2_b64 16-aligned", sink, n_cu);
  return 0;
}
