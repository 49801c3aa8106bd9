// PMC calibration probe (tooling, not product): FETCH_SIZE / WRITE_SIZE against a known byte
// count, in the access shapes decode_lpb2_kernel uses.  Every byte of a 1 GiB region is read
// (or written) exactly once per launch, far beyond L2 + MALL, so the HBM bytes are known:
//   read_g1   16 B per lane, every lane its own stream        (row/far-copy shape)
//   read_g4   lanes 4i..4i+3 read one 64-byte run             (the transposed refill)
//   read_g64  fully coalesced 1 KiB per wave-instruction       (reference shape of the guide)
//   write_g4_sc1  64-byte runs, sc1                            (the transposed flush)
//   write_g1_sc1  16 B per lane, sc1                           (row descriptors)
// Run each under its own `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` pass; tools/fetch_calib.py
// folds the CSVs into the ratio counter-bytes / real bytes per shape.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr uint64_t kBytes = 1ull << 30;
constexpr uint32_t kThreads = 256;

// lane -> byte offset of its k-th 16-byte access, so that the launch covers [0, kBytes) once.
// Each wave owns a contiguous span; inside it, G lanes form one run of 16*G bytes per access and
// the 64/G runs of one instruction are spread over the span (their own sub-streams).
template <int G>
__device__ __forceinline__ uint32_t offset_of(uint32_t wave, uint32_t lane, uint32_t k, uint32_t per_wave_iters) {
  const uint32_t seg = lane / G, in_seg = lane % G;
  const uint64_t span = uint64_t(per_wave_iters) * 64 * 16;       // bytes per wave
  const uint64_t seg_span = span / (64 / G);                          // bytes per sub-stream
  return uint32_t(uint64_t(wave) * span + seg * seg_span + uint64_t(k) * 16 * G + in_seg * 16);
}

template <int G>
__global__ __launch_bounds__(kThreads) void read_shape(const uint8_t* buf, uint32_t iters, uint32_t* sink) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(buf), 0, int(0x7FFFFFFF), 0x00020000);
  const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * kThreads + threadIdx.x) >> 6;
  v4u acc = {0, 0, 0, 0};
  for (uint32_t k = 0; k < iters; k++) acc ^= __builtin_amdgcn_raw_buffer_load_b128(r, offset_of<G>(wave, lane, k, iters), 0, 0);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[wave] = 1;
}

template <int G>
__global__ __launch_bounds__(kThreads) void write_shape(uint8_t* buf, uint32_t iters) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, int(0x7FFFFFFF), 0x00020000);
  const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * kThreads + threadIdx.x) >> 6;
  for (uint32_t k = 0; k < iters; k++) {
    v4u v = {k, lane, wave, 7};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, offset_of<G>(wave, lane, k, iters), 0, 16);  // sc1, as the kernel
  }
}

int main() {
  uint8_t* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, kBytes);
  const uint32_t waves = 16384, iters = uint32_t(kBytes / (uint64_t(waves) * 64 * 16));  // 64 accesses per lane
  const uint32_t grid = waves * 64 / kThreads;
  for (int rep = 0; rep < 3; rep++) {
    read_shape<1><<<grid, kThreads>>>(buf, iters, sink);
    read_shape<4><<<grid, kThreads>>>(buf, iters, sink);
    read_shape<64><<<grid, kThreads>>>(buf, iters, sink);
    write_shape<4><<<grid, kThreads>>>(buf, iters);
    write_shape<1><<<grid, kThreads>>>(buf, iters);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("fetch_calib: %llu bytes per launch, %u waves x %u accesses x 64 lanes x 16 B\n",
         (unsigned long long)kBytes, waves, iters);
  return 0;
}
