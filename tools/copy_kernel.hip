// Device-to-device streaming copy (measurement aid for bench.py's measured_copy_GBps): 16 bytes per
// lane, nontemporal loads and stores, four loads in flight per lane, grid-stride over the buffer.
// It sets the practical HBM read+write ceiling the decode kernels are compared against
// (roofline.frac_of_measured_copy); torch's copy_ is reported beside it.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_copy_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                          size_t n16) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride),
              c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// n: bytes (a multiple of 16); stream: a hipStream_t (0: the null stream); grid_per_cu workgroups of
// 256 lanes per CU.  Returns the hipError_t of the launch.
extern "C" int slate_probe_stream_copy(const void* src, void* dst, size_t n, void* stream, int num_cus,
                                       int grid_per_cu) {
  const size_t n16 = n / 16;
  const unsigned grid = unsigned(num_cus > 0 ? num_cus : 256) * unsigned(grid_per_cu > 0 ? grid_per_cu : 8);
  stream_copy_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(static_cast<const v4u*>(src),
                                                                          static_cast<v4u*>(dst), n16);
  return int(hipGetLastError());
}
