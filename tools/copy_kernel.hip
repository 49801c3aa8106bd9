// Device-to-device streaming copy (measurement aid for bench.py's measured_copy_GBps): the practical
// HBM read+write ceiling the decode kernels are compared against (roofline.frac_of_measured_copy).
// Several shapes of the same 16-byte-per-lane copy, so that the ceiling is the best of them rather
// than one guess: grid-stride loops with U loads in flight per lane (plain or nontemporal), and a
// one-pass form whose grid covers the buffer (each workgroup U x 4 KiB, no loop), the shape of the
// guide's float4-copy measurement.  torch's copy_ is reported beside it.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

namespace {
template <bool kNt>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if constexpr (kNt) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool kNt>
__device__ __forceinline__ void st(v4u* p, v4u v) {
  if constexpr (kNt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride, U loads in flight per lane before the U stores
template <int U, bool kNtLoad, bool kNtStore>
__global__ __launch_bounds__(256) void stride_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n16) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    v4u r[U];
#pragma unroll
    for (int k = 0; k < U; k++) r[k] = ld<kNtLoad>(src + i + k * stride);
#pragma unroll
    for (int k = 0; k < U; k++) st<kNtStore>(dst + i + k * stride, r[k]);
  }
  for (; i < n16; i += stride) st<kNtStore>(dst + i, ld<kNtLoad>(src + i));
}

// one pass: workgroup g copies 16-byte elements [g * 256 * U, (g + 1) * 256 * U), lane t the
// elements g * 256 * U + k * 256 + t
template <int U, bool kNtLoad, bool kNtStore>
__global__ __launch_bounds__(256) void pass_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n16) {
  const size_t base = size_t(blockIdx.x) * 256 * U + threadIdx.x;
  v4u r[U];
#pragma unroll
  for (int k = 0; k < U; k++)
    if (base + k * 256 < n16) r[k] = ld<kNtLoad>(src + base + k * 256);
#pragma unroll
  for (int k = 0; k < U; k++)
    if (base + k * 256 < n16) st<kNtStore>(dst + base + k * 256, r[k]);
}
}  // namespace

// variant: 0 grid-stride U=4 nt/nt (the round-4 kernel), 1 U=4 plain, 2 U=8 plain, 3 U=8 nt/nt,
// 4 U=4 plain loads / nt stores, 5 one pass U=1 plain, 6 one pass U=4 plain, 7 one pass U=4 nt/nt.
// n: bytes (a multiple of 16); stream: a hipStream_t (0: the null stream); grid_per_cu: workgroups
// of 256 lanes per CU for the grid-stride forms.  Returns the hipError_t of the launch (or 1 for an
// unknown variant).
extern "C" int slate_probe_stream_copy_v(const void* src, void* dst, size_t n, void* stream, int num_cus,
                                         int grid_per_cu, int variant) {
  const size_t n16 = n / 16;
  const unsigned grid = unsigned(num_cus > 0 ? num_cus : 256) * unsigned(grid_per_cu > 0 ? grid_per_cu : 8);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const v4u* a = static_cast<const v4u*>(src);
  v4u* b = static_cast<v4u*>(dst);
  auto pass_grid = [&](size_t u) { return unsigned((n16 + 256 * u - 1) / (256 * u)); };
  switch (variant) {
    case 0: stride_copy<4, true, true><<<grid, 256, 0, s>>>(a, b, n16); break;
    case 1: stride_copy<4, false, false><<<grid, 256, 0, s>>>(a, b, n16); break;
    case 2: stride_copy<8, false, false><<<grid, 256, 0, s>>>(a, b, n16); break;
    case 3: stride_copy<8, true, true><<<grid, 256, 0, s>>>(a, b, n16); break;
    case 4: stride_copy<4, false, true><<<grid, 256, 0, s>>>(a, b, n16); break;
    case 5: pass_copy<1, false, false><<<pass_grid(1), 256, 0, s>>>(a, b, n16); break;
    case 6: pass_copy<4, false, false><<<pass_grid(4), 256, 0, s>>>(a, b, n16); break;
    case 7: pass_copy<4, true, true><<<pass_grid(4), 256, 0, s>>>(a, b, n16); break;
    default: return 1;
  }
  return int(hipGetLastError());
}

extern "C" int slate_probe_stream_copy(const void* src, void* dst, size_t n, void* stream, int num_cus,
                                       int grid_per_cu) {
  return slate_probe_stream_copy_v(src, dst, n, stream, num_cus, grid_per_cu, 0);
}
