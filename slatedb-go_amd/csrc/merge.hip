// K-way merge with first-iterator precedence: iter.MergeSort (internal/iter/merge.go:12-111),
// the step of executeCompaction (compaction/executor.go:92-151) between decoding the input
// sorted runs and re-encoding the output SSTs.
//
// The heap merge is serial; on the GPU every element finds its place on its own.  For element
// e at position p of iterator i, the merged position is
//   rank(e) = p + sum_{j<i} upper_bound_j(key e) + sum_{j>i} lower_bound_j(key e),
// which is exactly the heap's (key, iterator index) order when each iterator is sorted
// (merge.go:88-95), so M[rank(e)] = e is a permutation.  An entry is returned when its key
// differs from the previous merged key (merge.go:67-72: lastKey only changes on a return, and
// equal keys are adjacent), and never when the key is empty (lastKey starts nil and
// bytes.Equal(empty, nil) is true).  The kept entries are compacted with a tile scan.
//
// Keys are compared through a 16-byte big-endian head (zero padded) plus the length: equal
// heads with min(len) <= 16 are ordered by length; longer keys compare their tails in HBM.
// Work per element is (k-1) binary searches over 16-byte heads: this is L2/HBM latency work
// (integer compares, no MFMA).
#include "common.h"
#include "kernels.h"

namespace slate {
namespace {

constexpr int kMergeThreads = 256;
constexpr uint32_t kMergeTile = 2048;  // ranks per workgroup in the keep / scatter kernels

struct Head {
  uint64_t h0, h1;  // key bytes 0..7 and 8..15, big-endian, zero padded
};

__global__ __launch_bounds__(kMergeThreads) void merge_heads_kernel(const uint8_t* keys, const uint64_t* key_off,
                                                                    uint32_t n, Head* heads, uint32_t* lens) {
  const uint32_t e = blockIdx.x * kMergeThreads + threadIdx.x;
  if (e >= n) return;
  const uint64_t o = key_off[e];
  const uint64_t len = key_off[e + 1] - o;
  uint64_t h[2] = {0, 0};
  const uint32_t m = len < 16 ? uint32_t(len) : 16u;
  for (uint32_t b = 0; b < m; b++) h[b >> 3] |= uint64_t(keys[o + b]) << (56 - 8 * (b & 7));
  heads[e] = Head{h[0], h[1]};
  lens[e] = len > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(len);
}

// bytes.Compare(key a, key b) given their heads
__device__ __forceinline__ int key_cmp(const Head& ha, uint32_t la, uint64_t a, const Head& hb, uint32_t lb,
                                       uint64_t b, const uint8_t* keys, const uint64_t* key_off) {
  if (ha.h0 != hb.h0) return ha.h0 < hb.h0 ? -1 : 1;
  if (ha.h1 != hb.h1) return ha.h1 < hb.h1 ? -1 : 1;
  const uint32_t m = min(la, lb);
  if (m > 16) {
    const uint8_t* pa = keys + key_off[a];
    const uint8_t* pb = keys + key_off[b];
    for (uint32_t i = 16; i < m; i++) {
      const uint32_t x = pa[i], y = pb[i];
      if (x != y) return x < y ? -1 : 1;
    }
  }
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

// rank of every element; also flags an iterator that is not sorted (merge.go assumes sorted input)
__global__ __launch_bounds__(kMergeThreads) void merge_rank_kernel(const uint8_t* keys, const uint64_t* key_off,
                                                                   const Head* heads, const uint32_t* lens,
                                                                   const uint32_t* src_start, uint32_t k,
                                                                   uint32_t n, uint32_t* M, uint32_t* flags) {
  const uint32_t e = blockIdx.x * kMergeThreads + threadIdx.x;
  if (e >= n) return;
  // the iterator holding e: last i with src_start[i] <= e
  uint32_t lo = 0, hi = k;  // src_start[lo] <= e < src_start[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (src_start[mid] <= e) lo = mid;
    else hi = mid;
  }
  const uint32_t i = lo;
  const Head he = heads[e];
  const uint32_t le = lens[e];
  uint32_t rank = e - src_start[i];
  if (e + 1 < src_start[i + 1] &&
      key_cmp(he, le, e, heads[e + 1], lens[e + 1], e + 1, keys, key_off) > 0)
    atomicOr(flags, 1u);
  for (uint32_t j = 0; j < k; j++) {
    if (j == i) continue;
    // j < i: count keys <= e (upper bound); j > i: keys < e (lower bound)
    const int lim = j < i ? 0 : -1;
    uint32_t a = src_start[j], b = src_start[j + 1];
    const uint32_t base = a;
    while (a < b) {
      const uint32_t mid = a + ((b - a) >> 1);
      const int c = key_cmp(heads[mid], lens[mid], mid, he, le, e, keys, key_off);
      if (c <= lim) a = mid + 1;
      else b = mid;
    }
    rank += a - base;
  }
  M[rank] = e;
}

__device__ __forceinline__ bool keep_at(uint32_t r, uint32_t n, const uint32_t* M, const Head* heads, const uint32_t* lens,
                                        const uint8_t* keys, const uint64_t* key_off) {
  // M holds a permutation when every iterator is sorted; otherwise (reported as an error)
  // some slots keep the 0xFFFFFFFF fill and are skipped here, so nothing reads out of range
  const uint32_t e = M[r];
  if (e >= n) return false;
  const uint32_t le = lens[e];
  if (le == 0) return false;
  if (r == 0) return true;
  const uint32_t p = M[r - 1];
  if (p >= n) return true;
  return key_cmp(heads[p], lens[p], p, heads[e], le, e, keys, key_off) != 0;
}

// wave-local exclusive prefix of a boolean, and the wave's total
__device__ __forceinline__ uint32_t wave_prefix(bool f, uint32_t* total) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(f);
  *total = uint32_t(__popcll(m));
  return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

// keep flags (one byte per rank) and the kept count of each tile
__global__ __launch_bounds__(kMergeThreads) void merge_keep_kernel(const uint32_t* M, const Head* heads,
                                                                   const uint32_t* lens, const uint8_t* keys,
                                                                   const uint64_t* key_off, uint32_t n,
                                                                   uint8_t* keep, uint32_t* tile_cnt) {
  __shared__ uint32_t wsum[kMergeThreads / 64];
  const uint32_t t0 = blockIdx.x * kMergeTile;
  uint32_t cnt = 0;
  for (uint32_t r = t0 + threadIdx.x; r < min(t0 + kMergeTile, n); r += kMergeThreads) {
    const bool f = keep_at(r, n, M, heads, lens, keys, key_off);
    keep[r] = f ? 1 : 0;
    cnt += f ? 1u : 0u;
  }
  // workgroup sum
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kMergeThreads / 64; w++) s += wsum[w];
    tile_cnt[blockIdx.x] = s;
  }
}

// exclusive scan of the tile counts (one workgroup), total into *n_out
__global__ __launch_bounds__(1024) void merge_scan_kernel(uint32_t* tile_cnt, uint32_t tiles, uint64_t* n_out) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < tiles; c0 += 1024) {
    const uint32_t t = c0 + threadIdx.x;
    const uint32_t v = t < tiles ? tile_cnt[t] : 0u;
    // inclusive wave scan
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if ((threadIdx.x & 63) >= uint32_t(o)) x += y;
    }
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t wo = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) wo += wsum[w];
    const uint32_t base = carry;
    if (t < tiles) tile_cnt[t] = base + wo + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = base + wo + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_out = carry;
}

// kept entries, in merged order, to their compacted positions
__global__ __launch_bounds__(kMergeThreads) void merge_scatter_kernel(const uint32_t* M, const uint8_t* keep,
                                                                      const uint32_t* tile_off, uint32_t n,
                                                                      uint32_t* out_idx) {
  __shared__ uint32_t wsum[kMergeThreads / 64];
  __shared__ uint32_t carry;
  const uint32_t t0 = blockIdx.x * kMergeTile;
  if (threadIdx.x == 0) carry = tile_off[blockIdx.x];
  __syncthreads();
  for (uint32_t c0 = t0; c0 < min(t0 + kMergeTile, n); c0 += kMergeThreads) {
    const uint32_t r = c0 + threadIdx.x;
    const bool f = r < n && keep[r];
    uint32_t wt;
    const uint32_t lp = wave_prefix(f, &wt);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = wt;
    __syncthreads();
    uint32_t wo = 0, all = 0;
    for (uint32_t w = 0; w < kMergeThreads / 64; w++) {
      wo += w < (threadIdx.x >> 6) ? wsum[w] : 0u;
      all += wsum[w];
    }
    const uint32_t base = carry;
    if (f) out_idx[base + wo + lp] = M[r];
    __syncthreads();
    if (threadIdx.x == 0) carry = base + all;
    __syncthreads();
  }
}

}  // namespace

size_t merge_scratch_bytes(uint32_t n, uint32_t k) {
  const size_t tiles = (size_t(n) + kMergeTile - 1) / kMergeTile;
  return 16 * size_t(n) + 4 * size_t(n) + 4 * size_t(n) + size_t(n) + 4 * tiles + 4 * (size_t(k) + 1) + 256;
}

hipError_t launch_merge(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint32_t n,
                        const uint32_t* h_src_start, uint32_t k, void* scratch, uint32_t* out_idx, uint64_t* n_out,
                        uint32_t* d_flags) {
  const uint32_t tiles = (n + kMergeTile - 1) / kMergeTile;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  Head* heads = reinterpret_cast<Head*>(p);
  p += 16 * size_t(n);
  uint32_t* lens = reinterpret_cast<uint32_t*>(p);
  p += 4 * size_t(n);
  uint32_t* M = reinterpret_cast<uint32_t*>(p);
  p += 4 * size_t(n);
  uint32_t* tile_cnt = reinterpret_cast<uint32_t*>(p);
  p += 4 * size_t(tiles);
  uint32_t* src_start = reinterpret_cast<uint32_t*>(p);
  p += 4 * (size_t(k) + 1);
  uint8_t* keep = p;
  hipError_t e = hipMemcpyAsync(src_start, h_src_start, 4 * (size_t(k) + 1), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(d_flags, 0, 4, st);
  if (e != hipSuccess) return e;
  if (n == 0) return hipMemsetAsync(n_out, 0, 8, st);
  e = hipMemsetAsync(M, 0xFF, 4 * size_t(n), st);
  if (e != hipSuccess) return e;
  const uint32_t g = (n + kMergeThreads - 1) / kMergeThreads;
  hipLaunchKernelGGL(merge_heads_kernel, dim3(g), dim3(kMergeThreads), 0, st, keys, key_off, n, heads, lens);
  hipLaunchKernelGGL(merge_rank_kernel, dim3(g), dim3(kMergeThreads), 0, st, keys, key_off, heads, lens, src_start,
                     k, n, M, d_flags);
  hipLaunchKernelGGL(merge_keep_kernel, dim3(tiles), dim3(kMergeThreads), 0, st, M, heads, lens, keys, key_off, n,
                     keep, tile_cnt);
  hipLaunchKernelGGL(merge_scan_kernel, dim3(1), dim3(1024), 0, st, tile_cnt, tiles, n_out);
  hipLaunchKernelGGL(merge_scatter_kernel, dim3(tiles), dim3(kMergeThreads), 0, st, M, keep, tile_cnt, n, out_idx);
  return hipGetLastError();
}

}  // namespace slate
