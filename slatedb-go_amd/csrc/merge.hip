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

// heads from aligned dword loads (a lane's key bytes [o, o+16) are covered by five aligned words;
// a word that starts inside the key stays inside the allocation's last page)
__global__ __launch_bounds__(kMergeThreads) void merge_heads_kernel(const uint8_t* keys, const uint64_t* key_off,
                                                                    uint32_t n, Head* heads, uint32_t* lens) {
  const uint32_t e = blockIdx.x * kMergeThreads + threadIdx.x;
  if (e >= n) return;
  const uint64_t o = key_off[e];
  const uint64_t len = key_off[e + 1] - o;
  const uint32_t m = len < 16 ? uint32_t(len) : 16u;
  const uint64_t base = o & ~uint64_t(3);
  const uint32_t sh = uint32_t(o & 3);
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint64_t a = base + 4 * k;
    w[k] = a < o + m ? *reinterpret_cast<const uint32_t*>(keys + a) : 0u;
  }
  uint32_t x[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int32_t keep = min(max(int32_t(m) - 4 * k, 0), 4);  // key bytes in this dword
    const uint32_t mask = keep == 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u);
    x[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(w[k + 1], w[k], sh) & mask);
  }
  heads[e] = Head{(uint64_t(x[0]) << 32) | x[1], (uint64_t(x[2]) << 32) | x[3]};
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
  // The (k-1) binary searches are independent: run up to four of them interleaved, so their
  // dependent load chains overlap (the kernel is bound by load latency, not bandwidth; a
  // wave-window variant that cut the loads 3x but lengthened the chain ran slower).
  for (uint32_t j0 = 0; j0 < k; j0 += 4) {
    uint32_t a[4], b[4], base[4];
    int lim[4];
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const uint32_t j = j0 + g;
      const bool use = j < k && j != i;
      base[g] = use ? src_start[j] : 0u;
      a[g] = base[g];
      b[g] = use ? src_start[j + 1] : 0u;
      lim[g] = j < i ? 0 : -1;  // j < i: count keys <= e (upper bound); j > i: keys < e (lower bound)
    }
    while ((a[0] < b[0]) | (a[1] < b[1]) | (a[2] < b[2]) | (a[3] < b[3])) {
      uint32_t mid[4];
      Head hm[4];
      uint32_t lm[4];
#pragma unroll
      for (int g = 0; g < 4; g++) {
        mid[g] = a[g] + ((b[g] - a[g]) >> 1);
        const bool live = a[g] < b[g];
        hm[g] = live ? heads[mid[g]] : Head{0, 0};
        lm[g] = live ? lens[mid[g]] : 0u;
      }
#pragma unroll
      for (int g = 0; g < 4; g++) {
        if (a[g] < b[g]) {
          const int c = key_cmp(hm[g], lm[g], mid[g], he, le, e, keys, key_off);
          if (c <= lim[g]) a[g] = mid[g] + 1;
          else b[g] = mid[g];
        }
      }
    }
#pragma unroll
    for (int g = 0; g < 4; g++) rank += a[g] - base[g];
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

// ---------------------------------------------------------------- compaction rows (KV views)
// Between block decode and the merge, executeCompaction's iterators (sstable.Iterator ->
// block.Iterator, block/iterator.go:84-107) turn each row into (full key, value | tombstone):
// row 0 of a block is decoded against firstKey = nil, so its key is its suffix and becomes the
// block's firstKey; row i's key is firstKey[:prefixLen] || suffix (row.go:72-79).  Here every
// row does that on its own: lengths -> exclusive scans -> a copy pass, 16 lanes per row.
namespace {

constexpr uint32_t kScanTile = 4096;  // elements per workgroup in the u64 scan

// exclusive scan of n u32 lengths into n+1 u64 offsets: tile sums, one-workgroup scan of the
// tile sums, tile-local scans
__global__ __launch_bounds__(256) void scan_tile_sum_kernel(const uint32_t* len, uint64_t n, uint64_t* tile_sum) {
  __shared__ uint64_t ws[4];
  const uint64_t t0 = uint64_t(blockIdx.x) * kScanTile;
  uint64_t s = 0;
  for (uint64_t i = t0 + threadIdx.x; i < min(t0 + kScanTile, n); i += 256) s += len[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void scan_tiles_kernel(uint64_t* tile_sum, uint32_t tiles) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < tiles; c0 += 1024) {
    const uint32_t t = c0 + threadIdx.x;
    const uint64_t v = t < tiles ? tile_sum[t] : 0;
    uint64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if ((threadIdx.x & 63) >= uint32_t(o)) x += y;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t wo = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) wo += ws[w];
    const uint64_t base = carry;
    if (t < tiles) tile_sum[t] = base + wo + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = base + wo + x;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void scan_local_kernel(const uint32_t* len, uint64_t n, const uint64_t* tile_off,
                                                         uint64_t* off) {
  __shared__ uint64_t ws[4];
  __shared__ uint64_t carry;
  const uint64_t t0 = uint64_t(blockIdx.x) * kScanTile;
  if (threadIdx.x == 0) carry = tile_off[blockIdx.x];
  __syncthreads();
  for (uint64_t c0 = t0; c0 < min(t0 + kScanTile, n); c0 += 256) {
    const uint64_t i = c0 + threadIdx.x;
    const uint64_t v = i < n ? len[i] : 0;
    uint64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if ((threadIdx.x & 63) >= uint32_t(o)) x += y;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t wo = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) wo += ws[w];
    const uint64_t base = carry;
    if (i < n) off[i] = base + wo + x - v;
    if (i + 1 == n) off[n] = base + wo + x;
    __syncthreads();
    if (threadIdx.x == 255) carry = base + wo + x;
    __syncthreads();
  }
}

hipError_t scan_u32_to_u64(hipStream_t st, const uint32_t* len, uint64_t n, uint64_t* off, uint64_t* tile_scratch) {
  if (n == 0) return hipMemsetAsync(off, 0, 8, st);
  const uint32_t tiles = uint32_t((n + kScanTile - 1) / kScanTile);
  hipLaunchKernelGGL(scan_tile_sum_kernel, dim3(tiles), dim3(256), 0, st, len, n, tile_scratch);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, st, tile_scratch, tiles);
  hipLaunchKernelGGL(scan_local_kernel, dim3(tiles), dim3(256), 0, st, len, n, tile_scratch, off);
  return hipGetLastError();
}

__device__ __forceinline__ uint32_t block_of_row(const uint64_t* row_base, uint32_t n_blocks, uint64_t r) {
  uint32_t lo = 0, hi = n_blocks;  // row_base[lo] <= r < row_base[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (row_base[mid] <= r) lo = mid;
    else hi = mid;
  }
  return lo;
}

// row slots are planned with a capacity per block (decoded_len + 13) / 15: slot j of block b holds a
// row when j < n_rows.  valid[] marks them (a failed block or row sets flags bit 1 and keeps no rows)
__global__ __launch_bounds__(256) void rows_valid_kernel(const uint64_t* row_base, uint32_t n_blocks,
                                                         const slate_block_meta* meta, const slate_row* rows,
                                                         uint64_t n_slots, uint32_t* valid, uint32_t* flags) {
  const uint64_t r = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (r >= n_slots) return;
  const uint32_t b = block_of_row(row_base, n_blocks, r);
  const slate_block_meta m = meta[b];
  const uint64_t j = r - row_base[b];
  bool v = j < m.n_rows;
  const bool bad_block = m.status != SLATE_OK || (m.flags & SLATE_BLKF_ROWS_TRUNCATED) != 0;
  if (v && (bad_block || rows[r].status != SLATE_OK)) {
    atomicOr(flags, 2u);
    v = false;
  }
  if (bad_block && j == 0) atomicOr(flags, 2u);
  valid[r] = v ? 1u : 0u;
}

// Go's block.Iterator stops at the first row that fails to decode (block/iterator.go:92-96): the
// rows after it are not returned either.  Does work only when rows_valid_kernel found a failure.
__global__ __launch_bounds__(256) void rows_cut_kernel(const uint64_t* row_base, uint32_t n_blocks,
                                                       const slate_block_meta* meta, const slate_row* rows,
                                                       uint32_t* valid, const uint32_t* flags) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= n_blocks || !(*flags & 2u)) return;
  const uint64_t r0 = row_base[b], cap = row_base[b + 1] - r0;
  const uint64_t n = min<uint64_t>(meta[b].n_rows, cap);  // a failed block has no valid rows already
  bool cut = false;
  for (uint64_t j = 0; j < n; j++) {
    cut = cut || rows[r0 + j].status != SLATE_OK;
    if (cut) valid[r0 + j] = 0;
  }
}

// compacted row i -> its slot; lengths of row i (slots past the row count give zero lengths)
__global__ __launch_bounds__(256) void rows_slot_kernel(const uint32_t* valid, const uint64_t* pos, uint64_t n_slots,
                                                        uint32_t* slot) {
  const uint64_t r = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (r < n_slots && valid[r]) slot[pos[r]] = uint32_t(r);
}

__global__ __launch_bounds__(256) void rows_len_kernel(const uint64_t* row_base, uint32_t n_blocks,
                                                       const slate_row* rows, const uint32_t* slot,
                                                       const uint64_t* pos, uint64_t n_slots, uint32_t* klen,
                                                       uint32_t* vlen, uint8_t* tomb) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n_slots) return;
  if (i >= pos[n_slots]) {
    klen[i] = 0;
    vlen[i] = 0;
    return;
  }
  const uint32_t r = slot[i];
  const uint32_t b = block_of_row(row_base, n_blocks, r);
  const slate_row w = rows[r];
  const bool first = r == row_base[b];
  klen[i] = (first ? 0u : w.key_prefix_len) + w.key_suffix_len;
  const bool t = (w.flags & 1) != 0;
  vlen[i] = t ? 0u : w.value_len;
  tomb[i] = t ? 1 : 0;
}

// 16 lanes per row: key = firstKey[:pl] || suffix, value bytes
__global__ __launch_bounds__(256) void rows_copy_kernel(const uint8_t* data, const uint64_t* out_off,
                                                        const uint64_t* row_base, uint32_t n_blocks,
                                                        const slate_row* rows, const uint32_t* slot, const uint64_t* n_kv,
                                                        uint64_t n_slots, const uint64_t* key_off, uint8_t* keys,
                                                        const uint64_t* val_off, uint8_t* vals) {
  const uint64_t i = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 4;
  const uint32_t l = threadIdx.x & 15;
  if (i >= n_slots || i >= *n_kv) return;
  const uint32_t r = slot[i];
  const uint32_t b = block_of_row(row_base, n_blocks, r);
  const uint8_t* blk = data + out_off[b];
  const slate_row w = rows[r];
  const slate_row w0 = rows[row_base[b]];
  const uint64_t ko = key_off[i], kn = key_off[i + 1] - ko;
  const uint32_t pl = r == row_base[b] ? 0u : uint32_t(kn) - w.key_suffix_len;
  const uint8_t* fk = blk + w0.row_off + 4;  // row 0's suffix is the block's first key
  const uint8_t* sfx = blk + w.row_off + 4;
  for (uint32_t i = l; i < kn; i += 16) keys[ko + i] = i < pl ? fk[i] : sfx[i - pl];
  const uint64_t vo = val_off[i], vn = val_off[i + 1] - vo;
  const uint8_t* v = blk + w.row_off + 4 + w.key_suffix_len + w.meta_len;
  for (uint32_t i = l; i < vn; i += 16) vals[vo + i] = v[i];
}

// merged order: lengths of the returned entries
__global__ __launch_bounds__(256) void gather_len_kernel(const uint32_t* idx, uint64_t n, const uint64_t* key_off,
                                                         const uint64_t* val_off, const uint8_t* tomb,
                                                         uint32_t* klen, uint32_t* vlen, uint8_t* tomb_out) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = idx[i];
  klen[i] = uint32_t(key_off[e + 1] - key_off[e]);
  vlen[i] = uint32_t(val_off[e + 1] - val_off[e]);
  tomb_out[i] = tomb[e];
}

__global__ __launch_bounds__(256) void gather_copy_kernel(const uint32_t* idx, uint64_t n, const uint8_t* keys,
                                                          const uint64_t* key_off, const uint8_t* vals,
                                                          const uint64_t* val_off, uint8_t* okeys,
                                                          const uint64_t* okey_off, uint8_t* ovals,
                                                          const uint64_t* oval_off) {
  const uint64_t i = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 4;
  const uint32_t l = threadIdx.x & 15;
  if (i >= n) return;
  const uint32_t e = idx[i];
  const uint64_t ks = key_off[e], kd = okey_off[i], kn = okey_off[i + 1] - kd;
  for (uint64_t j = l; j < kn; j += 16) okeys[kd + j] = keys[ks + j];
  const uint64_t vs = val_off[e], vd = oval_off[i], vn = oval_off[i + 1] - vd;
  for (uint64_t j = l; j < vn; j += 16) ovals[vd + j] = vals[vs + j];
}

}  // namespace

// rows phase: klen, vlen, valid, slot (u32 each), pos (u64, n+1), tile sums
size_t kv_scratch_bytes(uint64_t n) { return 16 * n + 8 * (n + 1) + 8 * ((n + kScanTile - 1) / kScanTile) + 256; }

// scratch: klen | vlen | valid | slot (u32 x n_slots each) | pos (u64 x n_slots+1) | tile sums
hipError_t launch_rows_lengths(hipStream_t st, const uint64_t* row_base, uint32_t n_blocks,
                               const slate_block_meta* meta, const slate_row* rows, uint64_t n_slots,
                               uint64_t* key_off, uint64_t* val_off, uint8_t* tomb, uint64_t* n_kv, uint32_t* flags,
                               void* scratch) {
  uint32_t* klen = static_cast<uint32_t*>(scratch);
  uint32_t* vlen = klen + n_slots;
  uint32_t* valid = vlen + n_slots;
  uint32_t* slot = valid + n_slots;
  uint64_t* pos = reinterpret_cast<uint64_t*>(slot + n_slots);
  uint64_t* tiles = pos + n_slots + 1;
  hipError_t e = hipMemsetAsync(flags, 0, 4, st);
  if (e != hipSuccess) return e;
  const dim3 g(uint32_t((n_slots + 255) / 256));
  if (n_slots) {
    hipLaunchKernelGGL(rows_valid_kernel, g, dim3(256), 0, st, row_base, n_blocks, meta, rows, n_slots, valid, flags);
    hipLaunchKernelGGL(rows_cut_kernel, dim3((n_blocks + 255) / 256), dim3(256), 0, st, row_base, n_blocks, meta, rows,
                       valid, flags);
  }
  e = scan_u32_to_u64(st, valid, n_slots, pos, tiles);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(n_kv, pos + n_slots, 8, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  if (n_slots) {
    hipLaunchKernelGGL(rows_slot_kernel, g, dim3(256), 0, st, valid, pos, n_slots, slot);
    hipLaunchKernelGGL(rows_len_kernel, g, dim3(256), 0, st, row_base, n_blocks, rows, slot, pos, n_slots, klen, vlen,
                       tomb);
  }
  e = scan_u32_to_u64(st, klen, n_slots, key_off, tiles);
  if (e != hipSuccess) return e;
  return scan_u32_to_u64(st, vlen, n_slots, val_off, tiles);
}

// the slot map is read back from the scratch the lengths phase filled
hipError_t launch_rows_copy(hipStream_t st, const uint8_t* data, const uint64_t* out_off, const uint64_t* row_base,
                            uint32_t n_blocks, const slate_row* rows, uint64_t n_slots, const uint64_t* n_kv,
                            const void* scratch, const uint64_t* key_off, uint8_t* keys, const uint64_t* val_off,
                            uint8_t* vals) {
  if (n_slots == 0) return hipSuccess;
  const uint32_t* slot = static_cast<const uint32_t*>(scratch) + 3 * n_slots;
  hipLaunchKernelGGL(rows_copy_kernel, dim3(uint32_t((n_slots * 16 + 255) / 256)), dim3(256), 0, st, data, out_off,
                     row_base, n_blocks, rows, slot, n_kv, n_slots, key_off, keys, val_off, vals);
  return hipGetLastError();
}

hipError_t launch_gather_lengths(hipStream_t st, const uint32_t* idx, uint64_t n, const uint64_t* key_off,
                                 const uint64_t* val_off, const uint8_t* tomb, uint64_t* okey_off, uint64_t* oval_off,
                                 uint8_t* otomb, void* scratch) {
  uint32_t* klen = static_cast<uint32_t*>(scratch);
  uint32_t* vlen = klen + n;
  uint64_t* tiles = reinterpret_cast<uint64_t*>(vlen + n);
  if (n) {
    hipLaunchKernelGGL(gather_len_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, st, idx, n, key_off, val_off,
                       tomb, klen, vlen, otomb);
  }
  hipError_t e = scan_u32_to_u64(st, klen, n, okey_off, tiles);
  if (e != hipSuccess) return e;
  return scan_u32_to_u64(st, vlen, n, oval_off, tiles);
}

hipError_t launch_gather_copy(hipStream_t st, const uint32_t* idx, uint64_t n, const uint8_t* keys,
                              const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off, uint8_t* okeys,
                              const uint64_t* okey_off, uint8_t* ovals, const uint64_t* oval_off) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gather_copy_kernel, dim3(uint32_t((n * 16 + 255) / 256)), dim3(256), 0, st, idx, n, keys,
                     key_off, vals, val_off, okeys, okey_off, ovals, oval_off);
  return hipGetLastError();
}

}  // namespace slate

namespace slate {

// dst[i] = src[i] + delta: a KV view's offsets rebased when views are concatenated (slate_compact).
__global__ void u64_add_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, uint64_t n,
                               uint64_t delta) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    dst[i] = src[i] + delta;
}

hipError_t launch_u64_add(hipStream_t st, const uint64_t* src, uint64_t* dst, uint64_t n, uint64_t delta) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = uint32_t(std::min<uint64_t>((n + 255) / 256, 4096));
  u64_add_kernel<<<grid, 256, 0, st>>>(src, dst, n, delta);
  return hipGetLastError();
}

}  // namespace slate
