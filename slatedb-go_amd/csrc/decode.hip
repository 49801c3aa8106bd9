// Block decode on MI355X: block.Decode (internal/sstable/block/block.go:78-134)
// followed by the block iterator's per-row v0 decode (row.go:191-261,
// block/iterator.go:84-107), for a batch of independent blocks resident in HBM.
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   in   : encoded blocks back to back, block i = in[in_off[i] .. in_off[i+1])
//   out  : decoded block i (rows || BE16 offsets || BE16 count) at out + out_off[i];
//          out_off is 16-byte aligned so every block is written with aligned
//          dwordx4 stores
//   meta : one 16-byte slate_block_meta per block
//   rows : slate_row descriptors of block i at rows + row_base[i]
//
// Kernels:
//   plan_sizes_kernel     decoded length per block (Snappy varint header) -> sizes
//   scan_* (3 passes)     exclusive scans of the sizes -> out_off / row_base
//   decode_fast_kernel    one wavefront per block, block staged in LDS:
//                         CRC32 (64 lanes x 64-byte segments, GF(2) combine),
//                         Snappy tag walk (wave-uniform) with lane-parallel copies,
//                         offset checks, row descriptors, aligned write-back
//   decode_large_kernel   same device code for blocks that exceed the fast
//                         kernel's LDS budget (one wave per workgroup, ~150 KiB LDS)
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "encode.h"
#include "wave_crc.h"
#include "zstd.h"
#include "rows.h"

namespace slate {

// ------------------------------------------------------------------ sizes
// golang/snappy decode.go decodedLen: binary.Uvarint, n <= 0 || v > 0xffffffff
// => ErrCorrupt.  Returns false for a corrupt header.
__device__ inline bool snappy_header(const uint8_t* p, uint64_t n, uint64_t* dlen, uint32_t* hdr) {
  uint64_t x = 0;
  uint32_t s = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (i == 10) return false;
    uint32_t b = p[i];
    if (b < 0x80) {
      if (i == 9 && b > 1) return false;
      x |= uint64_t(b) << s;
      if (x > 0xffffffffull) return false;
      *dlen = x;
      *hdr = i + 1;
      return true;
    }
    x |= uint64_t(b & 0x7f) << s;
    s += 7;
  }
  return false;
}

// ------------------------------------------------------------------- LZ4
// compress.Decode CodecLz4 = io.ReadAll(lz4.NewReader(buf)) (compression.go:143-144), the
// LZ4 frame format read in order; oracle/slate_oracle.c lz4_frame is the restatement this
// follows step for step (same checks, same order, same status codes).
constexpr uint32_t kLz4Magic = 0x184D2204u;
__device__ inline uint32_t ld_le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
struct Lz4Hdr {
  int status;
  uint32_t flg, hl;  // FLG byte, descriptor length (FLG .. DictID)
  uint64_t bmax, content;
};
__device__ inline Lz4Hdr lz4_header(const uint8_t* in, uint64_t n) {
  Lz4Hdr h{SLATE_OK, 0, 0, 0, 0};
  if (n < 4) { h.status = SLATE_E_LZ4_CORRUPT; return h; }
  if (ld_le32(in) != kLz4Magic) { h.status = SLATE_E_LZ4_MAGIC; return h; }
  if (n < 7) { h.status = SLATE_E_LZ4_CORRUPT; return h; }
  const uint32_t flg = in[4], bd = in[5];
  if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8F) || ((bd >> 4) & 7) < 4) { h.status = SLATE_E_LZ4_CORRUPT; return h; }
  h.flg = flg;
  h.bmax = uint64_t(1) << (8 + 2 * ((bd >> 4) & 7));
  h.hl = 2 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
  if (n < 4 + h.hl + 1) { h.status = SLATE_E_LZ4_CORRUPT; return h; }
  if (flg & 8)
    for (int k = 7; k >= 0; k--) h.content = (h.content << 8) | in[6 + k];
  return h;
}
// Structure-only pass (no checksums): the decoded size of the blocks before the first
// structural error, which is what the in-order decoder can write before it fails.
__device__ inline void lz4_frame_len(const uint8_t* in, uint64_t n, uint64_t* dl) {
  *dl = 0;
  const Lz4Hdr h = lz4_header(in, n);
  if (h.status != SLATE_OK || (h.flg & 1)) return;
  const bool indep = (h.flg >> 5) & 1, bcheck = (h.flg >> 4) & 1;
  uint64_t pos = 4 + h.hl + 1, d = 0;
  for (;;) {
    if (n - pos < 4) return;
    const uint32_t bs = ld_le32(in + pos);
    pos += 4;
    if (bs == 0) return;
    const uint64_t sz = bs & 0x7FFFFFFFu;
    if (sz > h.bmax || n - pos < sz + (bcheck ? 4 : 0)) return;
    if (bs >> 31) {
      d += sz;
    } else {
      const uint8_t* src = in + pos;
      uint64_t s = 0, bd = 0;
      const uint64_t lo = indep ? d : 0;
      for (;;) {
        if (s >= sz) return;
        const uint32_t token = src[s++];
        uint64_t ll = token >> 4;
        if (ll == 15) {
          uint32_t b;
          do {
            if (s >= sz) return;
            b = src[s++];
            ll += b;
          } while (b == 255);
        }
        if (ll > sz - s || ll > h.bmax - bd) return;
        s += ll;
        bd += ll;
        if (s == sz) break;
        if (sz - s < 2) return;
        const uint64_t off = src[s] | uint64_t(src[s + 1]) << 8;
        s += 2;
        if (off == 0 || off > d + bd - lo) return;
        uint64_t ml = token & 15;
        if (ml == 15) {
          uint32_t b;
          do {
            if (s >= sz) return;
            b = src[s++];
            ml += b;
          } while (b == 255);
        }
        ml += 4;
        if (ml > h.bmax - bd) return;
        bd += ml;
      }
      d += bd;
    }
    *dl = d;
    pos += sz + (bcheck ? 4 : 0);
  }
}

// Decoded length of a block: false when the block cannot decode (too small,
// corrupt Snappy header, provably corrupt length, unsupported codec).
__device__ inline bool decoded_len(int codec, const uint8_t* in, uint64_t len, uint64_t* dl, uint32_t* hdr) {
  *hdr = 0;
  *dl = 0;
  if (len < 6) return false;
  uint64_t clen = len - 4;
  if (codec == SLATE_CODEC_NONE) {
    *dl = clen;
    return true;
  }
  if (codec == SLATE_CODEC_SNAPPY) {
    uint64_t v;
    if (!snappy_header(in, clen, &v, hdr)) return false;
    if (v > kSnappyMaxExpansion * clen) return false;
    *dl = v;
    return true;
  }
  if (codec == SLATE_CODEC_LZ4) {  // the size the in-order decoder writes (even when it then fails)
    lz4_frame_len(in, clen, dl);
    return true;
  }
  return false;
}

__global__ void plan_sizes_kernel(int codec, const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                  uint32_t n, uint64_t* __restrict__ out_sz, uint64_t* __restrict__ row_sz) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {  // the scans turn the trailing zero into the totals
    out_sz[n] = 0;
    row_sz[n] = 0;
    return;
  }
  uint64_t s0 = in_off[i];
  uint32_t hdr;
  uint64_t dl;
  decoded_len(codec, in + s0, in_off[i + 1] - s0, &dl, &hdr);
  out_sz[i] = align16(dl);
  row_sz[i] = row_capacity(dl);
}

// plan_sizes_kernel over a list of blocks (list[0 .. *count)): the CodecLz4 frames the lane plan
// hands back (decode_lpb2.hip plan_lz4_lane_kernel).
__global__ void plan_list_kernel(int codec, const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                 const uint32_t* list, const uint32_t* count, uint64_t* __restrict__ out_sz,
                                 uint64_t* __restrict__ row_sz) {
  const uint32_t items = *count;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < items; k += gridDim.x * blockDim.x) {
    const uint32_t i = list[k];
    const uint64_t s0 = in_off[i];
    uint32_t hdr;
    uint64_t dl;
    decoded_len(codec, in + s0, in_off[i + 1] - s0, &dl, &hdr);
    out_sz[i] = align16(dl);
    row_sz[i] = row_capacity(dl);
  }
}

// CodecZlib sizes: the bytes the in-order inflater writes (also when it then fails;
// oracle or_block_decode_batch), one wave per block reading the stream from HBM.
__global__ __launch_bounds__(256) void plan_zlib_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off, uint32_t n,
                                                        uint64_t* __restrict__ out_sz, uint64_t* __restrict__ row_sz,
                                                        const uint32_t* list, const uint32_t* count);

// ------------------------------------------------ exclusive scan (2 arrays)
constexpr int kScanThreads = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

template <typename T>
__device__ inline T block_exclusive_scan(T v, T* sh, T* total) {
  int t = threadIdx.x, lane = t & 63, w = t >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  T wsum = 0, all = 0;
  for (int k = 0; k < kScanThreads / 64; k++) {
    if (k < w) wsum += sh[k];
    all += sh[k];
  }
  __syncthreads();
  *total = all;
  return x - v + wsum;
}

__global__ void scan_reduce_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint32_t n,
                                   uint64_t* __restrict__ pa, uint64_t* __restrict__ pb) {
  __shared__ uint64_t sh[2][kScanThreads / 64];
  uint64_t base = uint64_t(blockIdx.x) * kScanTile;
  uint64_t sa = 0, sb = 0;
  for (int k = 0; k < kScanItems; k++) {
    uint64_t i = base + uint64_t(k) * kScanThreads + threadIdx.x;
    if (i < n) { sa += a[i]; if (b) sb += b[i]; }
  }
  uint64_t ta, tb;
  block_exclusive_scan(sa, sh[0], &ta);
  block_exclusive_scan(sb, sh[1], &tb);
  if (threadIdx.x == 0) { pa[blockIdx.x] = ta; pb[blockIdx.x] = tb; }
}

// CodecNone / CodecSnappy sizes (plan_sizes_kernel) and the scan's tile sums in one pass: the
// sizes are written and summed by the same threads (one launch and one re-read fewer).
__global__ void plan_reduce_kernel(int codec, const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                   uint32_t n, uint64_t* __restrict__ out_sz, uint64_t* __restrict__ row_sz,
                                   uint64_t* __restrict__ pa, uint64_t* __restrict__ pb) {
  __shared__ uint64_t sh[2][kScanThreads / 64];
  const uint64_t base = uint64_t(blockIdx.x) * kScanTile;
  uint64_t sa = 0, sb = 0;
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = base + uint64_t(k) * kScanThreads + threadIdx.x;
    if (i > n) continue;
    uint64_t o = 0, r = 0;  // (entry n: the trailing zero the scan turns into the totals)
    if (i < n) {
      const uint64_t s0 = in_off[i];
      uint32_t hdr;
      uint64_t dl;
      decoded_len(codec, in + s0, in_off[i + 1] - s0, &dl, &hdr);
      o = align16(dl);
      r = row_capacity(dl);
    }
    out_sz[i] = o;
    row_sz[i] = r;
    sa += o;
    sb += r;
  }
  uint64_t ta, tb;
  block_exclusive_scan(sa, sh[0], &ta);
  block_exclusive_scan(sb, sh[1], &tb);
  if (threadIdx.x == 0) {
    pa[blockIdx.x] = ta;
    pb[blockIdx.x] = tb;
  }
}

// The scan's last pass, each tile first summing the tile sums below it itself (the single-workgroup
// partials pass is then not needed: ~1000 tiles per 1 M blocks, a few loads per thread).
__global__ void scan_apply_sum_kernel(uint64_t* __restrict__ a, uint64_t* __restrict__ b, uint32_t n,
                                      const uint64_t* __restrict__ pa, const uint64_t* __restrict__ pb) {
  __shared__ uint64_t sh[2][kScanThreads / 64];
  uint64_t qa = 0, qb = 0;
  for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kScanThreads) {
    qa += pa[j];
    qb += pb[j];
  }
  uint64_t ba, bb;
  block_exclusive_scan(qa, sh[0], &ba);
  block_exclusive_scan(qb, sh[1], &bb);
  const uint64_t base = uint64_t(blockIdx.x) * kScanTile + uint64_t(threadIdx.x) * kScanItems;
  uint64_t va[kScanItems], vb[kScanItems], sa = 0, sb = 0;
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = base + k;
    va[k] = i < n ? a[i] : 0;
    vb[k] = (b && i < n) ? b[i] : 0;
    sa += va[k];
    sb += vb[k];
  }
  uint64_t ta, tb;
  uint64_t ea = block_exclusive_scan(sa, sh[0], &ta) + ba;
  uint64_t eb = block_exclusive_scan(sb, sh[1], &tb) + bb;
  for (int k = 0; k < kScanItems; k++) {
    const uint64_t i = base + k;
    if (i < n) {
      a[i] = ea;
      if (b) b[i] = eb;
    }
    ea += va[k];
    eb += vb[k];
  }
}

// ------------------------------------------------------------- Snappy decode
// golang/snappy v0.0.4 decode (decode_other.go), one wavefront: the tag walk is
// wave-uniform (scalar values), each literal/copy is spread over the 64 lanes.
// Returns SLATE_OK or SLATE_E_SNAPPY_CORRUPT.
__device__ int wave_snappy_decode(const uint8_t* src, uint32_t sn, uint32_t s, uint8_t* dst, uint32_t dn,
                                  int lane) {
  uint32_t d = 0;
  while (s < sn) {
    uint32_t c = __builtin_amdgcn_readfirstlane(src[s]);
    uint32_t t = c & 3;
    if (t == 0) {
      uint32_t x = c >> 2;
      if (x < 60) {
        s += 1;
      } else {
        uint32_t nb = x - 59;
        s += 1 + nb;
        if (s > sn) return SLATE_E_SNAPPY_CORRUPT;
        x = 0;
        for (uint32_t k = 0; k < nb; k++) x |= uint32_t(src[s - nb + k]) << (8 * k);
        x = __builtin_amdgcn_readfirstlane(x);
      }
      uint64_t len = uint64_t(x) + 1;
      if (len > uint64_t(dn - d) || len > uint64_t(sn - s)) return SLATE_E_SNAPPY_CORRUPT;
      for (uint32_t j = lane; j < uint32_t(len); j += kWave) dst[d + j] = src[s + j];
      d += uint32_t(len);
      s += uint32_t(len);
      continue;
    }
    uint32_t len, off;
    if (t == 1) {
      s += 2;
      if (s > sn) return SLATE_E_SNAPPY_CORRUPT;
      len = 4 + ((c >> 2) & 7);
      off = ((c & 0xe0) << 3) | __builtin_amdgcn_readfirstlane(src[s - 1]);
    } else if (t == 2) {
      s += 3;
      if (s > sn) return SLATE_E_SNAPPY_CORRUPT;
      len = 1 + (c >> 2);
      off = __builtin_amdgcn_readfirstlane(uint32_t(src[s - 2]) | uint32_t(src[s - 1]) << 8);
    } else {
      s += 5;
      if (s > sn) return SLATE_E_SNAPPY_CORRUPT;
      len = 1 + (c >> 2);
      off = __builtin_amdgcn_readfirstlane(uint32_t(src[s - 4]) | uint32_t(src[s - 3]) << 8 |
                                           uint32_t(src[s - 2]) << 16 | uint32_t(src[s - 1]) << 24);
    }
    if (off == 0 || d < off || len > dn - d) return SLATE_E_SNAPPY_CORRUPT;
    if (off >= len) {
      if (uint32_t(lane) < len) dst[d + lane] = dst[d - off + lane];
    } else {
      // forward byte-by-byte semantics: byte j repeats the off-byte pattern
      for (uint32_t j = lane; j < len; j += kWave) dst[d + j] = dst[d - off + (j % off)];
    }
    d += len;
  }
  return d == dn ? SLATE_OK : SLATE_E_SNAPPY_CORRUPT;
}

// ------------------------------------------------------------- LZ4 decode
// XXH32 (seed 0) of LDS bytes [off, off+n) of a 4-aligned buffer: lanes 0..3 run the four
// stripe accumulators, the tail and the avalanche are wave-uniform.
constexpr uint32_t kXP1 = 2654435761u, kXP2 = 2246822519u, kXP3 = 3266489917u, kXP4 = 668265263u,
                   kXP5 = 374761393u;
__device__ inline uint32_t xrotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ uint32_t wave_xxh32(const uint8_t* base, uint32_t off, uint32_t n, int lane) {
  uint32_t h;
  if (n >= 16) {
    uint32_t v = lane == 0 ? kXP1 + kXP2 : (lane == 1 ? kXP2 : (lane == 2 ? 0u : 0u - kXP1));
    const uint32_t stripes = n / 16;
    if (lane < 4) {
#pragma unroll 8
      for (uint32_t i = 0; i < stripes; i++)
        v = xrotl(v + lds_u32(base, int32_t(off + 16 * i + 4 * uint32_t(lane))) * kXP2, 13) * kXP1;
    }
    const uint32_t v1 = __builtin_amdgcn_readlane(v, 0), v2 = __builtin_amdgcn_readlane(v, 1),
                   v3 = __builtin_amdgcn_readlane(v, 2), v4 = __builtin_amdgcn_readlane(v, 3);
    h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
  } else {
    h = kXP5;
  }
  h += n;
  uint32_t i = n & ~15u;
  for (; i + 4 <= n; i += 4) h = xrotl(h + __builtin_amdgcn_readfirstlane(lds_u32(base, int32_t(off + i))) * kXP3, 17) * kXP4;
  for (; i < n; i++) h = xrotl(h + uint32_t(base[off + i]) * kXP5, 11) * kXP1;
  h ^= h >> 15;
  h *= kXP2;
  h ^= h >> 13;
  h *= kXP3;
  h ^= h >> 16;
  return __builtin_amdgcn_readfirstlane(h);
}

// The frame in LDS (in, n bytes; `base`/`off` address it for 4-aligned reads) decoded in
// order into out[0, cap): wave-uniform parse, lane-parallel copies.  The checks and
// their order are oracle/slate_oracle.c lz4_frame's; out == nullptr is its sizes-only pass
// (no writes, no checksums).
__device__ int wave_lz4_decode(const uint8_t* base, uint32_t off, uint32_t n, uint8_t* out, uint32_t cap, int lane,
                               uint32_t* out_len) {
  const uint8_t* in = base + off;
  *out_len = 0;
  const Lz4Hdr h = lz4_header(in, n);
  if (h.status != SLATE_OK) return h.status;
  if (out && in[4 + h.hl] != ((wave_xxh32(base, off + 4, h.hl, lane) >> 8) & 0xFF)) return SLATE_E_LZ4_HEADER_CHECKSUM;
  if (h.flg & 1) return SLATE_E_LZ4_CORRUPT;  // no dictionaries are configured
  const bool indep = (h.flg >> 5) & 1, bcheck = (h.flg >> 4) & 1, ccheck = (h.flg >> 2) & 1, csize = (h.flg >> 3) & 1;
  uint32_t pos = 4 + h.hl + 1, d = 0;
  for (;;) {
    if (n - pos < 4) return SLATE_E_LZ4_CORRUPT;
    const uint32_t bs = __builtin_amdgcn_readfirstlane(ld_le32(in + pos));
    pos += 4;
    if (bs == 0) break;
    const uint32_t sz = bs & 0x7FFFFFFFu;
    if (sz > h.bmax || n - pos < sz + (bcheck ? 4u : 0u)) return SLATE_E_LZ4_CORRUPT;
    if (out && bcheck && wave_xxh32(base, off + pos, sz, lane) != __builtin_amdgcn_readfirstlane(ld_le32(in + pos + sz)))
      return SLATE_E_LZ4_BLOCK_CHECKSUM;
    const uint8_t* src = in + pos;
    // sequence headers are read through a 64-byte window held one byte per lane
    // (v_readlane with a uniform index): one LDS round trip per 64 input bytes instead
    // of one per header byte
    uint32_t wbase = 0x80000000u, win = 0;  // p - wbase >= 64 for every p < 2^31: the first read loads
    auto byte_at = [&](uint32_t p) -> uint32_t {  // src[p], p < sz (wave-uniform)
      if (p - wbase >= uint32_t(kWave)) {
        wbase = p;
        win = (p + uint32_t(lane) < sz) ? uint32_t(src[p + lane]) : 0u;
      }
      return __builtin_amdgcn_readlane(win, int(p - wbase));
    };
    if (bs >> 31) {  // stored block
      if (sz > cap - d) return SLATE_E_LZ4_CORRUPT;
      if (out)
        for (uint32_t j = lane; j < sz; j += kWave) out[d + j] = src[j];
      d += sz;
    } else {
      const uint32_t d0 = d, lo = indep ? d : 0u;
      uint32_t s = 0;
      for (;;) {
        if (s >= sz) return SLATE_E_LZ4_CORRUPT;
        const uint32_t token = byte_at(s);
        s++;
        uint32_t ll = token >> 4;
        if (ll == 15) {
          uint32_t b;
          do {
            if (s >= sz) return SLATE_E_LZ4_CORRUPT;
            b = byte_at(s);
            s++;
            ll += b;
          } while (b == 255);
        }
        if (ll > sz - s || ll > h.bmax - (d - d0) || ll > cap - d) return SLATE_E_LZ4_CORRUPT;
        if (out)
          for (uint32_t j = lane; j < ll; j += kWave) out[d + j] = src[s + j];
        s += ll;
        d += ll;
        if (s == sz) break;  // the last sequence has literals only
        if (sz - s < 2) return SLATE_E_LZ4_CORRUPT;
        const uint32_t mo = byte_at(s) | (byte_at(s + 1) << 8);
        s += 2;
        if (mo == 0 || mo > d - lo) return SLATE_E_LZ4_CORRUPT;
        uint32_t ml = token & 15;
        if (ml == 15) {
          uint32_t b;
          do {
            if (s >= sz) return SLATE_E_LZ4_CORRUPT;
            b = byte_at(s);
            s++;
            ml += b;
          } while (b == 255);
        }
        ml += 4;
        if (ml > h.bmax - (d - d0) || ml > cap - d) return SLATE_E_LZ4_CORRUPT;
        // byte j repeats the mo-byte pattern (overlapping copies); every read is below d
        if (!out) {
        } else if (mo >= ml) {  // wave-uniform: no overlap, no modulo
          if (uint32_t(lane) < ml) out[d + lane] = out[d - mo + lane];
          for (uint32_t j = lane + kWave; j < ml; j += kWave) out[d + j] = out[d - mo + j];
        } else {
          for (uint32_t j = lane; j < ml; j += kWave) out[d + j] = out[d - mo + (j % mo)];
        }
        d += ml;
      }
    }
    *out_len = d;
    pos += sz + (bcheck ? 4u : 0u);
  }
  if (ccheck) {
    if (n - pos < 4) return SLATE_E_LZ4_CORRUPT;
    __builtin_amdgcn_wave_barrier();
#ifdef SLATE_NO_CONTENT_XXH  // profiling variants only (tools/payload_probe.py): the check skipped
    if (false)
#else
    if (out && wave_xxh32(out, 0, d, lane) != __builtin_amdgcn_readfirstlane(ld_le32(in + pos)))
#endif
      return SLATE_E_LZ4_FRAME_CHECKSUM;
    pos += 4;
  }
  if (csize && h.content != d) return SLATE_E_LZ4_CORRUPT;
  if (pos != n) return SLATE_E_LZ4_CORRUPT;
  *out_len = d;
  return SLATE_OK;
}

// ------------------------------------------------------------ Zlib (inflate)
// compress.Decode CodecZlib = io.ReadAll(zlib.NewReader(buf)) (compression.go:134-140):
// oracle/slate_oracle.c zlib_stream is the restatement this follows check for check.  One
// wave per stream: the bit reader is wave-uniform (bytes come through a 64-byte window
// held one byte per lane), each Huffman symbol is found by lanes 1..15 testing the code of
// their length at once (the shortest match wins, as in a bit-serial canonical decoder),
// and copies are spread over the lanes.
struct ZHuff {
  uint32_t count[16], first[16], index[16];
  uint16_t sym[288];
  uint32_t max, ok;
};
struct ZScratch {  // per wave
  ZHuff lit, dist, clen;
  uint8_t lens[320];
};
constexpr uint32_t kZScratch = (sizeof(ZScratch) + 15) & ~15u;
constexpr uint32_t kZFixed = (2 * sizeof(ZHuff) + 15) & ~15u;

// Canonical tables from code lengths (flate huffmanDecoder.init's acceptance: complete
// codes, the empty tree, or one code of length 1).  Symbols of a length are ranked in
// symbol order with ballots, 64 symbols at a time.
__device__ void zbuild(ZHuff* h, const uint8_t* lens, uint32_t n, int lane) {
  uint32_t cnt = 0;  // lane l: number of codes of length l
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    const uint32_t i = c0 + lane;
    const uint32_t my = i < n ? lens[i] : 0u;
    for (uint32_t l = 1; l < 16; l++) {
      const uint32_t k = uint32_t(__builtin_popcountll(__ballot(my == l)));
      cnt += (uint32_t(lane) == l) ? k : 0u;
    }
  }
  // lane-uniform prefix over lengths
  uint32_t max = 0, first = 0, idx = 0, c = 0;
  for (uint32_t l = 1; l < 16; l++) {
    const uint32_t k = __builtin_amdgcn_readlane(cnt, int(l));
    if (uint32_t(lane) == l) {
      h->count[l] = k;
      h->first[l] = first;
      h->index[l] = idx;
    }
    first = (first + k) << 1;
    idx += k;
    if (k) max = l;
  }
  for (uint32_t l = 1; l <= max; l++) c = (c << 1) + __builtin_amdgcn_readlane(cnt, int(l));
  if (lane == 0) {
    h->count[0] = 0;
    h->max = max;
    h->ok = (max == 0 || c == (1u << max) || (c == 1 && max == 1)) ? 1u : 0u;
  }
  // symbols of length l at index[l] + rank (rank = earlier symbols of that length)
  uint32_t base = 0;  // lane l: symbols of length l placed so far
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    const uint32_t i = c0 + lane;
    const uint32_t my = i < n ? lens[i] : 0u;
    uint32_t pos = 0;
    for (uint32_t l = 1; l < 16; l++) {
      const uint64_t m = __ballot(my == l);
      const uint32_t before = __builtin_amdgcn_readlane(base, int(l));
      if (my == l) pos = before + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)));
      base += (uint32_t(lane) == l) ? uint32_t(__builtin_popcountll(m)) : 0u;
    }
    if (my) h->sym[h->index[my] + pos] = uint16_t(i);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}

struct ZBits {  // wave-uniform bit reader over src[0, n)
  const uint8_t* src;
  uint32_t n, pos, nb;
  uint64_t bits;
  uint32_t wbase, win;
};
__device__ inline uint32_t zbyte(ZBits& z, uint32_t p, int lane) {
  if (p - z.wbase >= uint32_t(kWave)) {
    z.wbase = p;
    z.win = (p + uint32_t(lane) < z.n) ? uint32_t(z.src[p + lane]) : 0u;
  }
  return __builtin_amdgcn_readlane(z.win, int(p - z.wbase));
}
__device__ inline void zfill(ZBits& z, int lane) {  // as many whole bytes as fit (>= 56 bits when available)
  while (z.nb <= 56 && z.pos < z.n) {
    z.bits |= uint64_t(zbyte(z, z.pos, lane)) << z.nb;
    z.pos++;
    z.nb += 8;
  }
}
// -1: out of input, -2: no code matches
// A table's per-length values, lane l holding length l's (1 <= l < 16): read from LDS once per
// table instead of once per symbol.
struct ZLane {
  const ZHuff* h;
  uint32_t first, count, index, max;
};
__device__ inline ZLane zlane(const ZHuff* h, int lane) {
  const uint32_t l = uint32_t(lane);
  return ZLane{h, l < 16 ? h->first[l] : 0u, l < 16 ? h->count[l] : 0u, l < 16 ? h->index[l] : 0u,
               uint32_t(__builtin_amdgcn_readfirstlane(h->max))};
}
// The next symbol: lanes 1..15 test the code of their length at once, the shortest match wins
// (a bit-serial canonical decoder's result); -1: the input ends first, -2: no code matches.
__device__ inline int zsym(ZBits& z, const ZLane& t, int lane) {
  zfill(z, lane);
  const uint32_t l = uint32_t(lane);
  const uint32_t mx = t.max;
  const uint32_t peek = uint32_t(z.bits) & 0x7FFFu;
  const bool test = l >= 1 && l <= mx && l <= z.nb && l < 16;
  const uint32_t code = (l >= 1 && l < 16) ? (__builtin_bitreverse32(peek) >> (32 - l)) : 0u;
  const bool hit = test && code - t.first < t.count;
  const uint64_t m = __ballot(hit);
  if (m == 0) return (z.nb < mx) ? -1 : -2;
  const int L = __builtin_ctzll(m);
  const uint32_t at = __builtin_amdgcn_readlane(t.index + code - t.first, L);
  z.bits >>= L;
  z.nb -= uint32_t(L);
  return int(t.h->sym[at]);
}
__device__ inline int zsym(ZBits& z, const ZHuff* h, int lane) { return zsym(z, zlane(h, lane), lane); }
__device__ inline bool zneed(ZBits& z, uint32_t k, int lane) {
  zfill(z, lane);
  return z.nb >= k;
}
__device__ inline uint32_t ztake(ZBits& z, uint32_t k) {
  const uint32_t v = uint32_t(z.bits) & ((1u << k) - 1u);
  z.bits >>= k;
  z.nb -= k;
  return v;
}

__constant__ uint16_t kZLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                       31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kZLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kZDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                        193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kZDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kZClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// RFC 1951 3.2.6 fixed tables, built once per workgroup
__device__ void zfixed_build(ZHuff* fl, ZHuff* fd, uint8_t* lens, int lane) {
  for (uint32_t i = lane; i < 288; i += kWave) lens[i] = i < 144 ? 8 : (i < 256 ? 9 : (i < 280 ? 7 : 8));
  __builtin_amdgcn_s_waitcnt(0);
  zbuild(fl, lens, 288, lane);
  for (uint32_t i = lane; i < 30; i += kWave) lens[i] = 5;
  __builtin_amdgcn_s_waitcnt(0);
  zbuild(fd, lens, 30, lane);
}

// The stream in[0, n) decoded in order into out[0, cap) (out == nullptr: sizes only, no
// Adler-32).  *out_len: bytes written so far (also on failure).
// kSeg (zlib_payload_segs_kernel): in[0, n) is a raw deflate segment of a larger stream that
// starts with a block header and ends either after an empty non-final stored block whose bytes
// end exactly at n (a piece of this builder's streams) or after the final block at the byte
// boundary n; no zlib header, no Adler-32; distances may not reach before the segment.
template <bool kSeg = false>
__device__ int wave_inflate(const uint8_t* in, uint32_t n, uint8_t* out, uint32_t cap, ZScratch* zs,
                            const ZHuff* fixl, const ZHuff* fixd, int lane, uint32_t* out_len) {
  *out_len = 0;
  if (n == 0) return SLATE_E_EOF;
  if (n < 2) return SLATE_E_UNEXPECTED_EOF;
  const uint32_t b0 = __builtin_amdgcn_readfirstlane(in[0]), b1 = __builtin_amdgcn_readfirstlane(in[1]);
  if (!kSeg && ((b0 & 0x0f) != 8 || (b0 >> 4) > 7 || ((b0 << 8) | b1) % 31 != 0)) return SLATE_E_ZLIB_HEADER;
  uint32_t start = kSeg ? 0u : 2u;
  if (!kSeg && (b1 & 0x20)) {
    if (n < 6) return SLATE_E_UNEXPECTED_EOF;
    const uint32_t id = __builtin_amdgcn_readfirstlane(ld_be32(in + 2));
    if (id != 1) return SLATE_E_ZLIB_DICTIONARY;
    start = 6;
  }
  ZBits z{in, n, start, 0, 0, 0x80000000u, 0};
  uint32_t d = 0;
  bool final = false;
  while (!final) {
    if (!zneed(z, 3, lane)) return SLATE_E_UNEXPECTED_EOF;
    final = ztake(z, 1) != 0;
    const uint32_t type = ztake(z, 2);
    if (type == 0) {  // stored: to the byte boundary, LEN, NLEN, bytes
      ztake(z, z.nb & 7);
      const uint32_t p = z.pos - z.nb / 8;  // next unread byte
      z.pos = p;
      z.nb = 0;
      z.bits = 0;
      if (n - p < 4) return SLATE_E_UNEXPECTED_EOF;
      const uint32_t len = zbyte(z, p, lane) | (zbyte(z, p + 1, lane) << 8);
      const uint32_t nlen = zbyte(z, p + 2, lane) | (zbyte(z, p + 3, lane) << 8);
      z.pos = p + 4;
      if (len != (~nlen & 0xffffu)) return SLATE_E_FLATE_CORRUPT;
      if (len > cap - d) return SLATE_E_FLATE_CORRUPT;
      const uint32_t avail = min(n - z.pos, len);
      if (out)
        for (uint32_t j = lane; j < avail; j += kWave) out[d + j] = in[z.pos + j];
      d += avail;
      z.pos += avail;
      *out_len = d;
      if (avail < len) return SLATE_E_UNEXPECTED_EOF;
      if (kSeg && !final && len == 0 && z.pos == n) return SLATE_OK;  // the piece's byte-aligning end
      continue;
    }
    if (type == 3) return SLATE_E_FLATE_CORRUPT;
    const ZHuff *hl = fixl, *hd = fixd;
    if (type == 2) {
      if (!zneed(z, 14, lane)) return SLATE_E_UNEXPECTED_EOF;
      const uint32_t nlit = ztake(z, 5) + 257, ndist = ztake(z, 5) + 1, nclen = ztake(z, 4) + 4;
      if (nlit > 286 || ndist > 30) return SLATE_E_FLATE_CORRUPT;
      uint32_t cl = 0;  // lane i < 19: the code length of code-length symbol i
      for (uint32_t i = 0; i < 19; i++) {
        uint32_t v = 0;
        if (i < nclen) {
          if (!zneed(z, 3, lane)) return SLATE_E_UNEXPECTED_EOF;
          v = ztake(z, 3);
        }
        if (uint32_t(lane) == kZClenOrder[i]) cl = v;
      }
      if (lane < 19) zs->lens[lane] = uint8_t(cl);
      __builtin_amdgcn_s_waitcnt(0);
      zbuild(&zs->clen, zs->lens, 19, lane);
      if (!zs->clen.ok) return SLATE_E_FLATE_CORRUPT;
      uint32_t i = 0, prev = 0;
      while (i < nlit + ndist) {
        const int sym = zsym(z, &zs->clen, lane);
        if (sym == -1) return SLATE_E_UNEXPECTED_EOF;
        if (sym < 0) return SLATE_E_FLATE_CORRUPT;
        if (sym < 16) {
          if (lane == 0) zs->lens[i] = uint8_t(sym);
          prev = uint32_t(sym);
          i++;
          continue;
        }
        uint32_t rep, val = 0;
        if (sym == 16) {
          if (i == 0) return SLATE_E_FLATE_CORRUPT;
          val = prev;
          if (!zneed(z, 2, lane)) return SLATE_E_UNEXPECTED_EOF;
          rep = 3 + ztake(z, 2);
        } else if (sym == 17) {
          if (!zneed(z, 3, lane)) return SLATE_E_UNEXPECTED_EOF;
          rep = 3 + ztake(z, 3);
        } else {
          if (!zneed(z, 7, lane)) return SLATE_E_UNEXPECTED_EOF;
          rep = 11 + ztake(z, 7);
        }
        if (i + rep > nlit + ndist) return SLATE_E_FLATE_CORRUPT;
        for (uint32_t j = lane; j < rep; j += kWave) zs->lens[i + j] = uint8_t(val);
        prev = val;
        i += rep;
      }
      __builtin_amdgcn_s_waitcnt(0);
      zbuild(&zs->lit, zs->lens, nlit, lane);
      zbuild(&zs->dist, zs->lens + nlit, ndist, lane);
      if (!zs->lit.ok || !zs->dist.ok) return SLATE_E_FLATE_CORRUPT;
      if (__builtin_amdgcn_readfirstlane(zs->lens[256]) == 0) return SLATE_E_FLATE_CORRUPT;
      hl = &zs->lit;
      hd = &zs->dist;
    }
    const ZLane tl = zlane(hl, lane), td = zlane(hd, lane);
    for (;;) {
      int sym = zsym(z, tl, lane);
      if (sym == -1) return SLATE_E_UNEXPECTED_EOF;
      if (sym < 0) return SLATE_E_FLATE_CORRUPT;
      if (sym < 256) {
        if (d >= cap) return SLATE_E_FLATE_CORRUPT;
        if (out && lane == 0) out[d] = uint8_t(sym);
        d++;
        *out_len = d;
        continue;
      }
      if (sym == 256) break;
      sym -= 257;
      if (sym >= 29) return SLATE_E_FLATE_CORRUPT;
      const uint32_t le = kZLenExtra[sym];
      if (!zneed(z, le, lane)) return SLATE_E_UNEXPECTED_EOF;
      const uint32_t len = kZLenBase[sym] + ztake(z, le);
      const int ds = zsym(z, td, lane);
      if (ds == -1) return SLATE_E_UNEXPECTED_EOF;
      if (ds < 0 || ds >= 30) return SLATE_E_FLATE_CORRUPT;
      const uint32_t de = kZDistExtra[ds];
      if (!zneed(z, de, lane)) return SLATE_E_UNEXPECTED_EOF;
      const uint32_t dist = kZDistBase[ds] + ztake(z, de);
      if (dist > d || dist > 32768) return SLATE_E_FLATE_CORRUPT;
      if (len > cap - d) return SLATE_E_FLATE_CORRUPT;
      if (out) {
        __builtin_amdgcn_wave_barrier();
        if (dist >= len) {
          for (uint32_t j = lane; j < len; j += kWave) out[d + j] = out[d - dist + j];
        } else {
          for (uint32_t j = lane; j < len; j += kWave) out[d + j] = out[d - dist + (j % dist)];
        }
      }
      d += len;
      *out_len = d;
    }
  }
  // the Adler-32 trailer starts at the next byte boundary
  ztake(z, z.nb & 7);
  const uint32_t p = z.pos - z.nb / 8;
  if (kSeg) return p == n ? SLATE_OK : SLATE_E_FLATE_CORRUPT;  // the last segment ends the stream
  if (n - p < 4) return SLATE_E_UNEXPECTED_EOF;
  if (out) {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint64_t sa = 0, sb = 0;  // sum x_i and sum (d - i) x_i
    for (uint32_t i = lane; i < d; i += kWave) {
      const uint64_t x = out[i];
      sa += x;
      sb += uint64_t(d - i) * x;
    }
    for (int o = 32; o >= 1; o >>= 1) {
      sa += __shfl_xor(sa, o, 64);
      sb += __shfl_xor(sb, o, 64);
    }
    const uint32_t a = uint32_t((1 + sa) % 65521u), b = uint32_t((uint64_t(d) + sb) % 65521u);
    const uint32_t want = __builtin_amdgcn_readfirstlane((zbyte(z, p, lane) << 24) | (zbyte(z, p + 1, lane) << 16) |
                                                         (zbyte(z, p + 2, lane) << 8) | zbyte(z, p + 3, lane));
    if (((b << 16) | a) != want) return SLATE_E_ZLIB_CHECKSUM;
  }
  *out_len = d;
  return SLATE_OK;
}

// list: the blocks to plan (list[0 .. *count): the ones the lane-per-block plan left), or nullptr
// for all n
__global__ __launch_bounds__(256) void plan_zlib_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off, uint32_t n,
                                                        uint64_t* __restrict__ out_sz, uint64_t* __restrict__ row_sz,
                                                        const uint32_t* list, const uint32_t* count) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kZFixed + 4 * kZScratch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  ZHuff* fix = reinterpret_cast<ZHuff*>(smem);
  ZScratch* zs = reinterpret_cast<ZScratch*>(smem + kZFixed + wave * kZScratch);
  if (wave == 0) zfixed_build(fix, fix + 1, zs->lens, lane);
  __syncthreads();
  const uint32_t waves = gridDim.x * 4;
  const uint32_t items = list ? *count : n;
  for (uint32_t k = blockIdx.x * 4 + wave; k < items; k += waves) {
    const uint32_t b = list ? list[k] : k;
    const uint64_t s0 = in_off[b], len = in_off[b + 1] - s0;
    uint32_t dl = 0;
    if (len >= 6 && len - 4 < 0xFFFFFFFFull) wave_inflate(in + s0, uint32_t(len - 4), nullptr, 0xFFFFFFFFu, zs, fix, fix + 1, lane, &dl);
    if (lane == 0) {
      out_sz[b] = align16(dl);
      row_sz[b] = row_capacity(dl);
    }
  }
}

// CodecZstd sizes (oracle or_zstd_plan): one wave per block reading the frames from HBM.
// list: the blocks to plan (list[0 .. *count)), or nullptr for all n.
__global__ __launch_bounds__(256) void plan_zstd_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off, uint32_t n,
                                                        uint64_t* __restrict__ out_sz, uint64_t* __restrict__ row_sz,
                                                        const uint32_t* list, const uint32_t* count) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kZsShared + 4 * kZsScratch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t items = list ? *count : n;
  if (blockIdx.x * 4 >= items) return;  // (workgroup-uniform) nothing to plan: skip the table build
  ZsShared* sh = reinterpret_cast<ZsShared*>(smem);
  ZsScratch* sc = reinterpret_cast<ZsScratch*>(smem + kZsShared + wave * kZsScratch);
  if (wave == 0) zs_shared_build(sh, sc, lane);
  __syncthreads();
  const uint32_t waves = gridDim.x * 4;
  for (uint32_t k = blockIdx.x * 4 + wave; k < items; k += waves) {
    const uint32_t b = list ? list[k] : k;
    const uint64_t s0 = in_off[b], len = in_off[b + 1] - s0;
    uint64_t dl = 0;
    if (len >= 6 && len - 4 < 0x7FFFFFFFull) {
      const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(in + s0) & ~uintptr_t(3));
      dl = wave_zstd_plan(base, int32_t((in + s0) - base), uint32_t(len - 4), sc, sh, lane);
    }
    if (lane == 0) {
      out_sz[b] = align16(dl);
      row_sz[b] = row_capacity(dl);
    }
  }
}

// ------------------------------------------------------------ one block
struct WaveBufs {
  const uint32_t* tab;  // CRC tables in LDS (4 x 256)
  uint8_t* in;          // staging for the encoded block (in_cap bytes, 16-aligned)
  uint8_t* out;         // decoded block (out_cap bytes, 16-aligned)
  uint32_t in_cap, out_cap;
  ZScratch* zs = nullptr;  // CodecZlib only: this wave's Huffman tables
  const ZHuff* zfix = nullptr;  // CodecZlib only: the workgroup's fixed literal/length + distance tables
  ZsScratch* zss = nullptr;     // CodecZstd only: this wave's tables
  const ZsShared* zsh = nullptr;  // CodecZstd only: the workgroup's predefined tables
};

// Returns false when the block does not fit this wave's LDS budget (caller defers it).
// CK: the codec class compiled in (0: None/Snappy/LZ4, 1: Zlib, 2: Zstd), so each kernel
// instance carries only its codec's registers.
// G (decode_payload_kernel): no LDS staging; the decoders read the encoded bytes and write
// the decoded ones in HBM (the lanes of one wave see each other's global stores in program
// order, so the copies read back what earlier lanes wrote), for payloads of any size.
// a.raw: the payload is an index or filter buffer, not a block: CRC + decompress only.
template <int CK, bool G = false>
__device__ bool decode_block_wave(const DecodeArgs& a, uint32_t b, const WaveBufs& w0, int lane, bool defer_large) {
  slate_block_meta m{};
  uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
  const uint8_t* gin = a.in + s0;
  WaveBufs w = w0;
  if (G) {
    w.in = const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(gin) & ~uintptr_t(15)));
    w.out = a.out + a.out_off[b];
    w.in_cap = w.out_cap = 0xFFFFFFFFu;
  }
  if (len < (a.raw ? 4u : 6u)) {
    m.status = SLATE_E_BLOCK_TOO_SMALL;
    write_meta(&a.meta[b], m, lane);
    return true;
  }
  uint32_t hdr = 0;
  uint64_t dl = 0;
  // LZ4/Zlib: the plan's capacity (>= what the in-order decoder writes); others: the header
  const bool dl_ok = (a.codec == SLATE_CODEC_LZ4 || a.codec == SLATE_CODEC_ZLIB || a.codec == SLATE_CODEC_ZSTD)
                         ? (dl = a.out_off[b + 1] - a.out_off[b], true)
                         : decoded_len(a.codec, gin, len, &dl, &hdr);
  uint32_t shift = uint32_t(reinterpret_cast<uintptr_t>(gin) & 15);
  if (len > 0xFFFFFF00ull || shift + len > w.in_cap || (a.codec != SLATE_CODEC_NONE && dl > w.out_cap)) {
    if (defer_large) return false;
    m.status = SLATE_E_CAPACITY;  // beyond the large kernel's LDS budget (its caller then takes the HBM mode)
    write_meta(&a.meta[b], m, lane);
    return true;
  }
  // ---- stage the encoded block into LDS with aligned 16-byte loads
  if (!G) {
    const uint4* src = reinterpret_cast<const uint4*>(gin - shift);
    uint4* dst = reinterpret_cast<uint4*>(w.in);
    uint32_t chunks = uint32_t((shift + len + 15) / 16);
    for (uint32_t c = lane; c < chunks; c += kWave) dst[c] = src[c];
  }
  __builtin_amdgcn_s_waitcnt(0);  // LDS stores visible to the whole wave (in-order LDS)
  __builtin_amdgcn_wave_barrier();
  uint32_t clen = uint32_t(len - 4);
  uint32_t stored = ld_be32(w.in + shift + clen);
  uint32_t crc = (dbg_bits(a) & 1) ? stored : wave_crc32(w.tab, w.in, int32_t(shift), clen, lane);
  if (stored != crc) {
    m.status = SLATE_E_BLOCK_CHECKSUM;
    write_meta(&a.meta[b], m, lane);
    return true;
  }
  // ---- an index / filter (DecodeIndex, ReadFilter): compress.Decode after the oracle's
  // or_decompress_len, whose status comes first and whose size is the capacity
  if (G && a.raw && (a.codec == SLATE_CODEC_LZ4 || a.codec == SLATE_CODEC_ZLIB || a.codec == SLATE_CODEC_ZSTD)) {
    uint32_t pl = 0;
    int pst = SLATE_OK;
    if (CK == 0 && a.codec == SLATE_CODEC_LZ4) {
      pst = wave_lz4_decode(w.in, shift, clen, nullptr, 0xFFFFFFFFu, lane, &pl);
    } else if (CK == 1 && a.codec == SLATE_CODEC_ZLIB) {
      pst = wave_inflate(w.in + shift, clen, nullptr, 0xFFFFFFFFu, w.zs, w.zfix, w.zfix + 1, lane, &pl);
    } else if (CK == 2 && a.codec == SLATE_CODEC_ZSTD) {
      const uint64_t z = wave_zstd_plan(w.in, int32_t(shift), clen, w.zss, w.zsh, lane);
      if (z > a.out_off[b + 1] - a.out_off[b]) pst = SLATE_E_CAPACITY;  // cannot happen: the host planned with it
      pl = uint32_t(z);
    }
    if (pst != SLATE_OK) {
      m.status = int16_t(pst);
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    dl = pl;
  }
  // ---- decompress (compress.Decode, compression.go:126-157)
  const uint8_t* buf;  // decoded buffer in LDS
  uint32_t n;
  if (a.codec == SLATE_CODEC_NONE) {
    buf = w.in + shift;
    n = clen;
  } else if (CK == 0 && a.codec == SLATE_CODEC_SNAPPY) {
    if (!dl_ok) {  // corrupt varint header or provably corrupt length
      m.status = SLATE_E_SNAPPY_CORRUPT;
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    int st = (dbg_bits(a) & 2) ? SLATE_OK : wave_snappy_decode(w.in + shift, clen, hdr, w.out, uint32_t(dl), lane);
    if (st != SLATE_OK) {
      m.status = int16_t(st);
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    buf = w.out;
    n = uint32_t(dl);
  } else if (CK == 0 && a.codec == SLATE_CODEC_LZ4) {
    uint32_t outn = 0;
    int st = (dbg_bits(a) & 2) ? (outn = uint32_t(dl), SLATE_OK)  // profiling: skip the decompression
                           : wave_lz4_decode(w.in, shift, clen, w.out, uint32_t(dl), lane, &outn);
    if (st != SLATE_OK) {
      m.status = int16_t(st);
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    buf = w.out;
    n = outn;
  } else if (CK == 1 && a.codec == SLATE_CODEC_ZLIB) {
    uint32_t outn = 0;
    int st = (dbg_bits(a) & 2) ? (outn = uint32_t(dl), SLATE_OK)
                           : wave_inflate(w.in + shift, clen, w.out, uint32_t(dl), w.zs, w.zfix, w.zfix + 1, lane, &outn);
    if (st != SLATE_OK) {
      m.status = int16_t(st);
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    buf = w.out;
    n = outn;
  } else if (CK == 2 && a.codec == SLATE_CODEC_ZSTD) {
    uint32_t outn = 0;
    int st = (dbg_bits(a) & 2) ? (outn = uint32_t(dl), SLATE_OK)
                           : wave_zstd_decode(w.in, int32_t(shift), clen, w.out, uint32_t(dl), w.zss, w.zsh, lane, &outn,
                                              dbg_bits(a));
    if (st != SLATE_OK) {
      m.status = int16_t(st);
      write_meta(&a.meta[b], m, lane);
      return true;
    }
    buf = w.out;
    n = outn;
  } else {
    m.status = SLATE_E_INVALID_CODEC;
    write_meta(&a.meta[b], m, lane);
    return true;
  }
  __builtin_amdgcn_wave_barrier();
  // ---- write the decoded buffer back (16-aligned destination); a.no_data (CodecNone aliased in
  // place): the bytes are already there
  if (a.no_data) {
  } else if (G) {
    if (buf != w.out)
      for (uint32_t c = lane; c < n; c += kWave) w.out[c] = buf[c];
  } else if (!(dbg_bits(a) & 8)) {
    uint8_t* gout = a.out + a.out_off[b];
    uint32_t chunks = (n + 15) / 16;
    if (buf == w.out) {
      const uint4* s = reinterpret_cast<const uint4*>(buf);
      for (uint32_t c = lane; c < chunks; c += kWave) reinterpret_cast<uint4*>(gout)[c] = s[c];
    } else {
      uint32_t base = uint32_t(buf - w.in);
      for (uint32_t c = lane; c < chunks; c += kWave) {
        int32_t o = int32_t(base + 16 * c);
        uint4 v;
        v.x = lds_u32(w.in, o);
        v.y = lds_u32(w.in, o + 4);
        v.z = lds_u32(w.in, o + 8);
        v.w = lds_u32(w.in, o + 12);
        reinterpret_cast<uint4*>(gout)[c] = v;
      }
    }
  }
  if (a.raw) {  // an index / filter payload: decoded length only
    m.data_len = n;
    write_meta(&a.meta[b], m, lane);
    return true;
  }
  block_finish(a, b, buf, n, lane, m);
  return true;
}

// CodecZlib LDS after the per-wave buffers: fixed tables (one per workgroup), then a
// ZScratch per wave; the fixed tables are built by wave 0.
__device__ inline void zlib_lds(WaveBufs& w, uint8_t* zbase, int waves, int wave, int lane) {
  ZHuff* fix = reinterpret_cast<ZHuff*>(zbase);
  w.zfix = fix;
  w.zs = reinterpret_cast<ZScratch*>(zbase + kZFixed + size_t(wave) * kZScratch);
  if (wave == 0) zfixed_build(fix, fix + 1, w.zs->lens, lane);
  (void)waves;
  __syncthreads();
}

// CodecZstd LDS after the per-wave buffers: the predefined tables (one per workgroup, built
// by wave 0), then a ZsScratch per wave.
__device__ inline void zstd_lds(WaveBufs& w, uint8_t* zbase, int wave, int lane) {
  ZsShared* sh = reinterpret_cast<ZsShared*>(zbase);
  w.zsh = sh;
  w.zss = reinterpret_cast<ZsScratch*>(zbase + kZsShared + size_t(wave) * kZsScratch);
  if (wave == 0) zs_shared_build(sh, w.zss, lane);
  __syncthreads();
}

template <int CK>
__global__ __launch_bounds__(kDecodeThreads) void decode_fast_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // CodecZstd: trimmed staging (two workgroups per CU with the tables); larger blocks
  // take the large-block kernel
  constexpr uint32_t in_cap = CK == 2 ? kZsFastInCap : kFastInCap, out_cap = CK == 2 ? kZsFastOutCap : kFastOutCap;
  const uint32_t per_wave = in_cap + out_cap;
  WaveBufs w{tab, smem + kTabBytes + wave * per_wave, smem + kTabBytes + wave * per_wave + in_cap, in_cap, out_cap};
  if (CK == 1) zlib_lds(w, smem + kTabBytes + (kDecodeThreads / 64) * per_wave, kDecodeThreads / 64, wave, lane);
  if (CK == 2) zstd_lds(w, smem + kTabBytes + (kDecodeThreads / 64) * per_wave, wave, lane);
  const uint32_t waves = gridDim.x * (kDecodeThreads / 64);
  for (uint32_t b = blockIdx.x * (kDecodeThreads / 64) + wave; b < a.n; b += waves) {
    if (!decode_block_wave<CK>(a, b, w, lane, true)) {
      if (lane == 0) a.large_list[atomicAdd(a.large_count, 1u)] = b;
    }
  }
}

// decode_fast_kernel over a list of blocks (list[0 .. *count)): the CodecZstd blocks the fast
// path hands back (zstd_fast.hip).
template <int CK>
__global__ __launch_bounds__(kDecodeThreads) void decode_list_kernel(DecodeArgs a, const uint32_t* list,
                                                                     const uint32_t* count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t items = *count;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.handbacks && items) atomicAdd(a.handbacks, uint64_t(items));
  if (blockIdx.x * (kDecodeThreads / 64) >= items) return;  // (workgroup-uniform) no block: skip the tables
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t in_cap = CK == 2 ? kZsFastInCap : kFastInCap, out_cap = CK == 2 ? kZsFastOutCap : kFastOutCap;
  const uint32_t per_wave = in_cap + out_cap;
  WaveBufs w{tab, smem + kTabBytes + wave * per_wave, smem + kTabBytes + wave * per_wave + in_cap, in_cap, out_cap};
  if (CK == 1) zlib_lds(w, smem + kTabBytes + (kDecodeThreads / 64) * per_wave, kDecodeThreads / 64, wave, lane);
  if (CK == 2) zstd_lds(w, smem + kTabBytes + (kDecodeThreads / 64) * per_wave, wave, lane);
  const uint32_t waves = gridDim.x * (kDecodeThreads / 64);
  for (uint32_t k = blockIdx.x * (kDecodeThreads / 64) + wave; k < items; k += waves) {
    const uint32_t b = list[k];
    if (!decode_block_wave<CK>(a, b, w, lane, true)) {
      if (lane == 0) a.large_list[atomicAdd(a.large_count, 1u)] = b;
    }
  }
}

template <int CK>
__global__ __launch_bounds__(64) void decode_large_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t count = *a.large_count;
  if (blockIdx.x >= count) return;  // (workgroup-uniform) no block: skip the tables (~50 us for Zstd's)
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63;
  // CodecZlib: its tables take the top of the input staging area
  const uint32_t in_cap = CK == 1 ? kLargeInCap - kZFixed - kZScratch
                          : CK == 2 ? kLargeInCap - kZsShared - kZsScratch
                                    : kLargeInCap;
  WaveBufs w{tab, smem + kTabBytes, smem + kTabBytes + kLargeInCap, in_cap, kLargeOutCap};
  if (CK == 1) zlib_lds(w, smem + kTabBytes + in_cap, 1, 0, lane);
  if (CK == 2) zstd_lds(w, smem + kTabBytes + in_cap, 0, lane);
  for (uint32_t k = blockIdx.x; k < count; k += gridDim.x) {
    // beyond this kernel's LDS budget (encoded > 64 KiB or decoded > 88 KiB: a block holding one
    // large value): the same wave decoder with input and output in HBM
    const uint32_t b = a.large_list[k];
    if (!decode_block_wave<CK>(a, b, w, lane, true)) decode_block_wave<CK, true>(a, b, w, lane, false);
  }
}

// Index / filter payloads of any size (LZ4 / Zlib / Zstd; raw mode): one wave per payload,
// input and output in HBM (decode_block_wave<CK, true>), LDS for the CRC and codec tables only.
template <int CK>
__global__ __launch_bounds__(64) void decode_payload_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63;
  WaveBufs w{tab, nullptr, nullptr, 0u, 0u};
  if (CK == 1) zlib_lds(w, smem + kTabBytes, 1, 0, lane);
  if (CK == 2) zstd_lds(w, smem + kTabBytes, 0, lane);
  for (uint32_t b = blockIdx.x; b < a.n; b += gridDim.x) decode_block_wave<CK, true>(a, b, w, lane, false);
}

// ---------------------------------------------- CodecZlib payloads split by piece
// An index or filter written by this builder is one deflate stream whose pieces each end with an
// empty stored block, so piece k starts byte-aligned right after the k-th `00 00 FF FF`.  The host
// cuts the stream at those markers (a marker inside a piece's data makes that piece fail here, and
// the serial path takes over); one wave per segment inflates it in LDS (wave_inflate<true>).
// seg = nseg x (stream offset, length); sizes[k] = decoded bytes at slots + k * 64 KiB, or ~0u.
constexpr uint32_t kZPayIn = 66 * 1024 + 32, kZPayOut = 65536;
__global__ __launch_bounds__(64) void zlib_payload_segs_kernel(const uint8_t* __restrict__ in,
                                                               const uint32_t* __restrict__ seg, uint32_t nseg,
                                                               uint8_t* __restrict__ slots,
                                                               uint32_t* __restrict__ sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* lin = smem;
  uint8_t* lout = smem + kZPayIn;
  ZHuff* fix = reinterpret_cast<ZHuff*>(lout + kZPayOut);
  ZScratch* zs = reinterpret_cast<ZScratch*>(reinterpret_cast<uint8_t*>(fix) + kZFixed);
  const int lane = int(threadIdx.x);
  zfixed_build(fix, fix + 1, zs->lens, lane);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  for (uint32_t k = blockIdx.x; k < nseg; k += gridDim.x) {
    const uint32_t pos = seg[2 * k], n = seg[2 * k + 1];
    const uint8_t* g = in + pos;
    const uint32_t shift = uint32_t(reinterpret_cast<uintptr_t>(g) & 15);
    if (shift + n + 16 > kZPayIn) {
      if (lane == 0) sizes[k] = ~0u;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    {
      const uint4* src4 = reinterpret_cast<const uint4*>(g - shift);
      uint4* dst4 = reinterpret_cast<uint4*>(lin);
      for (uint32_t c = uint32_t(lane); c < (shift + n + 15) / 16; c += kWave) dst4[c] = src4[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint32_t d = 0;
    const bool ok = wave_inflate<true>(lin + shift, n, lout, kZPayOut, zs, fix, fix + 1, lane, &d) == SLATE_OK;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (ok) {
      uint4* o4 = reinterpret_cast<uint4*>(slots + size_t(k) * kZPayOut);
      const uint4* l4 = reinterpret_cast<const uint4*>(lout);
      for (uint32_t c = uint32_t(lane); c < (d + 15) / 16; c += kWave) o4[c] = l4[c];
    }
    if (lane == 0) sizes[k] = ok ? d : ~0u;
  }
}

// Adler-32 partial sums of a device buffer: slice t = bytes [4096 t, 4096 t + 4096) (the last one
// shorter): part[t] = (sum x_j, sum (end_t - j) x_j); the host folds them (api_sst.cpp).
__global__ __launch_bounds__(256) void adler_slices_kernel(const uint8_t* __restrict__ p, uint32_t n,
                                                           uint64_t* __restrict__ part) {
  const uint32_t nsl = (n + 4095) / 4096;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < nsl; t += gridDim.x * 4) {
    const uint32_t s0 = 4096 * t, e = min(n, s0 + 4096);
    uint64_t sa = 0, sb = 0;
    for (uint32_t j = s0 + lane; j < e; j += kWave) {
      const uint64_t x = p[j];
      sa += x;
      sb += uint64_t(e - j) * x;
    }
    for (int o = 32; o >= 1; o >>= 1) {
      sa += __shfl_xor(sa, o, 64);
      sb += __shfl_xor(sb, o, 64);
    }
    if (lane == 0) {
      part[2 * t] = sa;
      part[2 * t + 1] = sb;
    }
  }
}

hipError_t launch_zlib_payload_segs(hipStream_t st, const uint8_t* in, const uint32_t* seg, uint32_t nseg,
                                    uint8_t* slots, uint32_t* sizes, int num_cus) {
  if (nseg == 0) return hipGetLastError();
  const size_t lds = size_t(kZPayIn) + kZPayOut + kZFixed + kZScratch;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zlib_payload_segs_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  zlib_payload_segs_kernel<<<min(nseg, uint32_t(num_cus)), 64, lds, st>>>(in, seg, nseg, slots, sizes);
  return hipGetLastError();
}

hipError_t launch_adler_slices(hipStream_t st, const uint8_t* p, uint32_t n, uint64_t* part) {
  const uint32_t nsl = (n + 4095) / 4096;
  if (nsl) adler_slices_kernel<<<min((nsl + 3) / 4, 4096u), 256, 0, st>>>(p, n, part);
  return hipGetLastError();
}

// ------------------------------------------- CodecLz4 payloads split by data block
// An index or filter written as an LZ4 frame of independent data blocks (this builder's frames:
// one block per 64 KiB piece) decodes block by block in parallel: one wave per data block, the
// compressed block and its output in LDS.  sizes[k] = the decoded bytes (the output at
// slots + k * kLz4PaySlot), or ~0u when block k needs the serial path (an output above 64 KiB, or
// any check of wave_lz4_decode's failing).  Frame header, block list, content size and checksum
// are the host's and lz4_payload_xxh32_kernel's (api_sst.cpp lz4_payload_split).
constexpr uint32_t kLz4PayIn = 65536 + 32, kLz4PayOut = 65536, kLz4PaySlot = 65536;
__global__ __launch_bounds__(64) void lz4_payload_blocks_kernel(const uint8_t* __restrict__ in,
                                                                const uint32_t* __restrict__ blk, uint32_t nblk,
                                                                uint32_t bmax, uint8_t* __restrict__ slots,
                                                                uint32_t* __restrict__ sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* lin = smem;
  uint8_t* lout = smem + kLz4PayIn;
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const uint32_t pos = blk[2 * k], bs = blk[2 * k + 1];
    const uint32_t sz = bs & 0x7FFFFFFFu;
    const bool stored = (bs >> 31) != 0;
    const uint8_t* g = in + pos;
    const uint32_t shift = uint32_t(reinterpret_cast<uintptr_t>(g) & 15);
    if (shift + sz + 16 > kLz4PayIn || (stored && sz > kLz4PayOut) || sz > bmax) {
      if (lane == 0) sizes[k] = ~0u;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    {
      const uint4* src4 = reinterpret_cast<const uint4*>(g - shift);
      uint4* dst4 = reinterpret_cast<uint4*>(lin);
      const uint32_t chunks = (shift + sz + 15) / 16;
      for (uint32_t c = lane; c < chunks; c += kWave) dst4[c] = src4[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const uint8_t* src = lin + shift;
    uint32_t d = 0;
    bool ok = true;
    if (stored) {
      for (uint32_t j = lane; j < sz; j += kWave) lout[j] = src[j];
      d = sz;
    } else {
      // wave_lz4_decode's sequence loop for one independent block (lo = d0 = 0), cap = 64 KiB
      uint32_t wbase = 0x80000000u, win = 0;
      auto byte_at = [&](uint32_t p) -> uint32_t {
        if (p - wbase >= uint32_t(kWave)) {
          wbase = p;
          win = (p + lane < sz) ? uint32_t(src[p + lane]) : 0u;
        }
        return __builtin_amdgcn_readlane(win, int(p - wbase));
      };
      const uint32_t cap = min(kLz4PayOut, bmax);
      uint32_t s = 0;
      for (;;) {
        if (s >= sz) { ok = false; break; }
        const uint32_t token = byte_at(s);
        s++;
        uint32_t ll = token >> 4;
        if (ll == 15) {
          uint32_t b;
          do {
            if (s >= sz) { ok = false; break; }
            b = byte_at(s);
            s++;
            ll += b;
          } while (b == 255);
          if (!ok) break;
        }
        if (ll > sz - s || ll > cap - d) { ok = false; break; }
        for (uint32_t j = lane; j < ll; j += kWave) lout[d + j] = src[s + j];
        s += ll;
        d += ll;
        if (s == sz) break;  // the last sequence has literals only
        if (sz - s < 2) { ok = false; break; }
        const uint32_t mo = byte_at(s) | (byte_at(s + 1) << 8);
        s += 2;
        if (mo == 0 || mo > d) { ok = false; break; }
        uint32_t ml = token & 15;
        if (ml == 15) {
          uint32_t b;
          do {
            if (s >= sz) { ok = false; break; }
            b = byte_at(s);
            s++;
            ml += b;
          } while (b == 255);
          if (!ok) break;
        }
        ml += 4;
        if (ml > cap - d) { ok = false; break; }
        __builtin_amdgcn_wave_barrier();  // the literals / earlier matches are in LDS
        if (mo >= ml) {
          for (uint32_t j = lane; j < ml; j += kWave) lout[d + j] = lout[d - mo + j];
        } else {
          for (uint32_t j = lane; j < ml; j += kWave) lout[d + j] = lout[d - mo + (j % mo)];
        }
        __builtin_amdgcn_wave_barrier();
        d += ml;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (ok) {
      uint4* o4 = reinterpret_cast<uint4*>(slots + size_t(k) * kLz4PaySlot);
      const uint4* l4 = reinterpret_cast<const uint4*>(lout);
      for (uint32_t c = lane; c < (d + 15) / 16; c += kWave) o4[c] = l4[c];
    }
    if (lane == 0) sizes[k] = ok ? d : ~0u;
  }
}

// XXH32 (seed 0) of a device buffer by one wave: 1 KiB of stripes per step staged in LDS
// (loaded one step ahead), the four accumulators on lanes 0-3; *out = the hash.
__global__ __launch_bounds__(64) void lz4_payload_xxh32_kernel(const uint8_t* __restrict__ p, uint32_t n,
                                                               uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 buf[2][64];
  const uint32_t lane = threadIdx.x;
  const uint32_t stripes = n / 16, steps = (stripes + 63) / 64;
  uint32_t v = lane == 0 ? kXP1 + kXP2 : (lane == 1 ? kXP2 : (lane == 2 ? 0u : 0u - kXP1));
  const uint4* p4 = reinterpret_cast<const uint4*>(p);  // (a 16-byte aligned device buffer)
  uint4 nxt = (steps && lane < stripes) ? p4[lane] : make_uint4(0, 0, 0, 0);
  for (uint32_t t = 0; t < steps; t++) {
    buf[t & 1][lane] = nxt;
    const uint32_t q = 64 * (t + 1) + lane;
    nxt = q < stripes ? p4[q] : make_uint4(0, 0, 0, 0);  // in flight during this step
    __builtin_amdgcn_s_waitcnt(0xc07f);                   // lgkmcnt(0): the LDS store landed
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (lane < 4) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(buf[t & 1]);
      const uint32_t m = min(64u, stripes - 64 * t);
      for (uint32_t i = 0; i < m; i++) v = xrotl(v + w[4 * i + lane] * kXP2, 13) * kXP1;
    }
    __builtin_amdgcn_wave_barrier();
  }
  uint32_t h = n >= 16 ? xrotl(__builtin_amdgcn_readlane(v, 0), 1) + xrotl(__builtin_amdgcn_readlane(v, 1), 7) +
                             xrotl(__builtin_amdgcn_readlane(v, 2), 12) + xrotl(__builtin_amdgcn_readlane(v, 3), 18)
                       : kXP5;
  h += n;
  uint32_t i = n & ~15u;
  for (; i + 4 <= n; i += 4) h = xrotl(h + ld_le32(p + i) * kXP3, 17) * kXP4;
  for (; i < n; i++) h = xrotl(h + uint32_t(p[i]) * kXP5, 11) * kXP1;
  h ^= h >> 15;
  h *= kXP2;
  h ^= h >> 13;
  h *= kXP3;
  h ^= h >> 16;
  if (lane == 0) *out = h;
}

// CodecZstd payloads split by block: a frame whose compressed blocks decode on their own (fresh
// state: predefined or own tables, no treeless literals, no repeat offsets, no match reaching
// before the block) -- the frames this builder writes: one block per 64 KiB piece.  blk = nblk x
// (frame offset, block header); one wave per block with the block, its output and the tables in
// LDS; sizes[k] = decoded bytes at slots + k * 64 KiB, or ~0u for the serial path.
constexpr uint32_t kZsPayIn = 65536 + 32, kZsPayOut = 65536;
__global__ __launch_bounds__(64) void zstd_payload_blocks_kernel(const uint8_t* __restrict__ in,
                                                                 const uint32_t* __restrict__ blk, uint32_t nblk,
                                                                 uint32_t bmax, uint8_t* __restrict__ slots,
                                                                 uint32_t* __restrict__ sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* lin = smem;
  uint8_t* lout = smem + kZsPayIn;
  ZsShared* sh = reinterpret_cast<ZsShared*>(lout + kZsPayOut);
  ZsScratch* sc = reinterpret_cast<ZsScratch*>(reinterpret_cast<uint8_t*>(sh) + kZsShared);
  const int lane = int(threadIdx.x);
  zs_shared_build(sh, sc, lane);
  zs_sync();
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const uint32_t pos = blk[2 * k], bh = blk[2 * k + 1];
    const uint32_t bt = (bh >> 1) & 3, bs = bh >> 3;
    const uint8_t* g = in + pos;
    const uint32_t shift = uint32_t(reinterpret_cast<uintptr_t>(g) & 15);
    const uint32_t clen = bt == 1 ? 1u : bs;  // bytes of the block body
    if (bt == 3 || shift + clen + 16 > kZsPayIn || bs > bmax || (bt != 2 && bs > kZsPayOut)) {
      if (lane == 0) sizes[k] = ~0u;
      continue;
    }
    zs_sync();
    {
      const uint4* src4 = reinterpret_cast<const uint4*>(g - shift);
      uint4* dst4 = reinterpret_cast<uint4*>(lin);
      const uint32_t chunks = (shift + clen + 15) / 16;
      for (uint32_t c = uint32_t(lane); c < chunks; c += kWave) dst4[c] = src4[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    zs_sync();
    uint32_t d = 0;
    bool ok = true;
    if (bt == 0) {
      for (uint32_t j = uint32_t(lane); j < bs; j += kWave) lout[j] = lin[shift + j];
      d = bs;
    } else if (bt == 1) {
      const uint8_t v = lin[shift];
      for (uint32_t j = uint32_t(lane); j < bs; j += kWave) lout[j] = v;
      d = bs;
    } else {
      ZsState st{nullptr, nullptr, nullptr, 0, 0, 0, 0, 0, {1, 4, 8}, 0};
      const int r = zs_block(lin, int32_t(shift), bs, lout, kZsPayOut, &d, 0u, bmax, sc, sh, st, lane);
      ok = r == SLATE_OK && !st.rep_used;
    }
    zs_sync();
    __builtin_amdgcn_s_waitcnt(0);
    if (ok) {
      uint4* o4 = reinterpret_cast<uint4*>(slots + size_t(k) * kZsPayOut);
      const uint4* l4 = reinterpret_cast<const uint4*>(lout);
      for (uint32_t c = uint32_t(lane); c < (d + 15) / 16; c += kWave) o4[c] = l4[c];
    }
    if (lane == 0) sizes[k] = ok ? d : ~0u;
  }
}

// XXH64 (seed 0) of a 16-byte aligned device buffer by one wave (2 KiB of 32-byte stripes per
// step staged in LDS, loaded one step ahead; accumulators on lanes 0-3); out = the low 32 bits
// as the frame stores them.
__global__ __launch_bounds__(64) void zstd_payload_xxh64_kernel(const uint8_t* __restrict__ p, uint32_t n,
                                                                uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 buf[2][128];
  const uint32_t lane = threadIdx.x;
  const uint32_t stripes = n / 32, steps = (stripes + 63) / 64;
  uint64_t v = lane == 0 ? kX64P1 + kX64P2 : (lane == 1 ? kX64P2 : (lane == 2 ? 0ull : 0ull - kX64P1));
  const uint4* p4 = reinterpret_cast<const uint4*>(p);
  const uint32_t q16 = 2 * stripes;  // 16-byte chunks in whole stripes
  uint4 n0 = lane < q16 ? p4[lane] : make_uint4(0, 0, 0, 0), n1 = 64 + lane < q16 ? p4[64 + lane] : make_uint4(0, 0, 0, 0);
  for (uint32_t t = 0; t < steps; t++) {
    buf[t & 1][lane] = n0;
    buf[t & 1][64 + lane] = n1;
    const uint32_t q = 128 * (t + 1) + lane;
    n0 = q < q16 ? p4[q] : make_uint4(0, 0, 0, 0);
    n1 = q + 64 < q16 ? p4[q + 64] : make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (lane < 4) {
      const uint64_t* w = reinterpret_cast<const uint64_t*>(buf[t & 1]);
      const uint32_t m = min(64u, stripes - 64 * t);
      for (uint32_t i = 0; i < m; i++) v = x64round(v, w[4 * i + lane]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  uint64_t vv[4];
  for (int l = 0; l < 4; l++)
    vv[l] = uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v), l))) |
            (uint64_t(uint32_t(__builtin_amdgcn_readlane(uint32_t(v >> 32), l))) << 32);
  uint64_t h;
  if (n >= 32) {
    h = x64rotl(vv[0], 1) + x64rotl(vv[1], 7) + x64rotl(vv[2], 12) + x64rotl(vv[3], 18);
    for (int l = 0; l < 4; l++) h = (h ^ x64round(0, vv[l])) * kX64P1 + kX64P4;
  } else {
    h = kX64P5;
  }
  h += n;
  uint32_t i = n & ~31u;
  auto le64 = [&](uint32_t o) {
    uint64_t x = 0;
    for (int b = 7; b >= 0; b--) x = (x << 8) | p[o + b];
    return x;
  };
  for (; i + 8 <= n; i += 8) h = x64rotl(h ^ x64round(0, le64(i)), 27) * kX64P1 + kX64P4;
  if (i + 4 <= n) {
    h = x64rotl(h ^ uint64_t(ld_le32(p + i)) * kX64P1, 23) * kX64P2 + kX64P3;
    i += 4;
  }
  for (; i < n; i++) h = x64rotl(h ^ uint64_t(p[i]) * kX64P5, 11) * kX64P1;
  h ^= h >> 33;
  h *= kX64P2;
  h ^= h >> 29;
  h *= kX64P3;
  h ^= h >> 32;
  if (lane == 0) *out = uint32_t(h);
}

hipError_t launch_zstd_payload_blocks(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                      uint32_t bmax, uint8_t* slots, uint32_t* sizes, int num_cus) {
  if (nblk == 0) return hipGetLastError();
  const size_t lds = size_t(kZsPayIn) + kZsPayOut + kZsShared + kZsScratch;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zstd_payload_blocks_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  zstd_payload_blocks_kernel<<<min(nblk, uint32_t(num_cus)), 64, lds, st>>>(in, blk, nblk, bmax, slots, sizes);
  return hipGetLastError();
}

hipError_t launch_xxh64_lo(hipStream_t st, const uint8_t* p, uint32_t n, uint32_t* out) {
  zstd_payload_xxh64_kernel<<<1, 64, 0, st>>>(p, n, out);
  return hipGetLastError();
}

hipError_t launch_lz4_payload_blocks(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                     uint32_t bmax, uint8_t* slots, uint32_t* sizes, int num_cus) {
  if (nblk == 0) return hipGetLastError();
  const size_t lds = size_t(kLz4PayIn) + kLz4PayOut;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&lz4_payload_blocks_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  lz4_payload_blocks_kernel<<<min(nblk, uint32_t(num_cus)), 64, lds, st>>>(in, blk, nblk, bmax, slots, sizes);
  return hipGetLastError();
}

hipError_t launch_xxh32(hipStream_t st, const uint8_t* p, uint32_t n, uint32_t* out) {
  lz4_payload_xxh32_kernel<<<1, 64, 0, st>>>(p, n, out);
  return hipGetLastError();
}

// --------------------------------------------------------------- launchers
hipError_t decode_kernels_available() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&decode_fast_kernel<0>));
}

size_t decode_scratch_bytes(uint32_t n) {
  size_t tiles = (size_t(n) + 1 + kScanTile - 1) / kScanTile;
  return align16(2 * tiles * sizeof(uint64_t)) + 16 + align16(size_t(n) * sizeof(uint32_t)) + 16 +
         // CodecZstd fast path: count, list, records, sequences
         16 + 3 * align16(size_t(n) * sizeof(uint32_t)) + size_t(n) * sizeof(ZsFastRec) +
         size_t(n) * kZfSeqSlot * sizeof(uint32_t) +
         // its Huffman-literal slots (H1 -> H2): tables and stream records
         size_t(zf_huf_cap(n)) * (kZhTab + 64);
}

// The scratch one codec's plan + decode touch (carve's layout, cut after the last region the
// codec uses): CodecNone / Snappy need the scan tiles, the large-block list, the round counter and
// the list count (~8 B per block instead of ~560); LZ4, Zlib and Zstd keep every region (their fast
// paths' lists, records and sequence slots).
size_t decode_scratch_bytes_codec(uint32_t n, int codec) {
  if (codec != SLATE_CODEC_NONE && codec != SLATE_CODEC_SNAPPY) return decode_scratch_bytes(n);
  const size_t tiles = (size_t(n) + 1 + kScanTile - 1) / kScanTile;
  // scan tiles, large count, large list, round counter, list count, list
  return align16(2 * tiles * sizeof(uint64_t)) + 16 + align16(size_t(n) * sizeof(uint32_t)) + 16 + 16 +
         align16(size_t(n) * sizeof(uint32_t));
}

static DecodeScratch carve(void* scratch, uint32_t n) {
  DecodeScratch s;
  size_t tiles = (size_t(n) + 1 + kScanTile - 1) / kScanTile;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  s.pa = reinterpret_cast<uint64_t*>(p);
  s.pb = s.pa + tiles;
  p += align16(2 * tiles * sizeof(uint64_t));
  s.large_count = reinterpret_cast<uint32_t*>(p);
  p += 16;
  s.large_list = reinterpret_cast<uint32_t*>(p);
  p += align16(size_t(n) * sizeof(uint32_t));
  s.round_counter = reinterpret_cast<uint32_t*>(p);
  p += 16;
  s.zf.count = reinterpret_cast<uint32_t*>(p);
  p += 16;
  s.zf.list = reinterpret_cast<uint32_t*>(p);
  p += align16(size_t(n) * sizeof(uint32_t));
  s.zf.hlist = reinterpret_cast<uint32_t*>(p);
  p += align16(size_t(n) * sizeof(uint32_t));
  s.zf.flist = reinterpret_cast<uint32_t*>(p);
  p += align16(size_t(n) * sizeof(uint32_t));
  s.zf.rec = reinterpret_cast<ZsFastRec*>(p);
  p += size_t(n) * sizeof(ZsFastRec);
  s.zf.seq = reinterpret_cast<uint32_t*>(p);
  p += size_t(n) * kZfSeqSlot * sizeof(uint32_t);
  s.zf.hcap = zf_huf_cap(n);
  s.zf.htab = p;
  p += size_t(s.zf.hcap) * kZhTab;
  s.zf.hdesc = reinterpret_cast<uint32_t*>(p);
  p += size_t(s.zf.hcap) * 64;
  s.tiles = uint32_t(tiles);
  return s;
}

size_t zl_stage_bytes(uint32_t n) {
  return align16(size_t(n) * sizeof(ZsFastRec)) + size_t(n) * kZfSeqSlot * sizeof(uint32_t) +
         align16(size_t(n) * sizeof(uint32_t)) + 16 + size_t(n) * kZlStageStride;
}

ZlStage zl_stage_carve(void* base, uint32_t n) {
  ZlStage g;
  uint8_t* p = static_cast<uint8_t*>(base);
  g.rec = reinterpret_cast<ZsFastRec*>(p);
  p += align16(size_t(n) * sizeof(ZsFastRec));
  g.seq = reinterpret_cast<uint32_t*>(p);
  p += size_t(n) * kZfSeqSlot * sizeof(uint32_t);
  g.list = reinterpret_cast<uint32_t*>(p);
  p += align16(size_t(n) * sizeof(uint32_t));
  g.count = reinterpret_cast<uint32_t*>(p);
  p += 16;
  g.lit = p;
  return g;
}

hipError_t launch_decode_plan(hipStream_t st, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                              uint64_t* out_off, uint64_t* row_base, void* scratch, const ZlStage* stage,
                              int num_cus) {
  DecodeScratch s = carve(scratch, n);
  uint32_t m = n + 1;
  if (codec == SLATE_CODEC_LZ4 && n >= 64) {
    // one-block frames lane per block; the rest by the serial structure walk over a list (small
    // batches, e.g. one index or filter payload, take the serial walk directly)
    (void)hipMemsetAsync(s.zf.count, 0, sizeof(uint32_t), st);
    hipError_t e = launch_lz4_plan(st, in, in_off, n, out_off, row_base, s.zf.list, s.zf.count);
    if (e != hipSuccess) return e;
    if (n > 0) plan_list_kernel<<<min((n + 255) / 256, 1024u), 256, 0, st>>>(codec, in, in_off, s.zf.list, s.zf.count,
                                                                            out_off, row_base);
  } else if (codec == SLATE_CODEC_NONE || codec == SLATE_CODEC_SNAPPY) {
    // sizes + tile sums, then the apply pass with its own prefix of the tile sums: two launches
    plan_reduce_kernel<<<s.tiles, kScanThreads, 0, st>>>(codec, in, in_off, n, out_off, row_base, s.pa, s.pb);
    scan_apply_sum_kernel<<<s.tiles, kScanThreads, 0, st>>>(out_off, row_base, m, s.pa, s.pb);
    return hipGetLastError();
  } else {
    plan_sizes_kernel<<<(m + 255) / 256, 256, 0, st>>>(codec, in, in_off, n, out_off, row_base);
  }
  if (codec == SLATE_CODEC_ZLIB && n >= 64) {
    // block-sized streams lane per block (zlib_fast.hip; staged: parsed once, for the decode too);
    // the rest: the wave plan
    uint32_t* list = stage ? stage->list : s.zf.list;
    uint32_t* count = stage ? stage->count : s.zf.count;
    (void)hipMemsetAsync(count, 0, stage ? 3 * sizeof(uint32_t) : sizeof(uint32_t), st);
    hipError_t e = launch_zlib_plan_fast(st, in, in_off, n, out_off, row_base, list, count, num_cus, stage);
    if (e != hipSuccess) return e;
    plan_zlib_kernel<<<min((n + 3) / 4, 4096u), 256, 0, st>>>(in, in_off, n, out_off, row_base, list, count);
  } else if (codec == SLATE_CODEC_ZLIB && n > 0) {
    plan_zlib_kernel<<<min((n + 3) / 4, 4096u), 256, 0, st>>>(in, in_off, n, out_off, row_base, nullptr, nullptr);
  }
  if (codec == SLATE_CODEC_ZSTD && n > 0) {
    // single-frame blocks with a content size: lane per block; the rest: the wave plan
    (void)hipMemsetAsync(s.zf.count, 0, sizeof(uint32_t), st);
    hipError_t e = launch_zstd_plan_fast(st, in, in_off, n, out_off, row_base, s.zf.list, s.zf.count);
    if (e != hipSuccess) return e;
    plan_zstd_kernel<<<min((n + 3) / 4, 4096u), 256, 0, st>>>(in, in_off, n, out_off, row_base, s.zf.list, s.zf.count);
  }
  scan_reduce_kernel<<<s.tiles, kScanThreads, 0, st>>>(out_off, row_base, m, s.pa, s.pb);
  scan_apply_sum_kernel<<<s.tiles, kScanThreads, 0, st>>>(out_off, row_base, m, s.pa, s.pb);
  return hipGetLastError();
}

size_t scan_scratch_bytes(uint32_t m) { return 2 * size_t((m + kScanTile - 1) / kScanTile + 1) * sizeof(uint64_t); }

hipError_t launch_scan_u64(hipStream_t st, uint64_t* a, uint32_t m, void* scratch) {
  uint32_t tiles = (m + kScanTile - 1) / kScanTile;
  uint64_t* pa = static_cast<uint64_t*>(scratch);
  uint64_t* pb = pa + tiles + 1;
  scan_reduce_kernel<<<tiles, kScanThreads, 0, st>>>(a, nullptr, m, pa, pb);
  scan_apply_sum_kernel<<<tiles, kScanThreads, 0, st>>>(a, nullptr, m, pa, pb);
  return hipGetLastError();
}

// ------------------------------------------------------------- dense rows (host transfers)
__global__ void rows_count_kernel(const slate_block_meta* __restrict__ meta, const uint64_t* __restrict__ row_base,
                                  uint32_t n, uint64_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    cnt[n] = 0;
    return;
  }
  const uint64_t cap = row_base[i + 1] - row_base[i];
  cnt[i] = meta[i].status == SLATE_OK ? min(uint64_t(meta[i].n_rows), cap) : 0;
}

// one wave per block: its rows as 16-byte stores, consecutive lanes consecutive rows
__global__ __launch_bounds__(256) void rows_pack_kernel(const uint64_t* __restrict__ row_base, uint32_t n,
                                                        const slate_row* __restrict__ rows,
                                                        const uint64_t* __restrict__ dense_off,
                                                        slate_row* __restrict__ dense) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
    const uint64_t d0 = dense_off[i], c = dense_off[i + 1] - d0, r0 = row_base[i];
    for (uint64_t r = lane; r < c; r += 64)
      reinterpret_cast<uint4*>(dense)[d0 + r] = reinterpret_cast<const uint4*>(rows)[r0 + r];
  }
}

size_t rows_pack_scratch_bytes(uint32_t n) { return scan_scratch_bytes(n + 1) + 64; }

// One wave per block: the block's decoded bytes and rows written straight into the caller's
// page-locked buffers through their device addresses (host decode with pinned outputs: no
// staging, no host copy).  Block i lands at g_out[i] / g_row[i] when given (sharded batch), else
// at out_base + out_off[i] / row_base0 + row_base[i].  Bytes go as 16-byte stores (16-aligned
// destinations: every plan offset is), the rows of a decoded block as 16-byte stores.
__global__ __launch_bounds__(256) void blocks_to_host_kernel(const uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             const uint64_t* __restrict__ row_base,
                                                             const slate_block_meta* __restrict__ meta,
                                                             const slate_row* __restrict__ rows, uint32_t n,
                                                             uint8_t* dst_out, slate_row* dst_rows,
                                                             const uint64_t* __restrict__ g_out,
                                                             const uint64_t* __restrict__ g_row, uint64_t out_base,
                                                             uint64_t row_base0) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
    const uint64_t o0 = out_off[i], ob = out_off[i + 1] - o0;
    const uint64_t od = g_out ? g_out[i] : out_base + o0;
    for (uint64_t k = lane; k < ob / 16; k += 64)
      reinterpret_cast<uint4*>(dst_out + od)[k] = reinterpret_cast<const uint4*>(out + o0)[k];
    const slate_block_meta m = meta[i];
    const uint64_t r0 = row_base[i], cap = row_base[i + 1] - r0;
    const uint64_t c = m.status == SLATE_OK ? min(uint64_t(m.n_rows), cap) : 0;
    const uint64_t rd = g_row ? g_row[i] : row_base0 + r0;
    for (uint64_t r = lane; r < c; r += 64)
      reinterpret_cast<uint4*>(dst_rows)[rd + r] = reinterpret_cast<const uint4*>(rows)[r0 + r];
  }
}

// One block at the lowest latency (slate_block_decode, CodecNone / CodecSnappy): one launch, one
// wave.  The plan (decoded length -> output and row capacity) is the host's (the same
// decoded_len rules), so the offsets arrive as kernel arguments and sit in LDS; the encoded block
// is read once from the caller's page-locked staging through its device address into HBM
// (a.in), decoded by the large-kernel wave with its LDS budget (the host checks the block fits),
// and the decoded bytes go to page-locked host memory (host_out) the same way.  a.meta may be
// host memory too.  Replaces the generic path's plan kernel, scans, transfers and two waits.
__device__ __forceinline__ void decode_one(DecodeArgs a, const uint8_t* __restrict__ host_in, uint64_t in_len,
                                           uint64_t out_sz, uint64_t row_sz, uint8_t* __restrict__ host_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint64_t offs[6];
  const int lane = threadIdx.x;
  if (lane < 6) offs[lane] = lane == 1 ? in_len : lane == 3 ? out_sz : lane == 5 ? row_sz : 0;
  uint8_t* din = const_cast<uint8_t*>(a.in);
  // four 16-byte chunks per lane in flight per round trip over the link (loads first, clamped
  // indices: no predicated register arrays)
  const uint32_t nch = uint32_t((in_len + 15) / 16);
  for (uint32_t k0 = 0; k0 < nch; k0 += 256) {
    uint4 v[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++)
      v[u] = reinterpret_cast<const uint4*>(host_in)[min(k0 + 64 * u + uint32_t(lane), nch - 1)];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++)
      if (k0 + 64 * u + uint32_t(lane) < nch) reinterpret_cast<uint4*>(din)[k0 + 64 * u + lane] = v[u];
  }
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the staged block, before the wave reads it
  __syncthreads();
  a.in_off = offs;
  a.out_off = offs + 2;
  a.row_base = offs + 4;
  WaveBufs w{tab, smem + kTabBytes, smem + kTabBytes + kLargeInCap, kLargeInCap, kLargeOutCap};
  decode_block_wave<0>(a, 0, w, lane, false);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the decoded bytes, before the copy out
  __syncthreads();
  for (uint64_t k = lane; k < out_sz / 16; k += 64)
    reinterpret_cast<uint4*>(host_out)[k] = reinterpret_cast<const uint4*>(a.out)[k];
}
__global__ __launch_bounds__(64) void decode_one_kernel(DecodeArgs a, const uint8_t* __restrict__ host_in,
                                                        uint64_t in_len, uint64_t out_sz, uint64_t row_sz,
                                                        uint8_t* __restrict__ host_out) {
  decode_one(a, host_in, in_len, out_sz, row_sz, host_out);
}

// One CodecSnappy block for a single-block call (slate_block_decode: sstable.Iterator's one block per
// nextBlockIter, a point read), by a whole 1024-thread workgroup instead of one wave walking the
// ~170-tag chain serially (~70 us).  golang/snappy decode (decode_other.go:19-110) in parallel
// passes over the block staged in LDS:
//   1. every payload position p: the tag that would start there -- the next tag's position
//      (END at the payload end, ERR for a tag running past it) and its decoded length;
//   2. pointer doubling to 4- and 16-tag hops, one thread walks the 16-tag hops from the header
//      (~11 steps), their 4-tag sub-hops are found in parallel, and those are expanded in parallel:
//      the chain's tags with their output offsets;
//   3. every output byte finds its tag (binary search): a literal byte takes its value, a copied
//      byte points at the byte it repeats; pointer jumping until every byte holds a value;
// with the CRC32 on wave 0 beside pass 1.  Any check the serial decoder would fail (a tag past the
// payload, offset 0 or beyond the output, a length beyond the header's) sends the block to that
// decoder (wave 0), which then reports it; block.Decode's checks and rows are wave 0's block_finish.
constexpr uint32_t kOneParIn = 6144, kOneParOut = 12288, kOneParThreads = 1024;
constexpr uint32_t kOneParTags = kOneParIn / 2;
constexpr uint16_t kPEnd = 0xFFFE, kPErr = 0xFFFF;
constexpr size_t kOneParLds = kTabBytes + (kOneParIn + 32) + (kOneParOut + 16) + 8 * 2 * (kOneParIn + 16) +
                              4 * kOneParTags + 4 * (kOneParTags / 4 + 16) + 4 * (kOneParTags / 16 + 16) + 64;
static_assert(kOneParLds <= 160 * 1024, "decode_one_par_kernel's LDS");

__device__ __forceinline__ void snappy_tag_at(const uint8_t* in, uint32_t p, uint32_t clen, uint32_t* np, uint32_t* dl,
                                              uint32_t* hl, uint32_t* off, bool* lit) {
  const uint32_t c = in[p], t = c & 3;
  uint32_t len, h, o = 0;
  if (t == 0) {
    const uint32_t x = c >> 2;
    if (x < 60) {
      len = x + 1;
      h = 1;
    } else {
      const uint32_t nb = x - 59;
      uint32_t v = 0;
      for (uint32_t k = 0; k < nb; k++) v |= uint32_t(p + 1 + k < clen ? in[p + 1 + k] : 0u) << (8 * k);
      len = v + 1;  // (v + 1 == 0: wraps, fails below)
      h = 1 + nb;
    }
  } else if (t == 1) {
    len = 4 + ((c >> 2) & 7);
    o = ((c >> 5) << 8) | (p + 1 < clen ? in[p + 1] : 0u);
    h = 2;
  } else {
    len = 1 + (c >> 2);
    h = t == 2 ? 3 : 5;
    for (uint32_t k = 0; k < h - 1; k++) o |= uint32_t(p + 1 + k < clen ? in[p + 1 + k] : 0u) << (8 * k);
  }
  const uint64_t e = uint64_t(p) + h + (t == 0 ? uint64_t(len) : 0);
  *np = (len == 0 || e > clen) ? kPErr : uint32_t(e);
  *dl = len;
  *hl = h;
  *off = o;
  *lit = t == 0;
}

__device__ __forceinline__ void decode_one_par(DecodeArgs a, const uint8_t* __restrict__ host_in, uint64_t in_len,
                                               uint64_t out_sz, uint64_t row_sz, uint8_t* __restrict__ host_out,
                                               uint32_t stop) {
  // stop (profiling builds, SLATE_ONE_STOP): end after phase 1 staging, 2 pass 1, 3 the hop walk,
  // 4 the expansion, 5 pass 3, 6 before block_finish and the copy-out (the time per phase)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint64_t offs[6];
  __shared__ uint32_t sh_crc, sh_bad, sh_ntags, sh_nhops;
  const uint32_t tid = threadIdx.x;
  const int lane = int(tid & 63), wave = int(tid >> 6);
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  uint8_t* in = smem + kTabBytes;
  uint8_t* out = in + kOneParIn + 32;
  uint16_t* nxt = reinterpret_cast<uint16_t*>(out + kOneParOut + 16);
  uint16_t* dln = nxt + (kOneParIn + 16);
  uint16_t* j2 = dln + (kOneParIn + 16);
  uint16_t* s2 = j2 + (kOneParIn + 16);
  uint16_t* j4 = s2 + (kOneParIn + 16);
  uint16_t* s4 = j4 + (kOneParIn + 16);
  uint16_t* j16 = s4 + (kOneParIn + 16);
  uint16_t* s16 = j16 + (kOneParIn + 16);
  uint16_t* j8 = j2;  // (8-tag hops: j2 / s2 are not needed once j4 / s4 exist)
  uint16_t* s8 = s2;
  uint16_t* P = j2;  // the output bytes' pointers reuse j2 / s2 (2 * kOneParOut <= 4 * (kOneParIn + 16))
  uint32_t* T = reinterpret_cast<uint32_t*>(s16 + (kOneParIn + 16));  // tags: position | output offset << 16
  uint32_t* H = T + kOneParTags;                                      // 4-tag hops: position | offset << 16
  uint32_t* H16 = H + (kOneParTags / 4 + 16);                         // 16-tag hops
  if (tid < 6) offs[tid] = tid == 1 ? in_len : tid == 3 ? out_sz : tid == 5 ? row_sz : 0;
  if (tid == 0) {
    sh_bad = 0;
    sh_ntags = 0;
    sh_nhops = 0;
  }
  // ---- stage the block and the CRC tables
  const uint32_t nch = uint32_t((in_len + 15) / 16);
  for (uint32_t c = tid; c < nch; c += kOneParThreads)
    reinterpret_cast<uint4*>(in)[c] = reinterpret_cast<const uint4*>(host_in)[c];
  for (uint32_t i = tid; i < 1024; i += kOneParThreads) tab[i] = g_crc_tables.t[0][i];
  __syncthreads();
  if (stop == 1) return;
  const uint32_t clen = uint32_t(in_len - 4);
  uint64_t dl64 = 0;
  uint32_t hdr = 0;
  const bool hdr_ok = decoded_len(SLATE_CODEC_SNAPPY, in, in_len, &dl64, &hdr);
  const uint32_t dn = uint32_t(dl64);
  // ---- pass 1: the tag at every position (wave 0: the CRC32 first)
  if (wave == 0) {
    const uint32_t crc = wave_crc32(tab, in, 0, clen, lane);
    if (lane == 0) sh_crc = crc;
  }
  for (uint32_t p = hdr + tid; p < clen; p += kOneParThreads) {
    uint32_t np, dl, hl, off;
    bool lit;
    snappy_tag_at(in, p, clen, &np, &dl, &hl, &off, &lit);
    nxt[p] = uint16_t(np == clen ? kPEnd : np);
    dln[p] = uint16_t(min(dl, 0xFFFFu));
  }
  __syncthreads();
  if (stop == 2) return;
  const uint32_t stored = ld_be32(in + clen);
  auto fin = [&](slate_block_meta m, bool decoded) {
    // wave 0: block.Decode's checks and rows over the decoded block (or the status), then the copy-out
    if (wave == 0) {
      a.in_off = offs;
      a.out_off = offs + 2;
      a.row_base = offs + 4;
      if (decoded) block_finish(a, 0, out, dn, lane, m);
      else write_meta(&a.meta[0], m, lane);
    }
    __syncthreads();
    if (decoded)
      for (uint32_t k = tid; k < (dn + 15) / 16; k += kOneParThreads)
        reinterpret_cast<uint4*>(host_out)[k] = reinterpret_cast<const uint4*>(out)[k];
  };
  if (sh_crc != stored) {
    slate_block_meta m{};
    m.status = SLATE_E_BLOCK_CHECKSUM;
    fin(m, false);
    return;
  }
  bool bad = !hdr_ok || hdr > clen;
  if (!bad) {
    // ---- pass 2: 2- and 4-tag hops (END stays END, ERR propagates)
    auto hop = [&](const uint16_t* J, const uint16_t* S, uint16_t* J2, uint16_t* S2) {
      for (uint32_t p = hdr + tid; p < clen; p += kOneParThreads) {
        const uint32_t q = J[p];
        if (q >= kPEnd) {
          J2[p] = uint16_t(q);
          S2[p] = S[p];
        } else {
          J2[p] = J[q];
          S2[p] = uint16_t(min(uint32_t(S[p]) + S[q], 0xFFFFu));
        }
      }
    };
    hop(nxt, dln, j2, s2);
    __syncthreads();
    hop(j2, s2, j4, s4);
    __syncthreads();
    hop(j4, s4, j8, s8);
    __syncthreads();
    hop(j8, s8, j16, s16);
    __syncthreads();
    // one thread walks the chain in 16-tag hops from the header
    if (tid == 0) {
      uint32_t p = hdr, o = 0, k = 0, b = 0;
      while (p < clen) {
        if (k >= kOneParTags / 16 + 16 || o > dn) {
          b = 1;
          break;
        }
        H16[k++] = p | (o << 16);
        o += s16[p];
        const uint32_t q = j16[p];
        p = q == kPEnd ? clen : q;
        if (q == kPErr) {
          b = 1;
          break;
        }
      }
      if (o != dn) b = 1;  // the tags' bytes are exactly the header's length
      sh_nhops = k;
      sh_bad = b;
    }
    __syncthreads();
    // each 16-tag hop's four 4-tag sub-hops (all four but in the last: the chain goes on)
    const uint32_t n16 = sh_bad ? 0u : sh_nhops;
    for (uint32_t k = tid; k < n16; k += kOneParThreads) {
      uint32_t p = H16[k] & 0xFFFF, o = H16[k] >> 16, i = 0;
      for (; i < 4 && p < clen; i++) {
        H[4 * k + i] = p | (o << 16);
        o += s4[p];
        const uint32_t q = j4[p];
        p = q >= kPEnd ? clen : q;  // (no ERR: the 16-tag hop holds none)
      }
      if (k == n16 - 1) sh_ntags = 4 * k + i;  // (sh_ntags: the number of 4-tag hops, until below)
    }
    __syncthreads();
    if (stop == 3) return;
    bad = sh_bad != 0;
  }
  if (!bad) {
    const uint32_t nh = sh_ntags;
    __syncthreads();  // (every thread has read the hop count before sh_ntags becomes the tag count)
    // hops expanded: the chain's tags with their output offsets, checked as decode_other.go does
    uint32_t b = 0;
    for (uint32_t t = tid; t < nh; t += kOneParThreads) {
      uint32_t p = H[t] & 0xFFFF, o = H[t] >> 16, i = 0;
      for (; i < 4 && p < clen; i++) {
        T[4 * t + i] = p | (o << 16);
        uint32_t np, dl, hl, off;
        bool lit;
        snappy_tag_at(in, p, clen, &np, &dl, &hl, &off, &lit);
        if (!lit && (off == 0 || off > o)) b = 1;
        o += dl;
        const uint32_t q = nxt[p];
        p = q == kPEnd ? clen : q;
      }
      if (t == nh - 1) sh_ntags = 4 * t + i;
    }
    if (b) sh_bad = 1;
    __syncthreads();
    if (stop == 4) return;
    bad = sh_bad != 0;
  }
  if (!bad) {
    // ---- pass 3: every output byte from its tag; copies as pointers, then pointer jumping
    const uint32_t nt = sh_ntags;
    for (uint32_t x = tid; x < dn; x += kOneParThreads) {
      uint32_t lo = 0, hi = nt;  // the last tag with offset <= x
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((T[mid] >> 16) <= x) lo = mid;
        else hi = mid;
      }
      const uint32_t p = T[lo] & 0xFFFF, o = T[lo] >> 16;
      uint32_t np, dl, hl, off;
      bool lit;
      snappy_tag_at(in, p, clen, &np, &dl, &hl, &off, &lit);
      P[x] = lit ? uint16_t(0x8000u | in[p + hl + (x - o)]) : uint16_t(x - off);
    }
    __syncthreads();
    // The round's verdict is the barrier's own OR (one barrier per round, no shared flag that
    // thread 0 could reset while a late wave still reads the previous round's value).
    bool resolved = false;
    for (uint32_t round = 0; round < 16; round++) {
      uint32_t more = 0;
      for (uint32_t x = tid; x < dn; x += kOneParThreads) {
        const uint32_t v = P[x];
        if (!(v & 0x8000u)) {
          const uint32_t w = P[v];
          P[x] = uint16_t(w);
          more |= (w & 0x8000u) ? 0u : 1u;
        }
      }
      if (!__syncthreads_or(int(more))) {
        resolved = true;
        break;
      }
    }
    if (stop == 5) return;
    if (resolved) {  // (every byte resolved: 16 rounds cover any chain in kOneParOut bytes)
      for (uint32_t x = tid; x < dn; x += kOneParThreads) out[x] = uint8_t(P[x]);
      __syncthreads();
      if (stop == 6) return;
      fin(slate_block_meta{}, true);
      return;
    }
  }
  // ---- anything the passes refused: the serial decoder reports it (or decodes it)
  slate_block_meta m{};
  int st = SLATE_E_SNAPPY_CORRUPT;
  __syncthreads();  // every wave has read sh_bad (pass 2) before lane 0 of wave 0 rewrites it
  if (wave == 0 && hdr_ok) st = wave_snappy_decode(in, clen, hdr, out, dn, lane);
  if (wave == 0 && lane == 0) sh_bad = uint32_t(st);
  __syncthreads();
  st = int(sh_bad);
  m.status = int16_t(st);
  fin(m, st == SLATE_OK);
}
__global__ __launch_bounds__(kOneParThreads) void decode_one_par_kernel(DecodeArgs a, const uint8_t* __restrict__ host_in,
                                                                        uint64_t in_len, uint64_t out_sz, uint64_t row_sz,
                                                                        uint8_t* __restrict__ host_out, uint32_t stop) {
  decode_one_par(a, host_in, in_len, out_sz, row_sz, host_out, stop);
}

// Small batches (the read-ahead block reader's read_ahead blocks): one workgroup per block, so a
// batch of 64 blocks takes one block's latency instead of the lane-per-block kernel's one round
// (~0.3 ms for 64 blocks on one wave).  Descriptor k (host-mapped, one read per workgroup) names
// block b's staged input (16-byte aligned), its decoded bytes' place and its row slots; meta and rows
// are written through host-mapped pointers, the decoded bytes too.  Blocks [0, n_par) take the
// workgroup-parallel Snappy decoder, [n_par, n) the one-wave decoder (CodecNone, larger blocks),
// each in its own launch (their LDS budgets differ).
__global__ __launch_bounds__(kOneParThreads) void decode_small_par_kernel(DecodeArgs a, const SmallDesc* __restrict__ d,
                                                                          const uint8_t* hin, uint8_t* hout) {
  const SmallDesc x = d[blockIdx.x];
  DecodeArgs ab = a;
  ab.n = 1;
  ab.meta = a.meta + x.block;
  ab.rows = a.rows + x.row_base;
  decode_one_par(ab, hin + x.in_off, x.in_len, x.out_sz, x.row_sz, hout + x.out_off, 0);
}
__global__ __launch_bounds__(64) void decode_small_wave_kernel(DecodeArgs a, const SmallDesc* __restrict__ d,
                                                               const uint8_t* hin, uint8_t* hout, uint8_t* dscr) {
  const SmallDesc x = d[blockIdx.x];
  DecodeArgs ab = a;
  ab.n = 1;
  ab.meta = a.meta + x.block;
  ab.rows = a.rows + x.row_base;
  // device staging for the wave decoder: the block's input at its staging offset, its decoded bytes
  // at dev_out (after every input)
  ab.in = dscr + x.in_off;
  ab.out = dscr + x.dev_out;
  decode_one(ab, hin + x.in_off, x.in_len, x.out_sz, x.row_sz, hout + x.out_off);
}

hipError_t launch_decode_small(hipStream_t st, const DecodeArgs& args_in, const SmallDesc* descs, uint32_t n_par,
                               uint32_t n, const uint8_t* hin, uint8_t* hout, uint8_t* dscr) {
  DecodeArgs a = args_in;
  a.debug = 0;
  a.raw = 0;
  a.rt_zero = 0;
  if (n_par) {
    static const hipError_t attr_p = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_small_par_kernel),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(kOneParLds));
    if (attr_p != hipSuccess) return attr_p;
    decode_small_par_kernel<<<n_par, kOneParThreads, kOneParLds, st>>>(a, descs, hin, hout);
  }
  if (n > n_par) {
    constexpr size_t lds = kTabBytes + kLargeInCap + kLargeOutCap;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_small_wave_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (attr != hipSuccess) return attr;
    decode_small_wave_kernel<<<n - n_par, 64, lds, st>>>(a, descs + n_par, hin, hout, dscr);
  }
  return hipGetLastError();
}

bool small_par_fits(int codec, uint64_t in_len, uint64_t out_sz) {
  return codec == SLATE_CODEC_SNAPPY && in_len >= 6 && in_len + 16 <= kOneParIn && out_sz <= kOneParOut;
}
bool small_wave_fits(uint64_t in_len, uint64_t out_sz) { return in_len + 15 <= kLargeInCap && out_sz <= kLargeOutCap; }

hipError_t launch_decode_one(hipStream_t st, const DecodeArgs& args_in, const uint8_t* host_in, uint64_t in_len,
                             uint64_t out_sz, uint64_t row_sz, uint8_t* host_out) {
  DecodeArgs a = args_in;
  a.n = 1;
  a.debug = 0;
  a.raw = 0;
  a.rt_zero = 0;
  if ((a.codec != SLATE_CODEC_NONE && a.codec != SLATE_CODEC_SNAPPY) || in_len + 15 > kLargeInCap ||
      out_sz > kLargeOutCap)
    return hipErrorInvalidValue;
  static const bool par_off = getenv("SLATE_ONE_SERIAL") != nullptr;  // A/B runs: the one-wave decoder
  if (a.codec == SLATE_CODEC_SNAPPY && !par_off && in_len >= 6 && in_len + 16 <= kOneParIn && out_sz <= kOneParOut &&
      (reinterpret_cast<uintptr_t>(host_in) & 15) == 0) {
    static const hipError_t attr_p = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_one_par_kernel),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(kOneParLds));
    if (attr_p != hipSuccess) return attr_p;
#ifdef SLATE_PROFILING_BUILD
    static const uint32_t stop = getenv("SLATE_ONE_STOP") ? uint32_t(atoi(getenv("SLATE_ONE_STOP"))) : 0u;
#else
    constexpr uint32_t stop = 0;
#endif
    decode_one_par_kernel<<<1, kOneParThreads, kOneParLds, st>>>(a, host_in, in_len, out_sz, row_sz, host_out, stop);
    return hipGetLastError();
  }
  constexpr size_t lds = kTabBytes + kLargeInCap + kLargeOutCap;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_one_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  decode_one_kernel<<<1, 64, lds, st>>>(a, host_in, in_len, out_sz, row_sz, host_out);
  return hipGetLastError();
}

hipError_t launch_blocks_to_host(hipStream_t st, const uint8_t* out, const uint64_t* out_off, const uint64_t* row_base,
                                 const slate_block_meta* meta, const slate_row* rows, uint32_t n, uint8_t* dst_out,
                                 slate_row* dst_rows, const uint64_t* g_out, const uint64_t* g_row, uint64_t out_base,
                                 uint64_t row_base0) {
  if (n == 0) return hipSuccess;
  blocks_to_host_kernel<<<min((n + 3) / 4, 8192u), 256, 0, st>>>(out, out_off, row_base, meta, rows, n, dst_out,
                                                                 dst_rows, g_out, g_row, out_base, row_base0);
  return hipGetLastError();
}

hipError_t launch_rows_pack(hipStream_t st, const slate_block_meta* meta, const uint64_t* row_base, uint32_t n,
                            const slate_row* rows, uint64_t* dense_off, void* scratch, slate_row* dense) {
  if (n == 0) return hipSuccess;
  rows_count_kernel<<<(n + 256) / 256, 256, 0, st>>>(meta, row_base, n, dense_off);
  hipError_t e = launch_scan_u64(st, dense_off, n + 1, scratch);
  if (e != hipSuccess) return e;
  rows_pack_kernel<<<min((n + 3) / 4, 8192u), 256, 0, st>>>(row_base, n, rows, dense_off, dense);
  return hipGetLastError();
}

hipError_t launch_decode_payload(hipStream_t st, const DecodeArgs& args_in, int num_cus) {
  DecodeArgs a = args_in;
  a.debug = 0;
  a.raw = 1;
  if (a.n == 0) return hipGetLastError();
  const uint32_t grid = min(a.n, uint32_t(num_cus) * 4u);
  if (a.codec == SLATE_CODEC_ZLIB) {
    decode_payload_kernel<1><<<grid, 64, kTabBytes + kZFixed + kZScratch, st>>>(a);
  } else if (a.codec == SLATE_CODEC_ZSTD) {
    decode_payload_kernel<2><<<grid, 64, kTabBytes + kZsShared + kZsScratch, st>>>(a);
  } else {
    decode_payload_kernel<0><<<grid, 64, kTabBytes, st>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_decode(hipStream_t st, const DecodeArgs& args_in, void* scratch, int num_cus, const ZlStage* stage) {
  DecodeArgs a = args_in;
#ifdef SLATE_PROFILING_BUILD
  const char* dbg = getenv("SLATE_DEBUG_MODE");  // profiling variants only (tools/variant.sh)
  a.debug = dbg ? uint32_t(strtoul(dbg, nullptr, 0)) : 0u;
#else
  a.debug = 0;
#endif
  a.rt_zero = 0;
  DecodeScratch s = carve(scratch, a.n);
  a.large_list = s.large_list;
  a.large_count = s.large_count;
  a.round_counter = s.round_counter;
  (void)hipMemsetAsync(s.large_count, 0, sizeof(uint32_t), st);
  (void)hipMemsetAsync(s.round_counter, 0, sizeof(uint32_t), st);
  if (a.n == 0) return hipGetLastError();
  // Snappy: the lane-per-block streaming decoder (any block size); ablation bit 16 (profiling
  // variants only) selects the wave-per-block path instead
  if (a.codec == SLATE_CODEC_SNAPPY && !(dbg_bits(a) & 16)) return launch_decode_lpb2(st, a, num_cus);
  const size_t lds = a.codec == SLATE_CODEC_ZSTD
                         ? kTabBytes + (kDecodeThreads / 64) * size_t(kZsFastInCap + kZsFastOutCap + kZsScratch) + kZsShared
                         : kTabBytes + (kDecodeThreads / 64) * size_t(kFastInCap + kFastOutCap) +
                               (a.codec == SLATE_CODEC_ZLIB ? kZFixed + (kDecodeThreads / 64) * size_t(kZScratch) : 0);
  uint32_t wgs_needed = (a.n + kDecodeThreads / 64 - 1) / (kDecodeThreads / 64);
  uint32_t grid = min(wgs_needed, uint32_t(num_cus) * kDecodeWgPerCu);
  const size_t lds_large = kTabBytes + size_t(kLargeInCap) + kLargeOutCap;
  if (a.codec == SLATE_CODEC_ZLIB && !a.raw && !(dbg_bits(a) & 16)) {
    // the fast path (zlib_fast.hip phase Z + zstd_fast.hip phases A2 and B), then the exact path
    // over the blocks it handed back.  After a staged plan, phase Z's output is the plan's: records,
    // sequences, literals and hand-back list from the stage
    if (stage) {
      s.zf.rec = stage->rec;
      s.zf.seq = stage->seq;
      s.zf.list = stage->list;
      s.zf.count = stage->count;
      s.zf.lit = stage->lit;
    } else {
      (void)hipMemsetAsync(s.zf.count, 0, 3 * sizeof(uint32_t), st);
    }
    hipError_t e = launch_zlib_fast(st, a, s.zf, num_cus, stage != nullptr);
    if (e != hipSuccess) return e;
    decode_list_kernel<1><<<grid, kDecodeThreads, lds, st>>>(a, s.zf.list, s.zf.count);
    decode_large_kernel<1><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
  } else if (a.codec == SLATE_CODEC_ZLIB) {
    decode_fast_kernel<1><<<grid, kDecodeThreads, lds, st>>>(a);
    decode_large_kernel<1><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
  } else if (a.codec == SLATE_CODEC_ZSTD) {
    // the fast path (zstd_fast.hip), then the exact path over the blocks it handed back
    (void)hipMemsetAsync(s.zf.count, 0, 4 * sizeof(uint32_t), st);
    hipError_t e = launch_zstd_fast(st, a, s.zf, num_cus);
    if (e != hipSuccess) return e;
    decode_list_kernel<2><<<grid, kDecodeThreads, lds, st>>>(a, s.zf.list, s.zf.count);
    decode_large_kernel<2><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
#ifdef SLATE_PROFILING_BUILD
    if (getenv("SLATE_ZF_STATS")) {  // profiling variants only: how many blocks the fast path handed back
      uint32_t cnt = 0;
      std::vector<ZsFastRec> rec(a.n);
      (void)hipMemcpyAsync(&cnt, s.zf.count, 4, hipMemcpyDeviceToHost, st);
      (void)hipMemcpyAsync(rec.data(), s.zf.rec, a.n * sizeof(ZsFastRec), hipMemcpyDeviceToHost, st);
      (void)hipStreamSynchronize(st);
      std::vector<uint32_t> lst(cnt);
      (void)hipMemcpy(lst.data(), s.zf.list, cnt * 4, hipMemcpyDeviceToHost);
      uint32_t fast = 0, sum_fail = 0;
      for (const ZsFastRec& r : rec) fast += (r.info >> 16) & kZfFast;
      for (uint32_t b : lst) sum_fail += (rec[b].info >> 16) & kZfFast;
      FILE* f = fopen(getenv("SLATE_ZF_STATS"), "w");  // the value names the output file
      if (f) {
        fprintf(f, "%u %u %u %u\n", a.n, fast, cnt, sum_fail);
        for (uint32_t b : lst) fprintf(f, "%u %u\n", b, (rec[b].info >> 16) & kZfFast);
        fclose(f);
      }
    }
#endif
  } else if (a.codec == SLATE_CODEC_LZ4 && !a.raw && !(dbg_bits(a) & 16)) {
    // one-block frames lane per block (decode_lpb2.hip), then the exact path over the hand-backs
    (void)hipMemsetAsync(s.zf.count, 0, 3 * sizeof(uint32_t), st);
    hipError_t e = launch_lz4_fast(st, a, s.zf, num_cus);
    if (e != hipSuccess) return e;
    decode_list_kernel<0><<<grid, kDecodeThreads, lds, st>>>(a, s.zf.list, s.zf.count);
    decode_large_kernel<0><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
  } else if (a.codec == SLATE_CODEC_NONE && !a.raw && !(dbg_bits(a) & 16)) {
    // CodecNone blocks: the streaming wave-per-block decoder (decode_none.hip); blocks beyond its
    // size window take the exact wave path through large_list
    hipError_t e = launch_decode_none(st, a, num_cus);
    if (e != hipSuccess) return e;
    decode_large_kernel<0><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
  } else {
    decode_fast_kernel<0><<<grid, kDecodeThreads, lds, st>>>(a);
    decode_large_kernel<0><<<uint32_t(num_cus), 64, lds_large, st>>>(a);
  }
  return hipGetLastError();
}

}  // namespace slate

