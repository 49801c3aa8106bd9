// SST block encode on MI355X: the data-parallel part of sstable.Builder
// (internal/sstable/builder.go:160-213) + block.Builder (block/block.go:136-204)
// + block.Encode (block.go:54-75) for a batch of sorted KVs resident in HBM,
// plus the bloom filter build (bloom/bloom.go:107-172) and a large-buffer CRC32.
//
// Pipeline for one batch of n KVs (all launched on one stream):
//   enc_kv_kernel      per KV: FNV-1 64 hash (bloom.go:141), LCP with the previous
//                      key, sortedness flag
//   enc_next_kernel    per KV j: next[j] = first KV that does not fit in a block
//                      starting at j (greedy fill rule, block.go:171) + its size
//   enc_exit_kernel    per 4096-KV chunk: pointer jumping in LDS -> exit[j] =
//                      first position >= chunk end on j's block chain
//   enc_chain_kernel   one workgroup chains chunk entries e_{c+1} = exit[e_c]
//                      (windowed prefetch into LDS)
//   enc_mark_kernel    per chunk: walk the true block starts from its entry
//   enc_blocks_kernel  compact starts -> block list, encoded block sizes
//   enc_pack_kernel    one wavefront per block: rows packed in LDS (v0 row codec,
//                      row.go:149-189), BE16 offsets + count, CRC32, byte-exact
//                      write into the SST byte stream
//   bloom kernels      probes (enhanced double hashing) -> atomicOr bitset
//   crc kernels        CRC32 of a large device buffer (filter / index)
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "encode.h"
#include "wave_crc.h"
#include "lpb_common.h"
#include "snappy_enc.h"

namespace slate {

constexpr uint32_t kNone = 0xFFFFFFFFu;
#ifndef SLATE_PACK_STAGE  // CodecNone pack: stage the block's keys and values in LDS first (1) or not (0)
#define SLATE_PACK_STAGE 1
#endif
constexpr bool kPackStage = SLATE_PACK_STAGE != 0;
// golang/snappy searches: serial probes before each 64-probe batch (snappy_enc.h) for the filter /
// index chunks and for the data blocks
#ifndef SLATE_SNAP_CHUNK_SERIAL
#define SLATE_SNAP_CHUNK_SERIAL 8
#endif
#ifndef SLATE_SNAP_PACK_SERIAL
#define SLATE_SNAP_PACK_SERIAL 0
#endif
constexpr uint32_t kSnapChunkSerialProbes = SLATE_SNAP_CHUNK_SERIAL;  // serial probes before a batch (snappy_enc.h)

// ------------------------------------------------------------------ KV pass
__device__ inline uint64_t row_slot(const EncodeArgs& a, uint32_t i, uint32_t p16);

// A key of at most kKvShort bytes as 8 little-endian dwords (bytes past its length zero), read as the
// aligned dwords that hold it -- all loads in flight at once, then realigned by alignbyte -- instead
// of one dependent byte load per step (the byte loops kept the KV pass latency-bound).  A dword
// holding one of the key's bytes lies inside the key buffer's pages, so no load can fault.
constexpr uint32_t kKvShort = 32;
__device__ inline void key_words(const uint8_t* k, uint32_t kl, uint32_t (&r)[8]) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(k);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(addr & ~uintptr_t(3));
  const uint32_t sh = uint32_t(addr & 3);
  const uint32_t nw = (sh + kl + 3) >> 2;  // aligned dwords holding the key (<= 9)
  uint32_t w[9];
#pragma unroll
  for (uint32_t t = 0; t < 9; t++) w[t] = t < nw ? base[t] : 0u;
#pragma unroll
  for (uint32_t t = 0; t < 8; t++) {
    const int rem = int(kl) - int(4 * t);
    const uint32_t mask = rem >= 4 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
    r[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh) & mask;
  }
}

__device__ inline uint64_t fnv_words(const uint32_t (&r)[8], uint32_t kl) {
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1 64 (hash/fnv New64)
#pragma unroll
  for (uint32_t b = 0; b < 16; b++) {
    const uint64_t hn = (h * 0x100000001b3ull) ^ ((r[b >> 2] >> (8 * (b & 3))) & 0xFFu);
    h = b < kl ? hn : h;
  }
  if (kl > 16) {
#pragma unroll
    for (uint32_t b = 16; b < 32; b++) {
      const uint64_t hn = (h * 0x100000001b3ull) ^ ((r[b >> 2] >> (8 * (b & 3))) & 0xFFu);
      h = b < kl ? hn : h;
    }
  }
  return h;
}

// slot0[i] (optional) = row_slot(i, 0) saturated to u32: enc_next_kernel's row sizes, prefix-free
__global__ void enc_kv_kernel(EncodeArgs a, uint64_t* __restrict__ hashes, uint32_t* __restrict__ adj,
                              uint32_t* __restrict__ flags, uint32_t* __restrict__ slot0 = nullptr) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  if (slot0) slot0[i] = uint32_t(min(row_slot(a, i, 0), uint64_t(0xFFFFFFFFu)));
  const uint8_t* k = a.keys + a.key_off[i];
  uint64_t kl = a.key_off[i + 1] - a.key_off[i];
  const uint64_t pl = i > 0 ? a.key_off[i] - a.key_off[i - 1] : 0;
  if (kl <= kKvShort && pl <= kKvShort) {
    uint32_t r[8], q[8];
    key_words(k, uint32_t(kl), r);
    hashes[i] = fnv_words(r, uint32_t(kl));
    uint32_t l = 0;
    if (i > 0) {
      key_words(a.keys + a.key_off[i - 1], uint32_t(pl), q);
      const uint32_t m = uint32_t(min(pl, kl));
      uint32_t d = 32, qd = 0, rd = 0;  // first differing byte (bytes past both lengths are zero)
#pragma unroll
      for (uint32_t t = 0; t < 8; t++) {
        const uint32_t x = r[t] ^ q[t];
        const bool first = d == 32 && x != 0;
        d = first ? 4 * t + (__builtin_ctz(x) >> 3) : d;
        qd = first ? q[t] : qd;
        rd = first ? r[t] : rd;
      }
      const uint32_t o = min(d, m);
      l = o;
      const uint32_t s8 = 8 * (d & 3);
      const bool desc = (o < m) ? (((qd >> s8) & 0xFFu) > ((rd >> s8) & 0xFFu)) : (pl > kl);
      if (desc) atomicOr(flags, 1u);  // not sorted: the min-LCP shortcut does not hold
    }
    adj[i] = l;
    return;
  }
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1 64 (hash/fnv New64)
  for (uint64_t b = 0; b < kl; b++) {
    h *= 0x100000001b3ull;
    h ^= k[b];
  }
  hashes[i] = h;
  uint32_t l = 0;
  if (i > 0) {
    const uint8_t* p = a.keys + a.key_off[i - 1];
    uint64_t m = pl < kl ? pl : kl, o = 0;
    while (o < m && p[o] == k[o]) o++;
    l = o > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(o);
    bool desc = (o < m) ? (p[o] > k[o]) : (pl > kl);
    if (desc) atomicOr(flags, 1u);  // not sorted: the min-LCP shortcut does not hold
  }
  adj[i] = l;
}

__device__ inline uint64_t value_len(const EncodeArgs& a, uint32_t i) {
  return a.tomb[i] ? 0 : a.val_off[i + 1] - a.val_off[i];
}

// v0Size (row.go:95-107) of KV i with prefix p16 against the block's first key,
// plus its 2-byte offset slot.  Seq 0, no timestamps on the builder path.
__device__ inline uint64_t row_slot(const EncodeArgs& a, uint32_t i, uint32_t p16) {
  uint64_t kl = a.key_off[i + 1] - a.key_off[i];
  uint64_t sz = 4 + (kl - p16) + 9;
  if (!a.tomb[i]) sz += 4 + value_len(a, i);
  return sz + 2;
}

__device__ inline uint32_t lcp_direct(const EncodeArgs& a, uint32_t x, uint32_t y) {
  const uint8_t* p = a.keys + a.key_off[x];
  const uint8_t* q = a.keys + a.key_off[y];
  uint64_t m = min(a.key_off[x + 1] - a.key_off[x], a.key_off[y + 1] - a.key_off[y]), o = 0;
  while (o < m && p[o] == q[o]) o++;
  return o > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(o);
}

// block.Builder.Add fill rule (block.go:171): cur + 2 + v0Size(row) > blockSize
// rejects unless the block is empty.  prefix = uint16(computePrefixLen(first, key)).
// Sorted keys (the builder's case): the workgroup's KVs and the kNextWin - 256 after them have their
// LCP with the previous key and their prefix-free slot size (slot0) staged in LDS, so a KV's walk
// over the rows of its block reads LDS; a walk that leaves the window continues from HBM.
// row_slot(k, p16) = slot0[k] - p16 (p16 <= LCP <= key length).  A saturated slot0 (a row of
// >= 4 GiB) still ends the block when block_size < 2^32 - 2^16, the condition for this path.
constexpr uint32_t kNextThreads = 256, kNextWin = 1024;
__global__ __launch_bounds__(kNextThreads) void enc_next_kernel(EncodeArgs a, const uint32_t* __restrict__ adj,
                                                                const uint32_t* __restrict__ flags,
                                                                const uint32_t* __restrict__ slot0,
                                                                uint32_t* __restrict__ next,
                                                                uint64_t* __restrict__ bytes,
                                                                uint32_t* __restrict__ wg_max) {
  __shared__ uint32_t s_adj[kNextWin], s_slot[kNextWin];
  const uint32_t j0 = blockIdx.x * kNextThreads;
  const bool sorted = (*flags & 1u) == 0;
  const bool win = sorted && a.block_size < 0xFFFF0000ull;  // (workgroup-uniform)
  const uint32_t wend = win ? min(j0 + kNextWin, a.n) : j0;
  for (uint32_t x = threadIdx.x; j0 + x < wend; x += kNextThreads) {
    s_adj[x] = adj[j0 + x];
    s_slot[x] = slot0[j0 + x];
  }
  __syncthreads();
  const uint32_t j = j0 + threadIdx.x;
  uint32_t len = 0;
  if (j < a.n) {
    uint64_t cur = 2 + row_slot(a, j, 0);
    uint32_t p = 0xFFFFFFFFu, k = j + 1;
    bool full = false;
    for (; k < wend; k++) {
      p = min(p, s_adj[k - j0]);
      const uint64_t rs = uint64_t(s_slot[k - j0]) - (p & 0xFFFFu);
      if (cur + rs > a.block_size) {
        full = true;
        break;
      }
      cur += rs;
    }
    for (; !full && k < a.n; k++) {
      p = sorted ? min(p, adj[k]) : lcp_direct(a, j, k);
      uint64_t rs = row_slot(a, k, p & 0xFFFFu);
      if (cur + rs > a.block_size) break;
      cur += rs;
    }
    next[j] = k;
    bytes[j] = cur;
    len = k - j;
  }
  // the longest block in KVs, one word per workgroup (wg_max[blockIdx.x]; enc_chain_kernel reduces
  // them): an atomicMax per wave on one address serialised at ~11 ns each, 1.8 ms per 10 M KVs
  __shared__ uint32_t s_wmax[kNextThreads / 64];
#pragma unroll
  for (int o = 32; o; o >>= 1) len = max(len, uint32_t(__shfl_xor(int(len), o, 64)));
  if ((threadIdx.x & 63) == 0) s_wmax[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t w = 0; w < kNextThreads / 64; w++) m = max(m, s_wmax[w]);
    wg_max[blockIdx.x] = m;
  }
}

// ------------------------------------------------------------ block chains
constexpr uint32_t kChunk = 4096;
constexpr int kChunkThreads = 256;

__global__ __launch_bounds__(kChunkThreads) void enc_exit_kernel(uint32_t n, const uint32_t* __restrict__ next,
                                                                 uint32_t* __restrict__ exit_pos) {
  __shared__ uint32_t J[kChunk];
  uint32_t cs = blockIdx.x * kChunk, ce = min(cs + kChunk, n), m = ce - cs;
  for (uint32_t x = threadIdx.x; x < m; x += kChunkThreads) J[x] = next[cs + x];
  __syncthreads();
  // pointer jumping: after r rounds J[x] is >= 2^r hops ahead or has left the chunk
  for (int r = 0; r < 13; r++) {
    for (uint32_t x = threadIdx.x; x < m; x += kChunkThreads) {
      uint32_t v = J[x];
      if (v < ce) J[x] = J[v - cs];
    }
    __syncthreads();
  }
  for (uint32_t x = threadIdx.x; x < m; x += kChunkThreads) exit_pos[cs + x] = J[x];
}

// Sequential over chunks: entry[c] = first true block start in chunk c (kNone if
// a block spans the whole chunk).  Windows exit[cs .. cs+W) of upcoming chunks are
// prefetched into LDS; the true entry is always inside its chunk's window
// (W = longest block in KVs).
__global__ __launch_bounds__(kChunkThreads) void enc_chain_kernel(uint32_t n, const uint32_t* __restrict__ exit_pos,
                                                                  const uint32_t* __restrict__ wg_max,
                                                                  uint32_t n_wg, uint32_t* __restrict__ entry) {
  __shared__ uint32_t win[8192];
  __shared__ uint32_t e_sh;
  uint32_t nchunks = (n + kChunk - 1) / kChunk;
  {  // W = the longest block in KVs: the max over enc_next_kernel's per-workgroup words
    uint32_t m = 0;
    for (uint32_t x = threadIdx.x; x < n_wg; x += kChunkThreads) m = max(m, wg_max[x]);
    win[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t s = kChunkThreads / 2; s; s >>= 1) {
      if (threadIdx.x < s) win[threadIdx.x] = max(win[threadIdx.x], win[threadIdx.x + s]);
      __syncthreads();
    }
    m = win[0];
    __syncthreads();
    if (threadIdx.x == 0) e_sh = m;
  }
  __syncthreads();
  uint32_t W = min(e_sh, kChunk);
  __syncthreads();
  if (W == 0) W = 1;
  uint32_t G = max(1u, 8192u / W);
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nchunks; c0 += G) {
    uint32_t g = min(G, nchunks - c0);
    for (uint32_t t = threadIdx.x; t < g * W; t += kChunkThreads) {
      uint32_t c = c0 + t / W, x = c * kChunk + t % W;
      win[t] = x < n ? exit_pos[x] : n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t e = e_sh;
      for (uint32_t q = 0; q < g; q++) {
        uint32_t cs = (c0 + q) * kChunk, ce = min(cs + kChunk, n);
        if (e >= ce) {
          entry[c0 + q] = kNone;
        } else {
          entry[c0 + q] = e;
          e = win[q * W + (e - cs)];
        }
      }
      e_sh = e;
    }
    __syncthreads();
  }
}

// Per chunk: list the true block starts (walk next[] in LDS from the entry).
__global__ __launch_bounds__(kChunkThreads) void enc_mark_kernel(uint32_t n, const uint32_t* __restrict__ next,
                                                                 const uint32_t* __restrict__ entry,
                                                                 uint32_t* __restrict__ starts_tmp,
                                                                 uint64_t* __restrict__ counts) {
  __shared__ uint32_t J[kChunk];
  uint32_t c = blockIdx.x, cs = c * kChunk, ce = min(cs + kChunk, n), m = ce - cs;
  for (uint32_t x = threadIdx.x; x < m; x += kChunkThreads) J[x] = next[cs + x];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t e = entry[c], cnt = 0;
    if (e != kNone)
      while (e < ce) {
        starts_tmp[cs + cnt++] = e;
        e = J[e - cs];
      }
    counts[c] = cnt;
  }
}

// Block list: block b = KVs [start, next[start]).  The block whose end is n is
// still open unless this is the final flush.  Sizes of the encoded blocks
// (CodecNone: data + offsets + count + CRC).
__global__ void enc_blocks_kernel(uint32_t n, const uint32_t* __restrict__ starts_tmp,
                                  const uint64_t* __restrict__ chunk_base, const uint64_t* __restrict__ bytes,
                                  uint32_t* __restrict__ block_start, uint64_t* __restrict__ block_size) {
  uint32_t c = blockIdx.x, cs = c * kChunk;
  uint64_t base = chunk_base[c];
  // chunk_base is the exclusive scan of the per-chunk start counts
  uint32_t cnt = uint32_t(min<uint64_t>(chunk_base[c + 1] - base, kChunk));
  for (uint32_t t = threadIdx.x; t < cnt; t += blockDim.x) {
    if (base + t >= n) break;
    uint32_t s = starts_tmp[cs + t];
    block_start[base + t] = s;
    block_size[base + t] = bytes[s] + 4;
  }
}

// ------------------------------------------------------------- block packing
// One wavefront per block: rows assembled in LDS, then CRC and a byte-exact
// write into the SST stream at out + out_off[b].
__device__ inline void write_bytes_from_lds(uint8_t* gdst, const uint8_t* lds, uint32_t len, int lane) {
  // head bytes until gdst is 16-aligned, 16-byte chunks, tail bytes
  uint32_t head = uint32_t((16 - (reinterpret_cast<uintptr_t>(gdst) & 15)) & 15);
  if (head > len) head = len;
  if (uint32_t(lane) < head) gdst[lane] = lds[lane];
  uint32_t body = (len - head) / 16;
  uint4* d4 = reinterpret_cast<uint4*>(gdst + head);
  for (uint32_t c = lane; c < body; c += kWave) {
    int32_t o = int32_t(head + 16 * c);
    uint4 v;
    v.x = lds_u32(lds, o);
    v.y = lds_u32(lds, o + 4);
    v.z = lds_u32(lds, o + 8);
    v.w = lds_u32(lds, o + 12);
    d4[c] = v;
  }
  uint32_t tail0 = head + body * 16;
  for (uint32_t t = tail0 + lane; t < len; t += kWave) gdst[t] = lds[t];
}

// rows ‖ BE16 offsets ‖ BE16 count of the block holding KVs [s, e) into buf
// (block.go:162-182 Add, :54-64 Encode before compression); raw_len bytes.
// The block's keys and values staged in LDS (k == nullptr: read them from HBM): key bytes of KV i
// at k + (key_off[i] - kb), value bytes at v + (val_off[i] - vb); k and v 16-aligned.
struct KvStage {
  const uint8_t* k = nullptr;
  uint64_t kb = 0;
  const uint8_t* v = nullptr;
  uint64_t vb = 0;
};

// n bytes from the LDS stage (offset o of its 16-aligned base) to dst (any alignment), four at a
// time from two aligned dword reads
__device__ inline void copy_from_stage(uint8_t* dst, const uint8_t* base, uint32_t o, uint32_t n) {
  uint32_t b = 0;
  for (; b + 4 <= n; b += 4) {
    const uint32_t w = lds_u32(base, int32_t(o + b));
    dst[b] = uint8_t(w);
    dst[b + 1] = uint8_t(w >> 8);
    dst[b + 2] = uint8_t(w >> 16);
    dst[b + 3] = uint8_t(w >> 24);
  }
  for (; b < n; b++) dst[b] = base[o + b];
}

// Keys and values of KVs [s, e) into LDS at st (16-aligned, cap bytes) with 16-byte loads all in
// flight at once, so the rows are assembled from LDS instead of by dependent byte loads from HBM;
// an empty stage (read from HBM) when they do not fit.
__device__ inline KvStage stage_kvs(const EncodeArgs& a, uint32_t s, uint32_t e, uint8_t* st, uint32_t cap, int lane) {
  KvStage kst;
  const uint64_t k0 = a.key_off[s] & ~uint64_t(15), k1 = align16(a.key_off[e]);
  const uint64_t v0 = a.val_off[s] & ~uint64_t(15), v1 = align16(a.val_off[e]);
  const uint32_t nk = uint32_t((k1 - k0) / 16), nv = uint32_t((v1 - v0) / 16);
  if (16 * uint64_t(nk + nv) + 16 > cap) return kst;
  uint4* d = reinterpret_cast<uint4*>(st);
  const uint4* gk = reinterpret_cast<const uint4*>(a.keys + k0);
  const uint4* gv = reinterpret_cast<const uint4*>(a.vals + v0);
  for (uint32_t q0 = 0; q0 < nk + nv; q0 += 4 * kWave) {
    uint4 w[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t q = min(q0 + u * kWave + uint32_t(lane), nk + nv - 1);
      w[u] = q < nk ? gk[q] : gv[q - nk];
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t q = q0 + u * kWave + uint32_t(lane);
      if (q < nk + nv) d[q] = w[u];
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  kst.k = st;
  kst.kb = k0;
  kst.v = st + 16 * nk;
  kst.vb = v0;
  return kst;
}

__device__ void assemble_block(const EncodeArgs& a, const uint32_t* adj, bool sorted, uint32_t s, uint32_t e,
                               uint8_t* buf, uint32_t raw_len, int lane, const KvStage& kst = KvStage{}) {
  const uint32_t nrows = e - s;
  const uint32_t data_len = raw_len - 2 * nrows - 2;
  // rows, 64 at a time: prefix (running min of adjacent LCPs), row offset (scan)
  uint32_t carry_off = 0, carry_min = 0xFFFFFFFFu;
  for (uint32_t r0 = 0; r0 < nrows; r0 += kWave) {
    uint32_t r = r0 + lane;
    bool live = r < nrows;
    uint32_t i = s + r;
    uint32_t p = 0xFFFFFFFFu;
    if (live && r > 0) p = sorted ? adj[i] : lcp_direct(a, s, i);
    if (sorted) {  // inclusive min-scan over the rows of this group
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(p, o, 64);
        if (lane >= o) p = min(p, y);
      }
      p = min(p, carry_min);
    }
    uint32_t p16 = (live && r > 0) ? (p & 0xFFFFu) : 0;
    uint32_t sz = live ? uint32_t(row_slot(a, i, p16) - 2) : 0;
    uint32_t incl = sz;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    uint32_t off = carry_off + incl - sz;
    if (live) {
      const uint8_t* key = a.keys + a.key_off[i];
      uint32_t kl = uint32_t(a.key_off[i + 1] - a.key_off[i]);
      uint32_t sl = kl - p16;
      uint8_t* row = buf + off;
      st_be16(row, uint16_t(p16));
      st_be16(row + 2, uint16_t(sl));
      if (kst.k) copy_from_stage(row + 4, kst.k, uint32_t(a.key_off[i] - kst.kb) + p16, sl);
      else
        for (uint32_t b = 0; b < sl; b++) row[4 + b] = key[p16 + b];
      uint8_t* q = row + 4 + sl;
      for (int b = 0; b < 8; b++) q[b] = 0;  // seq 0 (builder.go:162 Row{Value: ...})
      bool tomb = a.tomb[i] != 0;
      q[8] = tomb ? 1 : 0;
      if (!tomb) {
        uint32_t vl = uint32_t(value_len(a, i));
        st_be32(q + 9, vl);
        const uint8_t* v = a.vals + a.val_off[i];
        if (kst.v) copy_from_stage(q + 13, kst.v, uint32_t(a.val_off[i] - kst.vb), vl);
        else
          for (uint32_t b = 0; b < vl; b++) q[13 + b] = v[b];
      }
      st_be16(buf + data_len + 2 * r, uint16_t(off));  // uint16(len(b.data)) (block.go:176)
    }
    carry_off += __shfl(incl, 63, 64);
    if (sorted) carry_min = __shfl(p, 63, 64);
  }
  if (lane == 0) st_be16(buf + data_len + 2 * nrows, uint16_t(nrows));
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0);
}

template <bool kLds>
__device__ void pack_block(const EncodeArgs& a, const uint32_t* adj, bool sorted, uint32_t s, uint32_t e,
                           uint8_t* buf, const uint32_t* tab, uint8_t* gdst, uint64_t enc_len, int lane,
                           const KvStage& kst = KvStage{}) {
  const uint32_t raw_len = uint32_t(enc_len - 4);
  assemble_block(a, adj, sorted, s, e, buf, raw_len, lane, kst);
  uint32_t crc = wave_crc32(tab, buf, 0, raw_len, lane);
  if (lane == 0) st_be32(buf + raw_len, crc);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0);
  write_bytes_from_lds(gdst, buf, uint32_t(enc_len), lane);
}

__global__ __launch_bounds__(kPackThreads) void enc_pack_kernel(EncodeArgs a, const uint32_t* __restrict__ adj,
                                                                const uint32_t* __restrict__ flags,
                                                                const uint32_t* __restrict__ block_start,
                                                                const uint32_t* __restrict__ next,
                                                                const uint64_t* __restrict__ out_off,
                                                                uint32_t nblocks, uint8_t* __restrict__ out,
                                                                uint32_t* __restrict__ big_list,
                                                                uint32_t* __restrict__ big_count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* buf = smem + kTabBytes + wave * kPackCap;
  const bool sorted = (*flags & 1u) == 0;
  const uint32_t waves = gridDim.x * (kPackThreads / 64);
  for (uint32_t b = blockIdx.x * (kPackThreads / 64) + wave; b < nblocks; b += waves) {
    uint64_t enc_len = out_off[b + 1] - out_off[b];
    if (enc_len + 8 > kPackCap) {
      if (lane == 0) big_list[atomicAdd(big_count, 1u)] = b;
      continue;
    }
    uint32_t s = block_start[b];
    // the KVs staged in the rest of the wave's buffer, past the block (+ CRC and slack)
    const uint32_t used = uint32_t(align16(enc_len + 16));
    const KvStage kst = kPackStage && used < kPackCap ? stage_kvs(a, s, next[s], buf + used, kPackCap - used, lane)
                                                      : KvStage{};
    pack_block<true>(a, adj, sorted, s, next[s], buf, tab, out + out_off[b], enc_len, lane, kst);
  }
}

// Blocks larger than the LDS budget: one wavefront per workgroup with the
// largest dynamic LDS allocation.
__global__ __launch_bounds__(64) void enc_pack_big_kernel(EncodeArgs a, const uint32_t* __restrict__ adj,
                                                          const uint32_t* __restrict__ flags,
                                                          const uint32_t* __restrict__ block_start,
                                                          const uint32_t* __restrict__ next,
                                                          const uint64_t* __restrict__ out_off,
                                                          uint8_t* __restrict__ out,
                                                          const uint32_t* __restrict__ big_list,
                                                          const uint32_t* __restrict__ big_count,
                                                          uint32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63;
  uint8_t* buf = smem + kTabBytes;
  const bool sorted = (*flags & 1u) == 0;
  uint32_t cnt = *big_count;
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    uint32_t b = big_list[k];
    uint64_t enc_len = out_off[b + 1] - out_off[b];
    if (enc_len + 8 > kPackBigCap) {
      if (lane == 0) atomicOr(status, 1u);  // beyond the LDS budget
      continue;
    }
    uint32_t s = block_start[b];
    pack_block<true>(a, adj, sorted, s, next[s], buf, tab, out + out_off[b], enc_len, lane);
  }
}

// ----------------------------------------------------------- Snappy blocks
// block.Encode with CodecSnappy (block.go:54-75): raw block assembled in LDS,
// golang/snappy encoded in LDS (snappy_enc.h), CRC32 of the compressed bytes,
// written to a per-block slot; a scan of the compressed sizes and a compaction
// pass place the blocks back to back.
__device__ inline uint64_t snap_slot_off(uint64_t raw_off, uint64_t b) { return align16(raw_off + raw_off / 6 + 48 * b); }

// per wave: the raw block (+16 readable bytes), the 4096-slot table and its owner bytes; the encoded
// block goes straight to its HBM slot (an LDS copy of it cost a quarter of the wave's LDS: with it,
// six waves per CU; without, nine)
constexpr uint32_t kSnapWaveBytes = kSnapRaw + 16 + 2 * kSnapRaw + kSnapOwner;

__global__ __launch_bounds__(kSnapThreads) void enc_pack_snappy_kernel(
    EncodeArgs a, const uint32_t* __restrict__ adj, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ block_start, const uint32_t* __restrict__ next, const uint64_t* __restrict__ raw_off,
    uint32_t nblocks, uint8_t* __restrict__ slots, uint64_t* __restrict__ csize, uint32_t* __restrict__ big_list,
    uint32_t* __restrict__ big_count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* raw = smem + kTabBytes + wave * kSnapWaveBytes;
  uint16_t* table = reinterpret_cast<uint16_t*>(raw + kSnapRaw + 16);
  uint8_t* owner = reinterpret_cast<uint8_t*>(table + kSnapRaw);
  const bool sorted = (*flags & 1u) == 0;
  // blocks handed out one at a time by a counter (flags word 4, zeroed with the flags): a wave that
  // drew cheap blocks takes more, so the launch ends when the work does
  uint32_t* work = const_cast<uint32_t*>(flags) + 4;
  auto draw = [&]() { return __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(work, 1u) : 0u); };
  for (uint32_t b = draw(); b < nblocks; b = draw()) {
    const uint64_t raw_len = raw_off[b + 1] - raw_off[b] - 4;
    if (raw_len > kSnapRaw) {
      if (lane == 0) big_list[atomicAdd(big_count, 1u)] = b;
      continue;
    }
    const uint32_t s = block_start[b];
    assemble_block(a, adj, sorted, s, next[s], raw, uint32_t(raw_len), lane);
    uint8_t* dst = slots + snap_slot_off(raw_off[b], b);
    const uint32_t clen =
        snappy_encode_wave<SLATE_SNAP_PACK_SERIAL>(raw, uint32_t(raw_len), dst, table, owner, lane, kSnapOwner - 1);
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence();  // the encoded bytes (stored by every lane) are read back by every lane
    const uint32_t crc = wave_crc32(tab, dst, 0, clen, lane);
    if (lane == 0) {
      st_be32(dst + clen, crc);
      csize[b] = clen + 4;
    }
  }
}

// Blocks above kSnapRaw bytes: one wave per workgroup, raw block staged in HBM,
// full 16 Ki-slot table in LDS.
__global__ __launch_bounds__(64) void enc_pack_snappy_big_kernel(
    EncodeArgs a, const uint32_t* __restrict__ adj, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ block_start, const uint32_t* __restrict__ next, const uint64_t* __restrict__ raw_off,
    uint8_t* __restrict__ rawbuf, uint8_t* __restrict__ slots, uint64_t* __restrict__ csize,
    const uint32_t* __restrict__ big_list, const uint32_t* __restrict__ big_count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  const int lane = threadIdx.x & 63;
  uint16_t* table = reinterpret_cast<uint16_t*>(smem + kTabBytes);
  uint8_t* owner = reinterpret_cast<uint8_t*>(table + kSnapMaxTable);
  const bool sorted = (*flags & 1u) == 0;
  const uint32_t cnt = *big_count;
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    const uint32_t b = big_list[k];
    const uint64_t raw_len = raw_off[b + 1] - raw_off[b] - 4;
    uint8_t* rp = rawbuf + raw_off[b];
    uint8_t* sp = slots + snap_slot_off(raw_off[b], b);
    const uint32_t s = block_start[b];
    assemble_block(a, adj, sorted, s, next[s], rp, uint32_t(raw_len), lane);
    __threadfence();
    const uint32_t clen = snappy_encode_wave(rp, uint32_t(raw_len), sp, table, owner, lane);
    __threadfence();
    const uint32_t crc = wave_crc32(tab, sp, 0, clen, lane);
    if (lane == 0) {
      st_be32(sp + clen, crc);
      csize[b] = clen + 4;
    }
  }
}

// slots -> back-to-back blocks at final_off (exclusive scan of csize)
__global__ void enc_compact_kernel(const uint8_t* __restrict__ slots, const uint64_t* __restrict__ raw_off,
                                   const uint64_t* __restrict__ final_off, uint32_t nblocks, uint8_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); b < nblocks; b += waves) {
    write_bytes_from_lds(out + final_off[b], slots + snap_slot_off(raw_off[b], b),
                         uint32_t(final_off[b + 1] - final_off[b]), lane);
  }
}

// snappy.Encode of one large buffer (bloom filter, index): one wave per 64 KiB
// chunk, chunk c's encoding at dst + c * kSnapChunkSlot, its length in len[c].
__global__ __launch_bounds__(64) void snappy_chunks_kernel(const uint8_t* __restrict__ src, uint64_t n,
                                                           uint8_t* __restrict__ dst, uint32_t* __restrict__ len) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  uint16_t* table = reinterpret_cast<uint16_t*>(smem);
  uint8_t* owner = reinterpret_cast<uint8_t*>(table + kSnapMaxTable);
  // the chunk itself is staged in LDS, so the match loop's dependent source reads come from LDS
  // (measured neutral on its own: the cost was the duplicate-slot scans, see snap_slot_neighbours)
  uint8_t* stage = smem + kSnapMaxTable * 3;
  const uint64_t nchunks = (n + kSnapMaxBlock - 1) / kSnapMaxBlock;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint8_t* p = src + c * kSnapMaxBlock;
    const uint32_t pn = uint32_t(min<uint64_t>(n - c * kSnapMaxBlock, kSnapMaxBlock));
    uint8_t* o = dst + c * kSnapChunkSlot;
    snap_sync();  // the previous chunk's reads of the stage are done
    // 16-byte loads for the whole chunks (the source is 16-aligned: chunk starts are 64 KiB apart
    // from an aligned buffer), bytes for the tail; all loads of a lane issue before its LDS stores
    const uint32_t nq = pn / 16;
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
#pragma unroll 4
      for (uint32_t q = uint32_t(lane); q < nq; q += kWave)
        reinterpret_cast<uint4*>(stage)[q] = reinterpret_cast<const uint4*>(p)[q];
      for (uint32_t i = 16 * nq + uint32_t(lane); i < pn; i += kWave) stage[i] = p[i];
    } else {
      for (uint32_t i = uint32_t(lane); i < pn; i += kWave) stage[i] = p[i];
    }
    if (lane < 16) stage[pn + lane] = 0;  // bytes past the chunk (never part of a match)
    snap_sync();
    uint32_t d;
    if (pn < kSnapMinNonLiteral) d = snap_emit_literal(o, 0, stage, pn, lane);
    else d = snappy_encode_block_wave<kSnapChunkSerialProbes>(stage, pn, o, table, owner, lane);
    if (lane == 0) len[c] = d;
  }
}

// ------------------------------------------------------------------- bloom
__device__ inline uint32_t mod_u32(uint32_t x, uint32_t m) { return x % m; }

// bloom.go:147-160 probesForKey in 32-bit arithmetic: every value is below filterBits (< 2^32), so
// the first two reductions are 32-bit and the later ones a conditional subtraction (h + delta <
// 2 filterBits; delta + i below filterBits + i, with the modulo kept for i >= filterBits) -- the
// same values as Go's uint64 % (the probes computed two 64-bit modulos each)
struct BloomProbes {
  uint32_t h, delta, m, k;
  __device__ BloomProbes(uint64_t h64, uint32_t filter_bits) : m(filter_bits), k(0) {
    h = uint32_t(h64) % m;
    delta = uint32_t(h64 >> 32) % m;
  }
  __device__ uint32_t next() {
    const uint64_t d = uint64_t(delta) + k;
    delta = d < m ? uint32_t(d) : (d - m < m ? uint32_t(d - m) : uint32_t(d % m));
    k++;
    const uint32_t p = h;
    const uint64_t hh = uint64_t(h) + delta;
    h = hh < m ? uint32_t(hh) : uint32_t(hh - m);
    return p;
  }
};

// bloom.go:147-160 probes for one key hash, setBit (bloom.go:169-172) as an
// atomicOr on the little-endian 32-bit word holding byte p/8.
__global__ void bloom_build_kernel(const uint64_t* __restrict__ hashes, uint64_t n, uint32_t num_probes,
                                   uint32_t filter_bits, uint32_t* __restrict__ words) {
  uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  BloomProbes pr(hashes[i], filter_bits);
  for (uint32_t k = 0; k < num_probes; k++) {
    const uint32_t p = pr.next();
    atomicOr(&words[p >> 5], 1u << (p & 31));
  }
}

// Bucketed build: the same probes, no global atomics.  ~70 M scattered device-scope atomicOr for a
// 10 M-key filter ran at ~30 G/s (2.35 ms); here a workgroup of keys counts its probes per 64 KiB
// slice of the filter (LDS histogram), a scan gives every (slice, workgroup) its range of a probe
// array, the workgroup scatters its probes there, and one workgroup per slice ORs the slice's probes
// into LDS and writes the slice out.  OR is order-free: the bits are the atomic kernel's.
constexpr uint32_t kBktThreads = 256, kBktKeysPerThread = 8, kBktKeys = kBktThreads * kBktKeysPerThread;
#ifndef SLATE_BKT_SLICE_LOG
#define SLATE_BKT_SLICE_LOG 19
#endif
#ifndef SLATE_BKT_OR_THREADS
#define SLATE_BKT_OR_THREADS 1024
#endif
constexpr uint32_t kBktSliceLog = SLATE_BKT_SLICE_LOG;  // 2^19 bits = 64 KiB of LDS per slice
constexpr uint32_t kBktMaxSlices = 8192, kBktOrThreads = SLATE_BKT_OR_THREADS;
constexpr uint64_t kBktMaxCells = 1ull << 24;  // (slices x key workgroups) counters


__global__ __launch_bounds__(kBktThreads) void bloom_count_kernel(const uint64_t* __restrict__ hashes, uint64_t n,
                                                                  uint32_t num_probes, uint32_t filter_bits,
                                                                  uint32_t n_slices, uint64_t* __restrict__ cells) {
  __shared__ uint32_t hist[kBktMaxSlices];
  for (uint32_t s = threadIdx.x; s < n_slices; s += kBktThreads) hist[s] = 0;
  __syncthreads();
  const uint64_t k0 = uint64_t(blockIdx.x) * kBktKeys;
  for (uint32_t r = 0; r < kBktKeysPerThread; r++) {
    const uint64_t i = k0 + r * kBktThreads + threadIdx.x;
    if (i >= n) break;
    BloomProbes pr(hashes[i], filter_bits);
    for (uint32_t q = 0; q < num_probes; q++) atomicAdd(&hist[pr.next() >> kBktSliceLog], 1u);
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < n_slices; s += kBktThreads) cells[uint64_t(s) * gridDim.x + blockIdx.x] = hist[s];
}

__global__ __launch_bounds__(kBktThreads) void bloom_scatter_kernel(const uint64_t* __restrict__ hashes, uint64_t n,
                                                                    uint32_t num_probes, uint32_t filter_bits,
                                                                    uint32_t n_slices,
                                                                    const uint64_t* __restrict__ cells,
                                                                    uint32_t* __restrict__ probes) {
  __shared__ uint32_t cur[kBktMaxSlices];
  for (uint32_t s = threadIdx.x; s < n_slices; s += kBktThreads)
    cur[s] = uint32_t(cells[uint64_t(s) * gridDim.x + blockIdx.x]);
  __syncthreads();
  const uint64_t k0 = uint64_t(blockIdx.x) * kBktKeys;
  for (uint32_t r = 0; r < kBktKeysPerThread; r++) {
    const uint64_t i = k0 + r * kBktThreads + threadIdx.x;
    if (i >= n) break;
    BloomProbes pr(hashes[i], filter_bits);
    for (uint32_t q = 0; q < num_probes; q++) {
      const uint32_t p = pr.next();
      probes[atomicAdd(&cur[p >> kBktSliceLog], 1u)] = p;
    }
  }
}

// one workgroup per slice: its probes (cells[s * n_wg] .. cells[(s + 1) * n_wg]) OR-ed into LDS
__global__ __launch_bounds__(kBktOrThreads) void bloom_or_kernel(const uint64_t* __restrict__ cells, uint32_t n_wg,
                                                                 const uint32_t* __restrict__ probes,
                                                                 uint32_t filter_bits, uint32_t* __restrict__ words) {
  __shared__ uint32_t slice[1u << (kBktSliceLog - 5)];
  const uint32_t s = blockIdx.x;
  for (uint32_t w = threadIdx.x; w < (1u << (kBktSliceLog - 5)); w += kBktOrThreads) slice[w] = 0;
  __syncthreads();
  const uint64_t lo = cells[uint64_t(s) * n_wg], hi = cells[uint64_t(s + 1) * n_wg];
  // eight loads in flight per thread before their ORs (one at a time: ~360 dependent round trips)
  constexpr uint32_t kU = 8;
  for (uint64_t j0 = lo + threadIdx.x; j0 < hi; j0 += kU * kBktOrThreads) {
    uint32_t p[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint64_t j = j0 + u * kBktOrThreads;
      p[u] = j < hi ? probes[j] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      if (j0 + u * kBktOrThreads < hi) {
        const uint32_t q = p[u] & ((1u << kBktSliceLog) - 1);
        atomicOr(&slice[q >> 5], 1u << (q & 31));
      }
    }
  }
  __syncthreads();
  const uint64_t w0 = uint64_t(s) << (kBktSliceLog - 5);
  const uint64_t total = (uint64_t(filter_bits) + 31) / 32;
  const uint32_t nw = uint32_t(min(uint64_t(1u << (kBktSliceLog - 5)), total - w0));
  for (uint32_t w = threadIdx.x; w < nw; w += kBktOrThreads) words[w0 + w] = slice[w];
}

__global__ void bloom_check_kernel(const uint8_t* __restrict__ keys, const uint64_t* __restrict__ key_off, uint64_t n,
                                   const uint8_t* __restrict__ bits, uint64_t bits_len, uint32_t num_probes,
                                   uint8_t* __restrict__ out) {
  uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (bits_len == 0) { out[i] = 0; return; }  // Filter.HasKey on an empty filter
  const uint8_t* k = keys + key_off[i];
  uint64_t kl = key_off[i + 1] - key_off[i];
  uint64_t h64 = 0xcbf29ce484222325ull;
  for (uint64_t b = 0; b < kl; b++) {
    h64 *= 0x100000001b3ull;
    h64 ^= k[b];
  }
  uint64_t m = bits_len * 8;
  m &= 0xFFFFFFFFull;  // uint32(len(f.Data)*8) (bloom.go:24)
  uint8_t res = 1;
  if (m == 0) { out[i] = 0; return; }
  BloomProbes pr(h64, uint32_t(m));
  for (uint32_t q = 0; q < num_probes; q++) {
    const uint32_t p = pr.next();
    if (!(bits[p >> 3] & (1u << (p & 7)))) { res = 0; break; }
  }
  out[i] = res;
}

// --------------------------------------------------------- large-buffer CRC
// crc32.ChecksumIEEE of a device buffer (the SST builder's filter and index payloads, up to tens of
// MB).  The buffer is cut into 16-byte chunks aligned to memory (chunk j = aligned bytes
// [16j, 16j + 16) from the 16-byte line of its first byte); the chunks wholly before the end form
// the "body", the bytes of the last partial chunk the "tail".  Each wave turns a stripe of 256
// body chunks into its raw CRC (slicing-by-16 per lane, lanes and rows joined by the zero-advance
// tables, as decode_none's block CRC), grid-stride, tables loaded once per workgroup; one wave
// then joins the stripes (GF(2) products) and the tail.  The 0xFFFFFFFF initial register is
// folded into message bytes 0..3 and the bytes before the message are zeroed.
constexpr uint32_t kCrcThreads = 256;
constexpr uint32_t kCrcStripeChunks = 256;
constexpr uint32_t kCrcLds = kTab16Bytes + kAdvN * 4096;

struct CrcGeo {
  const uint8_t* base;  // 16-byte line of the first byte
  uint32_t sh;          // message byte 0 = base[sh]
  uint64_t body;        // whole chunks
};
__device__ __forceinline__ CrcGeo crc_geo(const uint8_t* data, uint64_t n) {
  CrcGeo g;
  g.sh = uint32_t(reinterpret_cast<uintptr_t>(data) & 15);
  g.base = data - g.sh;
  g.body = (g.sh + n) / 16;
  // the initial register is folded into message bytes 0..3: the body must hold them (else the
  // whole message is the tail)
  if (16 * g.body < g.sh + 4) g.body = 0;
  return g;
}

__global__ __launch_bounds__(kCrcThreads) void crc_stripes_kernel(const uint8_t* __restrict__ data, uint64_t n,
                                                                  uint32_t* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  {
    const uint32_t* src = &g_crc16.t[0][0];
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = src[i];
    load_adv_tables(tab + 4096);
    __syncthreads();
  }
  const uint8_t* lds = smem;
  const uint32_t lane = threadIdx.x & 63;
  const CrcGeo g = crc_geo(data, n);
  const uint64_t stripes = (g.body + kCrcStripeChunks - 1) / kCrcStripeChunks;
  const uint64_t waves = uint64_t(gridDim.x) * (kCrcThreads / 64);
  for (uint64_t k = blockIdx.x * (kCrcThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); k < stripes;
       k += waves) {
    // the last stripe may be short: its chunks sit at the end of the 256 slots (zeros in front of
    // a zero register change nothing)
    const uint64_t c0 = k * kCrcStripeChunks;
    const uint32_t nck = uint32_t(min<uint64_t>(kCrcStripeChunks, g.body - c0));
    const uint32_t pad = kCrcStripeChunks - nck;
    const __amdgpu_buffer_rsrc_t R = make_rsrc(g.base + 16 * c0, 16 * uint64_t(nck));
    v4u v[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const int32_t j = int32_t(64 * q + lane) - int32_t(pad);
      v[q] = __builtin_amdgcn_raw_buffer_load_b128(R, j >= 0 ? uint32_t(16 * j) : kOOB, 0, 2);
    }
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const int32_t j = int32_t(64 * q + lane) - int32_t(pad);
      v4u c = v[q];
      if (k == 0 && __builtin_amdgcn_ballot_w64(j >= 0 && j < 2)) {
        // message bytes 0..3 take the initial register, the bytes before the message are zero:
        // chunk-relative message start at -sh + 16 j
        const int32_t m0 = 16 * j - int32_t(g.sh);  // message position of the chunk's byte 0
        const bool in = j >= 0 && j < 2;
        c.x = (in ? keep_mask(-m0, 16, 0) : ~0u) & c.x ^ (in ? keep_mask(-m0, 4 - m0, 0) : 0u);
        c.y = (in ? keep_mask(-m0, 16, 1) : ~0u) & c.y ^ (in ? keep_mask(-m0, 4 - m0, 1) : 0u);
        c.z = (in ? keep_mask(-m0, 16, 2) : ~0u) & c.z ^ (in ? keep_mask(-m0, 4 - m0, 2) : 0u);
        c.w = (in ? keep_mask(-m0, 16, 3) : ~0u) & c.w ^ (in ? keep_mask(-m0, 4 - m0, 3) : 0u);
      }
      const uint32_t r = crc_chunk0(lds, c);
      acc = (q == 0 ? 0u : adv_tab<5>(lds, acc)) ^ (j >= 0 ? r : 0u);
    }
    // lane l's chunks are followed by 63 - l chunks of their row: rows of 16 lanes by DPP, then
    // the four row heads
    acc = adv16(lds, acc) ^ row_shl<1>(acc);
    acc = adv_tab<0>(lds, acc) ^ row_shl<2>(acc);
    acc = adv_tab<1>(lds, acc) ^ row_shl<4>(acc);
    acc = adv_tab<2>(lds, acc) ^ row_shl<8>(acc);
    const uint32_t h1 = __builtin_amdgcn_readlane(acc, 16), h2 = __builtin_amdgcn_readlane(acc, 32),
                   h3 = __builtin_amdgcn_readlane(acc, 48);
    acc = adv_tab<3>(lds, acc) ^ h1;
    acc = adv_tab<3>(lds, acc) ^ h2;
    acc = adv_tab<3>(lds, acc) ^ h3;
    if (lane == 0) partial[k] = acc;
  }
}

// One wave: body = sum_k partial_k * x^(8 * bytes after stripe k), then the tail bytes (and the
// whole message when it has no whole chunk), inverted.
__global__ void crc_join_kernel(const uint8_t* __restrict__ data, uint64_t n, const uint32_t* __restrict__ partial,
                                uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const CrcGeo g = crc_geo(data, n);
  const uint64_t stripes = (g.body + kCrcStripeChunks - 1) / kCrcStripeChunks;
  uint32_t body = 0;
  if (stripes) {
    // stripes 0 .. S-2 are whole; stripe S-1 has nl chunks: Horner per lane over k = l, l+64, ...
    const uint64_t full = stripes - 1;
    const uint32_t nl = uint32_t(g.body - full * kCrcStripeChunks);
    const uint32_t x64 = x8n(uint64_t(16) * kCrcStripeChunks * 64);
    uint32_t acc = 0;
    uint64_t last = 0;
    bool any = false;
    for (uint64_t k = lane; k < full; k += 64) {
      acc = gf2_mulmod(acc, x64) ^ partial[k];
      last = k;
      any = true;
    }
    // lane's last stripe is followed by (full - 1 - last) whole stripes and the short one
    uint32_t v = any ? gf2_mulmod(acc, x8n(uint64_t(16) * kCrcStripeChunks * (full - 1 - last) + 16 * uint64_t(nl)))
                     : 0u;
    for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o, 64);
    body = v ^ partial[full];
  }
  if (lane == 0) {
    // tail: message bytes from 16 * body - sh on (all of them when there is no whole chunk, the
    // initial register then folded here)
    const uint64_t t0 = g.body ? 16 * g.body - g.sh : 0;
    uint32_t c = g.body ? body : 0xFFFFFFFFu;
    for (uint64_t i = t0; i < n; i++) c = g_crc16.t[0][(c ^ data[i]) & 0xff] ^ (c >> 8);
    *out = ~c;
  }
}

// --------------------------------------------------------------- launchers
static inline uint32_t blocks_for(uint64_t n, uint32_t t) { return uint32_t((n + t - 1) / t); }

hipError_t launch_kv_hashes(hipStream_t st, const EncodeArgs& a, uint64_t* hashes, uint32_t* adj, uint32_t* flags) {
  if (a.n) enc_kv_kernel<<<blocks_for(a.n, 256), 256, 0, st>>>(a, hashes, adj, flags);
  return hipGetLastError();
}

hipError_t launch_encode(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, int num_cus) {
  const uint32_t n = a.n;
  (void)hipMemsetAsync(w.flags, 0, 20, st);  // flags, maxlen, big_count, status, pack work counter
  if (n == 0) return hipGetLastError();
  // slot0 lives in exit_pos until enc_exit_kernel overwrites it
  enc_kv_kernel<<<blocks_for(n, 256), 256, 0, st>>>(a, w.hashes, w.adj, w.flags, w.exit_pos);
  // the per-workgroup longest blocks live in starts_tmp until enc_mark_kernel writes it
  const uint32_t n_wg = blocks_for(n, kNextThreads);
  enc_next_kernel<<<n_wg, kNextThreads, 0, st>>>(a, w.adj, w.flags, w.exit_pos, w.next, w.bytes, w.starts_tmp);
  uint32_t nchunks = blocks_for(n, kChunk);
  enc_exit_kernel<<<nchunks, kChunkThreads, 0, st>>>(n, w.next, w.exit_pos);
  enc_chain_kernel<<<1, kChunkThreads, 0, st>>>(n, w.exit_pos, w.starts_tmp, n_wg, w.entry);
  enc_mark_kernel<<<nchunks, kChunkThreads, 0, st>>>(n, w.next, w.entry, w.starts_tmp, w.counts);
  return hipGetLastError();
}

hipError_t launch_encode_blocks(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w) {
  uint32_t nchunks = blocks_for(a.n, kChunk);
  if (a.n == 0) return hipGetLastError();
  enc_blocks_kernel<<<nchunks, 256, 0, st>>>(a.n, w.starts_tmp, w.chunk_base, w.bytes, w.block_start,
                                             w.block_size);
  return hipGetLastError();
}

hipError_t launch_pack(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, uint32_t nblocks,
                       const uint64_t* out_off, uint8_t* out, int num_cus) {
  if (nblocks == 0) return hipGetLastError();
  const size_t lds = kTabBytes + (kPackThreads / 64) * size_t(kPackCap);
  uint32_t grid = min(blocks_for(nblocks, kPackThreads / 64), uint32_t(num_cus) * 8);
  enc_pack_kernel<<<grid, kPackThreads, lds, st>>>(a, w.adj, w.flags, w.block_start, w.next, out_off, nblocks, out,
                                                   w.big_list, w.big_count);
  enc_pack_big_kernel<<<uint32_t(num_cus), 64, kTabBytes + kPackBigCap, st>>>(
      a, w.adj, w.flags, w.block_start, w.next, out_off, out, w.big_list, w.big_count, w.status);
  return hipGetLastError();
}

size_t snappy_slots_bytes(uint64_t raw_total, uint64_t nblocks) {
  return align16(raw_total + raw_total / 6 + 48 * nblocks) + 64;
}

hipError_t launch_pack_snappy(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, uint32_t nblocks,
                              const uint64_t* raw_off, uint8_t* slots, uint64_t* csize, int num_cus) {
  if (nblocks == 0) return hipGetLastError();
  const size_t lds = kTabBytes + (kSnapThreads / 64) * size_t(kSnapWaveBytes);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&enc_pack_snappy_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  uint32_t grid = min(blocks_for(nblocks, kSnapThreads / 64), uint32_t(num_cus) * uint32_t(163840 / lds));
  enc_pack_snappy_kernel<<<grid, kSnapThreads, lds, st>>>(a, w.adj, w.flags, w.block_start, w.next, raw_off, nblocks,
                                                          slots, csize, w.big_list, w.big_count);
  return hipGetLastError();
}

hipError_t launch_pack_snappy_big(hipStream_t st, const EncodeArgs& a, const EncodeBufs& w, const uint64_t* raw_off,
                                  uint8_t* rawbuf, uint8_t* slots, uint64_t* csize, uint32_t big_count, int num_cus) {
  if (big_count == 0) return hipGetLastError();
  const size_t lds = kTabBytes + kSnapMaxTable * 3;
  enc_pack_snappy_big_kernel<<<min(big_count, uint32_t(num_cus) * 2), 64, lds, st>>>(
      a, w.adj, w.flags, w.block_start, w.next, raw_off, rawbuf, slots, csize, w.big_list, w.big_count);
  return hipGetLastError();
}

hipError_t launch_compact(hipStream_t st, const uint8_t* slots, const uint64_t* raw_off, const uint64_t* final_off,
                          uint32_t nblocks, uint8_t* out, int num_cus) {
  if (nblocks == 0) return hipGetLastError();
  enc_compact_kernel<<<min(blocks_for(nblocks, 4), uint32_t(num_cus) * 8), 256, 0, st>>>(slots, raw_off, final_off,
                                                                                       nblocks, out);
  return hipGetLastError();
}

hipError_t launch_snappy_chunks(hipStream_t st, const uint8_t* src, uint64_t n, uint8_t* dst, uint32_t* len,
                                int num_cus) {
  const uint64_t nchunks = (n + kSnapMaxBlock - 1) / kSnapMaxBlock;
  if (nchunks == 0) return hipGetLastError();
  const size_t lds = kSnapMaxTable * 3 + kSnapMaxBlock + 64;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_chunks_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  snappy_chunks_kernel<<<uint32_t(std::min<uint64_t>(nchunks, uint64_t(num_cus))), 64, lds, st>>>(src, n, dst, len);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void snappy_gather_kernel(const uint8_t* __restrict__ slots,
                                                            const uint32_t* __restrict__ len,
                                                            const uint64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  const uint64_t c = blockIdx.x;
  const uint32_t n = len[c];
  const uint8_t* s = slots + c * kSnapChunkSlot;
  uint8_t* o = dst + off[c];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) o[i] = s[i];
}

hipError_t launch_snappy_gather(hipStream_t st, const uint8_t* slots, const uint32_t* len, const uint64_t* off,
                                uint64_t nch, uint8_t* dst) {
  if (nch) snappy_gather_kernel<<<uint32_t(nch), 256, 0, st>>>(slots, len, off, dst);
  return hipGetLastError();
}

hipError_t launch_bloom_build(hipStream_t st, const uint64_t* hashes, uint64_t n, uint32_t num_probes,
                              uint32_t filter_bits, uint32_t* words) {
  if (n == 0) return hipGetLastError();
  bloom_build_kernel<<<uint32_t((n + 255) / 256), 256, 0, st>>>(hashes, n, num_probes, filter_bits, words);
  return hipGetLastError();
}

namespace {
struct BktShape {
  uint32_t n_slices = 0, n_wg = 0;
  uint64_t cells = 0;
  size_t o_scan = 0, o_probes = 0, bytes = 0;
};
BktShape bkt_shape(uint64_t n, uint32_t num_probes, uint32_t filter_bits) {
  BktShape b;
  if (n < 65536 || num_probes == 0 || filter_bits == 0) return b;  // small filters: the atomic kernel
  const uint64_t slices = (uint64_t(filter_bits) + (1ull << kBktSliceLog) - 1) >> kBktSliceLog;
  const uint64_t wg = (n + kBktKeys - 1) / kBktKeys;
  const uint64_t cells = slices * wg;
  if (slices > kBktMaxSlices || cells > kBktMaxCells || n * num_probes >= (1ull << 32)) return b;
  b.n_slices = uint32_t(slices);
  b.n_wg = uint32_t(wg);
  b.cells = cells;
  b.o_scan = ((cells + 1) * 8 + 255) & ~size_t(255);
  b.o_probes = b.o_scan + ((scan_scratch_bytes(uint32_t(cells + 1)) + 255) & ~size_t(255));
  b.bytes = b.o_probes + n * num_probes * 4 + 64;
  return b;
}
}  // namespace

size_t bloom_bucket_scratch_bytes(uint64_t n, uint32_t num_probes, uint32_t filter_bits) {
  return bkt_shape(n, num_probes, filter_bits).bytes;
}

hipError_t launch_bloom_build_bucketed(hipStream_t st, const uint64_t* hashes, uint64_t n, uint32_t num_probes,
                                       uint32_t filter_bits, uint32_t* words, void* scratch) {
  const BktShape b = bkt_shape(n, num_probes, filter_bits);
  if (!b.bytes || !scratch) return launch_bloom_build(st, hashes, n, num_probes, filter_bits, words);
  uint8_t* base = static_cast<uint8_t*>(scratch);
  uint64_t* cells = reinterpret_cast<uint64_t*>(base);
  uint32_t* probes = reinterpret_cast<uint32_t*>(base + b.o_probes);
  bloom_count_kernel<<<b.n_wg, kBktThreads, 0, st>>>(hashes, n, num_probes, filter_bits, b.n_slices, cells);
  hipError_t e = hipMemsetAsync(cells + b.cells, 0, 8, st);
  if (e == hipSuccess) e = launch_scan_u64(st, cells, uint32_t(b.cells + 1), base + b.o_scan);
  if (e != hipSuccess) return e;
  bloom_scatter_kernel<<<b.n_wg, kBktThreads, 0, st>>>(hashes, n, num_probes, filter_bits, b.n_slices, cells, probes);
  bloom_or_kernel<<<b.n_slices, kBktOrThreads, 0, st>>>(cells, b.n_wg, probes, filter_bits, words);
  return hipGetLastError();
}

hipError_t launch_bloom_check(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                              const uint8_t* bits, uint64_t bits_len, uint32_t num_probes, uint8_t* out) {
  if (n == 0) return hipGetLastError();
  bloom_check_kernel<<<uint32_t((n + 255) / 256), 256, 0, st>>>(keys, key_off, n, bits, bits_len, num_probes, out);
  return hipGetLastError();
}

size_t crc_scratch_bytes(uint64_t n) { return ((n + 16) / (16 * kCrcStripeChunks) + 2) * 4 + 16; }

hipError_t launch_crc32(hipStream_t st, const uint8_t* data, uint64_t n, uint32_t* scratch, uint32_t* out,
                        int num_cus) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&crc_stripes_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(kCrcLds));
  if (attr != hipSuccess) return attr;
  const uint64_t sh = reinterpret_cast<uintptr_t>(data) & 15;
  const uint64_t body = (sh + n) / 16 * 16 >= sh + 4 ? (sh + n) / 16 : 0;
  const uint64_t stripes = (body + kCrcStripeChunks - 1) / kCrcStripeChunks;
  if (stripes) {
    const uint64_t wgs = (stripes + kCrcThreads / 64 - 1) / (kCrcThreads / 64);
    const uint32_t grid = uint32_t(std::min<uint64_t>(wgs, uint64_t(std::max(num_cus, 1)) * 2));
    crc_stripes_kernel<<<grid, kCrcThreads, kCrcLds, st>>>(data, n, scratch);
  }
  crc_join_kernel<<<1, 64, 0, st>>>(data, n, scratch, out);
  return hipGetLastError();
}

// ------------------------------------------------------ builder KV staging (device side)
// Pending KVs live in device arrays; appended batches are rebased onto them.
__global__ void kv_rebase_kernel(const uint64_t* __restrict__ src, uint64_t n, uint64_t* __restrict__ dst,
                                 uint64_t base) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i <= n) dst[i] = base + (src[i] - src[0]);
}

__global__ void kv_tomb_kernel(const uint64_t* __restrict__ val_off, uint64_t n, uint8_t* __restrict__ tomb) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) tomb[i] = val_off[i + 1] == val_off[i] ? 1 : 0;
}

// index of the first empty key (block.go:163 assert), or n
__global__ void kv_first_empty_kernel(const uint64_t* __restrict__ key_off, uint64_t n, unsigned long long* out) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && key_off[i + 1] == key_off[i]) atomicMin(out, static_cast<unsigned long long>(i));
}

__global__ void kv_pick_len_kernel(const uint32_t* __restrict__ idx, uint64_t m, const uint64_t* __restrict__ key_off,
                                   uint64_t* __restrict__ len) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < m) len[i] = key_off[idx[i] + 1] - key_off[idx[i]];
  if (i == m) len[m] = 0;
}

// one lane per picked key (a block's first key: a few dozen bytes), 16 loads in flight per lane; a
// key longer than kPickLane bytes is copied by the whole wave afterwards, one such key at a time
constexpr uint32_t kPickLane = 256;
__global__ __launch_bounds__(256) void kv_pick_copy_kernel(const uint32_t* __restrict__ idx, uint64_t m,
                                                           const uint8_t* __restrict__ keys,
                                                           const uint64_t* __restrict__ key_off,
                                                           const uint64_t* __restrict__ out_off,
                                                           uint8_t* __restrict__ out) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t s = 0, l = 0, o = 0;
  if (i < m) {
    s = key_off[idx[i]];
    l = key_off[idx[i] + 1] - s;
    o = out_off[i];
  }
  if (l <= kPickLane) {
    for (uint64_t k = 0; k < l; k += 16) {
      uint8_t v[16];
#pragma unroll
      for (uint32_t t = 0; t < 16; t++) v[t] = k + t < l ? keys[s + k + t] : 0;
#pragma unroll
      for (uint32_t t = 0; t < 16; t++)
        if (k + t < l) out[o + k + t] = v[t];
    }
  }
  uint64_t longs = __ballot(l > kPickLane);
  while (longs) {
    const int src = __builtin_ctzll(longs);
    longs &= longs - 1;
    const uint64_t ws = __shfl(s, src, 64), wl = __shfl(l, src, 64), wo = __shfl(o, src, 64);
    for (uint64_t k = lane; k < wl; k += 64) out[wo + k] = keys[ws + k];
  }
}

hipError_t launch_kv_rebase(hipStream_t st, const uint64_t* src, uint64_t n, uint64_t* dst, uint64_t base) {
  kv_rebase_kernel<<<uint32_t((n + 256) / 256), 256, 0, st>>>(src, n, dst, base);
  return hipGetLastError();
}

hipError_t launch_kv_tomb_from_values(hipStream_t st, const uint64_t* val_off, uint64_t n, uint8_t* tomb) {
  if (n) kv_tomb_kernel<<<uint32_t((n + 255) / 256), 256, 0, st>>>(val_off, n, tomb);
  return hipGetLastError();
}

hipError_t launch_kv_first_empty(hipStream_t st, const uint64_t* key_off, uint64_t n, uint64_t* out) {
  hipError_t e = hipMemsetAsync(out, 0xFF, 8, st);
  if (e != hipSuccess) return e;
  if (n)
    kv_first_empty_kernel<<<uint32_t((n + 255) / 256), 256, 0, st>>>(key_off, n,
                                                                      reinterpret_cast<unsigned long long*>(out));
  return hipGetLastError();
}

size_t kv_pick_scratch_bytes(uint64_t m) { return scan_scratch_bytes(uint32_t(m + 1)) + 64; }

hipError_t launch_kv_pick_keys(hipStream_t st, const uint32_t* idx, uint64_t m, const uint8_t* keys,
                               const uint64_t* key_off, uint64_t* out_off, void* scratch, uint8_t* out) {
  kv_pick_len_kernel<<<uint32_t((m + 256) / 256), 256, 0, st>>>(idx, m, key_off, out_off);
  hipError_t e = launch_scan_u64(st, out_off, uint32_t(m + 1), scratch);
  if (e != hipSuccess) return e;
  if (m) kv_pick_copy_kernel<<<uint32_t((m + 255) / 256), 256, 0, st>>>(idx, m, keys, key_off, out_off, out);
  return hipGetLastError();
}

}  // namespace slate
