// Seeks for the point-read path (slatedb/db.go:291-315 reads through them):
//   block_seek_kernel  block.NewIteratorAtKey (internal/sstable/block/iterator.go:31-82) with
//                      firstFullKey's corrupted-first-key recovery (:117-132) and its warnings,
//                      over blocks decoded by the block decode kernels;
//   index_seek_kernel  sstable.Iterator.firstBlockIncludingOrAfterKey (iterator.go:123-153)
//                      over an SST index's first keys.
// One thread per query: each query is a short dependent chain (a binary search over a
// block's rows or an index), and a batch of point reads supplies the parallelism.
#include "common.h"
#include "kernels.h"

namespace slate {

namespace {

constexpr uint32_t kSeekWaveRows = 2048;  // rows of a block the wave-cooperative point read takes

__device__ inline int cmp_bytes(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  const uint32_t m = an < bn ? an : bn;
  for (uint32_t i = 0; i < m; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return an < bn ? -1 : (an > bn ? 1 : 0);
}

// row.go:265-288 PeekAtKey: status, prefix length, suffix length
__device__ inline int peek(const uint8_t* p, uint32_t n, uint32_t fk_len, uint32_t* pl, uint32_t* sl) {
  if (n < 4) return SLATE_E_ROW_PEEK_SHORT;
  *pl = ld_be16(p);
  *sl = ld_be16(p + 2);
  if (*pl > fk_len) return SLATE_E_ROW_PREFIX;
  if (n - 4 < *sl) return SLATE_E_ROW_SUFFIX;
  return SLATE_OK;
}

}  // namespace

__device__ __forceinline__ void seek_one(uint64_t q, const uint8_t* data, const uint64_t* out_off,
                                         const slate_block_meta* meta, const uint32_t* qblock, const uint8_t* qkeys,
                                         const uint64_t* qkey_off, slate_seek* res, slate_seek_warn* wout,
                                         uint32_t wcap);

__global__ void block_seek_kernel(const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                                  const uint32_t* qblock, const uint8_t* qkeys, const uint64_t* qkey_off, uint64_t nq,
                                  slate_seek* res, slate_seek_warn* wout, uint32_t wcap) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  seek_one(q, data, out_off, meta, qblock, qkeys, qkey_off, res, wout, wcap);
}

// One query by one wave (the point-read form with nq == 1): the same result and warnings as
// seek_one, with the per-row work done by all lanes at once.  The first-full-key scan classifies
// every row in parallel and takes the first that stops it; the binary search's probes are
// evaluated for every row in parallel (row h of the search: offset check, PeekAtKey, v0FullKey
// compare) into outcome[] (LDS), and lane 0 then walks the search over them, adding the warnings
// of the rows it visits in visit order -- so the warnings are exactly the serial search's.
__device__ void seek_one_wave(const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                              const uint32_t* qblock, const uint8_t* qkeys, const uint64_t* qkey_off, slate_seek* res,
                              slate_seek_warn* wout, uint32_t wcap, uint32_t lane, uint32_t* outcome) {
  slate_seek r{};
  r.first_idx = -1;
  uint32_t warn = 0;
  auto add = [&](uint32_t kind, int err, uint32_t x, uint32_t y) {  // (lane 0 only)
    if (wout && warn < wcap) {
      slate_seek_warn w{};
      w.kind = uint16_t(kind);
      w.err = int16_t(err);
      w.a = x;
      w.b = y;
      wout[warn] = w;
    }
    warn++;
  };
  const uint32_t b = qblock[0];
  const slate_block_meta m = meta[b];
  const uint8_t* key = qkeys + qkey_off[0];
  const uint32_t kl = uint32_t(qkey_off[1] - qkey_off[0]);
  if (m.status != SLATE_OK) {
    r.status = m.status;
    if (lane == 0) res[0] = r;
    return;
  }
  const uint8_t* d = data + out_off[b];
  const uint32_t dlen = m.data_len, n = m.n_rows;
  const uint8_t* offs = d + dlen;
  if (n == 0) {
    r.status = SLATE_E_SEEK_NO_OFFSETS;
    if (lane == 0) res[0] = r;
    return;
  }
  // firstFullKey: rows classified in parallel; the first panic or prefix-0 row ends the scan
  int32_t idx = -1;
  uint32_t fk_off = 0, fk_len = 0;
  bool panic = false;
  for (uint32_t i0 = 0; i0 < n && idx < 0 && !panic; i0 += 64) {
    const uint32_t i = i0 + lane;
    const bool in = i < n;
    const uint32_t o = in ? ld_be16(offs + 2 * i) : 0u;
    const bool pan = in && o > dlen;
    uint32_t pl = 0, sl = 0;
    const int e = (in && !pan) ? peek(d + o, dlen - o, 0, &pl, &sl) : SLATE_OK;
    const bool perr = in && !pan && e != SLATE_OK;
    const bool full = in && !pan && e == SLATE_OK && pl == 0;
    const uint64_t stop = __ballot(pan || full);
    const uint32_t f = stop ? uint32_t(__builtin_ctzll(stop)) : 64u;  // the row that ends the scan
    // the peek warnings of the rows before it, in order
    const uint64_t wm = __ballot(perr) & ((f < 64) ? ((uint64_t(1) << f) - 1) : ~uint64_t(0));
    for (uint64_t mm = wm; mm; mm &= mm - 1) {
      const int l = __builtin_ctzll(mm);
      const int el = __shfl(e, l, 64);
      const uint32_t ol = __shfl(o, l, 64);
      if (lane == 0) add(SLATE_WARN_PEEK_FIRST_KEY, el, ol, 0);
    }
    if (f < 64) {
      panic = __shfl(int(pan), int(f), 64) != 0;
      if (!panic) {
        idx = int32_t(i0 + f);
        fk_off = uint32_t(__shfl(o, int(f), 64)) + 4;
        fk_len = uint32_t(__shfl(sl, int(f), 64));
      }
    }
  }
  if (panic) {
    r.status = SLATE_E_SEEK_PANIC;
    r.n_warn = __builtin_amdgcn_readfirstlane(warn);
    if (lane == 0) res[0] = r;
    return;
  }
  if (idx < 0) {
    r.status = SLATE_E_SEEK_NO_FULL_KEY;
    if (lane == 0) add(SLATE_WARN_NO_FULL_KEY, SLATE_OK, 0, 0);
    r.n_warn = __builtin_amdgcn_readfirstlane(warn);
    if (lane == 0) res[0] = r;
    return;
  }
  r.first_idx = idx;
  r.first_len = uint16_t(fk_len);
  const uint8_t* fk = d + fk_off;
  if (cmp_bytes(fk, fk_len, key, kl) == 0) {
    r.start = 0;
    r.n_warn = __builtin_amdgcn_readfirstlane(warn);
    if (lane == 0) res[0] = r;
    return;
  }
  // every probe of the search, in parallel: outcome bit 0 = ok (row >= key), bits 1-2 = warning
  // kind (1 offset bounds, 2 peek), bits 16-31 = the offset or the peek status
  const uint32_t rows = n - uint32_t(idx);
  for (uint32_t h0 = 0; h0 < rows; h0 += 64) {
    const uint32_t h = h0 + lane;
    if (h < rows) {
      const uint32_t o = ld_be16(offs + 2 * (h + uint32_t(idx)));
      uint32_t out = 0;
      uint32_t pl, sl;
      int e = SLATE_OK;
      if (o > uint32_t(uint16_t(dlen))) {
        out = 2u | (o << 16);
      } else if ((e = peek(d + o, dlen - o, fk_len, &pl, &sl)) != SLATE_OK) {
        out = 4u | (uint32_t(uint16_t(int16_t(e))) << 16);
      } else {
        const uint32_t fl = pl + sl, mm = fl < kl ? fl : kl;
        int c = 0;
        for (uint32_t i = 0; i < mm && !c; i++) {
          const uint8_t x = i < pl ? fk[i] : d[o + 4 + (i - pl)];
          if (x != key[i]) c = x < key[i] ? -1 : 1;
        }
        if (!c) c = fl < kl ? -1 : (fl > kl ? 1 : 0);
        out = c >= 0 ? 1u : 0u;
      }
      outcome[h] = out;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    uint32_t lo = 0, hi = rows;
    while (lo < hi) {
      const uint32_t h = (lo + hi) >> 1;
      const uint32_t out = outcome[h];
      if (out & 2u) add(SLATE_WARN_OFFSET_BOUNDS, SLATE_OK, h + uint32_t(idx), out >> 16);
      else if (out & 4u) add(SLATE_WARN_PEEK_ROW, int(int16_t(uint16_t(out >> 16))), h + uint32_t(idx), 0);
      if (!(out & 1u)) lo = h + 1;
      else hi = h;
    }
    r.start = lo + uint32_t(idx);
    r.n_warn = warn;
    r.status = SLATE_OK;
    res[0] = r;
  }
}

// The point-read form (one workgroup, nq <= 256): the inputs, packed by the host into page-locked
// staging in the device layout, are copied into device memory by the kernel itself -- one burst
// over the link in place of a separate copy call -- then searched as above; the results go straight
// back into the staging through its device address.
// kLds: the staged inputs go to LDS (a point read's block and key: a few KiB), so the search's
// dependent reads are LDS round trips instead of L2 ones; otherwise to device memory at base.
template <bool kLds>
__global__ __launch_bounds__(256) void block_seek_staged_kernel(const uint4* __restrict__ hsrc, uint64_t chunks,
                                                                uint4* __restrict__ base, size_t o_data, size_t o_off,
                                                                size_t o_meta, size_t o_q, size_t o_keys,
                                                                size_t o_koff, uint64_t nq, slate_seek* res,
                                                                slate_seek_warn* wout, uint32_t wcap) {
  extern __shared__ __attribute__((aligned(16))) uint4 stage[];
  uint4* dst = kLds ? stage : base;
  for (uint64_t c = threadIdx.x; c < chunks; c += 4 * blockDim.x) {  // four 16-byte chunks in flight
    uint4 v[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) v[u] = hsrc[min(c + u * blockDim.x, chunks - 1)];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++)
      if (c + u * blockDim.x < chunks) dst[c + u * blockDim.x] = v[u];
  }
  __threadfence_block();
  __syncthreads();
  const uint8_t* b = reinterpret_cast<const uint8_t*>(dst);
  const slate_block_meta* mt = reinterpret_cast<const slate_block_meta*>(b + o_meta);
  if (kLds && nq == 1 && mt[reinterpret_cast<const uint32_t*>(b + o_q)[0]].n_rows <= kSeekWaveRows) {
    // a point read: the wave-cooperative form, its outcome table after the stage
    if (threadIdx.x < 64)
      seek_one_wave(b + o_data, reinterpret_cast<const uint64_t*>(b + o_off),
                    reinterpret_cast<const slate_block_meta*>(b + o_meta), reinterpret_cast<const uint32_t*>(b + o_q),
                    b + o_keys, reinterpret_cast<const uint64_t*>(b + o_koff), res, wout, wcap, threadIdx.x,
                    reinterpret_cast<uint32_t*>(dst + chunks));
    return;
  }
  const uint64_t q = threadIdx.x;
  if (q >= nq) return;
  seek_one(q, b + o_data, reinterpret_cast<const uint64_t*>(b + o_off), reinterpret_cast<const slate_block_meta*>(b + o_meta),
           reinterpret_cast<const uint32_t*>(b + o_q), b + o_keys, reinterpret_cast<const uint64_t*>(b + o_koff), res,
           wout, wcap);
}

__device__ __forceinline__ void seek_one(uint64_t q, const uint8_t* data, const uint64_t* out_off,
                                         const slate_block_meta* meta, const uint32_t* qblock, const uint8_t* qkeys,
                                         const uint64_t* qkey_off, slate_seek* res, slate_seek_warn* wout,
                                         uint32_t wcap) {
  uint32_t warn = 0;
  // types.ErrWarn.Add, in order: the first wcap warnings are recorded, all are counted
  auto add = [&](uint32_t kind, int err, uint32_t x, uint32_t y) {
    if (wout && warn < wcap) {
      slate_seek_warn w{};
      w.kind = uint16_t(kind);
      w.err = int16_t(err);
      w.a = x;
      w.b = y;
      wout[q * wcap + warn] = w;
    }
    warn++;
  };
  slate_seek r{};
  r.first_idx = -1;
  const uint32_t b = qblock[q];
  const slate_block_meta m = meta[b];
  const uint8_t* key = qkeys + qkey_off[q];
  const uint32_t kl = uint32_t(qkey_off[q + 1] - qkey_off[q]);
  if (m.status != SLATE_OK) {  // the block failed block.Decode: no iterator exists for it
    r.status = m.status;
    res[q] = r;
    return;
  }
  const uint8_t* d = data + out_off[b];
  const uint32_t dlen = m.data_len, n = m.n_rows;
  const uint8_t* offs = d + dlen;  // BE16 Offsets after Data
  if (n == 0) {
    r.status = SLATE_E_SEEK_NO_OFFSETS;  // iterator.go:32-34
    res[q] = r;
    return;
  }
  // firstFullKey: the first row that PeekAtKey(Data[off:], nil) accepts has keyPrefixLen 0
  int32_t idx = -1;
  uint32_t fk_off = 0, fk_len = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t o = ld_be16(offs + 2 * i);
    if (o > dlen) {  // block.Data[offset:] panics
      r.status = SLATE_E_SEEK_PANIC;
      r.n_warn = warn;
      res[q] = r;
      return;
    }
    uint32_t pl, sl;
    const int e = peek(d + o, dlen - o, 0, &pl, &sl);
    if (e != SLATE_OK) {
      add(SLATE_WARN_PEEK_FIRST_KEY, e, o, 0);  // iterator.go:121
      continue;
    }
    if (pl == 0) {
      idx = int32_t(i);
      fk_off = o + 4;
      fk_len = sl;
      break;
    }
  }
  if (idx < 0) {  // iterator.go:130-131 -> :41-47
    r.status = SLATE_E_SEEK_NO_FULL_KEY;
    add(SLATE_WARN_NO_FULL_KEY, SLATE_OK, 0, 0);  // iterator.go:130
    r.n_warn = warn;
    res[q] = r;
    return;
  }
  r.first_idx = idx;
  r.first_len = uint16_t(fk_len);
  const uint8_t* fk = d + fk_off;
  if (cmp_bytes(fk, fk_len, key, kl) == 0) {  // iterator.go:51-58: offsetIndex 0
    r.start = 0;
    r.n_warn = warn;
    res[q] = r;
    return;
  }
  // sort.Search(len(Offsets) - idx, ...) over PeekAtKey + v0FullKey (iterator.go:62-74)
  uint32_t lo = 0, hi = n - uint32_t(idx);
  while (lo < hi) {
    const uint32_t h = (lo + hi) >> 1;
    const uint32_t o = ld_be16(offs + 2 * (h + uint32_t(idx)));
    bool ok = false;
    uint32_t pl, sl;
    int e = SLATE_OK;
    if (o > uint32_t(uint16_t(dlen))) {
      add(SLATE_WARN_OFFSET_BOUNDS, SLATE_OK, h + uint32_t(idx), o);  // iterator.go:65
    } else if ((e = peek(d + o, dlen - o, fk_len, &pl, &sl)) != SLATE_OK) {
      add(SLATE_WARN_PEEK_ROW, e, h + uint32_t(idx), 0);  // iterator.go:70
    } else {
      // v0FullKey = firstKey[:prefixLen] || suffix, compared with the sought key
      const uint32_t fl = pl + sl, mm = fl < kl ? fl : kl;
      int c = 0;
      for (uint32_t i = 0; i < mm && !c; i++) {
        const uint8_t x = i < pl ? fk[i] : d[o + 4 + (i - pl)];
        if (x != key[i]) c = x < key[i] ? -1 : 1;
      }
      if (!c) c = fl < kl ? -1 : (fl > kl ? 1 : 0);
      ok = c >= 0;
    }
    if (!ok) lo = h + 1;
    else hi = h;
  }
  r.start = lo + uint32_t(idx);
  r.n_warn = warn;
  r.status = SLATE_OK;
  res[q] = r;
}

__global__ void index_seek_kernel(const uint8_t* keys, const uint64_t* key_off, uint64_t n_blocks, const uint8_t* qkeys,
                                  const uint64_t* qkey_off, uint64_t nq, uint64_t* out) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const uint8_t* key = qkeys + qkey_off[q];
  const uint32_t kl = uint32_t(qkey_off[q + 1] - qkey_off[q]);
  int64_t low = 0, high = int64_t(n_blocks) - 1, found = 0;
  while (low <= high) {
    const int64_t mid = low + (high - low) / 2;
    const int c = cmp_bytes(keys + key_off[mid], uint32_t(key_off[mid + 1] - key_off[mid]), key, kl);
    if (c < 0) {
      low = mid + 1;
      found = mid;
    } else if (c > 0) {
      if (mid > 0) high = mid - 1;
      else break;
    } else {
      found = mid;
      break;
    }
  }
  out[q] = uint64_t(found);
}

hipError_t launch_block_seek(hipStream_t st, const uint8_t* data, const uint64_t* out_off, const slate_block_meta* meta,
                             const uint32_t* qblock, const uint8_t* qkeys, const uint64_t* qkey_off, uint64_t nq,
                             slate_seek* res, slate_seek_warn* warn, uint32_t warn_cap) {
  if (nq == 0) return hipSuccess;
  block_seek_kernel<<<uint32_t((nq + 255) / 256), 256, 0, st>>>(data, out_off, meta, qblock, qkeys, qkey_off, nq, res,
                                                                 warn, warn_cap);
  return hipGetLastError();
}

hipError_t launch_block_seek_staged(hipStream_t st, const void* hsrc_dev, size_t bytes, void* base, size_t o_data,
                                    size_t o_off, size_t o_meta, size_t o_q, size_t o_keys, size_t o_koff, uint64_t nq,
                                    slate_seek* res, slate_seek_warn* warn, uint32_t warn_cap) {
  if (nq == 0) return hipSuccess;
  if (nq > 256 || (reinterpret_cast<uintptr_t>(hsrc_dev) & 15) || (reinterpret_cast<uintptr_t>(base) & 15))
    return hipErrorInvalidValue;
  const uint64_t chunks = (bytes + 15) / 16;
  // LDS: the staged bytes, then (one query) the search's outcome per row
  if (16 * chunks + 4 * kSeekWaveRows <= 65536)
    block_seek_staged_kernel<true><<<1, 256, 16 * chunks + (nq == 1 ? 4 * kSeekWaveRows : 0), st>>>(static_cast<const uint4*>(hsrc_dev), chunks,
                                                                 static_cast<uint4*>(base), o_data, o_off, o_meta, o_q,
                                                                 o_keys, o_koff, nq, res, warn, warn_cap);
  else
    block_seek_staged_kernel<false><<<1, 256, 0, st>>>(static_cast<const uint4*>(hsrc_dev), chunks,
                                                        static_cast<uint4*>(base), o_data, o_off, o_meta, o_q, o_keys,
                                                        o_koff, nq, res, warn, warn_cap);
  return hipGetLastError();
}

hipError_t launch_index_seek(hipStream_t st, const uint8_t* keys, const uint64_t* key_off, uint64_t n_blocks,
                             const uint8_t* qkeys, const uint64_t* qkey_off, uint64_t nq, uint64_t* out) {
  if (nq == 0) return hipSuccess;
  index_seek_kernel<<<uint32_t((nq + 255) / 256), 256, 0, st>>>(keys, key_off, n_blocks, qkeys, qkey_off, nq, out);
  return hipGetLastError();
}

}  // namespace slate
