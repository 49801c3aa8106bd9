// CodecZstd fast path: lane-per-block parse, wave-per-block build, lane-per-block checksum.
//
// compress.Decode(CodecZstd) (compression.go:146-153) is restated check for check by the
// wave-per-block decoder (zstd.h, the exact path).  That path is latency-bound: one wave walks a
// block's frame, FSE states and XXH64 as serial chains (20.6 ms per 1 M configs[4] blocks).
// Most blocks an SST holds are one simple shape -- one frame, one compressed block, raw or RLE
// literals, predefined or RLE sequence tables, a handful of sequences (configs[4]: 98.7 % of
// blocks, ~7 sequences, ~1.9 KB of raw literals) -- and for that shape the work splits well:
//
//   A  zs_fast_parse_kernel  one LANE per block: the frame header, literal header and the whole
//                            FSE sequence decode (64 blocks' state machines advance in one wave
//                            instruction), every check of zs_frame/zs_block replicated; emits
//                            the literal location and (ll, ml, offset) per sequence
//   A2 zs_fast_crc_kernel    one LANE per block: the SST block's CRC32 over its encoded bytes,
//                            streamed in 64-byte runs (slicing-by-16, 64 blocks per instruction)
//   B  zs_fast_build_kernel  one WAVE per block (the next block's record in flight): stage the
//                            frame in LDS, place all literal runs, then the matches in order (a
//                            byte or a dword per lane), write the block back, block.Decode checks
//                            and rows
//   C  zs_fast_sum_kernel    one LANE per block: the frame's XXH64 over the decoded block,
//                            streamed in 64-byte runs (the four accumulators' serial chains of
//                            64 blocks advance in one wave instruction)
//
// Anything outside the shape, or failing any check (A), or failing the frame checksum (C), is
// appended to a list and decoded by the exact path afterwards (decode.hip decode_list_kernel),
// which then writes that block's meta, bytes and rows; so every status and every byte of such a
// block is the exact path's.  A CRC32 mismatch (A2) is reported directly: it is the first check
// of both paths (block.go:83-89).
// The plan (decoded sizes) has the same split: plan_zstd_fast_kernel (lane per block) for
// single-frame blocks with a content size, the wave plan for the rest.
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"
#include "zstd.h"
#include "rows.h"

namespace slate {

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0xFFFFFFF0u;

// per-lane LDS windows of phase A: the frame's first 32 bytes (three chunks: any alignment)
// and 11 chunks around the sequences section (+16 bytes slack for 8-byte bit reads)
constexpr uint32_t kZfHead = 48;
constexpr uint32_t kZfTailChunks = 11;
constexpr uint32_t kZfTail = 16 * kZfTailChunks + 16;
constexpr uint32_t kZfLane = kZfHead + kZfTail;
constexpr uint32_t kZfParseThreads = 256;
// phase B: one wave per block, seven 4-wave workgroups per CU (72 VGPRs), the decoded block in LDS
// with the frame staged around its tail (the bytes after the literals and the 16-byte phase: +256)
constexpr uint32_t kZfBuildThreads = 256;
#ifndef SLATE_ZF_BUILD_WG
#define SLATE_ZF_BUILD_WG 7  // workgroups per CU (the VGPR budget: 7 -> 72 per lane)
#endif
constexpr uint32_t kZfIn = kZsFastInCap, kZfOut = kZsFastOutCap;
constexpr uint32_t kZfJunk = kZfOut + 256;      // 64 junk dwords (lanes' discarded writes)
constexpr uint32_t kZfOutLds = kZfJunk + 256;
// phase C: 256 bytes of LDS per lane; phase A2: 64 + the slicing-by-16 CRC tables
constexpr uint32_t kZfSumThreads = 256;
constexpr uint32_t kZfCrcThreads = 512;
// phase B': per wave the frame, the decoded block and the Huffman part of a ZsScratch; two 4-wave
// workgroups per CU (one-wave workgroups, eleven per CU, measured 18 % slower)
constexpr uint32_t kZfHufThreads = 256;
constexpr uint32_t kZfHufWave = kZsFastInCap + 16 + kZfOutLds + kZsHufScratch;
constexpr uint32_t kZfBuildLds = (kZfBuildThreads / 64) * kZfOutLds;
constexpr uint32_t kZfHufLds = (kZfHufThreads / 64) * kZfHufWave;
static_assert(SLATE_ZF_BUILD_WG * kZfBuildLds <= 160 * 1024, "phase B workgroups per CU exceed the LDS");
static_assert(2 * kZfHufLds <= 160 * 1024, "phase B' workgroups per CU exceed the LDS");

struct ZfShared {
  ZsShared fse;  // the predefined LL / ML / OF decoding tables
  uint32_t ll_base[36], ml_base[53];
  uint8_t ll_bits[36], ml_bits[53];
};

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
  return (uint64_t(hi) << 32) | lo;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint64_t b = uniform64(reinterpret_cast<uint64_t>(base));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes < kOOB ? uint32_t(bytes) : kOOB);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0, int(n), 0x00020000);
}
#ifndef SLATE_ZF_LDPOL  // cache policy of the phases' streaming loads (0 default, 2 nt)
#define SLATE_ZF_LDPOL 0
#endif
__device__ __forceinline__ v4u bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SLATE_ZF_LDPOL);
}
__device__ __forceinline__ void lds_put16(uint8_t* p, const v4u& v) { *reinterpret_cast<v4u*>(p) = v; }

// wave-aggregated append of the lanes with `want` to list[*count ...]
__device__ __forceinline__ void list_append(bool want, uint32_t item, uint32_t* list, uint32_t* count) {
  const uint64_t m = __ballot(want);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == uint32_t(__builtin_ctzll(m))) base = atomicAdd(count, uint32_t(__builtin_popcountll(m)));
  base = __shfl(base, __builtin_ctzll(m), 64);
  if (want) list[base + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)))] = item;
}

// The frame head of one block (zs_header + the first block header, oracle zs_header /
// zs_frame): bytes hb[i] = frame byte i for i < 32 (clen = frame bytes).  Fills the fields
// and returns true when the frame has the fast shape's head: magic at 0, a valid header
// without dictionary, exactly one block (last), the frame (and its checksum) ending at clen.
struct ZfHead {
  uint32_t body, bs, bt, checksum, has_fcs, bmax;
  uint64_t fcs;
};
__device__ bool zf_head(const uint8_t* hb, uint32_t clen, ZfHead& h) {
  if (clen < 4) return false;
  const uint32_t magic = uint32_t(hb[0]) | (uint32_t(hb[1]) << 8) | (uint32_t(hb[2]) << 16) | (uint32_t(hb[3]) << 24);
  if (magic != 0xFD2FB528u) return false;
  const uint32_t n = clen - 4;  // zs_header(base, off + 4, n - 4)
  if (n < 1) return false;
  const uint32_t fhd = hb[4], fcsf = fhd >> 6, ss = (fhd >> 5) & 1, dif = fhd & 3;
  if (fhd & 8) return false;
  const uint32_t dsz = dif == 3 ? 4 : dif, fl = fcsf == 0 ? ss : (2u << (fcsf - 1));
  const uint32_t hsize = 1 + (ss ? 0 : 1) + dsz + fl;
  if (n < hsize) return false;
  uint32_t q = 5;
  uint64_t window = 0;
  if (!ss) {
    const uint32_t wd = hb[q++], wl = 10 + (wd >> 3);
    window = (1ull << wl) + ((1ull << wl) >> 3) * (wd & 7);
  }
  uint32_t dict = 0;
  for (uint32_t i = 0; i < dsz; i++) dict |= uint32_t(hb[q++]) << (8 * i);
  if (dict != 0) return false;
  uint64_t f = 0;
  for (uint32_t i = 0; i < fl; i++) f |= uint64_t(hb[q + i]) << (8 * i);
  if (fl == 2) f += 256;
  if (ss) window = f;
  if (window > kZsMaxWindow) return false;
  h.has_fcs = fl != 0;
  h.fcs = f;
  h.checksum = (fhd >> 2) & 1;
  h.bmax = uint32_t(window < kZsBlockMax ? window : kZsBlockMax);
  uint32_t p = 4 + hsize;  // <= 18
  if (clen - p < 3) return false;
  const uint32_t bh = uint32_t(hb[p]) | (uint32_t(hb[p + 1]) << 8) | (uint32_t(hb[p + 2]) << 16);
  p += 3;
  h.bt = (bh >> 1) & 3;
  h.bs = bh >> 3;
  if (!(bh & 1) || h.bt == 3 || h.bs > h.bmax) return false;
  const uint32_t adv = h.bt == 1 ? 1 : h.bs;
  if (clen - p < adv) return false;
  h.body = p;
  p += adv;
  if (h.checksum) {
    if (clen - p < 4) return false;
    p += 4;
  }
  return p == clen;
}

// --------------------------------------------------------------- bits of phase A
// The sequences bitstream in a lane's tail window (LDS), read as zs_peek reads it.
struct ZfBits {
  const uint8_t* buf;
  int64_t S, bp;
};
// The stream through a 64-bit register window (phases A and A'): c holds stream bits [lo, lo + 64).
// zf_fill puts at least the 56 bits below bp there (all of them when bp <= 56); zf_take reads
// k <= bp - lo of them (or, with lo = 0, past the stream's start, as zs_peek: zeros below it).
// One LDS round trip per fill instead of one per read.
struct ZfReg {
  uint64_t c;
  int64_t lo;
};
__device__ __forceinline__ void zf_fill(const ZfBits& z, ZfReg& r) {
  r.lo = z.bp > 56 ? ((z.bp - 56) & ~int64_t(7)) : 0;
  const int32_t off = int32_t((z.S + r.lo) >> 3);  // (S is a byte boundary)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(z.buf + (off & ~3));
  const uint32_t sh = uint32_t(off) & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
  r.c = uint64_t(__builtin_amdgcn_alignbyte(w1, w0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32);
}
__device__ __forceinline__ uint32_t zf_take(ZfBits& z, const ZfReg& r, uint32_t k) {
  const int64_t t = z.bp - int64_t(k);
  const uint64_t x = t >= 0 ? r.c >> uint32_t(t - r.lo) : r.c << uint32_t(-t);
  const uint32_t v = z.bp > 0 ? uint32_t(x & ((1ull << k) - 1)) : 0u;
  z.bp = t;
  return v;
}

}  // namespace

// ------------------------------------------------------------------------------- plan
// Lane per block: single-frame blocks with a content size get or_zstd_plan's size here
// (min(content size, the block's bound)); every other block goes to `list` for the wave plan.
__global__ __launch_bounds__(kZfParseThreads) void plan_zstd_fast_kernel(const uint8_t* __restrict__ in,
                                                                         const uint64_t* __restrict__ in_off, uint32_t n,
                                                                         uint64_t* __restrict__ out_sz,
                                                                         uint64_t* __restrict__ row_sz, uint32_t* list,
                                                                         uint32_t* count) {
  __shared__ __attribute__((aligned(16))) uint8_t heads[kZfParseThreads * kZfHead];
  uint8_t* hb0 = heads + threadIdx.x * kZfHead;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); r0 < n; r0 += stride) {
    const uint32_t b = r0 + (threadIdx.x & 63);
    const uint32_t rend = min(r0 + 64, n);
    const uint8_t* lo = in + in_off[r0];
    const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(lo) & ~uintptr_t(15));
    const __amdgpu_buffer_rsrc_t R = make_rsrc(base, align16(uint64_t((in + in_off[rend]) - base)));
    bool fast = false;
    uint64_t dl = 0;
    uint32_t shift = 0, rel = kOOB;
    uint64_t len = 0;
    if (b < n) {
      const uint64_t s0 = in_off[b];
      len = in_off[b + 1] - s0;
      shift = uint32_t(reinterpret_cast<uintptr_t>(in + s0) & 15);
      if (len >= 6 && len - 4 < 0x7FFFFFFFull) rel = uint32_t(((in + s0) - shift) - base);
    }
    const v4u c0 = bload(R, rel), c1 = bload(R, rel == kOOB ? kOOB : rel + 16), c2 = bload(R, rel == kOOB ? kOOB : rel + 32);
    lds_put16(hb0, c0);
    lds_put16(hb0 + 16, c1);
    lds_put16(hb0 + 32, c2);
    if (rel != kOOB) {
      ZfHead h;
      if (zf_head(hb0 + shift, uint32_t(len - 4), h) && h.has_fcs) {
        const uint64_t bound = h.bt == 2 ? h.bmax : h.bs;
        dl = h.fcs < bound ? h.fcs : bound;
        fast = true;
      }
    }
    if (fast) {
      out_sz[b] = align16(dl);
      row_sz[b] = row_capacity(dl);
    }
    list_append(b < n && !fast, b, list, count);
  }
}

// ------------------------------------------------------------------------------- phase A
__global__ __launch_bounds__(kZfParseThreads) void zs_fast_parse_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  ZfShared* sh = reinterpret_cast<ZfShared*>(smem);
  uint8_t* lanes = smem + ((sizeof(ZfShared) + 15) & ~size_t(15));
  {
    // the predefined tables (wave 0, lane 0), with a temporary ZsScratch over the lane windows
    if (threadIdx.x < 64) zs_shared_build(&sh->fse, reinterpret_cast<ZsScratch*>(lanes), int(threadIdx.x));
    for (uint32_t i = threadIdx.x; i < 36; i += blockDim.x) {
      sh->ll_base[i] = kZsLLBase[i];
      sh->ll_bits[i] = kZsLLBits[i];
    }
    for (uint32_t i = threadIdx.x; i < 53; i += blockDim.x) {
      sh->ml_base[i] = kZsMLBase[i];
      sh->ml_bits[i] = kZsMLBits[i];
    }
    __syncthreads();
  }
  uint8_t* hb0 = lanes + threadIdx.x * kZfLane;
  uint8_t* tb0 = hb0 + kZfHead;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); r0 < a.n; r0 += stride) {
    const uint32_t b = r0 + (threadIdx.x & 63);
    const uint32_t rend = min(r0 + 64, a.n);
    const uint8_t* lo = a.in + a.in_off[r0];
    const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(lo) & ~uintptr_t(15));
    const __amdgpu_buffer_rsrc_t R = make_rsrc(base, align16(uint64_t((a.in + a.in_off[rend]) - base)));
    ZsFastRec rec{0, 0, 0, 0, 0, 0, {0, 0}};
    bool ok = false;
    uint32_t shift = 0, rel = kOOB, clen = 0, cap = 0;
    if (b < a.n) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      shift = uint32_t(reinterpret_cast<uintptr_t>(a.in + s0) & 15);
      const uint64_t cap64 = a.out_off[b + 1] - a.out_off[b];
      // the exact path's staging limits (decode_block_wave): beyond them it is not this shape
      if (len >= 6 && shift + len <= kZfIn && cap64 <= kZfOut) {
        rel = uint32_t(((a.in + s0) - shift) - base);
        clen = uint32_t(len - 4);
        cap = uint32_t(cap64);
        ok = true;
      }
    }
    {
      const v4u c0 = bload(R, rel), c1 = bload(R, ok ? rel + 16 : kOOB), c2 = bload(R, ok ? rel + 32 : kOOB);
      lds_put16(hb0, c0);
      lds_put16(hb0 + 16, c1);
      lds_put16(hb0 + 32, c2);
    }
    const uint8_t* hb = hb0 + shift;
    ZfHead h{};
    ok = ok && zf_head(hb, clen, h) && h.bt == 2;
    // ---- literals section header (zs_block): raw, RLE, or Huffman-coded with a new tree
    uint32_t nlit = 0, pos = 0, lit = 0, rle = 0, huf = 0, cs = 0;
    const uint32_t nb = h.bs, body = h.body;
    if (ok) {
      const uint32_t b0 = hb[body], type = b0 & 3, sf = (b0 >> 2) & 3;
      uint32_t hs;
      if (type == 3) {  // treeless: no earlier tree in a one-block frame (the exact path: corrupt)
        ok = false;
        hs = 1;
      } else if (type == 2) {
        huf = sf == 0 ? 1u : 4u;  // streams
        const uint64_t hh = uint64_t(b0) | (uint64_t(hb[body + 1]) << 8) | (uint64_t(hb[body + 2]) << 16) |
                            (uint64_t(hb[body + 3]) << 24) | (uint64_t(hb[body + 4]) << 32);
        hs = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
        ok = nb >= hs;
        nlit = sf <= 1 ? uint32_t((hh >> 4) & 0x3FF) : (sf == 2 ? uint32_t((hh >> 4) & 0x3FFF) : uint32_t((hh >> 4) & 0x3FFFF));
        cs = sf <= 1 ? uint32_t((hh >> 14) & 0x3FF) : (sf == 2 ? uint32_t((hh >> 18) & 0x3FFF) : uint32_t((hh >> 22) & 0x3FFFF));
        ok = ok && nlit <= h.bmax && nb - hs >= cs && nlit <= cap;
        lit = body + hs;
        pos = hs + cs;
      } else if (sf == 1) {
        hs = 2;
        ok = nb >= 2;
        nlit = (b0 >> 4) + (uint32_t(hb[body + 1]) << 4);
      } else if (sf == 3) {
        hs = 3;
        ok = nb >= 3;
        nlit = (b0 >> 4) + (uint32_t(hb[body + 1]) << 4) + (uint32_t(hb[body + 2]) << 12);
      } else {
        hs = 1;
        nlit = b0 >> 3;
      }
      if (type <= 1) {
        ok = ok && nb >= 1 && nlit <= h.bmax && (type == 0 ? nb - hs >= nlit : nb - hs >= 1) && nlit <= cap;
        rle = type == 1;
        lit = rle ? uint32_t(hb[body + hs]) : body + hs;
        pos = hs + (type == 0 ? nlit : 1);
      }
      ok = ok && pos < nb;
    }
    // ---- the sequences section: 11 chunks from the one holding its first byte
    const uint32_t s = body + pos;  // frame offset of the sequences section
    const uint32_t c_lo = (shift + s) >> 4;
    const uint32_t wend = 16 * (c_lo + kZfTailChunks) - shift;  // frame offset past the window
    // the whole section (and the checksum) in the window: needed by this parse, not by the
    // deferral to phase A' (which reads its own, larger window) -- a 4 KiB block of 100-byte KVs
    // can have a 164-byte section + checksum
    const bool inwin = body + nb + (h.checksum ? 4u : 0u) <= wend;
    {
      v4u t[kZfTailChunks];
#pragma unroll
      for (uint32_t k = 0; k < kZfTailChunks; k++) t[k] = bload(R, ok ? rel + 16 * (c_lo + k) : kOOB);
#pragma unroll
      for (uint32_t k = 0; k < kZfTailChunks; k++) lds_put16(tb0 + 16 * k, t[k]);
    }
    const uint8_t* tb = tb0 + shift - 16 * c_lo;  // tb[i] = frame byte i for i in [s, wend)
    uint32_t nseq = 0, produced = 0;
    bool defer = false;  // to phase A' (zs_fse_parse_kernel)
    if (ok) {
      const uint32_t sn = nb - pos;
      const uint32_t c0 = tb[s];
      uint32_t sp;
      if (c0 < 128) {
        nseq = c0;
        sp = 1;
      } else if (c0 < 255) {
        ok = sn >= 2;
        nseq = ((c0 - 128) << 8) + tb[s + 1];
        sp = 2;
      } else {
        ok = sn >= 3;
        nseq = uint32_t(tb[s + 1]) + (uint32_t(tb[s + 2]) << 8) + 0x7F00;
        sp = 3;
      }
      // FSE_Compressed tables, or more than kZsFastSeqs sequences (and no repeat tables, which a
      // one-block frame cannot use): phase A' decodes them
      {
        const uint32_t m0 = (ok && nseq != 0 && sp < sn) ? uint32_t(tb[s + sp]) : 0u;
        const uint32_t a_ll = m0 >> 6, a_of = (m0 >> 4) & 3, a_ml = (m0 >> 2) & 3;
        defer = ok && nseq != 0 && sp < sn && !(m0 & 3) && a_ll != 3 && a_of != 3 && a_ml != 3 &&
                (nseq > kZsFastSeqs || a_ll == 2 || a_of == 2 || a_ml == 2) && nseq <= kZsFseSeqs;
      }
      ok = ok && !defer && nseq <= kZsFastSeqs && inwin;
      uint32_t lp = 0, o = 0;
      const uint32_t lbase = cap - nlit;
      if (ok && nseq == 0) {
        ok = sp == sn;
      } else if (ok) {
        ok = sp < sn;
        const uint32_t modes = ok ? uint32_t(tb[s + sp++]) : 0u;
        ok = ok && !(modes & 3);
        // Symbol_Compression_Mode: predefined (0) or RLE (1) per table, in LL, OF, ML order
        uint32_t m_ll = modes >> 6, m_of = (modes >> 4) & 3, m_ml = (modes >> 2) & 3;
        ok = ok && m_ll <= 1 && m_of <= 1 && m_ml <= 1;
        uint32_t r_ll = 0, r_of = 0, r_ml = 0;
        if (ok && m_ll) {
          ok = sn - sp >= 1 && tb[s + sp] <= 35;
          r_ll = tb[s + sp++];
        }
        if (ok && m_of) {
          ok = sn - sp >= 1 && tb[s + sp] <= 31;
          r_of = tb[s + sp++];
        }
        if (ok && m_ml) {
          ok = sn - sp >= 1 && tb[s + sp] <= 52;
          r_ml = tb[s + sp++];
        }
        // zs_bstart
        const uint32_t bn = sn - sp;
        const uint32_t last = ok && bn ? uint32_t(tb[s + sn - 1]) : 0u;
        ok = ok && last != 0;
        ZfBits bits{tb0, 8 * int64_t(shift + s + sp - 16 * c_lo), ok ? 8 * int64_t(bn - 1) + (31 - __builtin_clz(last)) : 0};
        uint32_t sll = 0, sof = 0, sml = 0;
        ZfReg rg{};  // (the register window of phase A': one fill per sequence, more for long values)
        if (ok) {
          zf_fill(bits, rg);
          sll = zf_take(bits, rg, m_ll ? 0 : 6);
          sof = zf_take(bits, rg, m_of ? 0 : 5);
          sml = zf_take(bits, rg, m_ml ? 0 : 6);
        }
        uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
        uint2* seqs = reinterpret_cast<uint2*>(z.seq + size_t(b) * kZfSeqSlot);
        for (uint32_t i = 0; ok && i < nseq; i++) {
          const ZsFse ell = m_ll ? ZsFse{uint8_t(r_ll), 0, 0} : sh->fse.ll[sll];
          const ZsFse eof = m_of ? ZsFse{uint8_t(r_of), 0, 0} : sh->fse.of[sof];
          const ZsFse eml = m_ml ? ZsFse{uint8_t(r_ml), 0, 0} : sh->fse.ml[sml];
          const uint32_t ofc = eof.sym, llc = ell.sym, mlc = eml.sym;
          if (ofc > 31) {
            ok = false;
            break;
          }
          zf_fill(bits, rg);  // >= 56 bits: the offset's <= 31
          uint64_t ofv = (1ull << ofc);
          if (ofc > 24) {
            const uint32_t hi = zf_take(bits, rg, ofc - 24);
            ofv += (uint64_t(hi) << 24) + zf_take(bits, rg, 24);
          } else {
            ofv += zf_take(bits, rg, ofc);
          }
          const uint32_t mb = sh->ml_bits[mlc], lb = sh->ll_bits[llc];  // (<= 16 each)
          if (rg.lo > 0 && bits.bp - rg.lo < int64_t(mb + lb)) zf_fill(bits, rg);
          const uint32_t ml = sh->ml_base[mlc] + zf_take(bits, rg, mb);
          const uint32_t ll = sh->ll_base[llc] + zf_take(bits, rg, lb);
          uint64_t offv;
          if (ofv > 3) {
            offv = ofv - 3;
            rep2 = rep1;
            rep1 = rep0;
            rep0 = uint32_t(offv);
          } else {
            const uint32_t idx = uint32_t(ofv) - 1 + (ll == 0 ? 1u : 0u);
            offv = idx == 3 ? uint64_t(rep0) - 1 : (idx == 0 ? rep0 : idx == 1 ? rep1 : rep2);
            if (offv == 0) offv = 1;
            if (idx >= 2) rep2 = rep1;
            if (idx >= 1) {
              rep1 = rep0;
              rep0 = uint32_t(offv);
            }
          }
          if (i + 1 < nseq) {
            if (rg.lo > 0 && bits.bp - rg.lo < 18) zf_fill(bits, rg);  // (predefined logs 6 / 5 / 6)
            sll = uint32_t(ell.base) + zf_take(bits, rg, ell.nb);
            sml = uint32_t(eml.base) + zf_take(bits, rg, eml.nb);
            sof = uint32_t(eof.base) + zf_take(bits, rg, eof.nb);
          }
          if (bits.bp < 0 || ll > nlit - lp || uint64_t(o) + ll + ml > h.bmax || uint64_t(o) + ll + ml > cap ||
              uint64_t(o) + ll + ml > uint64_t(lbase) + lp + ll) {
            ok = false;
            break;
          }
          lp += ll;
          o += ll;
          if (offv > o) {  // fstart = 0: one frame
            ok = false;
            break;
          }
          seqs[i] = make_uint2(ll | (ml << 16), uint32_t(offv));
          o += ml;
        }
        ok = ok && bits.bp == 0;
      }
      const uint32_t rest = nlit - lp;
      ok = ok && uint64_t(o) + rest <= h.bmax && uint64_t(o) + rest <= cap;
      produced = o + rest;
      ok = ok && (!h.has_fcs || uint64_t(produced) == h.fcs);
    }
    if (ok) {
      rec.lit = lit;
      rec.nlit = nlit;
      rec.produced = produced;
      rec.info = nseq | ((kZfFast | (rle ? kZfRle : 0u) | (h.checksum ? kZfSum : 0u) | (huf ? kZfHuf | kZfHufOrig : 0u) |
                          (huf == 4 ? kZfHuf4 : 0u))
                         << 16);
      rec.cs = cs;
      const uint32_t q = body + nb;
      rec.want = h.checksum ? uint32_t(tb[q]) | (uint32_t(tb[q + 1]) << 8) | (uint32_t(tb[q + 2]) << 16) |
                                  (uint32_t(tb[q + 3]) << 24)
                            : 0u;
    }
    if (b < a.n) z.rec[b] = rec;
    list_append(b < a.n && !ok && !defer, b, z.list, z.count);
    list_append(b < a.n && ok && huf, b, z.hlist, z.count + 1);
    list_append(b < a.n && defer, b, z.flist, z.count + 2);
  }
}

// ------------------------------------------------------------------------------- phase A'
// Blocks whose sequence tables are FSE_Compressed -- libzstd's choice for a block of many short
// sequences: a 4 KiB block of 100-byte KVs (configs[1]'s shape) has ~112 sequences and LL / OF / ML
// tables of accuracy 6 / 5 / 7 -- or that have 17..128 sequences, from phase A's list: lane per
// block as phase A, each lane building its block's three decoding tables (RFC 8878 4.1.1, zs_ncount
// / zs_fse_build: FSE_Compressed, predefined or RLE) in its own LDS with 16-bit entries (accuracy
// logs <= 7, 224 entries in all), then the sequences as phase A, written as 4-byte records, four per
// store.  Anything else -- a larger table, a length or offset the record cannot hold, any failed
// check -- goes to the exact path, which decodes and reports it.
namespace {
// A lane's LDS: the three tables, then one window used three ways in turn -- the frame's first 48
// bytes (frame and literals headers); the sequences section's first kZfFseHdrChunks chunks (its
// counts, modes and table descriptions) with the table build's scratch after them; the sequences
// bitstream, kZfFseBitChunks chunks from the one holding its first byte (+16 bytes slack for 8-byte
// bit reads).  A 100 B-KV block's headers take <= 31 bytes and its bitstream <= 10 chunks from
// there (tools/kvwin.py over 20 k blocks); the section's chunks stay in registers between the
// stages.  624 bytes per lane: four one-wave workgroups per CU, one per SIMD.
constexpr uint32_t kZfFseThreads = 64;
constexpr uint32_t kZfFseHdrChunks = 4;
constexpr uint32_t kZfFseBitChunks = 10;
constexpr uint32_t kZfFseRegChunks = 14;  // chunks c_lo .. c_lo + 13 of the section held in registers
constexpr uint32_t kZfFseTab = 224;       // u16 entries, the LL, OF and ML tables back to back
constexpr uint32_t kZfFseScr = 112;       // int8 norm[53] + u8 next[53] (groups of eight: 56 each)
constexpr uint32_t kZfFseWin = 16 * kZfFseBitChunks + 16;
constexpr uint32_t kZfFseLane = 2 * kZfFseTab + kZfFseWin;
constexpr uint32_t kZfFseWgs = 4;  // per CU
static_assert(kZfFseLane % 16 == 0, "lane records stay 16-byte aligned");
static_assert(16 * kZfFseHdrChunks + kZfFseScr <= kZfFseWin && kZfHead <= kZfFseWin, "the window's three uses");
static_assert(kZfFseWgs * (kZfFseThreads * kZfFseLane + 512) <= 160 * 1024, "phase A' workgroups per CU exceed the LDS");

// A forward stream base[off, off + n) through a 64-bit register window: c holds stream bits
// [lo, lo + 64), lo a byte boundary, bits past the stream's end read as zeros (zs_fbits).
struct ZfFwd {
  uint64_t c;
  uint32_t lo;
};
__device__ __forceinline__ void zf_ffill(const uint8_t* base, int32_t off, uint32_t n, uint32_t bp, ZfFwd& r) {
  r.lo = bp & ~7u;
  const int32_t o = off + int32_t(r.lo >> 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (o & ~3));
  const uint32_t sh = uint32_t(o) & 3u, w0 = w[0], w1 = w[1], w2 = w[2];
  uint64_t c = uint64_t(__builtin_amdgcn_alignbyte(w1, w0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32);
  const uint32_t end = 8 * n;
  c = r.lo >= end ? 0ull : (end - r.lo >= 64 ? c : c & ((1ull << (end - r.lo)) - 1));
  r.c = c;
}
// k <= 32 bits at bp, which lie in the window (bp + k <= lo + 64)
__device__ __forceinline__ uint32_t zf_ftake(const ZfFwd& r, uint32_t bp, uint32_t k) {
  return uint32_t((r.c >> (bp - r.lo)) & ((1ull << k) - 1));
}

// FSE_readNCount (oracle zs_ncount, zstd.h zs_ncount) into int8 counts: bytes used or -1 (also for
// a count above 127, which this parse leaves to the exact path).  The bits come through a register
// window that every lane of the wave refills at once (when any lane has fewer than 26 bits left: a
// symbol takes <= 8 bits, and a run of zero-count flags 2 per read, which refill on their own), so a
// refill's LDS round trip is paid every few symbols, not per read.
__device__ int zf_ncount8(const uint8_t* base, int32_t off, uint32_t n, int8_t* norm, int maxs, int maxal) {
  if (n == 0) return -1;
  const int al = (base[off] & 15) + 5;
  if (al > maxal) return -1;
  uint32_t bp = 4;
  int remaining = (1 << al) + 1, threshold = 1 << al, nb = al + 1, s = 0;
  bool prev0 = false;
  for (int i = 0; i <= maxs; i++) norm[i] = 0;
  ZfFwd r;
  zf_ffill(base, off, n, bp, r);
  while (remaining > 1 && s <= maxs) {
    if (__ballot(bp + 26 > r.lo + 64)) zf_ffill(base, off, n, bp, r);
    if (prev0) {
      int n0 = s;
      for (;;) {
        if (bp + 2 > r.lo + 64) zf_ffill(base, off, n, bp, r);
        const uint32_t v = zf_ftake(r, bp, 2);
        bp += 2;
        n0 += int(v);
        if (v != 3) break;
      }
      if (n0 > maxs) return -1;
      s = n0;
      prev0 = false;
    }
    if (bp + uint32_t(nb) > r.lo + 64) zf_ffill(base, off, n, bp, r);
    const uint32_t v = zf_ftake(r, bp, uint32_t(nb));
    const int max = (2 * threshold - 1) - remaining;
    int count;
    if (int(v & uint32_t(threshold - 1)) < max) {
      count = int(v & uint32_t(threshold - 1));
      bp += uint32_t(nb - 1);
    } else {
      count = int(v & uint32_t(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bp += uint32_t(nb);
    }
    count--;
    if (count > 127) return -1;
    remaining -= count < 0 ? -count : count;
    norm[s++] = int8_t(count);
    prev0 = count == 0;
    while (remaining < threshold && nb > 1) {
      nb--;
      threshold >>= 1;
    }
  }
  if (remaining != 1 || (bp + 7) / 8 > n) return -1;
  return int((bp + 7) / 8) | (al << 16) | ((s - 1) << 24);  // used (< 2^16), the log, the last symbol
}

// FSE decoding table (oracle zs_fse_build) with 16-bit entries sym | nb << 6 | base << 9 (al <= 7).
// The LDS reads go eight at a time (one round trip per eight counts or cells): in the last pass the
// eight cells' next[] reads are issued together and a cell counts the same symbol among the earlier
// cells of its group; the stores then run in order (the last of a symbol holds its final count).
__device__ bool zf_fse_build16(uint16_t* t, const int8_t* norm, int last, int al, uint8_t* next) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t hi = size - 1;
  // (norm has room for 56 counts: groups of eight read past `last` harmlessly)
  for (int s0 = 0; s0 <= last; s0 += 8) {
    int c[8];
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = norm[s0 + j];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int s = s0 + j;
      if (s <= last) {
        if (c[j] == -1) {
          t[hi--] = uint16_t(s);
          next[s] = 1;
        } else {
          next[s] = uint8_t(c[j] > 0 ? c[j] : 0);
        }
      }
    }
  }
  uint32_t pos = 0;
  for (int s0 = 0; s0 <= last; s0 += 8) {
    int c[8];
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = norm[s0 + j];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int s = s0 + j;
      const int cn = s <= last ? c[j] : 0;
      for (int i = 0; i < cn; i++) {
        t[pos] = uint16_t(s);
        do pos = (pos + step) & mask;
        while (pos > hi);
      }
    }
  }
  if (pos != 0) return false;
  for (uint32_t u0 = 0; u0 < size; u0 += 8) {  // (size >= 32: accuracy logs >= 5)
    const uint4 q = *reinterpret_cast<const uint4*>(t + u0);
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
    uint32_t sym[8], x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) sym[j] = (qw[j >> 1] >> (16 * (j & 1))) & 63u;
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = next[sym[j]];
#pragma unroll
    for (int j = 1; j < 8; j++)
#pragma unroll
      for (int i = 0; i < j; i++) x[j] += sym[i] == sym[j] ? 1u : 0u;
    uint32_t e[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      next[sym[j]] = uint8_t(x[j] + 1);
      const uint32_t nbits = uint32_t(al) - (31 - __builtin_clz(x[j]));
      e[j] = sym[j] | (nbits << 6) | (((x[j] << nbits) - size) << 9);
    }
    *reinterpret_cast<uint4*>(t + u0) = make_uint4(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16),
                                                   e[6] | (e[7] << 16));
  }
  return true;
}

// The bytes of a table description at frame byte p that the header chunks hold (a description
// running past them fails its parse: its block goes to the exact path)
__device__ __forceinline__ uint32_t zf_hdr_n(uint32_t p, uint32_t n, int32_t hend) {
  const int32_t room = hend - int32_t(p);
  return room <= 0 ? 0u : (uint32_t(room) < n ? uint32_t(room) : n);
}

// One table (zs_table): mode 0 = the predefined distribution, 1 = RLE, 2 = FSE_Compressed at
// base[off, off + n).  Builds it at t (at most `room` entries); returns bytes used | accuracy log
// << 16, or -1.
__device__ int zf_table16(uint32_t mode, const uint8_t* base, int32_t off, uint32_t n, const int16_t* def, int defs,
                          int defal, int maxs, uint16_t* t, uint32_t room, int8_t* norm, uint8_t* next) {
  if (mode == 1) {
    if (n < 1 || int(base[off]) > maxs) return -1;
    t[0] = uint16_t(base[off]);  // nb 0, base 0
    return 1;
  }
  int a = defal, last = defs - 1, used = 0;
  if (mode == 0) {
    for (int i = 0; i < defs; i++) norm[i] = int8_t(def[i]);
  } else {
    const int r = zf_ncount8(base, off, n, norm, maxs, 7);
    if (r < 0) return -1;
    used = r & 0xFFFF;
    a = (r >> 16) & 0xFF;
    last = r >> 24;
  }
  if ((1u << a) > room || !zf_fse_build16(t, norm, last, a, next)) return -1;
  return used | (a << 16);
}
}  // namespace

// (one wave per SIMD: the registers need not be rationed)
__global__ __launch_bounds__(kZfFseThreads) __attribute__((amdgpu_waves_per_eu(1, 2))) void zs_fse_parse_kernel(
    DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t ll_base[36], ml_base[53];
  __shared__ uint8_t ll_bits[36], ml_bits[53];
  for (uint32_t i = threadIdx.x; i < 36; i += blockDim.x) {
    ll_base[i] = kZsLLBase[i];
    ll_bits[i] = kZsLLBits[i];
  }
  for (uint32_t i = threadIdx.x; i < 53; i += blockDim.x) {
    ml_base[i] = kZsMLBase[i];
    ml_bits[i] = kZsMLBits[i];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint16_t* tab = reinterpret_cast<uint16_t*>(smem + threadIdx.x * kZfFseLane);
  uint8_t* const hb0 = reinterpret_cast<uint8_t*>(tab + kZfFseTab);  // the window
  uint8_t* const tb0 = hb0;
  int8_t* norm = reinterpret_cast<int8_t*>(hb0 + 16 * kZfFseHdrChunks);
  uint8_t* next = reinterpret_cast<uint8_t*>(norm + 56);
  const uint32_t items = z.count[2];
  const uint32_t waves = gridDim.x * (kZfFseThreads / 64);
  for (uint32_t r0 = (blockIdx.x * (kZfFseThreads / 64) + (threadIdx.x >> 6)) * 64; r0 < items; r0 += waves * 64) {
    const bool have = r0 + lane < items;
    const uint32_t b = have ? z.flist[r0 + lane] : 0u;
    bool ok = false;
    uint32_t shift = 0, clen = 0, cap = 0;
    const uint8_t* gin = nullptr;
    if (have) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      gin = a.in + s0;
      shift = uint32_t(reinterpret_cast<uintptr_t>(gin) & 15);
      const uint64_t cap64 = a.out_off[b + 1] - a.out_off[b];
      if (len >= 6 && shift + len <= kZfIn && cap64 <= kZfOut) {  // (phase A checked these)
        clen = uint32_t(len - 4);
        cap = uint32_t(cap64);
        ok = true;
      }
    }
    // the block's aligned chunks 0 .. lastc (no read beyond the block: the input may end there)
    const v4u* gal = reinterpret_cast<const v4u*>(gin - shift);
    const uint32_t lastc = ok ? (shift + clen + 3) >> 4 : 0u;
    const v4u zero4 = {0, 0, 0, 0};
    if (ok) {
      lds_put16(hb0, gal[0]);
      lds_put16(hb0 + 16, lastc >= 1 ? gal[1] : zero4);
      lds_put16(hb0 + 32, lastc >= 2 ? gal[2] : zero4);
    }
    const uint8_t* hb = hb0 + shift;
    ZfHead h{};
    ok = ok && zf_head(hb, clen, h) && h.bt == 2;
    // the literals section header: raw or RLE (phase A sent Huffman-literal blocks here only when
    // their sequences need this parse; they take the exact path)
    uint32_t nlit = 0, pos = 0, lit = 0, rle = 0;
    const uint32_t nb = h.bs, body = h.body;
    if (ok) {
      const uint32_t b0 = hb[body], type = b0 & 3, sf = (b0 >> 2) & 3;
      uint32_t hs = 1;
      if (sf == 1) {
        hs = 2;
        nlit = (b0 >> 4) + (uint32_t(hb[body + 1]) << 4);
      } else if (sf == 3) {
        hs = 3;
        nlit = (b0 >> 4) + (uint32_t(hb[body + 1]) << 4) + (uint32_t(hb[body + 2]) << 12);
      } else {
        nlit = b0 >> 3;
      }
      ok = type <= 1 && nb >= hs && nlit <= h.bmax && (type == 0 ? nb - hs >= nlit : nb - hs >= 1) && nlit <= cap;
      rle = type == 1;
      lit = rle ? uint32_t(hb[body + hs]) : body + hs;
      pos = hs + (type == 0 ? nlit : 1);
      ok = ok && pos < nb;
    }
    // the sequences section: kZfFseRegChunks chunks from the one holding its first byte, into
    // registers; the first kZfFseHdrChunks into the window (the head is done with)
    const uint32_t s = body + pos;
    const uint32_t c_lo = (shift + s) >> 4;
    const uint32_t qend = body + nb + (h.checksum ? 4u : 0u);  // the frame's bytes this parse reads
    ok = ok && qend <= 16 * (c_lo + kZfFseRegChunks) - shift;
    v4u R[kZfFseRegChunks];
#pragma unroll
    for (uint32_t k = 0; k < kZfFseRegChunks; k++) R[k] = ok && c_lo + k <= lastc ? gal[c_lo + k] : zero4;
    if (ok) {
#pragma unroll
      for (uint32_t k = 0; k < kZfFseHdrChunks; k++) lds_put16(tb0 + 16 * k, R[k]);
    }
    const uint8_t* tb = tb0 + shift - 16 * c_lo;  // tb[i] = frame byte i for i in [s, 16 (c_lo + 4) - shift)
    const int32_t tofs = int32_t(shift) - int32_t(16 * c_lo);  // frame byte i = tb0[i + tofs]
    const int32_t hend = int32_t(16 * kZfFseHdrChunks) - tofs;  // the header chunks' end, in frame bytes
    uint32_t nseq = 0, produced = 0;
    v4u qv = {0, 0, 0, 0};  // the current group of four records
    uint32_t* seqs = z.seq + size_t(b) * kZfSeqSlot;
    if (ok) {
      const uint32_t sn = nb - pos;
      const uint32_t c0 = tb[s];
      uint32_t sp;
      if (c0 < 128) {
        nseq = c0;
        sp = 1;
      } else if (c0 < 255) {
        ok = sn >= 2;
        nseq = ((c0 - 128) << 8) + tb[s + 1];
        sp = 2;
      } else {
        ok = sn >= 3;
        nseq = uint32_t(tb[s + 1]) + (uint32_t(tb[s + 2]) << 8) + 0x7F00;
        sp = 3;
      }
      ok = ok && nseq != 0 && nseq <= kZsFseSeqs && sp < sn;
      const uint32_t modes = ok ? uint32_t(tb[s + sp++]) : 0u;
      ok = ok && !(modes & 3);
      const uint32_t m_ll = modes >> 6, m_of = (modes >> 4) & 3, m_ml = (modes >> 2) & 3;
      ok = ok && m_ll <= 2 && m_of <= 2 && m_ml <= 2;
      // the three tables, LL / OF / ML as they follow each other, back to back in the lane's LDS
      uint32_t al_ll = 0, al_of = 0, al_ml = 0, t_of = 0, t_ml = 0;
      if (ok) {
        const int u = zf_table16(m_ll, tb0, int32_t(s + sp) + tofs, zf_hdr_n(s + sp, sn - sp, hend), kZsLLDef, 36, 6, 35, tab,
                                 kZfFseTab, norm, next);
        ok = u >= 0;
        sp += ok ? uint32_t(u & 0xFFFF) : 0u;
        al_ll = ok ? uint32_t(u >> 16) : 0u;
      }
      if (ok) {
        t_of = 1u << al_ll;
        const int u = zf_table16(m_of, tb0, int32_t(s + sp) + tofs, zf_hdr_n(s + sp, sn - sp, hend), kZsOFDef, 29, 5, 31,
                                 tab + t_of, kZfFseTab - t_of, norm, next);
        ok = u >= 0;
        sp += ok ? uint32_t(u & 0xFFFF) : 0u;
        al_of = ok ? uint32_t(u >> 16) : 0u;
      }
      if (ok) {
        t_ml = t_of + (1u << al_of);
        const int u = zf_table16(m_ml, tb0, int32_t(s + sp) + tofs, zf_hdr_n(s + sp, sn - sp, hend), kZsMLDef, 53, 6, 52,
                                 tab + t_ml, kZfFseTab - t_ml, norm, next);
        ok = u >= 0;
        sp += ok ? uint32_t(u & 0xFFFF) : 0u;
        al_ml = ok ? uint32_t(u >> 16) : 0u;
      }
      ok = ok && !(dbg_bits(a) & (1u << 18));  // profiling: the tables only (every block handed back)
      // the bitstream's chunks from the registers into the window (over the headers and the scratch)
      const uint32_t d = ((shift + s + sp) >> 4) - c_lo;
      ok = ok && d + kZfFseBitChunks <= kZfFseRegChunks && qend <= 16 * (c_lo + d + kZfFseBitChunks) - shift;
      if (ok) {
#pragma unroll
        for (uint32_t k = 0; k < kZfFseRegChunks; k++)
          if (k >= d && k < d + kZfFseBitChunks) lds_put16(tb0 + 16 * (k - d), R[k]);
      }
      tb -= 16 * d;  // tb[i] = frame byte i for i in [s + sp, qend)
      // zs_bstart
      const uint32_t bn = ok ? sn - sp : 0u;
      const uint32_t last = bn ? uint32_t(tb[s + sn - 1]) : 0u;
      ok = ok && last != 0;
      ZfBits bits{tb0, 8 * (int64_t(int32_t(s + sp) + tofs) - 16 * int64_t(d)),
                  ok ? 8 * int64_t(bn - 1) + (31 - __builtin_clz(last)) : 0};
      uint32_t sll = 0, sof = 0, sml = 0;
      ZfReg rg{};
      if (ok) {
        zf_fill(bits, rg);
        sll = zf_take(bits, rg, al_ll);  // (<= 21 bits: accuracy logs <= 7)
        sof = zf_take(bits, rg, al_of);
        sml = zf_take(bits, rg, al_ml);
      }
      uint32_t rep0 = 1, rep1 = 4, rep2 = 8, lp = 0, o = 0;
      const uint32_t lbase = cap - nlit;
      for (uint32_t i = 0; ok && i < nseq; i++) {
        zf_fill(bits, rg);  // (issued beside the table reads: >= 56 bits for this sequence's values)
        const uint32_t ell = tab[sll], eof = tab[t_of + sof], eml = tab[t_ml + sml];
        const uint32_t llc = ell & 63u, ofc = eof & 63u, mlc = eml & 63u;
        // an offset code above 12 gives an offset above 4096, which the record cannot hold (the
        // check below): the block goes to the exact path either way; so the values take <= 12 +
        // 16 + 16 bits of the window
        if (ofc > 12) {
          ok = false;
          break;
        }
        const uint32_t ofv = (1u << ofc) + zf_take(bits, rg, ofc);
        const uint32_t ml = ml_base[mlc] + zf_take(bits, rg, ml_bits[mlc]);
        const uint32_t ll = ll_base[llc] + zf_take(bits, rg, ll_bits[llc]);
        uint64_t offv;
        if (ofv > 3) {
          offv = ofv - 3;
          rep2 = rep1;
          rep1 = rep0;
          rep0 = uint32_t(offv);
        } else {
          const uint32_t idx = uint32_t(ofv) - 1 + (ll == 0 ? 1u : 0u);
          offv = idx == 3 ? uint64_t(rep0) - 1 : (idx == 0 ? rep0 : idx == 1 ? rep1 : rep2);
          if (offv == 0) offv = 1;
          if (idx >= 2) rep2 = rep1;
          if (idx >= 1) {
            rep1 = rep0;
            rep0 = uint32_t(offv);
          }
        }
        if (i + 1 < nseq) {
          if (rg.lo > 0 && bits.bp - rg.lo < 21) zf_fill(bits, rg);  // (long values only)
          sll = (ell >> 9) + zf_take(bits, rg, (ell >> 6) & 7u);
          sml = (eml >> 9) + zf_take(bits, rg, (eml >> 6) & 7u);
          sof = (eof >> 9) + zf_take(bits, rg, (eof >> 6) & 7u);
        }
        if (bits.bp < 0 || ll > nlit - lp || uint64_t(o) + ll + ml > h.bmax || uint64_t(o) + ll + ml > cap ||
            uint64_t(o) + ll + ml > uint64_t(lbase) + lp + ll) {
          ok = false;
          break;
        }
        lp += ll;
        o += ll;
        // fstart = 0: one frame; the record holds ll < 1024, ml - 3 < 1024, offset - 1 < 4096
        if (offv > o || ll > 1023 || ml - 3 > 1023 || offv > 4096) {
          ok = false;
          break;
        }
        const uint32_t r = ll | ((ml - 3) << 10) | (uint32_t(offv - 1) << 20);
        qv.x = (i & 3) == 0 ? r : qv.x;
        qv.y = (i & 3) == 1 ? r : qv.y;
        qv.z = (i & 3) == 2 ? r : qv.z;
        qv.w = (i & 3) == 3 ? r : qv.w;
        if ((i & 3) == 3) reinterpret_cast<v4u*>(seqs)[i >> 2] = qv;
        o += ml;
      }
      ok = ok && bits.bp == 0;
      const uint32_t rest = nlit - lp;
      ok = ok && uint64_t(o) + rest <= h.bmax && uint64_t(o) + rest <= cap;
      produced = o + rest;
      ok = ok && (!h.has_fcs || uint64_t(produced) == h.fcs);
    }
    if (ok && (nseq & 3)) reinterpret_cast<v4u*>(seqs)[nseq >> 2] = qv;
    // the record (ZsFastRec: lit, nlit, produced, info | want, cs, pad), as two 16-byte stores
    v4u w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0};
    if (ok) {
      const uint32_t qq = body + nb;
      w0.x = lit;
      w0.y = nlit;
      w0.z = produced;
      w0.w = nseq | ((kZfFast | kZfSeq4 | (rle ? kZfRle : 0u) | (h.checksum ? kZfSum : 0u)) << 16);
      w1.x = h.checksum ? uint32_t(tb[qq]) | (uint32_t(tb[qq + 1]) << 8) | (uint32_t(tb[qq + 2]) << 16) |
                              (uint32_t(tb[qq + 3]) << 24)
                        : 0u;
    }
    static_assert(sizeof(ZsFastRec) == 32, "record layout");
    if (have) {
      reinterpret_cast<v4u*>(z.rec + b)[0] = w0;
      reinterpret_cast<v4u*>(z.rec + b)[1] = w1;
    }
    list_append(have && !ok, b, z.list, z.count);
  }
}

// ------------------------------------------------------------------------------- phase B
namespace {
// What phase B needs of one block: its record, offsets and sequences, loaded by independent
// loads (no branch on their values) so that they can be issued one block ahead.
struct ZfRaw {
  ZsFastRec rec;
  uint64_t i0, i1, o0, o1;
  uint2 seq;  // lane i: dwords 2i, 2i + 1 of the block's sequence slot
  uint32_t b;
};
__device__ __forceinline__ ZfRaw zf_load(const DecodeArgs& a, const ZsFastArgs& z, uint32_t b, uint32_t lane) {
  ZfRaw r{};
  r.b = b;
  if (b < a.n) {
    r.rec = z.rec[b];
    r.i0 = a.in_off[b];
    r.i1 = a.in_off[b + 1];
    r.o0 = a.out_off[b];
    r.o1 = a.out_off[b + 1];
    r.seq = reinterpret_cast<const uint2*>(z.seq + size_t(b) * kZfSeqSlot)[lane];
  }
  return r;
}
// A block's sequences, two slots per lane: 8-byte records put sequence i on lane i (slot A),
// 4-byte records (kZfSeq4) sequences 2i and 2i + 1 on lane i (slots A and B); a slot past the
// block's sequences holds zeros.
struct ZfBlock {
  uint32_t b, fast, shift, len, cap, nseq, nlit, produced, lit, rle, huf, cs, s4, outlit, adler, want, hufo;
  const uint8_t* gin;
  uint8_t* gout;
  uint32_t llA, mlA, offA, llB, mlB, offB;
};
__device__ __forceinline__ ZfBlock zf_decode(const DecodeArgs& a, const ZfRaw& r, uint32_t lane) {
  ZfBlock k{};
  k.b = r.b;
  if (r.b >= a.n) return k;
  const uint32_t fl = __builtin_amdgcn_readfirstlane(r.rec.info >> 16);
  k.fast = fl & kZfFast;
  k.gin = a.in + r.i0;
  k.gout = a.out + r.o0;
  k.len = uint32_t(r.i1 - r.i0);
  k.shift = uint32_t(reinterpret_cast<uintptr_t>(k.gin) & 15);
  k.cap = uint32_t(r.o1 - r.o0);
  k.nseq = __builtin_amdgcn_readfirstlane(r.rec.info & 0xFFFFu);
  k.nlit = __builtin_amdgcn_readfirstlane(r.rec.nlit);
  k.produced = __builtin_amdgcn_readfirstlane(r.rec.produced);
  k.lit = __builtin_amdgcn_readfirstlane(r.rec.lit);
  k.rle = fl & kZfRle;
  k.huf = (fl & kZfHuf) ? ((fl & kZfHuf4) ? 4u : 1u) : 0u;
  k.hufo = fl & kZfHufOrig;
  k.cs = __builtin_amdgcn_readfirstlane(r.rec.cs);
  k.s4 = (fl & kZfSeq4) ? 1u : 0u;
  k.outlit = fl & kZfOutLit;  // (CodecZlib: the literals are at the start of the output slot)
  k.adler = fl & kZfAdler;
  k.want = __builtin_amdgcn_readfirstlane(r.rec.want);
  if (!k.fast) return k;
  if (k.s4) {
    const bool va = 2 * lane < k.nseq, vb = 2 * lane + 1 < k.nseq;
    const uint32_t x = va ? r.seq.x : 0u, y = vb ? r.seq.y : 0u;
    k.llA = x & 1023u;
    k.mlA = va ? ((x >> 10) & 1023u) + 3 : 0u;
    k.offA = va ? (x >> 20) + 1 : 0u;
    k.llB = y & 1023u;
    k.mlB = vb ? ((y >> 10) & 1023u) + 3 : 0u;
    k.offB = vb ? (y >> 20) + 1 : 0u;
  } else {
    const bool va = lane < k.nseq;
    k.llA = va ? r.seq.x & 0xFFFFu : 0u;
    k.mlA = va ? r.seq.x >> 16 : 0u;
    k.offA = va ? r.seq.y : 0u;
  }
  return k;
}
}  // namespace

// Build one block in wout from its sequences (lane i: sequence i) and its literals at wout[lb...]
// (or the RLE byte), write it back, then block.Decode's checks and rows (phases B and B').
// CodecZlib blocks (kZfAdler) are checked against the stream's Adler-32 first: false = mismatch,
// nothing written (the caller hands the block to the exact path, which reports it).
__device__ __forceinline__ bool zf_build(const DecodeArgs& a, const ZfBlock& cur, uint8_t* wout, uint32_t lb, uint32_t out_nt,
                                         uint32_t lane, uint32_t dbg) {
  const uint32_t lit = cur.lit;
  slate_block_meta m{};
  // exclusive scans over the lanes (two sequences per lane) give each sequence's literal source
  // and output position
  const uint32_t nseq = cur.nseq, nlit = cur.nlit;
  const uint32_t llA = cur.llA, mlA = cur.mlA, llB = cur.llB, mlB = cur.mlB;
  const uint32_t t_ll = llA + llB, t_out = llA + mlA + llB + mlB;
  uint32_t x_ll = t_ll, x_out = t_out;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y1 = __shfl_up(x_ll, d, 64), y2 = __shfl_up(x_out, d, 64);
    if (int(lane) >= d) {
      x_ll += y1;
      x_out += y2;
    }
  }
  const uint32_t lsrcA = x_ll - t_ll, dposA = x_out - t_out;  // exclusive
  const uint32_t lsrcB = lsrcA + llA, dposB = dposA + llA + mlA;
  const uint32_t tot_ll = __shfl(x_ll, 63, 64), tot_out = __shfl(x_out, 63, 64);
  const uint32_t rle4 = (lit & 0xFF) * 0x01010101u;
  uint8_t* junk = wout + kZfJunk + 4 * lane;
  // One 16-byte piece of a literal run: output dwords w .. w + 12 of the run [dst, end), moved down
  // by delta (output byte p = wout[p + delta]).  Only the dwords that hold run bytes are written
  // (the others go to the lane's junk dword); the (up to three) bytes the first or last of them
  // spills over lie in the neighbouring match (>= 3 bytes), written afterwards, or past the block,
  // and never reach literals still to be moved (the cursor rule: o + ml <= cap - nlit + lp, ml >= 3).
  // A run moves down, and a later run's source lies above every earlier run's destination, so
  // pieces read in one instruction and written in the next may come from any runs.
  auto piece = [&](bool go, uint32_t w, uint32_t end, int32_t delta) {
    uint32_t o[4];
    if (cur.rle) {
      o[0] = o[1] = o[2] = o[3] = rle4;
    } else {
      const int32_t sa = int32_t(w) + delta;
      const uint32_t* sp = reinterpret_cast<const uint32_t*>(wout + (go ? (sa & ~3) : 0));
      const uint32_t sh = uint32_t(sa) & 3;
      const uint32_t d0 = sp[0], d1 = sp[1], d2 = sp[2], d3 = sp[3], d4 = sp[4];
      o[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
      o[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
      o[2] = __builtin_amdgcn_alignbyte(d3, d2, sh);
      o[3] = __builtin_amdgcn_alignbyte(d4, d3, sh);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t k = 0; k < 4; k++)
      *reinterpret_cast<uint32_t*>((go && w + 4 * k < end) ? wout + w + 4 * k : junk) = o[k];
  };
  if (!(dbg & (1u << 22))) {
    // the sequences' runs: piece j of all of them (lane-major, A before B) on lane j mod 64; a
    // piece finds its lane by a binary search over the lanes' exclusive piece counts
    const uint32_t pcA = llA ? (dposA + llA - (dposA & ~3u) + 15) / 16 : 0u;
    const uint32_t pcB = llB ? (dposB + llB - (dposB & ~3u) + 15) / 16 : 0u;
    const uint32_t t_pc = pcA + pcB;
    uint32_t x_pc = t_pc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x_pc, d, 64);
      if (int(lane) >= d) x_pc += y;
    }
    const uint32_t e_pc = x_pc - t_pc, n_pc = __shfl(x_pc, 63, 64);
    for (uint32_t j0 = 0; j0 < n_pc; j0 += kWave) {
      const uint32_t j = j0 + lane;
      uint32_t k = 0;
#pragma unroll
      for (uint32_t st = 32; st >= 1; st >>= 1) k = uint32_t(__shfl(e_pc, int(k + st), 64)) <= j ? k + st : k;
      // (every lane takes part in every shuffle: a ds_bpermute reads nothing from a lane the exec
      // mask leaves out, so no shuffle sits in a divergent select)
      const uint32_t q = j - uint32_t(__shfl(e_pc, int(k), 64));
      const uint32_t qa = __shfl(pcA, int(k), 64);
      const uint32_t dA = __shfl(dposA, int(k), 64), dB = __shfl(dposB, int(k), 64);
      const uint32_t sA = __shfl(lsrcA, int(k), 64), sB = __shfl(lsrcB, int(k), 64);
      const uint32_t lA = __shfl(llA, int(k), 64), lB = __shfl(llB, int(k), 64);
      const bool inA = q < qa;
      const uint32_t dst = inA ? dA : dB, src = inA ? sA : sB, L = inA ? lA : lB;
      const uint32_t p = inA ? q : q - qa;
      piece(j < n_pc, (dst & ~3u) + 16 * p, dst + L, int32_t(lb + src) - int32_t(dst));
      zs_sync();
    }
    // the trailing run (after the last match)
    const uint32_t L = nlit - tot_ll, dst = tot_out, end = dst + L;
    const int32_t delta = int32_t(lb + tot_ll) - int32_t(dst);
    for (uint32_t w = (dst & ~3u) + 16 * lane; __ballot(L != 0 && w < end); w += 16 * kWave) piece(w < end, w, end, delta);
  }
  zs_sync();
  // Matches in order: each reads only bytes before its own position.  Non-overlapping ones
  // (offset >= length) a dword per lane, the edge dwords merged with the bytes around the
  // match; overlapping ones a byte per lane.
  const uint32_t offA = cur.offA, offB = cur.offB, s4 = cur.s4;
  // (lane li holds sequence li, or with 4-byte records sequences 2li and 2li + 1: slots A and B)
  const uint32_t pkA = cur.mlA | (offA << 16), pkB = cur.mlB | (offB << 16);  // ml < 2^16, offset <= 4112
  const uint32_t mpA = dposA + llA, mpB = dposB + llB;
  auto match = [&](uint32_t pk, uint32_t mp) {
    const uint32_t M = pk & 0xFFFFu, O = pk >> 16;
    if (M <= kWave) {
      // most matches: one byte per lane (an overlapping one repeats every O bytes, all before mp)
      if (lane < M) {
        const uint32_t t = O >= M ? lane : lane % O;
        wout[mp + lane] = wout[mp - O + t];
      }
    } else if (O >= M) {
      const uint32_t me = mp + M;
      const uint32_t lo_keep = (1u << (8 * (mp & 3))) - 1u, hi_keep = (me & 3) ? ~((1u << (8 * (me & 3))) - 1u) : 0u;
      for (uint32_t w = (mp & ~3u) + 4 * lane; w < me; w += 4 * kWave) {
        uint32_t v = lds_u32(wout, int32_t(w) - int32_t(O));
        const uint32_t keep = (w < mp ? lo_keep : 0u) | (w + 4 > me ? hi_keep : 0u);
        if (keep) v = (v & ~keep) | (*reinterpret_cast<const uint32_t*>(wout + w) & keep);
        *reinterpret_cast<uint32_t*>(wout + w) = v;
      }
    } else {
      for (uint32_t j = lane; j < M; j += kWave) wout[mp + j] = wout[mp - O + (j % O)];
    }
    zs_sync();
  };
  const uint32_t nl = (dbg & (1u << 21)) ? 0u : (s4 ? (nseq + 1) / 2 : nseq);
  for (uint32_t li = 0; li < nl; li++) {
    match(__builtin_amdgcn_readlane(pkA, li), __builtin_amdgcn_readlane(mpA, li));
    if (s4 && 2 * li + 1 < nseq) match(__builtin_amdgcn_readlane(pkB, li), __builtin_amdgcn_readlane(mpB, li));
  }
  const uint32_t n = cur.produced;
  if (cur.adler) {
    // Adler-32 (RFC 1950 8.2) of wout[0, n): a = 1 + sum x_i, b = n + sum (n - i) x_i, mod 65521
    // (the sums stay below 2^32 for n <= 4112); a dword per lane per step
    uint32_t sa = 0, sb = 0;
    for (uint32_t j = lane; 4 * j < n; j += kWave) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(wout + 4 * j);
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = 4 * j + q;
        const uint32_t x = i < n ? (w >> (8 * q)) & 0xFFu : 0u;
        sa += x;
        sb += (n - i) * x;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {
      sa += __shfl_xor(sa, o, 64);
      sb += __shfl_xor(sb, o, 64);
    }
    const uint32_t ad = (((n + sb) % 65521u) << 16) | ((1u + sa) % 65521u);
    if (__builtin_amdgcn_readfirstlane(ad) != cur.want) return false;
  }
  {
    uint8_t* gout = cur.gout;
    const uint32_t oc = (dbg & (1u << 27)) ? 0u : (n + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(wout);
    if (out_nt) {
      const v4u* s4 = reinterpret_cast<const v4u*>(wout);
      for (uint32_t c = lane; c < oc; c += kWave) __builtin_nontemporal_store(s4[c], reinterpret_cast<v4u*>(gout) + c);
    } else {
      for (uint32_t c = lane; c < oc; c += kWave) reinterpret_cast<uint4*>(gout)[c] = src[c];
    }
  }
  if (dbg & (1u << 20)) write_meta(&a.meta[cur.b], m, int(lane));
  else block_finish(a, cur.b, wout, n, int(lane), m);
  return true;
}

// One wave per block, the next block's record and sequences loaded while this one is built.  The frame is staged in the output buffer at the 16-byte phase of its address, placed
// so that its raw literals start at lb >= cap - nlit: phase A checked zs_block's rule that the
// write cursor never passes the unread literals (o + ml <= cap - nlit + lp before each literal
// run), so the runs can be moved down in place, in order.
__global__ __launch_bounds__(kZfBuildThreads, SLATE_ZF_BUILD_WG) void zs_fast_build_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  uint8_t* wout = smem + wave * kZfOutLds;
  const uint32_t waves = gridDim.x * (kZfBuildThreads / 64);
  // profiling ablations (SLATE_DEBUG_MODE, profiling variants only): 1<<20 no block_finish,
  // 1<<21 no matches, 1<<22 no literal runs, 1<<24 no XXH64 rounds, 1<<26 no hand-back from C,
  // 1<<27 no output write, 1<<28 no frame staging
  const uint32_t dbg = dbg_bits(a);
  const uint32_t first = blockIdx.x * (kZfBuildThreads / 64) + wave;
  // list mode (z.blist): item i is block blist[i], for the H2-prepared blocks only
  const uint32_t i_end = z.blist ? min(z.count[1], z.hcap) : a.n;
  auto block_at = [&](uint32_t i) { return z.blist ? (i < i_end ? z.blist[i] : a.n) : i; };
  uint32_t g0 = 0, gi = 0;
  auto draw4 = [&]() { return __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(z.count + 3, z.draw) : 0u); };
  auto next_of = [&](uint32_t i) {
    if (!z.draw) return i + waves;
    if (++gi == z.draw) {
      g0 = draw4();
      gi = 0;
    }
    return g0 + gi;
  };
  uint32_t i = first;
  if (z.draw) i = g0 = draw4();
  ZfRaw nr = zf_load(a, z, block_at(i), lane);
  while (i < i_end) {
    const ZfRaw cr = nr;
    i = next_of(i);
    nr = zf_load(a, z, block_at(i), lane);  // in flight while this block is built
    const ZfBlock cur = zf_decode(a, cr, lane);
    if (!cur.fast || cur.huf || (z.skip_hufo && cur.hufo)) continue;  // (Huffman literals: phase B' / the list pass)
    // CodecZlib (kZfOutLit): the literal bytes at the start of the (16-aligned) output slot take
    // the frame's place: shift 0, literals from byte 0, nlit bytes
    const uint32_t lbase = cur.cap - cur.nlit, lit = cur.outlit ? 0u : cur.lit, shift = cur.outlit ? 0u : cur.shift;
    const uint32_t slen = cur.outlit ? cur.nlit : cur.len;
    // frame byte 0 at wout[F], F = 16-aligned base + shift, literals at lb = F + lit >= lbase
    uint32_t base16 = 16;
    if (!cur.rle && lbase > lit + shift + 16) base16 = (lbase - lit - shift + 15) & ~15u;
    const uint32_t F = base16 + shift, lb = F + lit;
    {
      const uint32_t chunks = (dbg & (1u << 28)) ? 0u : (shift + slen + 15) / 16;
      const uint8_t* lsrc = z.lit ? z.lit + size_t(cur.b) * kZlStageStride : cur.gout;  // (a staged plan's)
      const uint4* src = reinterpret_cast<const uint4*>(cur.outlit ? lsrc : cur.gin - shift);
      uint4* dst = reinterpret_cast<uint4*>(wout + base16);
      for (uint32_t c = lane; c < chunks; c += kWave) dst[c] = src[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    zs_sync();
    if (!zf_build(a, cur, wout, lb, z.out_nt, lane, dbg) && lane == 0) {  // (the block's CRC32 held: phase A2)
      z.rec[cur.b].info = 0;
      z.list[atomicAdd(z.count, 1u)] = cur.b;  // the Adler-32 failed: the exact path reports it
    }
  }
}

// ------------------------------------------------------------------------------- phase B'
// Blocks whose literals are Huffman-coded with a new tree (zs_block literal type 2; configs[4]:
// ~1 %), one wave per block from phase A's list: the tree (zs_huf_read) and the one or four
// streams decoded as zs_block does, into the tail of the output buffer, then built like phase B.
// Any failed check hands the block to the exact path.
__global__ __launch_bounds__(kZfHufThreads) void zs_fast_huf_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // (the list's first z.hcap entries are phases H1 / H2's)
  const uint32_t items = z.count[1];
  if (z.hcap + blockIdx.x * (kZfHufThreads / 64) >= items) return;  // (workgroup-uniform)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* win = smem + wave * kZfHufWave;
  uint8_t* wout = win + kZfIn + 16;
  ZsScratch* sc = reinterpret_cast<ZsScratch*>(wout + kZfOutLds);
  for (uint32_t k = z.hcap + blockIdx.x * (kZfHufThreads / 64) + wave; k < items; k += gridDim.x * (kZfHufThreads / 64)) {
    const uint32_t b = z.hlist[k];
    const ZfBlock cur = zf_decode(a, zf_load(a, z, b, lane), lane);
    if (!cur.fast) continue;  // the CRC32 failed (phase A2)
    const uint32_t shift = cur.shift;
    {
      const uint32_t chunks = (shift + cur.len + 15) / 16;
      const uint4* src = reinterpret_cast<const uint4*>(cur.gin - shift);
      uint4* dst = reinterpret_cast<uint4*>(win);
      for (uint32_t c = lane; c < chunks; c += kWave) dst[c] = src[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    zs_sync();
    const uint32_t nlit = cur.nlit, lbase = cur.cap - nlit;
    uint32_t tl = 0;
    // 1<<30: profiling, no tree (a flat 8-bit table is assumed)
    const int t = (dbg_bits(a) & (1u << 30)) ? (tl = 8, 1) : zs_huf_read(win, int32_t(shift + cur.lit), cur.cs, sc, int(lane), &tl, dbg_bits(a));
    bool fail = t < 0;
    if (!fail) {
      const uint32_t q = shift + cur.lit + uint32_t(t), qn = cur.cs - uint32_t(t);
      auto bN = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(win[q + i])); };
      // stream l on lane l: bytes [sb, sb + sl) of win, m literals to wout[lbase + lo]
      uint32_t sb = 0, sl = 0, m = 0, lo = 0;
      if (cur.huf == 1) {
        sb = q;
        sl = qn;
        m = nlit;
      } else if (qn < 10) {
        fail = true;
      } else {
        const uint32_t l1 = bN(0) | (bN(1) << 8), l2 = bN(2) | (bN(3) << 8), l3 = bN(4) | (bN(5) << 8);
        const uint32_t seg = (nlit + 3) / 4;
        fail = l1 + l2 + l3 + 6 > qn || 3 * seg > nlit;
        const uint32_t l4 = qn - 6 - l1 - l2 - l3, s0 = q + 6;
        sb = lane == 0 ? s0 : lane == 1 ? s0 + l1 : lane == 2 ? s0 + l1 + l2 : s0 + l1 + l2 + l3;
        sl = lane == 0 ? l1 : lane == 1 ? l2 : lane == 2 ? l3 : l4;
        m = lane < 3 ? seg : nlit - 3 * seg;
        lo = seg * (lane < 3 ? lane : 3u);
      }
      bool badl = false;
      if (!fail && lane < cur.huf && !(dbg_bits(a) & (1u << 29))) {  // 1<<29: profiling, no streams
        int64_t bp = zs_bstart(win, int32_t(sb), sl);
        if (bp < 0) {
          badl = true;
        } else {
          const int64_t S = 8 * int64_t(sb);
          const uint32_t tmask = (1u << tl) - 1;
          uint8_t* dst = wout + lbase + lo;
          int64_t clo = 0;
          uint64_t cv = 0;
          bool have = false;
          for (uint32_t i = 0; i < m; i++) {  // a 56-bit register window, as zs_block
            const int64_t lo2 = bp - int64_t(tl);
            uint32_t v;
            if (have && lo2 >= clo) {
              v = uint32_t(cv >> (lo2 - clo)) & tmask;
            } else if (lo2 >= 0) {
              clo = bp > 56 ? bp - 56 : 0;
              cv = zs_bits(win, S + clo, 56);
              have = true;
              v = uint32_t(cv >> (lo2 - clo)) & tmask;
            } else {
              v = uint32_t(zs_peek(win, S, bp, tl));
            }
            const uint32_t e = sc->huf[v];
            dst[i] = uint8_t(e);
            bp -= e >> 8;
          }
          badl = bp != 0;
        }
      }
      fail = fail || __ballot(badl) != 0;
    }
    if (fail) {  // to the exact path: not summed (C), decoded and reported by D
      if (lane == 0) {
        z.rec[b].info = 0;
        z.list[atomicAdd(z.count, 1u)] = b;
      }
      continue;
    }
    zs_sync();
    (void)zf_build(a, cur, wout, lbase, z.out_nt, lane, 0);  // (Zstd frames only: no Adler-32)
  }
}

// ------------------------------------------------------------------------------ phases H1, H2
// Huffman-literal blocks (zs_block literal type 2 with a new tree; configs[4]: ~1.1 % of blocks)
// in two passes instead of phase B's wave per block with four busy lanes:
//   H1 zs_huf_tree_kernel    one WAVE per block, many per CU: the tree description (zs_huf_read)
//                            into the block's decoding table in HBM (2^tl 16-bit entries) and its
//                            one or four streams' records (start, length, symbols, output place)
//   H2 zs_huf_stream_kernel  one LANE per stream, 16 blocks per wave: the 16 tables in LDS, each
//                            lane's backward bitstream through a 64-bit register window fed from a
//                            per-lane LDS ring of 16-byte chunks (one chunk prefetched), a table
//                            read per symbol, the literal bytes to the start of the block's output
//                            slot; the block then leaves as a kZfOutLit block (phase B builds it
//                            from there, as it builds CodecZlib blocks) or, on any failed check
//                            (the stream does not end exactly at its first bit), to the exact path.
// Both run on the main stream after A2 (the rec flags they rewrite are A2's too). Entries of the
// Huffman list beyond the slots (zf_huf_cap) take phase B'.
constexpr uint32_t kZhTreeThreads = 256;
constexpr uint32_t kZhWin = 192;  // the tree description's window: <= 15 + 1 + 127 bytes + 8 slack
// the tree decode's scratch without its 4 KiB table (H1 writes the table straight to HBM): small
// waves, so many fit beside phase A2 on the side stream
constexpr uint32_t kZhScrTail = kZsHufScratch - uint32_t(offsetof(ZsScratch, wt));
constexpr uint32_t kZhTreeWave = kZhWin + kZhScrTail;
constexpr uint32_t kZhTreeLds = (kZhTreeThreads / 64) * kZhTreeWave;
constexpr uint32_t kZhBlocks = 15;  // blocks per H2 wave (four stream lanes each; 64 KiB of LDS with
                                    // the rings, so it fits beside two phase-A2 workgroups)
// per-lane LDS ring: four 16-byte chunks at a 17-dword stride (an odd stride puts the lanes' ring
// dwords at one offset in distinct banks; a 16-dword one put all of them in two), written as dwords;
// lanes 60..63 hold no stream and no ring
constexpr uint32_t kZhRing = 68;
constexpr uint32_t kZhStreamLds = kZhBlocks * kZhTab + 4 * kZhBlocks * kZhRing;
static_assert(4 * kZhBlocks * kZhRing <= 4096, "the rings fit the 4 KiB after the tables");
static_assert(2 * kZhStreamLds <= 160 * 1024, "phase H2 workgroups per CU exceed the LDS");

__global__ __launch_bounds__(kZhTreeThreads) void zs_huf_tree_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t items = min(z.count[1], z.hcap);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* win = smem + wave * kZhTreeWave;
  // sc's fields from wt on lie in this wave's tail; its huf table is never touched (huf_out below)
  ZsScratch* sc = reinterpret_cast<ZsScratch*>(win + kZhWin - offsetof(ZsScratch, wt));
  const uint32_t waves = gridDim.x * (kZhTreeThreads / 64);
  for (uint32_t k = blockIdx.x * (kZhTreeThreads / 64) + wave; k < items; k += waves) {
    const uint32_t b = z.hlist[k];
    const ZsFastRec rec = z.rec[b];
    const uint32_t fl = zrfl(rec.info >> 16);
    uint4* dk = reinterpret_cast<uint4*>(z.hdesc + 16 * size_t(k));
    if (!(fl & kZfFast)) {  // the CRC32 failed (phase A2): H2 skips it
      continue;
    }
    const uint64_t i0 = a.in_off[b];
    const uint32_t len = uint32_t(a.in_off[b + 1] - i0);
    const uint32_t shift = uint32_t(reinterpret_cast<uintptr_t>(a.in + i0) & 15);
    const uint8_t* F = a.in + i0 - shift;
    const __amdgpu_buffer_rsrc_t R = make_rsrc(F, align16(uint64_t(shift) + len));
    const uint32_t lit = zrfl(rec.lit), cs = zrfl(rec.cs), nlit = zrfl(rec.nlit);
    const uint32_t nstr = (fl & kZfHuf4) ? 4u : 1u;
    // the tree description's window: chunks from the one holding its first byte
    const uint32_t c0 = (shift + lit) >> 4, off = (shift + lit) & 15;
    if (lane < kZhWin / 16) lds_put16(win + 16 * lane, bload(R, 16 * (c0 + lane)));
    __builtin_amdgcn_s_waitcnt(0);
    zs_sync();
    uint32_t tl = 0;
    const int t = zs_huf_read(win, int32_t(off), cs, sc, int(lane), &tl, 0u,
                              reinterpret_cast<uint16_t*>(z.htab + size_t(k) * kZhTab));
    bool fail = t < 0;
    uint32_t sb = 0, sl = 0, m = 0, lo = 0;  // lane l < nstr: stream l
    if (!fail) {
      const uint32_t q = off + uint32_t(t), qn = cs - uint32_t(t), fq = lit + uint32_t(t);
      if (nstr == 1) {
        sb = fq;
        sl = qn;
        m = nlit;
      } else if (qn < 10) {
        fail = true;
      } else {
        auto bN = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(win[q + i])); };
        const uint32_t l1 = bN(0) | (bN(1) << 8), l2 = bN(2) | (bN(3) << 8), l3 = bN(4) | (bN(5) << 8);
        const uint32_t seg = (nlit + 3) / 4;
        fail = l1 + l2 + l3 + 6 > qn || 3 * seg > nlit;
        const uint32_t l4 = qn - 6 - l1 - l2 - l3, s0 = fq + 6;
        sb = lane == 0 ? s0 : lane == 1 ? s0 + l1 : lane == 2 ? s0 + l1 + l2 : s0 + l1 + l2 + l3;
        sl = lane == 0 ? l1 : lane == 1 ? l2 : lane == 2 ? l3 : l4;
        m = lane < 3 ? seg : nlit - 3 * seg;
        lo = seg * (lane < 3 ? lane : 3u);
      }
    }
    if (fail) {  // to the exact path, as phase B' hands a block back
      if (lane == 0) {
        z.rec[b].info = 0;
        z.list[atomicAdd(z.count, 1u)] = b;
      }
      continue;
    }
    // (the table went to the slot); the stream records (absolute frame-relative starts)
    if (lane < 4) dk[lane] = lane < nstr ? make_uint4(shift + sb, sl, m, lo | (tl << 16)) : make_uint4(0, 0, 0, 0);
    zs_sync();
  }
}

// H1, lane per block (shipped; the wave-per-block zs_huf_tree_kernel above stays for A/B runs,
// SLATE_ZF_H1_WAVE): the tree description as zs_huf_read reads it -- direct 4-bit weights, or
// FSE-coded ones (zf_ncount8 / zf_fse_build16 as phase A' builds its tables, then the two-state
// decode of zs_weights_fse) -- the weight checks, and the weight-major table written to the slot
// with stores of 1, 2, 4 or 8 entries (a weight-w symbol's 2^(w-1) entries start at a multiple of
// 2^(w-1)).  Stricter than the exact path where it is cheaper (more than 16 weight symbols, counts
// above 127): such blocks go to the exact path, which decodes and reports them.  One wave per
// 64 blocks: configs[4]'s ~11 k Huffman blocks are ~170 waves, so the LDS is not rationed.
constexpr uint32_t kZhLWin = 176;   // 11 chunks from the one holding the description's first byte
// LDS, by region (per-lane accesses at one offset land in distinct banks where they are hot):
//   window   lane l at 180 l (45 dwords: odd), written as dwords -- the weight decode's bit reads
//   norm/next lane l at kZhLNn + 96 l (the FSE build's counts, brief)
//   ft       lane l at kZhLFt + 144 l (the FSE table as zf_fse_build16 builds it: 16-byte aligned)
//   fti      entry i of lane l at kZhLFti + 2 (64 i + l) (the same table interleaved: the decode's reads)
//   w        weight k of lane l at kZhLW + 64 k + l (interleaved bytes)
constexpr uint32_t kZhLWinStride = 180;
constexpr uint32_t kZhLNn = 64 * kZhLWinStride, kZhLFt = kZhLNn + 64 * 96, kZhLFti = kZhLFt + 64 * 144,
                   kZhLW = kZhLFti + 64 * 64 * 2, kZhLLds = kZhLW + 64 * 256;
static_assert(kZhLWinStride % 4 == 0 && (kZhLWinStride / 4) % 2 == 1 && kZhLWinStride >= kZhLWin, "window stride");

// packed per-weight counters (9 bits each, weights 1..11) and table cursors (12 bits each)
__device__ __forceinline__ void zh_cnt_add(uint64_t& c0, uint64_t& c1, uint32_t my) {
  c0 += (my >= 1 && my <= 6) ? uint64_t(1) << (9 * (my - 1)) : 0ull;
  c1 += (my >= 7 && my <= 11) ? uint64_t(1) << (9 * (my - 7)) : 0ull;
}
__device__ __forceinline__ uint32_t zh_cnt(uint64_t c0, uint64_t c1, uint32_t q) {
  return uint32_t((q <= 6 ? c0 >> (9 * (q - 1)) : c1 >> (9 * (q - 7))) & 511u);
}

__global__ __launch_bounds__(64) void zs_huf_tree_lanes_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t items = min(z.count[1], z.hcap);
  const uint32_t lane = threadIdx.x & 63;
  uint8_t* win = smem + lane * kZhLWinStride;
  uint32_t* wind = reinterpret_cast<uint32_t*>(win);
  int8_t* norm = reinterpret_cast<int8_t*>(smem + kZhLNn + 96 * lane);
  uint8_t* next = smem + kZhLNn + 96 * lane + 32;
  uint16_t* ft = reinterpret_cast<uint16_t*>(smem + kZhLFt + 144 * lane);
  uint16_t* fti = reinterpret_cast<uint16_t*>(smem + kZhLFti) + lane;  // entry i at fti[64 i]
  uint8_t* w = smem + kZhLW + lane;                                      // weight k at w[64 k]
  for (uint32_t r0 = blockIdx.x * 64; r0 < items; r0 += gridDim.x * 64) {
    const uint32_t k = r0 + lane;
    uint32_t b = 0, fl = 0;
    ZsFastRec rec{};
    if (k < items) {
      b = z.hlist[k];
      rec = z.rec[b];
      fl = rec.info >> 16;
    }
    const bool act = k < items && (fl & kZfFast);  // (else the CRC32 failed in phase A2)
    bool ok = act;
    uint32_t shift = 0, off = 0, lit = rec.lit, cs = rec.cs, nlit = rec.nlit;
    if (act) {
      const uint64_t i0 = a.in_off[b];
      const uint32_t len = uint32_t(a.in_off[b + 1] - i0);
      shift = uint32_t(reinterpret_cast<uintptr_t>(a.in + i0) & 15);
      const uint8_t* F = a.in + i0 - shift;
      const uint32_t c0 = (shift + lit) >> 4, cend = (shift + len + 15) >> 4;
      off = (shift + lit) & 15;
      v4u ch[kZhLWin / 16];
#pragma unroll
      for (uint32_t c = 0; c < kZhLWin / 16; c++)
        ch[c] = c0 + c < cend ? *reinterpret_cast<const v4u*>(F + 16 * (c0 + c)) : v4u{0, 0, 0, 0};
#pragma unroll
      for (uint32_t c = 0; c < kZhLWin / 16; c++) {
        wind[4 * c] = ch[c].x;
        wind[4 * c + 1] = ch[c].y;
        wind[4 * c + 2] = ch[c].z;
        wind[4 * c + 3] = ch[c].w;
      }
    }
    // ---- the weights (zs_huf_read / zs_weights_fse)
    uint32_t nw = 0, used = 0;
    ok = ok && cs >= 1;
    const uint32_t hb = ok ? uint32_t(win[off]) : 0u;
    if (ok && hb >= 128) {
      nw = hb - 127;
      const uint32_t nbytes = (nw + 1) / 2;
      ok = 1 + nbytes <= cs;
      for (uint32_t i = 0; ok && i < nw; i++) {
        const uint32_t by = win[off + 1 + i / 2];
        w[64 * i] = uint8_t((i & 1) ? (by & 15) : (by >> 4));
      }
      used = 1 + nbytes;
    } else if (ok) {
      ok = 1 + hb <= cs;
      int r = -1;
      if (ok) r = zf_ncount8(win, int32_t(off + 1), hb, norm, 15, 6);
      ok = ok && r >= 0;
      const uint32_t hs = ok ? uint32_t(r & 0xFFFF) : 0u, al = ok ? uint32_t((r >> 16) & 0xFF) : 0u;
      const int last = ok ? (r >> 24) : 0;
      ok = ok && zf_fse_build16(ft, norm, last, int(al), next);
      if (ok)
        for (uint32_t i = 0; i < (1u << al); i++) fti[64 * i] = ft[i];
      const uint32_t so = off + 1 + hs, bn = hb - hs;
      ok = ok && bn != 0;
      const uint32_t lastb = ok ? uint32_t(win[so + bn - 1]) : 0u;
      ok = ok && lastb != 0;
      int32_t pos = ok ? int32_t(8 * (bn - 1) + (31 - __builtin_clz(lastb | 1u))) : 0;
      // the backward stream's bits through a 64-bit register window [wlo, wlo + 64) (wlo a multiple
      // of 32; stream dword d = bytes so + 4d .. +3, zeros below the stream's first bit: rd's
      // semantics for pos < kb), refilled from the lane's window when a read would leave it
      int32_t wlo = INT32_MAX;
      uint64_t wv = 0;
      auto sdw = [&](int32_t d) -> uint32_t { return d >= 0 ? lds_u32(win, int32_t(so) + 4 * d) : 0u; };
      auto rd = [&](uint32_t kb) -> uint32_t {
        const int32_t lo = pos - int32_t(kb);
        if (lo < wlo) {
          wlo = ((pos + 31) & ~31) - 64;
          const int32_t d = wlo >> 5;
          wv = uint64_t(sdw(d)) | (uint64_t(sdw(d + 1)) << 32);
        }
        const uint32_t v = uint32_t(wv >> uint32_t(lo - wlo)) & ((1u << kb) - 1u);
        pos = lo;
        return v;
      };
      if (ok) {
        uint32_t s1 = rd(al), s2 = rd(al);
        for (;;) {  // two interleaved states until the stream overreads (FSE_decompress tail)
          if (nw > 253) {
            ok = false;
            break;
          }
          uint32_t e = fti[64 * s1];
          w[64 * nw++] = uint8_t(e & 63u);
          s1 = (e >> 9) + rd((e >> 6) & 7u);
          if (pos < 0) {
            w[64 * nw++] = uint8_t(fti[64 * s2] & 63u);
            break;
          }
          if (nw > 253) {
            ok = false;
            break;
          }
          e = fti[64 * s2];
          w[64 * nw++] = uint8_t(e & 63u);
          s2 = (e >> 9) + rd((e >> 6) & 7u);
          if (pos < 0) {
            w[64 * nw++] = uint8_t(fti[64 * s1] & 63u);
            break;
          }
        }
      }
      used = 1 + hb;
    }
    // ---- weight statistics (zs_huf_read): counts per weight, the implied last weight, tl
    uint32_t tl = 0;
    uint64_t c0 = 0, c1 = 0;
    if (ok) {
      uint32_t total = 0;
      for (uint32_t i = 0; i < nw; i++) {
        const uint32_t my = w[64 * i];
        ok = ok && my <= 11;
        total += (my && my <= 11) ? (1u << (my - 1)) : 0u;
        zh_cnt_add(c0, c1, my);
      }
      ok = ok && total != 0;
      tl = 32 - __builtin_clz(total | 1u);
      ok = ok && tl <= 11;
      const uint32_t rest = (1u << tl) - total;
      ok = ok && rest != 0 && !(rest & (rest - 1));
      const uint32_t lastw = 32 - __builtin_clz(rest | 1u);
      if (ok) {
        w[64 * nw] = uint8_t(lastw);
        zh_cnt_add(c0, c1, lastw);
      }
      const uint32_t r1 = zh_cnt(c0, c1, 1);
      ok = ok && r1 >= 2 && !(r1 & 1);
    }
    // ---- the weight-major table into the slot: symbol s of weight my at cur[my], 2^(my-1) entries
    if (ok) {
      uint64_t p0 = 0, p1 = 0, p2 = 0;  // cursors, 12 bits each: weights 1..5, 6..10, 11
      uint32_t acc = 0;
      for (uint32_t q = 1; q <= tl; q++) {
        const uint64_t v = uint64_t(acc);
        p0 |= q <= 5 ? v << (12 * (q - 1)) : 0ull;
        p1 |= (q >= 6 && q <= 10) ? v << (12 * (q - 6)) : 0ull;
        p2 |= q == 11 ? v : 0ull;
        acc += zh_cnt(c0, c1, q) << (q - 1);
      }
      uint8_t* tab = z.htab + size_t(k) * kZhTab;
      for (uint32_t sy = 0; sy <= nw; sy++) {
        const uint32_t my = w[64 * sy];
        if (!my) continue;
        const uint32_t sh = my <= 5 ? 12 * (my - 1) : (my <= 10 ? 12 * (my - 6) : 0u);
        const uint64_t word = my <= 5 ? p0 : (my <= 10 ? p1 : p2);
        const uint32_t p = uint32_t(word >> sh) & 4095u, ne = 1u << (my - 1);
        const uint64_t inc = uint64_t(ne) << sh;
        p0 += my <= 5 ? inc : 0ull;
        p1 += (my >= 6 && my <= 10) ? inc : 0ull;
        p2 += my == 11 ? inc : 0ull;
        const uint32_t e = ((tl + 1 - my) << 8) | sy, e2 = e | (e << 16);
        uint8_t* dst = tab + 2 * p;
        if (ne >= 8) {
          for (uint32_t c = 0; c < ne / 8; c++) *reinterpret_cast<uint4*>(dst + 16 * c) = make_uint4(e2, e2, e2, e2);
        } else if (ne == 4) {
          *reinterpret_cast<uint2*>(dst) = make_uint2(e2, e2);
        } else if (ne == 2) {
          *reinterpret_cast<uint32_t*>(dst) = e2;
        } else {
          *reinterpret_cast<uint16_t*>(dst) = uint16_t(e);
        }
      }
    }
    // ---- the streams (as phase B': one, or four behind a 6-byte jump table)
    const uint32_t nstr = (fl & kZfHuf4) ? 4u : 1u;
    uint4 sd[4] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (ok) {
      const uint32_t q = off + used, qn = cs - used, fq = lit + used;
      if (nstr == 1) {
        sd[0] = make_uint4(shift + fq, qn, nlit, tl << 16);
      } else if (qn < 10) {
        ok = false;
      } else {
        const uint32_t l1 = win[q] | (uint32_t(win[q + 1]) << 8), l2 = win[q + 2] | (uint32_t(win[q + 3]) << 8),
                       l3 = win[q + 4] | (uint32_t(win[q + 5]) << 8);
        const uint32_t seg = (nlit + 3) / 4;
        ok = !(l1 + l2 + l3 + 6 > qn || 3 * seg > nlit);
        const uint32_t l4 = qn - 6 - l1 - l2 - l3, s0 = shift + fq + 6;
        sd[0] = make_uint4(s0, l1, seg, 0 | (tl << 16));
        sd[1] = make_uint4(s0 + l1, l2, seg, seg | (tl << 16));
        sd[2] = make_uint4(s0 + l1 + l2, l3, seg, (2 * seg) | (tl << 16));
        sd[3] = make_uint4(s0 + l1 + l2 + l3, l4, nlit - 3 * seg, (3 * seg) | (tl << 16));
      }
    }
    if (ok) {
      uint4* dk = reinterpret_cast<uint4*>(z.hdesc + 16 * size_t(k));
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) dk[i] = sd[i];
    }
    // any failed check: to the exact path, as phase B' hands a block back
    if (act && !ok) z.rec[b].info = 0;
    list_append(act && !ok, b, z.list, z.count);
  }
}

namespace {
// chunk c of the frame (16-byte aligned base F) as a stream starting at frame byte fs sees it: the
// bytes before fs read as zeros (a backward stream's bits below its start: zs_peek), so a peek
// needs no end-of-stream case
__device__ __forceinline__ uint4 zh_chunk(const uint8_t* F, int32_t c, uint32_t fs) {
  const int32_t c0 = int32_t(fs >> 4);
  if (c < c0) return make_uint4(0, 0, 0, 0);
  uint4 v = *reinterpret_cast<const uint4*>(F + 16 * c);
  if (c == c0) {
    const uint32_t z = fs & 15;  // bytes [0, z) zeroed
    auto keep = [&](uint32_t k) -> uint32_t {  // dword k's mask
      const int32_t n = int32_t(z) - int32_t(4 * k);  // its bytes below fs
      return n <= 0 ? 0xFFFFFFFFu : (n >= 4 ? 0u : ~((1u << (8 * n)) - 1u));
    };
    v.x &= keep(0);
    v.y &= keep(1);
    v.z &= keep(2);
    v.w &= keep(3);
  }
  return v;
}
}  // namespace

__global__ __launch_bounds__(64) void zs_huf_stream_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t items = min(z.count[1], z.hcap);
  const uint32_t lane = threadIdx.x & 63, j = lane >> 2, l = lane & 3;
  uint8_t* ring = smem + kZhBlocks * kZhTab + min(lane, 4 * kZhBlocks - 1) * kZhRing;
  uint32_t* rd = reinterpret_cast<uint32_t*>(ring);
  for (uint32_t k0 = blockIdx.x * kZhBlocks; k0 < items; k0 += gridDim.x * kZhBlocks) {
    // the 16 blocks' tables (whole slots; entries past 2^tl are never read)
    {
      const uint32_t nb = min(kZhBlocks, items - k0);
      const uint4* src = reinterpret_cast<const uint4*>(z.htab + size_t(k0) * kZhTab);
      uint4* dst = reinterpret_cast<uint4*>(smem);
      for (uint32_t c = lane; c < nb * (kZhTab / 16); c += kWave) dst[c] = src[c];
    }
    const uint32_t k = k0 + j;
    const bool mine = j < kZhBlocks && k < items;  // (lanes 60..63 idle)
    uint32_t b = 0, fl = 0;
    uint4 d = make_uint4(0, 0, 0, 0);
    if (mine) {
      b = z.hlist[k];
      fl = z.rec[b].info >> 16;
      d = reinterpret_cast<const uint4*>(z.hdesc + 16 * size_t(k))[l];
    }
    const uint32_t tl = d.w >> 16, lo = d.w & 0xFFFFu, m = d.z, sl = d.y, fs = d.x;
    // the lane's stream: frame bytes [fs, fs + sl) from the 16-aligned frame base F
    bool act = mine && (fl & kZfFast) && tl != 0;
    const uint8_t* F = nullptr;
    uint8_t* out = nullptr;
    if (act) {
      const uint64_t i0 = a.in_off[b];
      F = a.in + i0 - (reinterpret_cast<uintptr_t>(a.in + i0) & 15);
      out = a.out + a.out_off[b] + lo;
    }
    bool bad = act && sl == 0;
    act = act && !bad;
    // the top chunk (the stream's last byte: zs_bstart) and the one below into the ring
    const int32_t T = act ? int32_t((fs + sl - 1) >> 4) : 0;
    const uint4 cT = act ? zh_chunk(F, T, fs) : make_uint4(0, 0, 0, 0);
    const uint4 cT1 = act ? zh_chunk(F, T - 1, fs) : make_uint4(0, 0, 0, 0);
    auto put = [&](int32_t c, const uint4& v) {  // (dwords: the ring is 4-byte aligned)
      uint32_t* q = rd + 4 * (c & 3);
      q[0] = v.x;
      q[1] = v.y;
      q[2] = v.z;
      q[3] = v.w;
    };
    if (mine) {
      put(T, cT);
      put(T - 1, cT1);
    }
    int32_t lowc = T - 1;
    uint4 pf = act ? zh_chunk(F, T - 2, fs) : make_uint4(0, 0, 0, 0);
    const uint32_t lb = (fs + sl - 1) & 15;
    const uint32_t lw = lb < 4 ? cT.x : lb < 8 ? cT.y : lb < 12 ? cT.z : cT.w;
    const uint32_t lastb = (lw >> (8 * (lb & 3))) & 0xFFu;
    bad = bad || (act && lastb == 0);
    act = act && lastb != 0;
    // P: the frame-relative bit just above the next code; the stream ends exactly at P0 = 8 fs
    const int32_t P0 = int32_t(8 * fs);
    int32_t P = act ? P0 + int32_t(8 * (sl - 1) + (31 - __builtin_clz(lastb | 1u))) : P0;
    int32_t clo = 0;
    uint64_t cv = 0;
    const uint32_t tmask = (1u << tl) - 1u;
    const uint16_t* tab = reinterpret_cast<const uint16_t*>(smem + min(j, kZhBlocks - 1) * kZhTab);
    zs_sync();
    // the window's first fill (below)
    clo = INT32_MAX;
    // the output through a 16-byte register stage aligned to the address (a store per 16 bytes,
    // so the chunk commit's wait finds the last store long done); the stage's partly covered
    // pieces at the stream's two ends go out as byte stores (the neighbouring stream owns the rest)
    const uint32_t ph = uint32_t(reinterpret_cast<uintptr_t>(out)) & 15u;
    uint64_t sg0 = 0, sg1 = 0;
    auto flush = [&](uint32_t i_last) {  // the stage holds output bytes up to symbol i_last
      const uint32_t e = ph + i_last + 1, c0 = (e - 1) & ~15u;  // the stage's piece [c0, c0 + 16)
      uint8_t* dst = out - ph + c0;
      const uint32_t lo_b = c0 < ph ? ph - c0 : 0u, hi_b = e - c0;  // covered bytes [lo_b, hi_b)
      if (lo_b == 0 && hi_b == 16) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(uint32_t(sg0), uint32_t(sg0 >> 32), uint32_t(sg1), uint32_t(sg1 >> 32));
      } else {
        for (uint32_t q = lo_b; q < hi_b; q++) dst[q] = uint8_t((q < 8 ? sg0 >> (8 * q) : sg1 >> (8 * (q - 8))) & 0xFF);
      }
      sg0 = sg1 = 0;
    };
    for (uint32_t i = 0; __ballot(act && i < m); i++) {
      const bool go = act && i < m;
      if (go && P - int32_t(tl) < clo) {
        // 64 bits from the dword boundary at or above P, down: two ring dwords
        clo = ((P + 31) & ~31) - 64;
        const int32_t D = clo >> 5;
        if ((D >> 2) < lowc) {  // one chunk lower: commit the prefetched one, fetch the next
          lowc -= 1;
          put(lowc, pf);
          pf = zh_chunk(F, lowc - 1, fs);
        }
        cv = uint64_t(rd[D & 15]) | (uint64_t(rd[(D + 1) & 15]) << 32);
      }
      const uint32_t v = uint32_t(cv >> uint32_t(P - int32_t(tl) - clo)) & tmask;  // (zeros below the stream)
      const uint32_t e = tab[v];
      if (go) {
        const uint32_t q = (ph + i) & 15u;
        const uint64_t by = uint64_t(e & 0xFFu) << (8 * (q & 7));
        sg0 |= q < 8 ? by : 0ull;
        sg1 |= q < 8 ? 0ull : by;
        if (q == 15 || i + 1 == m) flush(i);
        P -= int32_t(e >> 8);
      }
    }
    bad = bad || (act && P != P0);
    // per block: any failing stream hands it back; else phase B builds it from the output slot
    const uint32_t bm = uint32_t(__ballot(bad) >> (4 * j)) & 15u;
    if (l == 0 && mine && (fl & kZfFast) && tl != 0) {
      if (bm) {
        z.rec[b].info = 0;
        z.list[atomicAdd(z.count, 1u)] = b;
      } else {
        // (atomics: phase A2 may clear the record at the same time on the main stream; a cleared
        // record stays without kZfFast, and B / C skip it)
        atomicAnd(&z.rec[b].info, ~((kZfHuf | kZfHuf4) << 16));
        atomicOr(&z.rec[b].info, kZfOutLit << 16);
      }
    }
    zs_sync();
  }
}

// ------------------------------------------------------------------------------- phase C
// The frame checksum of each fast block whose CRC32 held (phase B), lane per block: XXH64 (seed
// 0) of the decoded block, whose four accumulators' serial chains advance for 64 blocks in one
// wave instruction.  A mismatch goes to the exact path, which reports it.  Round of 64 blocks:
// each iteration brings the next 64 bytes of every block with transposed loads (in load j,
// lanes 4i..4i+3 read one 64-byte run of block 16j+i) issued one iteration ahead into
// registers; the loading lanes put them into the owner's LDS slot, and every lane runs two
// 32-byte stripes.
// kRun = 256 (phase C since round 5): 256-byte runs, lanes 16i..16i+15 of load j reading block 4j+i
// -- fewer address-unit requests per byte than 64-byte runs (tools/scatter_probe.hip: ~188 CU
// cycles per wave-instruction for 64-byte runs, ~98 for 128-byte ones), eight stripes per
// iteration, 64 KiB of LDS per workgroup.  Same-box A/Bs (profiles/round5/ab_zstd_runs.txt): C at
// 128 B +2.5 % on configs[4], at 256 B another +0.5 % (and +0.3 % on kv100); A2 at 128 B (256
// threads, for the LDS) 1 % slower than at 64 B with 512 threads, so A2 keeps 64.
#ifndef SLATE_ZF_SUM_RUN
#define SLATE_ZF_SUM_RUN 256
#endif
#ifndef SLATE_ZF_CRC_RUN
#define SLATE_ZF_CRC_RUN 64
#endif
namespace {
template <uint32_t kRun>
struct ZfGroup {
  v4u p[kRun / 16];
};
template <uint32_t kRun>
__device__ __forceinline__ ZfGroup<kRun> zf_load_group(__amdgpu_buffer_rsrc_t R, uint32_t t, uint32_t rel,
                                                       uint32_t groups, uint32_t lane) {
  constexpr uint32_t kL = kRun / 16;  // lanes per block in one load
  ZfGroup<kRun> g;
#pragma unroll
  for (uint32_t j = 0; j < kL; j++) {
    const uint32_t o = (64 / kL) * j + lane / kL, c = lane % kL;
    const uint32_t g_o = __shfl(groups, int(o), 64), rel_o = __shfl(rel, int(o), 64);
    g.p[j] = bload(R, t < g_o ? rel_o + kRun * t + 16 * c : kOOB);
  }
  return g;
}
template <uint32_t kRun>
__device__ __forceinline__ void zf_commit_group(const ZfGroup<kRun>& g, uint8_t* slots0, uint32_t t, uint32_t groups,
                                                uint32_t lane) {
  constexpr uint32_t kL = kRun / 16;
#pragma unroll
  for (uint32_t j = 0; j < kL; j++) {
    const uint32_t o = (64 / kL) * j + lane / kL, c = lane % kL;
    if (t < uint32_t(__shfl(groups, int(o), 64))) lds_put16(slots0 + o * kRun + 16 * c, g.p[j]);
  }
}
}  // namespace

__global__ __launch_bounds__(kZfSumThreads) void zs_fast_sum_kernel(DecodeArgs a, ZsFastArgs z) {
  constexpr uint32_t kRun = SLATE_ZF_SUM_RUN;
  __shared__ __attribute__((aligned(16))) uint8_t slots[kZfSumThreads * kRun];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_lane0 = threadIdx.x - lane;
  uint8_t* slots0 = slots + wave_lane0 * kRun;
  const uint8_t* mine = slots0 + lane * kRun;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x + wave_lane0; r0 < a.n; r0 += stride) {
    const uint32_t b = r0 + lane;
    const uint32_t rend = min(r0 + 64, a.n);
    const __amdgpu_buffer_rsrc_t R = make_rsrc(a.out + a.out_off[r0], a.out_off[rend] - a.out_off[r0]);
    uint32_t orel = 0, len = 0, want = 0;
    bool act = false;
    if (b < a.n) {
      const ZsFastRec rec = z.rec[b];
      const uint32_t fl = rec.info >> 16;
      act = (fl & kZfFast) && (fl & kZfSum) && a.meta[b].status != SLATE_E_BLOCK_CHECKSUM;
      len = act ? rec.produced : 0u;
      want = rec.want;
      orel = uint32_t(a.out_off[b] - a.out_off[r0]);
    }
    const uint32_t groups = (len + kRun - 1) / kRun, stripes = len / 32;
    uint64_t v0 = kX64P1 + kX64P2, v1 = kX64P2, v2 = 0, v3 = 0ull - kX64P1;
    ZfGroup<kRun> g = zf_load_group<kRun>(R, 0, orel, groups, lane);
    for (uint32_t t = 0; __ballot(t < groups); t++) {
      zf_commit_group<kRun>(g, slots0, t, groups, lane);
      g = zf_load_group<kRun>(R, t + 1, orel, groups, lane);  // in flight during this iteration
      zs_sync();
#pragma unroll
      for (uint32_t h = 0; h < kRun / 32; h++) {
        if ((kRun / 32) * t + h < stripes && !(dbg_bits(a) & (1u << 24))) {
          const uint64_t* w = reinterpret_cast<const uint64_t*>(mine + 32 * h);
          v0 = x64round(v0, w[0]);
          v1 = x64round(v1, w[1]);
          v2 = x64round(v2, w[2]);
          v3 = x64round(v3, w[3]);
        }
      }
      zs_sync();
    }
    bool bad = false;
    if (act) {
      // the tail (< 32 bytes) lies in the last group, still in this lane's slot
      uint64_t hh;
      if (len >= 32) {
        hh = x64rotl(v0, 1) + x64rotl(v1, 7) + x64rotl(v2, 12) + x64rotl(v3, 18);
        hh = (hh ^ x64round(0, v0)) * kX64P1 + kX64P4;
        hh = (hh ^ x64round(0, v1)) * kX64P1 + kX64P4;
        hh = (hh ^ x64round(0, v2)) * kX64P1 + kX64P4;
        hh = (hh ^ x64round(0, v3)) * kX64P1 + kX64P4;
      } else {
        hh = kX64P5;
      }
      hh += len;
      uint32_t i = len & ~31u;
      const uint8_t* tail = mine - kRun * ((len - 1) / kRun);  // tail[i] = decoded byte i (len > 0)
      for (; i + 8 <= len; i += 8)
        hh = x64rotl(hh ^ x64round(0, *reinterpret_cast<const uint64_t*>(tail + i)), 27) * kX64P1 + kX64P4;
      if (i + 4 <= len) {
        hh = x64rotl(hh ^ uint64_t(*reinterpret_cast<const uint32_t*>(tail + i)) * kX64P1, 23) * kX64P2 + kX64P3;
        i += 4;
      }
      for (; i < len; i++) hh = x64rotl(hh ^ uint64_t(tail[i]) * kX64P5, 11) * kX64P1;
      hh ^= hh >> 33;
      hh *= kX64P2;
      hh ^= hh >> 29;
      hh *= kX64P3;
      hh ^= hh >> 32;
      bad = uint32_t(hh) != want;
    }
    list_append(bad && !(dbg_bits(a) & (1u << 26)), b, z.list, z.count);
  }
}

// ------------------------------------------------------------------------------- phase A2
// The SST block CRC32 (block.go:83-89: the first check of block.Decode) of each block phase A
// took, lane per block, before anything is built: slicing-by-16 over whole 16-byte chunks, the
// payload's first and last chunk byte by byte, the encoded bytes streamed in 64-byte runs as in
// phase C.  A mismatch is reported here, as the exact path would (status only), and the block
// leaves the fast path.
__global__ __launch_bounds__(kZfCrcThreads) void zs_fast_crc_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  {
    const uint32_t* src = &g_crc16.t[0][0];
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = src[i];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_lane0 = threadIdx.x - lane;
  constexpr uint32_t kRun = SLATE_ZF_CRC_RUN;
  uint8_t* slots0 = smem + kTab16Bytes + wave_lane0 * kRun;
  const uint8_t* mine = slots0 + lane * kRun;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x + wave_lane0; r0 < a.n; r0 += stride) {
    const uint32_t b = r0 + lane;
    const uint32_t rend = min(r0 + 64, a.n);
    const uint8_t* ilo = a.in + a.in_off[r0];
    const uint8_t* ibase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(ilo) & ~uintptr_t(15));
    const __amdgpu_buffer_rsrc_t R = make_rsrc(ibase, align16(uint64_t((a.in + a.in_off[rend]) - ibase)));
    // lane's block: payload bytes [shift, shift + clen) of its aligned run, the stored CRC after
    uint32_t shift = 0, clen = 0, irel = 0, groups = 0;
    bool act = false;
    if (b < a.n) {
      act = (z.rec[b].info >> 16) & kZfFast;
      if (act) {
        const uint64_t s0 = a.in_off[b];
        shift = uint32_t(reinterpret_cast<uintptr_t>(a.in + s0) & 15);
        clen = uint32_t(a.in_off[b + 1] - s0) - 4;
        irel = uint32_t(((a.in + s0) - shift) - ibase);
        groups = (shift + clen + kRun - 1) / kRun;
      }
    }
    uint32_t stored = 0;
    {
      const uint32_t c = (shift + clen) >> 4;
      const v4u s0 = bload(R, act ? irel + 16 * c : kOOB), s1 = bload(R, act ? irel + 16 * c + 16 : kOOB);
      const uint32_t w[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const uint32_t p = (shift + clen) & 15;  // the stored CRC is bytes p..p+3 of the 32 loaded
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        lo = (p >> 2) == k ? w[k] : lo;
        hi = (p >> 2) + 1 == k ? w[k] : hi;
      }
      stored = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, p & 3));
    }
    uint32_t crc = 0xFFFFFFFFu;
    ZfGroup<kRun> g = zf_load_group<kRun>(R, 0, irel, groups, lane);
    for (uint32_t t = 0; __ballot(t < groups); t++) {
      zf_commit_group<kRun>(g, slots0, t, groups, lane);
      g = zf_load_group<kRun>(R, t + 1, irel, groups, lane);  // in flight during this iteration
      zs_sync();
#pragma unroll
      for (uint32_t k = 0; k < kRun / 16; k++) {
        const uint32_t c0 = kRun * t + 16 * k;  // aligned offset of the chunk
        const v4u v = *reinterpret_cast<const v4u*>(mine + 16 * k);
        const bool whole = t < groups && c0 >= shift && c0 + 16 <= shift + clen;
        const bool part = t < groups && !whole && c0 < shift + clen && c0 + 16 > shift;
        const uint32_t cw = crc16_step(tab, crc, v.x, v.y, v.z, v.w);
        crc = whole ? cw : crc;
        if (__ballot(part)) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t i = 0; i < 16; i++) {
            const uint32_t pos = c0 + i;
            const uint32_t byte = (w[i >> 2] >> (8 * (i & 3))) & 0xFF;
            const uint32_t cb = tab[(crc ^ byte) & 0xFF] ^ (crc >> 8);
            crc = (part && pos >= shift && pos < shift + clen) ? cb : crc;
          }
        }
      }
      zs_sync();
    }
    if (act && ~crc != stored) {
      slate_block_meta m{};
      m.status = SLATE_E_BLOCK_CHECKSUM;
      a.meta[b] = m;
      z.rec[b].info = 0;  // not built (B), not summed (C), not handed back
    }
  }
}

hipError_t launch_zstd_plan_fast(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n, uint64_t* out_sz,
                                 uint64_t* row_sz, uint32_t* list, uint32_t* count) {
  if (n == 0) return hipGetLastError();
  const uint32_t grid = min((n + kZfParseThreads - 1) / kZfParseThreads, 8192u);
  plan_zstd_fast_kernel<<<grid, kZfParseThreads, 0, st>>>(in, in_off, n, out_sz, row_sz, list, count);
  return hipGetLastError();
}

size_t zstd_fast_parse_lds() { return ((sizeof(ZfShared) + 15) & ~size_t(15)) + size_t(kZfParseThreads) * kZfLane; }

// Phase B' runs beside phase B: they take disjoint blocks (B skips Huffman-literal blocks, B' takes
// only those), B' keeps a few lanes of few waves busy for about a millisecond per 1 M configs[4]
// blocks, and B fills the chip.  On the caller's side stream (DecodeArgs::side, owned by its
// context), forked after phase A2 and joined before phase C.
// CodecZlib: phase Z (zlib_fast.hip) in place of A / A', then A2 and B (no Huffman-literal or
// XXH64 phase: B checks the Adler-32)
hipError_t launch_zlib_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus, bool parsed) {
  if (a.n == 0) return hipGetLastError();
  if (!parsed) {
    hipError_t e = launch_zlib_fast_parse(st, a, z, num_cus);
    if (e != hipSuccess) return e;
  }
  const size_t lds_crc = kTab16Bytes + size_t(kZfCrcThreads) * SLATE_ZF_CRC_RUN;
  const uint32_t grid_crc = min((a.n + kZfCrcThreads - 1) / kZfCrcThreads, uint32_t(num_cus) * 3u);
  zs_fast_crc_kernel<<<grid_crc, kZfCrcThreads, lds_crc, st>>>(a, z);
  const size_t lds_b = kZfBuildLds;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zs_fast_build_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_b));
  if (attr != hipSuccess) return attr;
  const uint32_t grid_b = min((a.n + kZfBuildThreads / 64 - 1) / (kZfBuildThreads / 64), uint32_t(num_cus) * SLATE_ZF_BUILD_WG);
  zs_fast_build_kernel<<<grid_b, kZfBuildThreads, lds_b, st>>>(a, z);
  return hipGetLastError();
}

hipError_t launch_zstd_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus) {
  if (a.n == 0) return hipGetLastError();
  const size_t lds_a = zstd_fast_parse_lds();
  const uint32_t grid_a = min((a.n + kZfParseThreads - 1) / kZfParseThreads, uint32_t(num_cus) * 2u);
  zs_fast_parse_kernel<<<grid_a, kZfParseThreads, lds_a, st>>>(a, z);
  // phase A': the blocks phase A listed for the FSE parse (four one-wave workgroups per CU)
  zs_fse_parse_kernel<<<uint32_t(num_cus) * kZfFseWgs, kZfFseThreads, size_t(kZfFseThreads) * kZfFseLane, st>>>(a, z);
  const size_t lds_crc = kTab16Bytes + size_t(kZfCrcThreads) * SLATE_ZF_CRC_RUN;
  // (read per call, for same-process A/B runs) SLATE_ZF_NO_H: phase B' takes every Huffman-literal
  // block; SLATE_ZF_H_SERIAL: phases H1 / H2 after A2 on the main stream instead of beside it;
  // SLATE_ZF_CRC_WG: phase A2's workgroups per CU (2 leave room for H1 / H2 beside it)
  const bool no_h = getenv("SLATE_ZF_NO_H") != nullptr;
  const bool h_serial = getenv("SLATE_ZF_H_SERIAL") != nullptr;
  const char* crc_wg_env = getenv("SLATE_ZF_CRC_WG");
  const uint32_t crc_wg = crc_wg_env && atoi(crc_wg_env) >= 1 && atoi(crc_wg_env) <= 3 ? uint32_t(atoi(crc_wg_env)) : 2u;
  const uint32_t grid_crc = min((a.n + kZfCrcThreads - 1) / kZfCrcThreads, uint32_t(num_cus) * crc_wg);
  ZsFastArgs zh = z;
  const uint32_t hmax = no_h ? 0u : min(a.n, z.hcap);
  if (no_h) zh.hcap = 0;
  SideStream* fh = (h_serial || !a.side || !hmax) ? nullptr : a.side;
  hipStream_t hs = st;
  if (fh && fh->get() && hipEventRecord(fh->fork, st) == hipSuccess && hipStreamWaitEvent(fh->s, fh->fork, 0) == hipSuccess)
    hs = fh->s;
  // phases H1 / H2: the Huffman-literal blocks' trees, then their streams lane per stream (the
  // workgroups of an empty list exit at once): beside A2 on the side stream, or after it
  static const hipError_t attr_t = hipFuncSetAttribute(reinterpret_cast<const void*>(&zs_huf_stream_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(kZhStreamLds));
  if (attr_t != hipSuccess) return attr_t;
  static const hipError_t attr_l = hipFuncSetAttribute(reinterpret_cast<const void*>(&zs_huf_tree_lanes_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(kZhLLds));
  if (attr_l != hipSuccess) return attr_l;
  const bool h1_wave = getenv("SLATE_ZF_H1_WAVE") != nullptr;
  const uint32_t grid_h1 = h1_wave ? min((hmax + 3) / 4, uint32_t(num_cus) * 8u) : min((hmax + 63) / 64, uint32_t(num_cus));
  auto launch_h1 = [&](hipStream_t q) {
    if (h1_wave) zs_huf_tree_kernel<<<grid_h1, kZhTreeThreads, kZhTreeLds, q>>>(a, z);
    else zs_huf_tree_lanes_kernel<<<grid_h1, 64, kZhLLds, q>>>(a, z);
  };
  const uint32_t grid_h2 = min((hmax + kZhBlocks - 1) / kZhBlocks, uint32_t(num_cus) * 2u);
  const size_t lds_b = kZfBuildLds;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zs_fast_build_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_b));
  if (attr != hipSuccess) return attr;
  const uint32_t grid_b = min((a.n + kZfBuildThreads / 64 - 1) / (kZfBuildThreads / 64), uint32_t(num_cus) * SLATE_ZF_BUILD_WG);
  const size_t lds_h = kZfHufLds;
  static const hipError_t attr_h = hipFuncSetAttribute(reinterpret_cast<const void*>(&zs_fast_huf_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_h));
  if (attr_h != hipSuccess) return attr_h;
  static const uint32_t huf_wg = [] {  // phase B' workgroups per CU (A/B runs: SLATE_ZF_HUF_WG, 1..3)
    const char* e = getenv("SLATE_ZF_HUF_WG");
    const uint32_t v = e ? uint32_t(atoi(e)) : 2u;
    return v >= 1 && v <= 163840 / kZfHufLds ? v : 2u;
  }();
  const uint32_t grid_c = min((a.n + kZfSumThreads - 1) / kZfSumThreads, uint32_t(num_cus) * 4u);
  // SLATE_ZF_B_EARLY=1 (read per call; off: slower on configs[4], profiles/round6/ab/ab_zstd_b_early.txt):
  // the main stream's B starts after A2 and skips the Huffman-literal blocks (kZfHufOrig); the side
  // stream runs H1, H2, then -- once A2 is done -- B over H2's blocks (list mode) and B' over the
  // list's rest, joined before C
  const char* early_env = getenv("SLATE_ZF_B_EARLY");
  const bool early = early_env && *early_env == '1';
  // SLATE_ZF_B_DRAW=G: phase B (main stream) draws G blocks at a time from a counter (0: static stride)
  const char* draw_env = getenv("SLATE_ZF_B_DRAW");
  const uint32_t bdraw = draw_env ? uint32_t(atoi(draw_env)) : 0u;
  ZsFastArgs zb = z;
  zb.draw = bdraw;
  // phase B's output stores non-temporal (SLATE_ZF_OUT_NT=0: default policy; read per call):
  // configs[4] 4.52 -> 4.33 ms, kv100 9.09 -> 9.04 (profiles/round6/ab/ab_zstd_out_nt.txt)
  const char* nt_env = getenv("SLATE_ZF_OUT_NT");
  zb.out_nt = nt_env && *nt_env == '0' ? 0u : 1u;
  if (hs != st && early) {
    launch_h1(hs);
    zs_huf_stream_kernel<<<grid_h2, 64, kZhStreamLds, hs>>>(a, z);
    zs_fast_crc_kernel<<<grid_crc, kZfCrcThreads, lds_crc, st>>>(a, z);
    hipError_t e = hipEventRecord(fh->fork, st);  // A2 done (fork's first wait was enqueued above)
    if (e == hipSuccess) e = hipStreamWaitEvent(hs, fh->fork, 0);
    if (e != hipSuccess) return e;
    ZsFastArgs zl = zb;
    zl.draw = 0;
    zl.blist = z.hlist;
    zs_fast_build_kernel<<<min((hmax + kZfBuildThreads / 64 - 1) / (kZfBuildThreads / 64), uint32_t(num_cus) * SLATE_ZF_BUILD_WG),
                           kZfBuildThreads, lds_b, hs>>>(a, zl);
    zs_fast_huf_kernel<<<uint32_t(num_cus) * huf_wg, kZfHufThreads, lds_h, hs>>>(a, zh);
    ZsFastArgs zm = zb;
    zm.skip_hufo = 1;
    zm.draw = bdraw;
    zs_fast_build_kernel<<<grid_b, kZfBuildThreads, lds_b, st>>>(a, zm);
    e = hipEventRecord(fh->join, hs);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, fh->join, 0);
    if (e != hipSuccess) return e;
    zs_fast_sum_kernel<<<grid_c, kZfSumThreads, 0, st>>>(a, z);
    return hipGetLastError();
  }
  if (hs != st) {
    launch_h1(hs);
    zs_huf_stream_kernel<<<grid_h2, 64, kZhStreamLds, hs>>>(a, z);
    zs_fast_crc_kernel<<<grid_crc, kZfCrcThreads, lds_crc, st>>>(a, z);
    hipError_t e = hipEventRecord(fh->join, hs);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, fh->join, 0);
    if (e != hipSuccess) return e;
  } else {
    zs_fast_crc_kernel<<<grid_crc, kZfCrcThreads, lds_crc, st>>>(a, z);
    if (hmax) {
      launch_h1(st);
      zs_huf_stream_kernel<<<grid_h2, 64, kZhStreamLds, st>>>(a, z);
    }
  }
  static const bool serial = getenv("SLATE_ZF_SERIAL") != nullptr;  // one stream (A/B runs)
  SideStream* f = (serial || !a.side) ? nullptr : a.side;
  hipStream_t sh = st;
  if (f && f->get() && hipEventRecord(f->fork, st) == hipSuccess && hipStreamWaitEvent(f->s, f->fork, 0) == hipSuccess)
    sh = f->s;
  zs_fast_huf_kernel<<<uint32_t(num_cus) * huf_wg, kZfHufThreads, lds_h, sh>>>(a, zh);
  zs_fast_build_kernel<<<grid_b, kZfBuildThreads, lds_b, st>>>(a, zb);
  if (sh != st) {
    hipError_t e = hipEventRecord(f->join, sh);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, f->join, 0);
    if (e != hipSuccess) return e;
  }
  zs_fast_sum_kernel<<<grid_c, kZfSumThreads, 0, st>>>(a, z);
  return hipGetLastError();
}

}  // namespace slate
