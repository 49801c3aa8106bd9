// Zstd index / filter payloads whose blocks depend on each other -- the frames klauspost/compress's
// streaming writer (compression.go:105-118) and libzstd produce: repeat offsets carried across
// blocks, treeless literals reusing the previous Huffman tree, FSE tables in repeat mode --
// decoded block-parallel.  compress.Decode CodecZstd is io.ReadAll(zstd.NewReader(buf))
// (compression.go:146-153); zstd.h zs_frame / zs_block is the exact GPU decoder this follows check
// for check (oracle/zstd_oracle.c the CPU restatement).
//
// Only the entropy state crosses blocks, so it is settled first and the rest runs per block:
//   1. zq_scan (one wave): every block's literal and sequence headers; FSE tables (own, RLE,
//      predefined) built into per-block slots, and for treeless literals / repeat tables the block
//      whose tree / table applies;
//   2. zq_huf (wave per tree): Huffman trees into per-block slots;
//   3. zq_lit (wave per block): literals (raw, RLE, 1 or 4 Huffman streams) into a literal buffer;
//   4. zq_seq (wave per block, bitstream in LDS): the sequences as (literal length, match length,
//      offset), a repeat offset kept symbolic -- max(rep_i at block start + delta, 1) -- and the
//      block's repeat-offset transform;
//   5. zq_chain (one lane): the transforms composed in block order: every block's starting repeat
//      offsets, its output offset, the frame's length;
//   6. zq_exec (wave per block): per decoded byte its literal (val[x], pa[x] = x) or the earlier
//      byte its match repeats (pa[x] = x - offset), then zlib_par.hip's pointer doubling + gather.
// Any check that fails sets flag[0] and the caller hands the payload to the exact decoder, which
// then decodes and reports it: a success here is the exact decoder's success with the same bytes.
#include <hip/hip_runtime.h>

#include <utility>

#include "kernels.h"
#include "zstd.h"

namespace slate {
namespace {

constexpr uint32_t kZqSlot = 512;     // FSE table slot entries (ll / ml accuracy <= 9, of <= 8)
constexpr uint32_t kZqHuf = 2048;     // Huffman slot entries (tree depth <= 11)
constexpr uint32_t kZqNone = ~0u;
constexpr uint32_t kZqSym = 0x80000000u;  // symbolic offset: slot << 29 | -delta

struct ZqBlk {
  uint32_t kind;      // 0 raw, 1 RLE, 2 compressed
  uint32_t body, bs;  // body offset in the payload, Block_Size
  uint32_t ltype, lsf, nlit, lhs, lcs, huf, hdesc;  // literal section; huf = tree block; hdesc = tree bytes
  uint32_t seq_off, seq_len, nseq;                   // sequence bitstream (after the table descriptions)
  uint32_t tslot[3], tal[3];                         // FSE tables (ll, of, ml): slot, accuracy log
  uint32_t seq_base, lit_base, out_base, out_len;
  uint32_t rep_t[3];  // the block's repeat-offset transform (symbolic slots, kZqSym form)
  uint32_t rep0[3];   // repeat offsets at its start (zq_chain)
};

struct ZqScratch {
  uint32_t* flag;  // [0] give up, [1] sequences, [2] literals, [3] decoded length
  ZqBlk* blk;
  ZsFse* fse;      // 3 slots per block + 3 predefined
  uint16_t* huf;   // one slot per block
  uint32_t* htl;   // tree depth per block
};

__host__ __device__ inline size_t zq_al(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline ZqScratch zq_carve(void* base, uint32_t nblk, size_t* bytes) {
  ZqScratch z;
  uint8_t* q = static_cast<uint8_t*>(base);
  auto take = [&](size_t b) {
    uint8_t* r = q;
    q += zq_al(b);
    return r;
  };
  z.flag = reinterpret_cast<uint32_t*>(take(64));
  z.blk = reinterpret_cast<ZqBlk*>(take(size_t(nblk) * sizeof(ZqBlk)));
  z.fse = reinterpret_cast<ZsFse*>(take((size_t(nblk) + 1) * 3 * kZqSlot * sizeof(ZsFse)));
  z.huf = reinterpret_cast<uint16_t*>(take(size_t(nblk) * kZqHuf * 2));
  z.htl = reinterpret_cast<uint32_t*>(take(size_t(nblk) * 4));
  if (bytes) *bytes = size_t(q - static_cast<uint8_t*>(base));
  return z;
}

// symbolic offsets: a value < 2^28, or max(rep_slot at block start - d, 1)
__device__ inline uint32_t zq_symbolic(uint32_t slot, uint32_t d) { return kZqSym | (slot << 29) | d; }
__device__ inline uint32_t zq_resolve(uint32_t v, const uint32_t* rep) {
  if (!(v & kZqSym)) return v;
  const uint32_t r = rep[(v >> 29) & 3], d = v & 0x1FFFFFFFu;
  return r > d + 1 ? r - d : 1u;
}
__device__ inline uint32_t zq_minus1(uint32_t v) {  // rep0 - 1, 0 -> 1 (zs_block)
  if (v & kZqSym) return v + 1;                     // the delta grows (max(x - d, 1) - 1 clamped)
  return v > 1 ? v - 1 : 1u;
}

// ---------------------------------------------------------------- 1. headers
// Symbol_Compression_Mode for one table type (zs_table), the table going to slot `own`; *slot is
// the type's current table (kZqNone: none yet in this frame).  Bytes used or -1.
__device__ int zq_table(uint32_t mode, const uint8_t* in, int32_t off, uint32_t n, uint32_t own, uint32_t pre,
                        uint32_t defal, int maxs, int maxal, ZsFse* fse, ZsScratch* sc, uint32_t* slot, uint32_t* al,
                        int lane) {
  if (mode == 0) {
    *slot = pre;
    *al = defal;
    return 0;
  }
  if (mode == 1) {
    if (n < 1) return -1;
    const uint32_t sym = zrfl(uint32_t(in[off]));
    if (int(sym) > maxs) return -1;
    if (lane == 0) {
      ZsFse e;
      e.sym = uint8_t(sym);
      e.nb = 0;
      e.base = 0;
      fse[size_t(own) * kZqSlot] = e;
    }
    *slot = own;
    *al = 0;
    return 1;
  }
  if (mode == 2) {
    int hs = 0, a = 0, last = 0;
    if (lane == 0) {  // built in LDS (the build's scattered read-modify-writes), then copied out
      hs = zs_ncount(in, off, n, sc->norm, maxs, maxal, &a, &last);
      if (hs >= 0 && zs_fse_build(sc->ll, sc->norm, last, a, sc->next)) hs = -1;
    }
    hs = zrfl(hs);
    a = zrfl(a);
    zs_sync();
    if (hs < 0) return -1;
    for (uint32_t i = uint32_t(lane); i < (1u << a); i += 64) fse[size_t(own) * kZqSlot + i] = sc->ll[i];
    zs_sync();
    *slot = own;
    *al = uint32_t(a);
    return hs;
  }
  return *slot != kZqNone ? 0 : -1;  // repeat
}

__global__ __launch_bounds__(64) void zq_scan_kernel(const uint8_t* __restrict__ in, const uint32_t* __restrict__ bl,
                                                     uint32_t nblk, uint32_t bmax, ZqScratch Z) {
  __shared__ __attribute__((aligned(16))) ZsScratch sc;
  const int lane = threadIdx.x;
  const uint32_t pre = 3 * nblk;  // predefined tables: slots pre + 0..2
  if (lane == 0) {  // in LDS, then copied out
    for (int i = 0; i < 36; i++) sc.norm[i] = kZsLLDef[i];
    zs_fse_build(sc.ll, sc.norm, 35, 6, sc.next);
    for (int i = 0; i < 29; i++) sc.norm[i] = kZsOFDef[i];
    zs_fse_build(sc.of, sc.norm, 28, 5, sc.next);
    for (int i = 0; i < 53; i++) sc.norm[i] = kZsMLDef[i];
    zs_fse_build(sc.ml, sc.norm, 52, 6, sc.next);
  }
  zs_sync();
  for (uint32_t i = uint32_t(lane); i < 64; i += 64) {
    Z.fse[size_t(pre) * kZqSlot + i] = sc.ll[i];
    Z.fse[size_t(pre + 2) * kZqSlot + i] = sc.ml[i];
  }
  for (uint32_t i = uint32_t(lane); i < 32; i += 64) Z.fse[size_t(pre + 1) * kZqSlot + i] = sc.of[i];
  zs_sync();
  uint32_t huf = kZqNone, cur[3] = {kZqNone, kZqNone, kZqNone}, cal[3] = {0, 0, 0};
  uint32_t nseq_all = 0, nlit_all = 0;
  bool bad = false;
  for (uint32_t k = 0; k < nblk && !bad; k++) {
    const uint32_t off = bl[2 * k], bh = bl[2 * k + 1], bt = (bh >> 1) & 3, bs = bh >> 3;
    ZqBlk B{};
    B.kind = bt;
    B.body = off;
    B.bs = bs;
    B.huf = kZqNone;
    B.seq_base = nseq_all;
    B.lit_base = nlit_all;
    B.out_len = bs;
    for (int t = 0; t < 3; t++) B.tslot[t] = kZqNone;
    if (bt == 2) {
      const int32_t o = int32_t(off);
      const uint32_t n = bs;
      auto bN = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(in[o + int32_t(i)])); };
      if (n < 1) { bad = true; break; }
      const uint32_t b0 = bN(0), type = b0 & 3, sf = (b0 >> 2) & 3;
      uint32_t pos, nlit, hs, cs = 0;
      if (type <= 1) {
        if (sf == 1) {
          hs = 2;
          if (n < 2) { bad = true; break; }
          nlit = (b0 >> 4) + (bN(1) << 4);
        } else if (sf == 3) {
          hs = 3;
          if (n < 3) { bad = true; break; }
          nlit = (b0 >> 4) + (bN(1) << 4) + (bN(2) << 12);
        } else {
          hs = 1;
          nlit = b0 >> 3;
        }
        if (nlit > bmax || (type == 0 ? (n - hs < nlit) : (n - hs < 1))) { bad = true; break; }
        pos = hs + (type == 0 ? nlit : 1);
      } else {
        if (sf <= 1) {
          hs = 3;
          if (n < 3) { bad = true; break; }
          const uint32_t h = b0 | (bN(1) << 8) | (bN(2) << 16);
          nlit = (h >> 4) & 0x3FF;
          cs = (h >> 14) & 0x3FF;
        } else if (sf == 2) {
          hs = 4;
          if (n < 4) { bad = true; break; }
          const uint32_t h = b0 | (bN(1) << 8) | (bN(2) << 16) | (bN(3) << 24);
          nlit = (h >> 4) & 0x3FFF;
          cs = (h >> 18) & 0x3FFF;
        } else {
          hs = 5;
          if (n < 5) { bad = true; break; }
          const uint64_t h = uint64_t(b0 | (bN(1) << 8) | (bN(2) << 16) | (bN(3) << 24)) | (uint64_t(bN(4)) << 32);
          nlit = uint32_t((h >> 4) & 0x3FFFF);
          cs = uint32_t((h >> 22) & 0x3FFFF);
        }
        if (nlit > bmax || n - hs < cs) { bad = true; break; }
        if (type == 2) huf = k;
        else if (huf == kZqNone) { bad = true; break; }
        B.huf = huf;
        pos = hs + cs;
      }
      B.ltype = type;
      B.lsf = sf;
      B.nlit = nlit;
      B.lhs = hs;
      B.lcs = cs;
      // Sequences_Section
      if (pos >= n) { bad = true; break; }
      const int32_t s = o + int32_t(pos);
      const uint32_t sn = n - pos;
      auto sB = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(in[s + int32_t(i)])); };
      uint32_t nseq, sp;
      const uint32_t c0 = sB(0);
      if (c0 < 128) {
        nseq = c0;
        sp = 1;
      } else if (c0 < 255) {
        if (sn < 2) { bad = true; break; }
        nseq = ((c0 - 128) << 8) + sB(1);
        sp = 2;
      } else {
        if (sn < 3) { bad = true; break; }
        nseq = sB(1) + (sB(2) << 8) + 0x7F00;
        sp = 3;
      }
      B.nseq = nseq;
      if (nseq == 0) {
        if (sp != sn) { bad = true; break; }
      } else {
        if (sp >= sn) { bad = true; break; }
        const uint32_t modes = sB(sp++);
        if (modes & 3) { bad = true; break; }
        int t = zq_table(modes >> 6, in, s + int32_t(sp), sn - sp, 3 * k, pre, 6, 35, 9, Z.fse, &sc, &cur[0], &cal[0], lane);
        if (t < 0) { bad = true; break; }
        sp += uint32_t(t);
        t = zq_table((modes >> 4) & 3, in, s + int32_t(sp), sn - sp, 3 * k + 1, pre + 1, 5, 31, 8, Z.fse, &sc, &cur[1],
                     &cal[1], lane);
        if (t < 0) { bad = true; break; }
        sp += uint32_t(t);
        t = zq_table((modes >> 2) & 3, in, s + int32_t(sp), sn - sp, 3 * k + 2, pre + 2, 6, 52, 9, Z.fse, &sc, &cur[2],
                     &cal[2], lane);
        if (t < 0) { bad = true; break; }
        sp += uint32_t(t);
        if (zs_bstart(in, s + int32_t(sp), sn - sp) < 0) { bad = true; break; }
        B.seq_off = uint32_t(s) + sp;
        B.seq_len = sn - sp;
        for (int q = 0; q < 3; q++) {
          B.tslot[q] = cur[q];
          B.tal[q] = cal[q];
        }
      }
      nseq_all += nseq;
      nlit_all += nlit;
    }
    // identity transform (zq_seq replaces it for blocks with sequences)
    for (uint32_t q = 0; q < 3; q++) B.rep_t[q] = zq_symbolic(q, 0);
    if (lane == 0) Z.blk[k] = B;
    if (nseq_all > (1u << 28) || nlit_all > (1u << 28)) bad = true;
  }
  if (lane == 0) {
    if (bad) Z.flag[0] = 1;
    Z.flag[1] = nseq_all;
    Z.flag[2] = nlit_all;
  }
}

// ---------------------------------------------------------------- 2. trees
__global__ __launch_bounds__(64) void zq_huf_kernel(const uint8_t* __restrict__ in, uint32_t nblk, ZqScratch Z) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kZsHufScratch];
  ZsScratch* sc = reinterpret_cast<ZsScratch*>(smem);
  const int lane = threadIdx.x;
  if (Z.flag[0]) return;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const ZqBlk& B = Z.blk[k];
    if (B.kind != 2 || B.ltype != 2) continue;
    uint32_t tl = 0;
    const int t = zs_huf_read(in, int32_t(B.body + B.lhs), B.lcs, sc, lane, &tl);
    if (t < 0) {
      if (lane == 0) atomicOr(Z.flag, 1u);
      continue;
    }
    uint16_t* dst = Z.huf + size_t(k) * kZqHuf;
    for (uint32_t i = uint32_t(lane); i < (1u << tl); i += 64) dst[i] = sc->huf[i];
    if (lane == 0) {
      Z.htl[k] = tl;
      Z.blk[k].hdesc = uint32_t(t);
    }
    zs_sync();
  }
}

// ---------------------------------------------------------------- 3. literals
// The literal section staged in LDS (<= 128 KiB), then zs_block's stream decode (streams on lanes
// 0..3) into the literal buffer.
__global__ __launch_bounds__(64) void zq_lit_kernel(const uint8_t* __restrict__ in, uint32_t nblk, ZqScratch Z,
                                                    uint8_t* __restrict__ lit) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  uint16_t* htab = reinterpret_cast<uint16_t*>(dyn);
  uint8_t* stage = dyn + kZqHuf * 2;
  const int lane = threadIdx.x;
  if (Z.flag[0]) return;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const ZqBlk B = Z.blk[k];
    if (B.kind != 2 || (B.nlit == 0 && B.ltype < 2)) continue;  // Huffman streams are checked even when empty
    uint8_t* dst = lit + B.lit_base;
    const uint32_t src = B.body + B.lhs;
    if (B.ltype == 0) {
      for (uint32_t j = uint32_t(lane); j < B.nlit; j += 64) dst[j] = in[src + j];
      continue;
    }
    if (B.ltype == 1) {
      const uint8_t v = in[src];
      for (uint32_t j = uint32_t(lane); j < B.nlit; j += 64) dst[j] = v;
      continue;
    }
    const uint32_t tl = Z.htl[B.huf];
    const uint16_t* hsrc = Z.huf + size_t(B.huf) * kZqHuf;
    for (uint32_t i = uint32_t(lane); i < (1u << tl); i += 64) htab[i] = hsrc[i];
    const uint32_t skip = B.ltype == 2 ? Z.blk[k].hdesc : 0u;
    if (skip > B.lcs) {
      if (lane == 0) atomicOr(Z.flag, 1u);
      continue;
    }
    const uint32_t q0 = src + skip, qn = B.lcs - skip;
    // stage [q0 & ~3, q0 + qn) (4-aligned base for the bit helpers) and 8 bytes of slack
    const uint32_t a0 = q0 & ~3u, sh = q0 - a0, tot = sh + qn;
    for (uint32_t j = uint32_t(lane) * 4; j < tot + 8; j += 256) {
      uint32_t v = 0;
      for (uint32_t b = 0; b < 4; b++) v |= (j + b < tot ? uint32_t(in[a0 + j + b]) : 0u) << (8 * b);
      *reinterpret_cast<uint32_t*>(stage + j) = v;
    }
    zs_sync();
    const uint32_t streams = B.lsf == 0 ? 1 : 4, nlit = B.nlit;
    uint32_t sb = 0, sl = 0, m = 0, lo = 0;
    bool fail = false;
    if (streams == 1) {
      sb = sh;
      sl = qn;
      m = nlit;
    } else {
      if (qn < 10) fail = true;
      if (!fail) {
        auto bS = [&](uint32_t i) -> uint32_t { return zrfl(uint32_t(stage[sh + i])); };
        const uint32_t l1 = bS(0) | (bS(1) << 8), l2 = bS(2) | (bS(3) << 8), l3 = bS(4) | (bS(5) << 8);
        const uint32_t seg = (nlit + 3) / 4;
        if (l1 + l2 + l3 + 6 > qn || 3 * seg > nlit) {
          fail = true;
        } else {
          const uint32_t l4 = qn - 6 - l1 - l2 - l3, s0 = sh + 6;
          sb = lane == 0 ? s0 : lane == 1 ? s0 + l1 : lane == 2 ? s0 + l1 + l2 : s0 + l1 + l2 + l3;
          sl = lane == 0 ? l1 : lane == 1 ? l2 : lane == 2 ? l3 : l4;
          m = lane < 3 ? seg : nlit - 3 * seg;
          lo = seg * uint32_t(lane < 3 ? lane : 3);
        }
      }
    }
    bool badl = false;
    if (!fail && uint32_t(lane) < streams) {
      int64_t bp = zs_bstart(stage, int32_t(sb), sl);
      if (bp < 0) {
        badl = true;
      } else {
        const int64_t S = 8 * int64_t(sb);
        const uint32_t tmask = (1u << tl) - 1;
        uint8_t* o = dst + lo;
        int64_t clo = 0;
        uint64_t cv = 0;
        bool have = false;
        for (uint32_t i = 0; i < m; i++) {
          const int64_t lo2 = bp - int64_t(tl);
          uint32_t v;
          if (have && lo2 >= clo) {
            v = uint32_t(cv >> (lo2 - clo)) & tmask;
          } else if (lo2 >= 0) {
            clo = bp > 56 ? bp - 56 : 0;
            cv = zs_bits(stage, S + clo, 56);
            have = true;
            v = uint32_t(cv >> (lo2 - clo)) & tmask;
          } else {
            v = uint32_t(zs_peek(stage, S, bp, tl));
          }
          const uint32_t e = htab[v];
          o[i] = uint8_t(e);
          bp -= e >> 8;
        }
        badl = bp != 0;
      }
    }
    if (fail || __ballot(badl)) {
      if (lane == 0) atomicOr(Z.flag, 1u);
    }
    zs_sync();
  }
}

// ---------------------------------------------------------------- 4. sequences
// The bitstream staged in LDS, the three tables copied next to it; zs_block's sequence loop and
// checks (those that need no concrete offset), offsets kept symbolic.
__global__ __launch_bounds__(64) void zq_seq_kernel(uint32_t nblk, uint32_t bmax, const uint8_t* __restrict__ in,
                                                    ZqScratch Z, uint32_t* __restrict__ sll, uint32_t* __restrict__ sml,
                                                    uint32_t* __restrict__ sof) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  ZsFse* tab = reinterpret_cast<ZsFse*>(dyn);  // ll | of | ml, kZqSlot each
  uint8_t* stage = dyn + 3 * kZqSlot * sizeof(ZsFse);
  const int lane = threadIdx.x;
  if (Z.flag[0]) return;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const ZqBlk B = Z.blk[k];
    if (B.kind != 2) continue;
    if (B.nseq == 0) {
      if (lane == 0) Z.blk[k].out_len = B.nlit;
      continue;
    }
    for (uint32_t t = 0; t < 3; t++) {
      const ZsFse* s = Z.fse + size_t(B.tslot[t]) * kZqSlot;
      const uint32_t n = 1u << B.tal[t];
      for (uint32_t i = uint32_t(lane); i < n; i += 64) tab[t * kZqSlot + i] = s[i];
    }
    const uint32_t a0 = B.seq_off & ~3u, sh = B.seq_off - a0, tot = sh + B.seq_len;
    for (uint32_t j = uint32_t(lane) * 4; j < tot + 8; j += 256) {
      uint32_t v = 0;
      for (uint32_t b = 0; b < 4; b++) v |= (j + b < tot ? uint32_t(in[a0 + j + b]) : 0u) << (8 * b);
      *reinterpret_cast<uint32_t*>(stage + j) = v;
    }
    zs_sync();
    const ZsFse *tll = tab, *tof = tab + kZqSlot, *tml = tab + 2 * kZqSlot;
    int64_t bp = zs_bstart(stage, int32_t(sh), B.seq_len);
    const int64_t S = 8 * int64_t(sh);
    auto rd = [&](uint32_t kb) -> uint32_t {
      const uint32_t v = zrfl(uint32_t(zs_peek(stage, S, bp, kb)));
      bp -= kb;
      return v;
    };
    uint32_t stl = rd(B.tal[0]), sto = rd(B.tal[1]), stm = rd(B.tal[2]);
    uint32_t rep[3] = {zq_symbolic(0, 0), zq_symbolic(1, 0), zq_symbolic(2, 0)};
    uint32_t lp = 0, o = 0;
    bool fail = bp < 0;
    uint32_t vll = 0, vml = 0, vof = 0;  // lane i & 63 keeps sequence i until the group of 64 is stored
    const uint32_t nseq = B.nseq, base = B.seq_base;
    for (uint32_t i = 0; i < nseq && !fail; i++) {
      const ZsFse ell = tll[stl], eof = tof[sto], eml = tml[stm];
      const uint32_t ofc = zrfl(uint32_t(eof.sym)), llc = zrfl(uint32_t(ell.sym)), mlc = zrfl(uint32_t(eml.sym));
      if (ofc > 31) {
        fail = true;
        break;
      }
      uint64_t ofv = (1ull << ofc);
      if (ofc > 24) {
        const uint32_t hi = rd(ofc - 24);
        ofv += (uint64_t(hi) << 24) + rd(24);
      } else {
        ofv += rd(ofc);
      }
      const uint32_t ml = kZsMLBase[mlc] + rd(kZsMLBits[mlc]);
      const uint32_t ll = kZsLLBase[llc] + rd(kZsLLBits[llc]);
      uint32_t offs;
      if (ofv > 3) {
        if (ofv - 3 >= (1ull << 28)) {  // beyond any output here: the exact decoder fails it
          fail = true;
          break;
        }
        offs = uint32_t(ofv - 3);
        rep[2] = rep[1];
        rep[1] = rep[0];
        rep[0] = offs;
      } else {
        const uint32_t idx = uint32_t(ofv) - 1 + (ll == 0 ? 1u : 0u);
        offs = idx == 3 ? zq_minus1(rep[0]) : rep[idx];
        if (idx >= 2) rep[2] = rep[1];
        if (idx >= 1) {
          rep[1] = rep[0];
          rep[0] = offs;
        }
      }
      if (i + 1 < nseq) {
        stl = zrfl(uint32_t(ell.base)) + rd(zrfl(uint32_t(ell.nb)));
        stm = zrfl(uint32_t(eml.base)) + rd(zrfl(uint32_t(eml.nb)));
        sto = zrfl(uint32_t(eof.base)) + rd(zrfl(uint32_t(eof.nb)));
      }
      if (bp < 0 || ll > B.nlit - lp || uint64_t(o) + ll + ml > bmax) {
        fail = true;
        break;
      }
      lp += ll;
      o += ll + ml;
      if (uint32_t(lane) == (i & 63)) {
        vll = ll;
        vml = ml;
        vof = offs;
      }
      if ((i & 63) == 63 || i + 1 == nseq) {
        const uint32_t g = i & ~63u;
        if (uint32_t(lane) <= (i & 63)) {
          sll[base + g + lane] = vll;
          sml[base + g + lane] = vml;
          sof[base + g + lane] = vof;
        }
      }
    }
    if (!fail && bp != 0) fail = true;
    const uint32_t rest = B.nlit - lp;
    if (!fail && uint64_t(o) + rest > bmax) fail = true;
    if (lane == 0) {
      if (fail) atomicOr(Z.flag, 1u);
      Z.blk[k].out_len = o + rest;
      for (int q = 0; q < 3; q++) Z.blk[k].rep_t[q] = rep[q];
    }
    zs_sync();
  }
}

// ---------------------------------------------------------------- 5. the chain of blocks
__global__ void zq_chain_kernel(uint32_t nblk, ZqScratch Z) {
  if (threadIdx.x != 0 || Z.flag[0]) return;
  uint32_t rep[3] = {1, 4, 8};
  uint64_t out = 0;
  for (uint32_t k = 0; k < nblk; k++) {
    ZqBlk& B = Z.blk[k];
    for (int q = 0; q < 3; q++) B.rep0[q] = rep[q];
    uint32_t nr[3];
    for (int q = 0; q < 3; q++) nr[q] = zq_resolve(B.rep_t[q], rep);
    for (int q = 0; q < 3; q++) rep[q] = nr[q];
    B.out_base = uint32_t(out);
    out += B.out_len;
    if (out > (1u << 28)) {
      Z.flag[0] = 1;
      return;
    }
  }
  Z.flag[3] = uint32_t(out);
}

// ---------------------------------------------------------------- 6. bytes
__global__ __launch_bounds__(64) void zq_exec_kernel(const uint8_t* __restrict__ in, uint32_t nblk, ZqScratch Z,
                                                     const uint8_t* __restrict__ lit, const uint32_t* __restrict__ sll,
                                                     const uint32_t* __restrict__ sml, const uint32_t* __restrict__ sof,
                                                     uint8_t* __restrict__ val, uint32_t* __restrict__ pa) {
  const int lane = threadIdx.x;
  if (Z.flag[0]) return;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const ZqBlk B = Z.blk[k];
    const uint32_t x0 = B.out_base;
    if (B.kind == 0 || B.kind == 1) {
      for (uint32_t j = uint32_t(lane); j < B.bs; j += 64) {
        val[x0 + j] = in[B.body + (B.kind == 0 ? j : 0u)];
        pa[x0 + j] = x0 + j;
      }
      continue;
    }
    const uint8_t* L = lit + B.lit_base;
    const uint32_t xend = x0 + B.out_len;
    uint32_t x = x0, lp = 0;
    bool fail = false;
    for (uint32_t g = 0; g < B.nseq && !fail; g += 64) {
      const uint32_t i = g + uint32_t(lane);
      const bool have = i < B.nseq;
      const uint32_t ll = have ? sll[B.seq_base + i] : 0u, ml = have ? sml[B.seq_base + i] : 0u;
      const uint32_t off = have ? zq_resolve(sof[B.seq_base + i], B.rep0) : 0u;
      const uint32_t cnt = min(64u, B.nseq - g);
      for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t a = __builtin_amdgcn_readlane(ll, int(j)), m = __builtin_amdgcn_readlane(ml, int(j));
        const uint32_t f = __builtin_amdgcn_readlane(off, int(j));
        if (uint64_t(x) + a + m > xend || lp + a > B.nlit) {
          fail = true;
          break;
        }
        for (uint32_t t = uint32_t(lane); t < a; t += 64) {
          val[x + t] = L[lp + t];
          pa[x + t] = x + t;
        }
        lp += a;
        x += a;
        if (f > x) {  // reaches before the frame (zs_block: offv > o - fstart)
          fail = true;
          break;
        }
        for (uint32_t t = uint32_t(lane); t < m; t += 64) pa[x + t] = x + t - f;
        x += m;
      }
    }
    if (!fail && x + (B.nlit - lp) != xend) fail = true;
    if (!fail) {
      const uint32_t rest = B.nlit - lp;
      for (uint32_t t = uint32_t(lane); t < rest; t += 64) {
        val[x + t] = L[lp + t];
        pa[x + t] = x + t;
      }
    }
    if (fail && lane == 0) atomicOr(Z.flag, 1u);
  }
}

}  // namespace

size_t zstd_par_scratch_bytes(uint32_t nblk) {
  size_t bytes = 0;
  zq_carve(nullptr, nblk, &bytes);
  return bytes + 256;
}

const uint32_t* zstd_par_result(const void* scratch) { return static_cast<const uint32_t*>(scratch); }

hipError_t launch_zstd_par_headers(hipStream_t st, const uint8_t* in, const uint32_t* blk, uint32_t nblk,
                                   uint32_t bmax, void* scratch, int num_cus) {
  const ZqScratch Z = zq_carve(scratch, nblk, nullptr);
  hipError_t e = hipMemsetAsync(Z.flag, 0, 64, st);
  if (e != hipSuccess) return e;
  zq_scan_kernel<<<1, 64, 0, st>>>(in, blk, nblk, bmax, Z);
  zq_huf_kernel<<<min(nblk, uint32_t(num_cus) * 8), 64, 0, st>>>(in, nblk, Z);
  return hipGetLastError();
}

hipError_t launch_zstd_par_body(hipStream_t st, const uint8_t* in, uint32_t nblk, uint32_t bmax, void* scratch,
                                uint8_t* lit, uint32_t* sll, uint32_t* sml, uint32_t* sof, int num_cus) {
  const ZqScratch Z = zq_carve(scratch, nblk, nullptr);
  const size_t lit_lds = kZqHuf * 2 + kZsBlockMax + 64;
  const size_t seq_lds = 3 * kZqSlot * sizeof(ZsFse) + kZsBlockMax + 64;
  static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&zq_lit_kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lit_lds));
  static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&zq_seq_kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(seq_lds));
  if (a1 != hipSuccess) return a1;
  if (a2 != hipSuccess) return a2;
  const uint32_t g = min(nblk, uint32_t(num_cus));
  hipLaunchKernelGGL(zq_lit_kernel, dim3(g), dim3(64), lit_lds, st, in, nblk, Z, lit);
  hipLaunchKernelGGL(zq_seq_kernel, dim3(g), dim3(64), seq_lds, st, nblk, bmax, in, Z, sll, sml, sof);
  zq_chain_kernel<<<1, 64, 0, st>>>(nblk, Z);
  return hipGetLastError();
}

hipError_t launch_zstd_par_bytes(hipStream_t st, const uint8_t* in, uint32_t nblk, uint32_t total, void* scratch,
                                 const uint8_t* lit, const uint32_t* sll, const uint32_t* sml, const uint32_t* sof,
                                 uint8_t* val, uint32_t* pa, uint32_t* pb, uint32_t* changed, uint8_t* out,
                                 int num_cus) {
  const ZqScratch Z = zq_carve(scratch, nblk, nullptr);
  zq_exec_kernel<<<min(nblk, uint32_t(num_cus) * 4), 64, 0, st>>>(in, nblk, Z, lit, sll, sml, sof, val, pa);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_ptr_gather(st, total, val, pa, pb, changed, Z.flag, out);
}

}  // namespace slate
