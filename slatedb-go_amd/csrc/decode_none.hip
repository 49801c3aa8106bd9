// CodecNone block decode: block.Decode (internal/sstable/block/block.go:78-134) for the DB's
// default codec (slatedb/config/config.go:85).  CodecNone blocks are `data || BE32 CRC32(data)`,
// so decode is: CRC check, the decoded block = data, then block.go's offset / FirstKey checks and
// the row descriptors of row.go:191-261 (the same arithmetic as rows.h block_finish).
//
// This is pure streaming work (read ~4.1 KiB, write ~4 KiB + ~0.6 KiB of rows per block), so the
// kernel is shaped for HBM, not for instructions:
//   * one wave per block, 16 waves per CU, and the next block's loads in flight while the
//     current one is processed (grid-stride over blocks);
//   * loads are coalesced: in register row q, lane l holds the 16-byte input chunk of virtual
//     slot v = 64q + l, where the block's chunks are placed so that its last data chunk lands on
//     slot 319 (front padding `pad`); the output is written by the same layout, 1 KiB per store
//     instruction;
//   * CRC32 is linear and a zero-initialised register ignores leading zeros, so every lane
//     folds its five 16-byte output chunks independently (slicing-by-16, no serial chain across
//     chunks), then the lanes' values are combined with x^(8N) multiplications done as four
//     byte-table lookups (Horner over the register rows: N = 1024; a six-level lane tree:
//     N = 16 .. 512).  The 0xFFFFFFFF initial value is folded into the first four data bytes,
//     the zero padding after the data into the stored value (x^(8t) mod P);
//   * the block is staged in LDS (one 5 KiB slot per wave) for the unaligned output chunks and
//     the row walk; the offsets and rows are decoded one lane per row.
// Blocks larger than 5088 data bytes, or with fewer than 4, take the exact wave path
// (decode_large_kernel, through large_list), which reports them identically.
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"
#include "lpb_common.h"

namespace slate {

namespace {

constexpr int kNoneThreads = 512;  // 8 waves; two workgroups per CU (LDS: 80 KiB each)
constexpr uint32_t kNoneWgPerCu = 2;
constexpr uint32_t kNoneSlots = 320;  // 5 register rows x 64 lanes of 16-byte chunks
constexpr uint32_t kNoneMaxData = (kNoneSlots - 2) * 16;  // 5088 data bytes at most on this path
constexpr uint32_t kNoneStage = 5120;  // per-wave LDS staging: input chunks 0 .. nout
constexpr uint32_t kNoneTabBytes = kTab16Bytes + kAdvN * 4096;
constexpr uint32_t kNoneLds = kNoneTabBytes + (kNoneThreads / 64) * kNoneStage;
// cache policy of the output / row stores (0 default, 2 nt, 16 sc1): nt, and nt block loads, measured
// 2.04 vs 2.12 ms per 1 M blocks (profiles/round3/none/ab_policy.txt)
#ifndef SLATE_NONE_CPOL
#define SLATE_NONE_CPOL 2
#endif
constexpr int kNoneCpol = SLATE_NONE_CPOL;
#ifndef SLATE_NONE_LDPOL  // cache policy of the block loads (0 default, 2 nt): default since round 6
#define SLATE_NONE_LDPOL 0   // (same-box A/Bs, 1 M blocks: nt 2.158 / 2.153 ms, default 2.082 / 2.074;
#endif                       // profiles/round6/ab/ab_none_policy.txt)
constexpr int kNoneLdpol = SLATE_NONE_LDPOL;
// The decoded block is stored as soon as its chunks are formed, before the CRC's lane tree, so the
// stores drain while the tree's dependent lookups run (round 6).  A block whose CRC then fails has
// its meta say so; its output slot's bytes are unspecified, as Go sets no Block.Data on an error
// (block.go:85-88) and the parity tests compare bytes only of blocks that decoded.
#ifndef SLATE_NONE_ALIGN_LOADS
#define SLATE_NONE_ALIGN_LOADS 0
#endif
#ifndef SLATE_NONE_EARLY_STORE
#define SLATE_NONE_EARLY_STORE 1
#endif
static_assert(kNoneWgPerCu * kNoneLds <= 163840, "workgroups per CU");

// 4 bytes at byte position p of a wave's LDS stage (two aligned dword reads)
__device__ __forceinline__ uint32_t st_u32(const uint8_t* stage, uint32_t p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(stage + (p & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], p & 3u);
}
__device__ __forceinline__ uint32_t st_be16(const uint8_t* stage, uint32_t p) { return be16_of(st_u32(stage, p)); }

// v0 row decode (row.go:191-261, rows.h decode_row) against the staged block: data byte k is
// stage[sh + k], data_len = offsetStartIndex.  Returns the descriptor; *sl_ok = suffix length of a
// row that decoded (for the first key), ~0u otherwise.
__device__ __forceinline__ v4u row_stage(const uint8_t* stage, uint32_t sh, uint32_t data_len, uint32_t off, int fk,
                                         uint32_t* sl_ok) {
  *sl_ok = 0xFFFFFFFFu;
  const uint32_t n = data_len - off;
  const uint32_t w = st_u32(stage, sh + off);
  const uint32_t pl = n >= 4 ? be16_of(w) : 0u, sl = n >= 4 ? be16_of(w >> 16) : 0u;
  v4u r;
  r.x = off;
  r.y = pl | (sl << 16);
  r.z = 0;
  uint32_t st = SLATE_OK;
  if (n < 13) {
    st = SLATE_E_ROW_TOO_SHORT;
  } else if (pl > uint32_t(fk < 0 ? 0 : fk)) {
    st = SLATE_E_ROW_PREFIX;
  } else if (n - 4 < sl) {
    st = SLATE_E_ROW_SUFFIX;
  } else if (n - 4 - sl < 9) {
    st = SLATE_E_ROW_PANIC;
  } else {
    uint32_t o = 4 + sl;
    const uint32_t flags = st_u32(stage, sh + off + o + 8) & 0xff;
    o += 9;
    if ((flags & 2) && n - o < 8) {
      st = SLATE_E_ROW_EXPIRE;
    } else {
      o += (flags & 2) ? 8u : 0u;
      if ((flags & 4) && n - o < 8) {
        st = SLATE_E_ROW_CREATE;
      } else {
        o += (flags & 4) ? 8u : 0u;
        uint32_t vl = 0;
        if (!(flags & 1)) {
          if (n - o < 4) {
            st = SLATE_E_ROW_VALUE_LEN;
          } else {
            vl = __builtin_bswap32(st_u32(stage, sh + off + o));
            o += 4;
            if (n - o < vl) st = SLATE_E_ROW_VALUE;
          }
        }
        if (st == SLATE_OK) {
          r.z = vl;
          r.w = (flags & 7) | ((o - 4 - sl) << 8);
          *sl_ok = sl;
        }
      }
    }
  }
  if (st != SLATE_OK) r.w = st << 16;
  return r;
}

// Block geometry (wave-uniform, from scalar loads of in_off).  kind: 0 = this kernel decodes it,
// 1 = too small (meta only), 2 = the exact wave path (large_list), 3 = past the end.
struct Geo {
  uint32_t kind, sh, clen, nout, pad, pin;
  const uint8_t* base;
};
__device__ __forceinline__ Geo geo_of(const DecodeArgs& a, uint32_t b) {
  Geo g{3u, 0u, 0u, 0u, 0u, 0u, a.in};
  if (b >= a.n) return g;
  const uint64_t s0 = sload(a.in_off + b), len = sload(a.in_off + b + 1) - s0;
  const uint8_t* gin = a.in + s0;
  g.sh = uint32_t(reinterpret_cast<uintptr_t>(gin) & 15);
  g.base = gin - g.sh;
  g.kind = len < 6 ? 1u : ((len - 4 > kNoneMaxData || len - 4 < 4) ? 2u : 0u);
  g.clen = g.kind == 0 ? uint32_t(len - 4) : 0u;
  g.nout = (g.clen + 15) / 16;
  g.pad = kNoneSlots - g.nout;
  g.pin = kNoneSlots - 1 - ((g.sh + g.clen + 3) >> 4);  // (kind 0: <= 319 - (nout - 1) - 2)
#if SLATE_NONE_ALIGN_LOADS
  // up to three slots earlier, so that every load instruction's 1 KiB starts on a 64-byte boundary of
  // the address (16 segments, not 17); the stage only moves with it
  {
    const uint32_t d = (g.pin - uint32_t(reinterpret_cast<uintptr_t>(g.base) >> 4)) & 3u;
    g.pin -= g.pin >= d ? d : 0u;
  }
#endif
  return g;
}

// The block's loads: register row q of lane l = input chunk 64q + l - pin, so that the chunk
// holding the stored CRC's last byte (after the tail of the last output chunk) lands on slot 319;
// nothing before chunk 0 (zeros).  They are staged slot by slot, so the stage holds input chunk c
// at 16 (c + pin): every lane stores, no divergent branch.
struct Loads {
  v4u p[5];
};
__device__ __forceinline__ void issue_loads(const Geo& g, uint32_t lane, Loads& L) {
  const bool go = g.kind == 0;
  const __amdgpu_buffer_rsrc_t R = make_rsrc(g.base, go ? align16(uint64_t(g.sh) + g.clen + 4) : 0);
#pragma unroll
  for (uint32_t q = 0; q < 5; q++) {
    const int32_t c = int32_t(64 * q + lane) - int32_t(g.pin);
    L.p[q] = __builtin_amdgcn_raw_buffer_load_b128(R, c >= 0 ? uint32_t(16 * c) : kOOB, 0, kNoneLdpol);
  }
}

// the 16 data bytes of output chunk j: stage bytes [sh + 16j, sh + 16j + 16), from three aligned
// 8-byte reads (gfx950 serialises misaligned LDS accesses)
__device__ __forceinline__ v4u out_chunk(const uint8_t* stage, uint32_t sh, int32_t j) {
  const uint32_t o = sh + 16 * uint32_t(max(j, 0));
  const uint32_t a = o & ~7u;
  const v2u A = *reinterpret_cast<const v2u*>(stage + a), B = *reinterpret_cast<const v2u*>(stage + a + 8),
            C = *reinterpret_cast<const v2u*>(stage + a + 16);
  const bool q = (o & 4) != 0;  // wave-uniform (sh is)
  const uint32_t e0 = q ? A.y : A.x, e1 = q ? B.x : A.y, e2 = q ? B.y : B.x, e3 = q ? C.x : B.y, e4 = q ? C.y : C.x;
  const uint32_t b = o & 3;
  v4u r;
  r.x = alignb(e1, e0, b);
  r.y = alignb(e2, e1, b);
  r.z = alignb(e3, e2, b);
  r.w = alignb(e4, e3, b);
  return r;
}

// One block: stage its chunks (LDS, the wave's 5 KiB at stage0), put the loads of the block two steps ahead into the same
// registers, then decode it.  b / g / L advance to that block.
__device__ __forceinline__ void none_block(const DecodeArgs& a, const uint32_t* tab, uint8_t* stage0, uint32_t lane,
                                           uint32_t step, uint32_t& b, Geo& g, Loads& L) {
  const uint8_t* lds = reinterpret_cast<const uint8_t*>(tab);
  slate_block_meta m{};
  const Geo gc = g;
  const uint32_t sh = gc.sh, clen = gc.clen, nout = gc.nout, pad = gc.pad, pin = gc.pin;
  if (gc.kind == 0) {
#pragma unroll
    for (uint32_t q = 0; q < 5; q++) wr128(stage0 + 16 * (64 * q + lane), L.p[q], a.rt_zero);
  }
  const uint8_t* stage = stage0 + 16 * pin;  // stage[i] = input byte i (from the 16-byte base)
  const uint32_t bc = b;
  b += step;
  g = geo_of(a, b);
  issue_loads(g, lane, L);
  if (gc.kind == 1) {
    m.status = SLATE_E_BLOCK_TOO_SMALL;
    if (lane == 0) a.meta[bc] = m;
  } else if (gc.kind == 2) {
    if (lane == 0) a.large_list[atomicAdd(a.large_count, 1u)] = bc;
  } else {
    // ---- output chunks (slot v = 64q + lane holds output chunk j = v - pad) and their CRC:
    // zero below chunk 0, the initial 0xFFFFFFFF folded into data bytes 0..3, the bytes after
    // the data zeroed in the last chunk (t = 16 nout - clen of them)
    v4u O[5];
    uint32_t acc = 0;
    const uint32_t r = clen - 16 * (nout - 1);  // data bytes in the last chunk (1..16)
    const uint32_t t = 16 - r;
#pragma unroll
    for (uint32_t q = 0; q < 5; q++) {
      const int32_t j = int32_t(64 * q + lane) - int32_t(pad);
      O[q] = out_chunk(stage, sh, j);
      v4u c = O[q];
      const bool first = j == 0, last = j == int32_t(nout) - 1, none = j < 0;
      c.x ^= first ? 0xFFFFFFFFu : 0u;
      if (q == 4) {  // the last chunk is slot 319: lane 63 of row 4
        c.x &= (last && r < 4) ? (1u << (8 * r)) - 1u : 0xFFFFFFFFu;
        c.y &= (last && r < 8) ? (r <= 4 ? 0u : (1u << (8 * (r - 4))) - 1u) : 0xFFFFFFFFu;
        c.z &= (last && r < 12) ? (r <= 8 ? 0u : (1u << (8 * (r - 8))) - 1u) : 0xFFFFFFFFu;
        c.w &= (last && r < 16) ? (r <= 12 ? 0u : (1u << (8 * (r - 12))) - 1u) : 0xFFFFFFFFu;
      }
      if (!(dbg_bits(a) & 1)) {  // (profiling variants only: bit 1 skips the CRC, 4 the rows, 8 the output stores)
        const uint32_t k = crc_chunk0(lds, c);
        // Horner over the rows: row q's chunks lie 1024 (4 - q) bytes before row 4's
        acc = (q == 0 ? 0u : adv_tab<5>(lds, acc)) ^ (none ? 0u : k);
      }
    }
    if (SLATE_NONE_EARLY_STORE) {
      const __amdgpu_buffer_rsrc_t RO = make_rsrc(a.out + sload(a.out_off + bc), 16 * uint64_t(nout));
#pragma unroll
      for (uint32_t q = 0; q < 5; q++) {
        const int32_t j = int32_t(64 * q + lane) - int32_t(pad);
        __builtin_amdgcn_raw_buffer_store_b128(O[q], RO, (j >= 0 && !(dbg_bits(a) & 8) && !a.no_data) ? uint32_t(16 * j) : kOOB,
                                               0, kNoneCpol);
      }
    }
    bool crc_ok = true;
    if (!(dbg_bits(a) & 1)) {
      // lane tree: lane l's chunks end 16 (63 - l) bytes before lane 63's; inside rows of 16 lanes
      // by DPP row shifts, then the four row heads (lanes 0, 16, 32, 48) combined.  At the level of
      // shift s only the lanes l = 0 mod 2s carry a partial CRC on, so only they do the lookups
      // (fewer lanes, fewer bank conflicts on the random table indices), and the row heads are
      // combined with wave-uniform addresses (broadcast reads)
      {
        uint32_t t = acc;
        if (!(lane & 1)) t = adv16(lds, acc);
        acc = t ^ row_shl<1>(acc);
        t = acc;
        if (!(lane & 3)) t = adv_tab<0>(lds, acc);
        acc = t ^ row_shl<2>(acc);
        t = acc;
        if (!(lane & 7)) t = adv_tab<1>(lds, acc);
        acc = t ^ row_shl<4>(acc);
        t = acc;
        if (!(lane & 15)) t = adv_tab<2>(lds, acc);
        acc = t ^ row_shl<8>(acc);
      }
      const uint32_t h1 = __builtin_amdgcn_readlane(acc, 16), h2 = __builtin_amdgcn_readlane(acc, 32),
                     h3 = __builtin_amdgcn_readlane(acc, 48);
      uint32_t total = __builtin_amdgcn_readfirstlane(acc);
      total = __builtin_amdgcn_readfirstlane(adv_tab<3>(lds, total) ^ h1);  // rows 0-1
      total = __builtin_amdgcn_readfirstlane(adv_tab<3>(lds, total) ^ h2);  // rows 0-2
      total = __builtin_amdgcn_readfirstlane(adv_tab<3>(lds, total) ^ h3);  // rows 0-3
      const uint32_t stored = __builtin_bswap32(st_u32(stage, sh + clen));
      crc_ok = total == adv_small(tab, ~stored, t);
    }
    if (!crc_ok) {
      m.status = SLATE_E_BLOCK_CHECKSUM;
      if (lane == 0) a.meta[bc] = m;
    } else {
      // ---- the decoded block (16-byte slots; bytes after the data are padding)
      const __amdgpu_buffer_rsrc_t RO = make_rsrc(a.out + sload(a.out_off + bc), 16 * uint64_t(nout));
#pragma unroll
      for (uint32_t q = 0; q < 5 && !SLATE_NONE_EARLY_STORE; q++) {
        const int32_t j = int32_t(64 * q + lane) - int32_t(pad);
        __builtin_amdgcn_raw_buffer_store_b128(O[q], RO, (j >= 0 && !(dbg_bits(a) & 8) && !a.no_data) ? uint32_t(16 * j) : kOOB,
                                               0, kNoneCpol);
      }
      // ---- block.go:101-134 and the rows (rows.h block_finish arithmetic)
      const uint32_t n = clen;
      const uint32_t cnt = __builtin_amdgcn_readfirstlane(st_be16(stage, sh + n - 2));
      const int32_t osi = int32_t(n) - 2 - 2 * int32_t(cnt);
      if (osi <= 0) {
        m.status = SLATE_E_BLOCK_INDEX_OFFSET;
        m.detail = osi;
      } else {
        const uint32_t osu = uint32_t(osi);  // < 65536 on this path: uint16(offsetStartIndex) == osi
        uint32_t bad = 0xFFFFFFFFu, bad_off = 0;
        for (uint32_t i0 = 0; i0 < cnt && bad == 0xFFFFFFFFu; i0 += 64) {
          const uint32_t i = i0 + lane;
          const uint32_t off = i < cnt ? st_be16(stage, sh + osu + 2 * i) : 0u;
          const uint64_t m64 = __ballot(i < cnt && off > osu);
          if (m64) {
            const uint32_t l0 = uint32_t(__builtin_ctzll(m64));
            bad = i0 + l0;
            bad_off = __builtin_amdgcn_readlane(off, l0);
          }
        }
        if (bad != 0xFFFFFFFFu) {
          m.status = SLATE_E_BLOCK_OFFSET_BOUNDS;
          m.aux = uint16_t(bad);
          m.detail = int32_t(bad_off);
        } else {
          m.data_len = osu;
          m.n_rows = uint16_t(cnt);
          if (cnt == 0) {
            m.status = SLATE_E_BLOCK_NO_OFFSETS;
          } else {
            // FirstKey (block.go:130-131): uint16 arithmetic, Go panics out of range
            const uint32_t off0 = __builtin_amdgcn_readfirstlane(st_be16(stage, sh + osu));
            if (osu - off0 < 2) {
              m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
            } else {
              const uint16_t kl = uint16_t(__builtin_amdgcn_readfirstlane(st_be16(stage, sh + off0)));
              const uint16_t lo = uint16_t(off0 + 2), hi = uint16_t(off0 + 2 + kl);
              if (lo > hi || hi > n) {
                m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
              } else {
                m.aux = kl;
                const uint64_t rb = sload(a.row_base + bc);
                const uint32_t rcap = uint32_t(min(uint64_t(0xFFFFFFFFu), sload(a.row_base + bc + 1) - rb));
                uint32_t nr = cnt;
                if (nr > rcap) {
                  nr = rcap;
                  m.flags |= SLATE_BLKF_ROWS_TRUNCATED;
                }
                // the first key's length: row 0 decoded against an empty first key
                uint32_t sl0;
                (void)row_stage(stage, sh, osu, off0, -1, &sl0);
                const int fk = sl0 == 0xFFFFFFFFu ? -1 : int(__builtin_amdgcn_readfirstlane(sl0));
                const __amdgpu_buffer_rsrc_t RR = make_rsrc(a.rows + rb, 16 * uint64_t(nr));
                if (dbg_bits(a) & 4) nr = 0;
                for (uint32_t i0 = 0; i0 < nr; i0 += 64) {
                  const uint32_t i = i0 + lane;
                  const uint32_t off = st_be16(stage, sh + osu + 2 * min(i, cnt - 1));
                  uint32_t sl;
                  const v4u row = row_stage(stage, sh, osu, off, i == 0 ? -1 : fk, &sl);
                  __builtin_amdgcn_raw_buffer_store_b128(row, RR, i < nr ? 16 * i : kOOB, 0, kNoneCpol);
                }
              }
            }
          }
        }
      }
      if (lane == 0) a.meta[bc] = m;
    }
  }
}

__global__ __launch_bounds__(kNoneThreads) void decode_none_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);  // slicing-by-16 (16 KiB)
  {
    const uint32_t* src = &g_crc16.t[0][0];
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = src[i];
    load_adv_tables(tab + 4096);  // kAdvN x 4 x 256
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* stage = smem + kNoneTabBytes + wave * kNoneStage;
  const uint32_t waves_total = gridDim.x * (kNoneThreads / 64);
  // two register sets: blocks b, b + W, b + 2W, ... alternate between them, so while one block
  // is decoded the next one's loads are in flight and the one after it is being issued
  uint32_t bA = blockIdx.x * (kNoneThreads / 64) + wave, bB = bA + waves_total;
  Geo gA = geo_of(a, bA), gB = geo_of(a, bB);
  Loads LA, LB;
  issue_loads(gA, lane, LA);
  issue_loads(gB, lane, LB);
  while (gA.kind != 3) {
    none_block(a, tab, stage, lane, 2 * waves_total, bA, gA, LA);
    if (gB.kind == 3) break;
    none_block(a, tab, stage, lane, 2 * waves_total, bB, gB, LB);
  }
}

}  // namespace

hipError_t launch_decode_none(hipStream_t st, const DecodeArgs& a, int num_cus) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_none_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(kNoneLds));
  if (attr != hipSuccess) return attr;
  const uint32_t waves = (a.n + 0u);
  uint32_t grid = min((waves + kNoneThreads / 64 - 1) / (kNoneThreads / 64), uint32_t(num_cus) * kNoneWgPerCu);
  grid = max(grid, 1u);
  decode_none_kernel<<<grid, kNoneThreads, kNoneLds, st>>>(a);
  return hipGetLastError();
}

}  // namespace slate
