// CodecZlib fast path, phase Z: compress/zlib streams of SST blocks (compress.Decode,
// internal/compress/compression.go:134-140: io.ReadAll(zlib.NewReader(buf)); the zlib framing of
// RFC 1950 around RFC 1951 deflate, as Go's compress/zlib and compress/flate read it) decoded ONE
// LANE PER BLOCK, 64 blocks per wave instruction, into what the CodecZstd build phase consumes:
//   * the block's literal bytes, in order, written to the start of the block's output slot;
//   * its (literal run, match length, distance) sequences as 4-byte records (kZfSeq4) in z.seq;
//   * a ZsFastRec with kZfOutLit (literals in the output slot) and kZfAdler (want = the stream's
//     Adler-32, checked by the build phase over the decoded block in LDS).
// Then phase A2 (the SST block CRC32, zstd_fast.hip) and phase B (wave per block: literal runs
// placed, matches in order, write-back, block.Decode's checks and rows) run unchanged.
// Plan mode: the same decode with no writes gives each block's decoded size.  Staged plan mode
// (slate_block_decode_plan_device for CodecZlib): the plan IS phase Z -- sizes as in plan mode, and
// the literals, sequences and record of each block kept in the context's stage (ZlStage, literals
// at a fixed kZlStageStride per block), so the decode call that follows runs only A2 and B over
// them (each stream inflated once per plan + decode, not twice).
//
// Per lane: a 64-bit bit buffer fed from 16-byte chunks of the block (two chunks loaded ahead);
// canonical Huffman decoding (RFC 1951 3.2.2) as in zlib's puff: the code of length L is found by
// comparing the bit-reversed 15-bit peek with the left-justified limits of lengths 1..14 held in
// registers, and the symbol read from the lane's table of symbols sorted by (length, value) in LDS
// (literal/length 288 x u8 and distance 32 x u8: 320 bytes per lane, byte k of lane l's tables at
// LDS byte 64 k + l; the code-length code's 19 sorted symbols in two registers, the fixed codes'
// tables computed; one-wave workgroups, eight per CU: the LDS exactly full).  A literal/length table byte is the symbol's low 8 bits: within one
// code length the literals sort before 256..287, so the symbol is >= 256 exactly when its sorted
// index reaches that length's first non-literal slot (per length, in registers).  The dynamic header's code lengths are decoded twice (count, then place), so no length
// array is kept.  Only complete codes are taken; a stored block with data, a distance beyond the
// output or the 4 KiB record limit, more than 128 sequences, a literal run of 1024 or more, a
// truncated or over-long stream, or anything else unusual is handed to the exact path
// (decode_list_kernel<1>, wave_inflate), which decodes and reports it.
#include "common.h"
#include "kernels.h"
#include "lpb_common.h"

namespace slate {

namespace {

constexpr uint32_t kZlThreads = 64;    // one wave per workgroup
constexpr uint32_t kZlWgPerCu = 8;     // (LDS)
constexpr uint32_t kZlLane = 320;      // per-lane tables (bytes)
constexpr uint32_t kZlDistOff = 288;
constexpr uint32_t kZlLds = kZlThreads * kZlLane;
static_assert(kZlWgPerCu * kZlLds <= 163840, "workgroups per CU");
constexpr uint32_t kZlMaxOut = kZsFastOutCap;  // the build phase's LDS window
constexpr uint32_t kZlMaxSeqs = kZsFseSeqs;    // two records per lane in the build phase

__device__ __forceinline__ void zl_list_append(bool want, uint32_t item, uint32_t* list, uint32_t* count) {
  const uint64_t m = __ballot(want);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == uint32_t(__builtin_ctzll(m))) base = atomicAdd(count, uint32_t(__builtin_popcountll(m)));
  base = __shfl(base, __builtin_ctzll(m), 64);
  if (want) list[base + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)))] = item;
}

// ---- the lane's bit reader: bits [0, nb) of bb are the next stream bits (LSB first)
struct ZlIn {
  uint64_t bb;
  uint32_t nb;
  uint32_t k;      // the next dword of cur to append
  uint32_t c;      // chunk index of cur (16-byte units from the aligned base)
  uint32_t used;   // stream bits consumed
  v4u cur, nxt, nx2;
};
__device__ __forceinline__ uint32_t dword_of(const v4u& v, uint32_t k) {
  return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}
// at least 33 bits in bb afterwards (one dword appended when nb <= 32)
__device__ __forceinline__ void zl_refill(ZlIn& z, __amdgpu_buffer_rsrc_t R, uint32_t rel, bool act) {
  const bool go = act && z.nb <= 32;
  const uint32_t dw = dword_of(z.cur, z.k);
  z.bb = go ? (z.bb | (uint64_t(dw) << z.nb)) : z.bb;
  z.nb += go ? 32u : 0u;
  const bool adv = go && z.k == 3;
  z.k = go ? ((z.k + 1) & 3) : z.k;
  if (__ballot(adv)) {
    const v4u ld = bload<0>(R, adv ? rel + 16 * (z.c + 3) : kOOB);
    z.cur = adv ? z.nxt : z.cur;
    z.nxt = adv ? z.nx2 : z.nxt;
    z.nx2 = adv ? ld : z.nx2;
    z.c += adv ? 1u : 0u;
  }
}
__device__ __forceinline__ uint32_t zl_take(ZlIn& z, uint32_t n) {  // n <= 32, n <= nb
  const uint32_t v = uint32_t(z.bb) & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
  z.bb >>= n;
  z.nb -= n;
  z.used += n;
  return v;
}

// ---- canonical tables: lim[l] = left-justified end of the length-l codes, off[l] = index of
// the first length-l symbol in the sorted table minus the first length-l code
struct ZlTab {
  uint32_t lim[16], off[16];
  uint32_t maxl;  // the longest code length in use
};
// cnt[1..15] -> the table; false unless the code is complete (RFC 1951 codes as zlib / Go build
// them; incomplete and over-subscribed ones go to the exact path).  nxt: the sorted-table start of
// each length (packed 9-bit fields, see zl_put).
__device__ __forceinline__ bool zl_canon(const uint32_t (&cnt)[16], ZlTab& t, uint64_t (&nxt)[3]) {
  uint32_t first = 0, idx = 0;
  nxt[0] = nxt[1] = nxt[2] = 0;
  t.maxl = 1;
#pragma unroll
  for (int l = 1; l <= 15; l++) {
    t.maxl = cnt[l] ? uint32_t(l) : t.maxl;
    if (l > 1) first = (first + cnt[l - 1]) << 1;
    t.lim[l] = (first + cnt[l]) << (15 - l);
    t.off[l] = idx - first;
    nxt[(l - 1) / 7] |= uint64_t(idx) << (9 * ((l - 1) % 7));
    idx += cnt[l];
  }
  t.lim[0] = 0;
  t.off[0] = 0;
  return t.lim[15] == 32768u;
}
// sorted-table slot of the next symbol of length l (1..15), advancing it (l == 0: no slot, 0)
__device__ __forceinline__ uint32_t zl_put(uint64_t (&nxt)[3], uint32_t l) {
  const uint32_t lm = l == 0 ? 1u : l;
  const uint32_t w = (lm - 1) / 7, sh = 9 * ((lm - 1) % 7);
  const uint64_t word = w == 0 ? nxt[0] : (w == 1 ? nxt[1] : nxt[2]);
  const uint32_t p = uint32_t(word >> sh) & 511u;
  const uint64_t inc = l == 0 ? 0 : uint64_t(1) << sh;
  nxt[0] += w == 0 ? inc : 0;
  nxt[1] += w == 1 ? inc : 0;
  nxt[2] += w == 2 ? inc : 0;
  return p;
}
__device__ __forceinline__ void zl_count(uint64_t (&cnt)[3], uint32_t l, uint32_t rep) {
  const uint32_t w = (l - 1) / 7, sh = 9 * ((l - 1) % 7);
  const uint64_t inc = uint64_t(rep) << sh;
  cnt[0] += (l != 0 && w == 0) ? inc : 0;
  cnt[1] += (l != 0 && w == 1) ? inc : 0;
  cnt[2] += (l != 0 && w == 2) ? inc : 0;
}
__device__ __forceinline__ void zl_unpack(const uint64_t (&p)[3], uint32_t (&cnt)[16]) {
  cnt[0] = 0;
#pragma unroll
  for (int l = 1; l <= 15; l++) cnt[l] = uint32_t(p[(l - 1) / 7] >> (9 * ((l - 1) % 7))) & 511u;
}

// The code at the head of z (z.nb >= 15 or the stream's end): its length L and sorted index.
// kMax: the longest length the tables can hold.
template <int kMax>
__device__ __forceinline__ void zl_find(const ZlIn& z, const ZlTab& t, uint32_t& L, uint32_t& idx) {
  const uint32_t rev = __builtin_bitreverse32(uint32_t(z.bb)) >> 17;
  uint32_t len = 1, o = t.off[1];
#pragma unroll
  for (int k = 1; k < kMax; k++) {  // (explicit selects: a select chain became a scratch-array index)
    const bool ge = rev >= t.lim[k];
    len += ge ? 1u : 0u;
    o = vsel(ge, t.off[k + 1], o);
  }
  L = len;
  idx = o + (rev >> (15 - len));
}
// the same over two tables chosen per lane (b: table B); kmax: the wave's longest code length
// (the compares beyond it cannot succeed)
__device__ __forceinline__ void zl_find2(const ZlIn& z, const ZlTab& ta, const ZlTab& tb, bool b, uint32_t kmax,
                                         uint32_t& L, uint32_t& idx) {
  const uint32_t rev = __builtin_bitreverse32(uint32_t(z.bb)) >> 17;
  uint32_t len = 1, o = vsel(b, tb.off[1], ta.off[1]);
#pragma unroll
  for (int k = 1; k < 15; k++) {
    if (uint32_t(k) < kmax) {  // (wave-uniform; a guarded step, not a loop exit: the indices stay constant)
      const bool ge = rev >= vsel(b, tb.lim[k], ta.lim[k]);
      len += ge ? 1u : 0u;
      o = vsel(ge, vsel(b, tb.off[k + 1], ta.off[k + 1]), o);
    }
  }
  L = len;
  idx = o + (rev >> (15 - len));
}

__constant__ uint8_t kZlClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// length symbol 257 + s (s < 29): base and extra bits (RFC 1951 3.2.5)
__device__ __forceinline__ uint32_t len_extra(uint32_t s) { return (s < 8 || s == 28) ? 0u : (s - 4) >> 2; }
__device__ __forceinline__ uint32_t len_base(uint32_t s) {
  return s < 8 ? s + 3 : (s == 28 ? 258u : ((4u + (s & 3u)) << ((s - 4) >> 2)) + 3u);
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t s) { return s < 4 ? 0u : (s >> 1) - 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t s) {
  return s < 4 ? s + 1 : ((2u + (s & 1u)) << ((s >> 1) - 1)) + 1u;
}

// the fixed codes' symbol at sorted index ci (RFC 1951 3.2.6; sorted by (length, symbol):
// 256..279 (7 bits), 0..143 and 280..287 (8), 144..255 (9); distances: the index)
__device__ __forceinline__ uint32_t zl_fixed_sym(bool dist, uint32_t ci) {
  return dist ? ci : (ci < 24 ? ci + 256 : (ci < 168 ? ci - 24 : (ci < 176 ? ci + 112 : ci - 32)));
}
// the symbol of a literal/length table byte: + 256 from the length's first non-literal slot
__device__ __forceinline__ uint32_t zl_hi_at(const uint64_t (&hi)[3], uint32_t L) {
  const uint32_t q = L - 1, w = q >= 14 ? 2u : (q >= 7 ? 1u : 0u), sh = 9 * (q - 7 * w);
  const uint64_t word = w == 0 ? hi[0] : (w == 1 ? hi[1] : hi[2]);
  return uint32_t(word >> sh) & 511u;
}
__device__ __forceinline__ void zl_fixed_counts(ZlTab& tl, ZlTab& td) {
  uint32_t cl[16] = {}, cd[16] = {};
  cl[7] = 24;
  cl[8] = 152;
  cl[9] = 112;
  cd[5] = 32;  // (30 used; 32 make the fixed distance code complete, as in zlib's fixed table)
  uint64_t nx[3];
  (void)zl_canon(cl, tl, nx);
  (void)zl_canon(cd, td, nx);
}

}  // namespace

// One lane per block.  kMode kZlDecode: the literal bytes to the output slot, the sequences and
// the record (failures to z.list for the exact path); kZlPlan: sizes only (out_sz / row_sz;
// failures to plist for the wave plan); kZlStage: both -- the sizes, and the literals to the
// stage slot (z.lit + kZlStageStride b), sequences and record (failures to plist, which is also
// the decode's exact-path list)
constexpr int kZlDecode = 0, kZlPlan = 1, kZlStage = 2;
template <int kMode>
__global__ __launch_bounds__(kZlThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void zl_fast_kernel(DecodeArgs a, ZsFastArgs z, uint64_t* out_sz,
                                                             uint64_t* row_sz, uint32_t* plist, uint32_t* pcount) {
  constexpr bool kPlan = kMode == kZlPlan;     // no literal / sequence writes
  constexpr bool kSizes = kMode != kZlDecode;  // out_sz / row_sz / plist
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_lane0 = threadIdx.x - lane;
  uint8_t* mine = smem + threadIdx.x;  // byte k of this lane's tables at mine[64 k]
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x + wave_lane0; r0 < a.n; r0 += stride) {
    const uint32_t b = r0 + lane;
    const uint32_t rend = min(r0 + 64, a.n);
    // the wave's input (and output) as one buffer resource each
    const uint8_t* ilo = a.in + a.in_off[r0];
    const uint8_t* ibase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(ilo) & ~uintptr_t(15));
    const __amdgpu_buffer_rsrc_t R = make_rsrc(ibase, align16(uint64_t((a.in + a.in_off[rend]) - ibase)));
    __amdgpu_buffer_rsrc_t RO = R, RS = R;
    if (kMode == kZlDecode) RO = make_rsrc(a.out + a.out_off[r0], a.out_off[rend] - a.out_off[r0]);
    if (kMode == kZlStage) RO = make_rsrc(z.lit + size_t(r0) * kZlStageStride, uint64_t(rend - r0) * kZlStageStride);
    if (!kPlan) RS = make_rsrc(z.seq + size_t(r0) * kZfSeqSlot, uint64_t(rend - r0) * kZfSeqSlot * 4);
    bool act = b < a.n, ok = act;
    uint32_t clen = 0, shift = 0, irel = 0, cap = 0, orel = 0;
    if (act) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      shift = uint32_t(reinterpret_cast<uintptr_t>(a.in + s0) & 15);
      irel = uint32_t(((a.in + s0) - shift) - ibase);
      ok = len >= 6 && len - 4 <= 0xFFFFFFu;
      clen = ok ? uint32_t(len - 4) : 0u;
      if (kMode == kZlDecode) {
        const uint64_t c64 = a.out_off[b + 1] - a.out_off[b];
        cap = uint32_t(min(c64, uint64_t(kZlMaxOut)));
        ok = ok && c64 <= kZlMaxOut;
        orel = uint32_t(a.out_off[b] - a.out_off[r0]);
      }
      if (kMode == kZlStage) {
        cap = kZlMaxOut;
        orel = (b - r0) * kZlStageStride;
      }
    }
    // the bit reader at the stream's first byte
    ZlIn zi;
    zi.cur = bload<0>(R, ok ? irel : kOOB);
    zi.nxt = bload<0>(R, ok ? irel + 16 : kOOB);
    zi.nx2 = bload<0>(R, ok ? irel + 32 : kOOB);
    zi.c = 0;
    zi.used = 0;
    {
      // the dword holding byte `shift`, its bytes from there on; then the next dword
      const uint32_t k0 = shift >> 2;
      zi.bb = dword_of(zi.cur, k0) >> (8 * (shift & 3));
      zi.nb = 32 - 8 * (shift & 3);
      const bool adv = k0 == 3;
      const v4u c3 = bload<0>(R, (ok && adv) ? irel + 48 : kOOB);
      zi.k = adv ? 0u : k0 + 1;
      zi.cur = adv ? zi.nxt : zi.cur;
      zi.nxt = adv ? zi.nx2 : zi.nxt;
      zi.nx2 = adv ? c3 : zi.nx2;
      zi.c = adv ? 1u : 0u;
    }
    const uint32_t ubits = 8 * clen;  // the stream's bits (its Adler-32 included)
    zl_refill(zi, R, irel, ok);
    // RFC 1950 header: CM 8, CINFO <= 7, FCHECK, no preset dictionary
    if (ok) {
      const uint32_t cmf = zl_take(zi, 8), flg = zl_take(zi, 8);
      ok = (cmf & 15) == 8 && (cmf >> 4) <= 7 && ((cmf << 8) | flg) % 31 == 0 && !(flg & 0x20);
    }
    uint32_t o = 0, nl = 0, ll = 0, nseq = 0;
    v4u lbuf = {0, 0, 0, 0}, qv = {0, 0, 0, 0};
    bool more = ok;  // deflate blocks left
    while (__ballot(more)) {
      // ---- a block header
      zl_refill(zi, R, irel, more);
      uint32_t bfinal = 0, btype = 0;
      if (more) {
        bfinal = zl_take(zi, 1);
        btype = zl_take(zi, 2);
      }
      bool huff = more && (btype == 1 || btype == 2);
      bool dyn = more && btype == 2;
      // stored: to the byte boundary, LEN and NLEN; only empty ones stay here (Go's closing block)
      {
        const bool st = more && btype == 0;
        if (__ballot(st)) {
          const uint32_t al = st ? (zi.nb & 7) : 0u;
          if (st) (void)zl_take(zi, al);
          zl_refill(zi, R, irel, st);
          uint32_t ln = 0, nln = 0;
          if (st) {
            ln = zl_take(zi, 16);
            nln = zl_take(zi, 16);
          }
          ok = ok && !(st && (ln != 0 || nln != 0xFFFFu));
        }
        ok = ok && !(more && btype == 3);
      }
      huff = huff && ok;
      dyn = dyn && ok;
      ZlTab tl, td;  // the block's tables (dynamic: built below; fixed: set after)
      bool own = false;  // the lane's own (dynamic) tables
      uint64_t hi_dyn[3] = {0, 0, 0};  // the dynamic literal/length table's first non-literal slots
      if (__ballot(dyn)) {
        // HLIT, HDIST, HCLEN, then the code-length code's lengths (3 bits each, in kZlClOrder)
        zl_refill(zi, R, irel, dyn);
        uint32_t hlit = 0, hdist = 0, hclen = 0;
        if (dyn) {
          hlit = zl_take(zi, 5) + 257;
          hdist = zl_take(zi, 5) + 1;
          hclen = zl_take(zi, 4) + 4;
        }
        ok = ok && !(dyn && (hlit > 286 || hdist > 30));
        dyn = dyn && ok;
        uint64_t clp = 0;  // symbol s's length at bits 3s
#pragma unroll
        for (uint32_t i = 0; i < 19; i++) {
          if (i % 8 == 0) zl_refill(zi, R, irel, dyn);
          const bool rd = dyn && i < hclen;
          const uint32_t v = rd ? zl_take(zi, 3) : 0u;
          clp |= uint64_t(v) << (3 * kZlClOrder[i]);
        }
        // the code-length code: counts, table, sorted symbols (lane's LDS)
        uint32_t cc[16] = {};
#pragma unroll
        for (uint32_t s = 0; s < 19; s++) {
          const uint32_t l = uint32_t(clp >> (3 * s)) & 7u;
#pragma unroll
          for (uint32_t k = 1; k < 8; k++) cc[k] += l == k ? 1u : 0u;
        }
        ZlTab tc;
        uint64_t cn[3], clw0 = 0, clw1 = 0;  // the sorted code-length symbols, 5 bits each
        ok = ok && !(dyn && !zl_canon(cc, tc, cn));
        dyn = dyn && ok;
#pragma unroll
        for (uint32_t s = 0; s < 19; s++) {
          const uint32_t l = uint32_t(clp >> (3 * s)) & 7u;
          const uint32_t p = zl_put(cn, l);
          if (dyn && l) {
            clw0 |= p < 12 ? uint64_t(s) << (5 * p) : 0ull;
            clw1 |= p >= 12 ? uint64_t(s) << (5 * (p - 12)) : 0ull;
          }
        }
        // the literal/length and distance code lengths, twice: counted, then placed
        const ZlIn save = zi;
        uint64_t cntl[3] = {0, 0, 0}, cntd[3] = {0, 0, 0}, cnt8[3] = {0, 0, 0}, nxl[3], nxd[3];
        bool eob = false;  // length of symbol 256 nonzero
        for (uint32_t pass = 0; pass < 2; pass++) {
          if (pass == 1) {
            zi = save;
            uint32_t cl16[16], cd16[16];
            zl_unpack(cntl, cl16);
            zl_unpack(cntd, cd16);
            const bool cl_ok = zl_canon(cl16, tl, nxl), cd_ok = zl_canon(cd16, td, nxd);
            // each length's first slot + its literals (fields < 512: no carries between them)
            hi_dyn[0] = nxl[0] + cnt8[0];
            hi_dyn[1] = nxl[1] + cnt8[1];
            hi_dyn[2] = nxl[2] + cnt8[2];
            ok = ok && !(dyn && (!cl_ok || !cd_ok || !eob));
            dyn = dyn && ok;
          }
          uint32_t i = 0, prev = 0;
          bool go = dyn;
          const uint32_t nall = hlit + hdist;
          while (__ballot(go)) {
            zl_refill(zi, R, irel, go);
            uint32_t L = 1, idx = 0;
            zl_find<7>(zi, tc, L, idx);
            const uint32_t ci = min(idx, 18u);
            const uint32_t sym = go ? uint32_t((ci < 12 ? clw0 >> (5 * ci) : clw1 >> (5 * (ci - 12))) & 31u) : 0u;
            if (go) (void)zl_take(zi, L);
            uint32_t rep = 1, val = sym;
            const uint32_t xb = sym == 16 ? 2u : (sym == 17 ? 3u : (sym == 18 ? 7u : 0u));
            const uint32_t x = go ? zl_take(zi, xb) : 0u;
            if (sym == 16) {
              rep = 3 + x;
              val = prev;
            } else if (sym == 17) {
              rep = 3 + x;
              val = 0;
            } else if (sym == 18) {
              rep = 11 + x;
              val = 0;
            }
            const bool bad = go && ((sym == 16 && i == 0) || i + rep > nall || zi.used > ubits);
            ok = ok && !bad;
            go = go && !bad;
            if (go) {
              // symbols i .. i + rep - 1 get length val: [i, min(end, hlit)) literal/length, the rest distance
              const uint32_t nlit = i < hlit ? min(i + rep, hlit) - i : 0u;
              const uint32_t nd = rep - nlit;
              if (pass == 0) {
                zl_count(cntl, val, nlit);
                zl_count(cntd, val, nd);
                const uint32_t l8 = min(hlit, 256u);  // the literals 0..255 among them
                zl_count(cnt8, val, i < l8 ? min(i + rep, l8) - i : 0u);
                eob = eob || (val != 0 && i <= 256 && 256 < i + nlit);
              } else if (val != 0) {
                for (uint32_t j = 0; j < rep; j++) {  // (rep <= 138; usually 1)
                  const uint32_t s = i + j;
                  if (s < hlit) {
                    const uint32_t p = zl_put(nxl, val);
                    mine[64 * p] = uint8_t(s);
                  } else {
                    const uint32_t p = zl_put(nxd, val);
                    mine[64 * (kZlDistOff + p)] = uint8_t(s - hlit);
                  }
                }
              }
              prev = val;
              i += rep;
              go = i < nall;
            }
          }
        }
        own = dyn;
      }
      if (!own) {  // fixed codes (RFC 1951 3.2.6), or a lane that has no Huffman block here
        ZlTab fl, fd;
        zl_fixed_counts(fl, fd);
        tl = fl;
        td = fd;
      }
      huff = huff && ok;
      // ---- the block's symbols: st 0 = a literal/length code next, 1 = a distance code
      uint32_t st = 0, ml = 0;
      bool inb = huff;
      uint32_t kmax = inb ? max(tl.maxl, td.maxl) : 1u;
      for (int sh = 32; sh >= 1; sh >>= 1) kmax = max(kmax, uint32_t(__shfl_xor(int(kmax), sh, 64)));
      kmax = __builtin_amdgcn_readfirstlane(kmax);
      while (__ballot(inb)) {
        zl_refill(zi, R, irel, inb);
        uint32_t L = 1, idx = 0;
        zl_find2(zi, tl, td, st == 1, kmax, L, idx);
        const uint32_t ci = st == 1 ? min(idx, 31u) : min(idx, 287u);
        const uint32_t tb = uint32_t(mine[64 * ((st == 1 ? kZlDistOff : 0u) + ci)]);  // (own tables)
        const uint32_t sym = own ? tb + ((st == 0 && idx >= zl_hi_at(hi_dyn, L)) ? 256u : 0u) : zl_fixed_sym(st == 1, ci);
        if (inb) (void)zl_take(zi, L);
        const bool lit = inb && st == 0 && sym < 256;
        const bool end = inb && st == 0 && sym == 256;
        const bool len = inb && st == 0 && sym > 256;
        const bool dst = inb && st == 1;
        // a literal byte: into the 16-byte staging, stored when it fills
        if (!kPlan) {
          const uint32_t q = nl & 15, sh = 8 * (q & 3), wd = q >> 2;
          const uint32_t keep = ~(0xFFu << sh), put = (sym & 0xFFu) << sh;
          lbuf.x = (lit && wd == 0) ? ((lbuf.x & keep) | put) : lbuf.x;
          lbuf.y = (lit && wd == 1) ? ((lbuf.y & keep) | put) : lbuf.y;
          lbuf.z = (lit && wd == 2) ? ((lbuf.z & keep) | put) : lbuf.z;
          lbuf.w = (lit && wd == 3) ? ((lbuf.w & keep) | put) : lbuf.w;
          const bool full = lit && q == 15 && ok;
          __builtin_amdgcn_raw_buffer_store_b128(lbuf, RO, full ? orel + (nl & ~15u) : kOOB, 0, 0);
        }
        nl += lit ? 1u : 0u;
        ll += lit ? 1u : 0u;
        o += lit ? 1u : 0u;
        // a length code's extra bits, then a distance code next
        const uint32_t ls = len ? sym - 257 : 0u;
        const uint32_t lx = len ? len_extra(ls) : 0u;
        const uint32_t lxv = len ? zl_take(zi, lx) : 0u;
        ml = len ? len_base(ls) + lxv : ml;
        // a distance code and its extra bits: the sequence (ll, ml, dist)
        const uint32_t dx = dst ? dist_extra(sym) : 0u;
        zl_refill(zi, R, irel, dst && dx > 0);
        const uint32_t dxv = dst ? zl_take(zi, dx) : 0u;
        const uint32_t dist = dist_base(sym) + dxv;
        const bool bad = (len && ls >= 29) || (dst && (sym >= 30 || dist > o || dist > 4096 || ll >= 1024 ||
                                                       nseq >= kZlMaxSeqs)) ||
                         (inb && zi.used > ubits) || (!kPlan && inb && o + (dst ? ml : 0u) > cap) ||
                         (kPlan && o > kZlMaxOut);
        if (!kPlan && dst && !bad) {
          const uint32_t r = ll | ((ml - 3) << 10) | ((dist - 1) << 20);
          qv.x = (nseq & 3) == 0 ? r : qv.x;
          qv.y = (nseq & 3) == 1 ? r : qv.y;
          qv.z = (nseq & 3) == 2 ? r : qv.z;
          qv.w = (nseq & 3) == 3 ? r : qv.w;
          const bool st4 = (nseq & 3) == 3;
          __builtin_amdgcn_raw_buffer_store_b128(qv, RS, st4 ? (b - r0) * kZfSeqSlot * 4 + 16 * (nseq >> 2) : kOOB, 0,
                                                 0);
        }
        o += (dst && !bad) ? ml : 0u;
        nseq += (dst && !bad) ? 1u : 0u;
        ll = (dst && !bad) ? 0u : ll;
        ok = ok && !bad;
        st = (len && !bad) ? 1u : ((dst || bad) ? 0u : st);
        inb = inb && !bad && !end;
      }
      more = more && ok && bfinal == 0;
    }
    // ---- the Adler-32 after the last block, at the next byte boundary
    uint32_t want = 0;
    if (ok) {
      (void)zl_take(zi, zi.nb & 7);
      zl_refill(zi, R, irel, true);
      const uint32_t w = zl_take(zi, 32);
      want = __builtin_bswap32(w);
      ok = zi.used <= ubits;
    }
    if (kSizes) {
      if (act && ok) {
        out_sz[b] = align16(o);
        row_sz[b] = row_capacity(o);
      }
      zl_list_append(act && !ok, b, plist, pcount);
    }
    if (!kPlan) {
      // the last literals and the last sequences
      __builtin_amdgcn_raw_buffer_store_b128(lbuf, RO, (ok && (nl & 15)) ? orel + (nl & ~15u) : kOOB, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(qv, RS, (ok && (nseq & 3)) ? (b - r0) * kZfSeqSlot * 4 + 16 * (nseq >> 2) : kOOB,
                                             0, 0);
      v4u w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0};
      if (ok) {
        w0.y = nl;
        w0.z = o;
        w0.w = nseq | ((kZfFast | kZfSeq4 | kZfOutLit | kZfAdler) << 16);
        w1.x = want;
      }
      if (act) {
        reinterpret_cast<v4u*>(z.rec + b)[0] = w0;
        reinterpret_cast<v4u*>(z.rec + b)[1] = w1;
      }
      if (!kSizes) zl_list_append(act && !ok, b, z.list, z.count);
    }
  }
}

hipError_t launch_zlib_fast_parse(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zl_fast_kernel<kZlDecode>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(kZlLds));
  if (attr != hipSuccess) return attr;
  const uint32_t grid = min((a.n + kZlThreads - 1) / kZlThreads, uint32_t(num_cus) * kZlWgPerCu);
  zl_fast_kernel<kZlDecode><<<grid, kZlThreads, kZlLds, st>>>(a, z, nullptr, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_zlib_plan_fast(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                                 uint64_t* out_sz, uint64_t* row_sz, uint32_t* list, uint32_t* count, int num_cus,
                                 const ZlStage* stage) {
  if (n == 0) return hipGetLastError();
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&zl_fast_kernel<kZlPlan>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(kZlLds));
  static const hipError_t attr_s = hipFuncSetAttribute(reinterpret_cast<const void*>(&zl_fast_kernel<kZlStage>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(kZlLds));
  if (attr != hipSuccess) return attr;
  if (attr_s != hipSuccess) return attr_s;
  DecodeArgs a{};
  a.in = in;
  a.in_off = in_off;
  a.n = n;
  const uint32_t grid = min((n + kZlThreads - 1) / kZlThreads, uint32_t(num_cus > 0 ? num_cus : 256) * kZlWgPerCu);
  if (stage) {
    ZsFastArgs z{};
    z.rec = stage->rec;
    z.seq = stage->seq;
    z.lit = stage->lit;
    zl_fast_kernel<kZlStage><<<grid, kZlThreads, kZlLds, st>>>(a, z, out_sz, row_sz, list, count);
  } else {
    ZsFastArgs z{};
    zl_fast_kernel<kZlPlan><<<grid, kZlThreads, kZlLds, st>>>(a, z, out_sz, row_sz, list, count);
  }
  return hipGetLastError();
}

}  // namespace slate
