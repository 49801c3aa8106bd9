// Snappy block decode in two phases: a lane-per-block walk, then a wave-per-block build.
//
// block.Decode (internal/sstable/block/block.go:78-134) with CodecSnappy: CRC32 verify ->
// golang/snappy v0.0.4 decode (decode_other.go:19-110) -> offset checks -> row descriptors
// (row.go:191-261 as block/iterator.go walks the rows).
//
// The Snappy tag chain is serial inside a block: where a tag starts depends on the length of
// the one before.  The lane-per-block decoder (decode_lpb2.hip) runs 64 blocks' chains in
// lockstep and moves every decoded byte through a 128-byte ring per lane; that ring (272 B of
// LDS per lane) caps it at two waves per SIMD, and each step carries the whole machinery
// (rings, holes for far copies, throttles) whether or not the block needs it.  Here the two
// halves of the work get the shapes they want:
//
//  W  snappy_walk_kernel, lane per block, 64 blocks per wave in lockstep: the chain walk only.
//     It streams the block through a small LDS input ring (128-byte transposed refills: lanes
//     8i..8i+7 load one 128-byte run of a block), folds every chunk into the block CRC32, parses
//     each tag with golang/snappy's checks, and records every 8th tag's position (an "anchor":
//     input offset, decoded offset, first piece index).  No byte is copied.  Per block it writes
//     a 16-byte record and the anchors.
//  D  snappy_build_kernel, wave per block, the whole block in LDS: the compressed bytes are
//     staged with coalesced loads; one lane per anchor re-parses its 8 tags into copy pieces of
//     at most 60 bytes (a copy whose source lies inside the literal just before it becomes a
//     read of that literal's input bytes); the pieces are then executed in groups of up to
//     four -- 16 lanes per piece, 4 bytes per lane -- where a piece joins a group only if its
//     source bytes were final before the group started; then block.go's checks, the rows
//     (one lane per row, the exact row.go field order) and coalesced stores of the block, its
//     rows and its meta.
//  F  anything either phase does not take on its happy path -- a failed CRC or Snappy check,
//     a block larger than D's LDS staging, more tags than anchors, a failed block.go or row
//     check -- is decoded by decode_lpb2_kernel, which skips every block D completed
//     (DecodeArgs::wpb).  Statuses, bytes and rows are therefore always the exact decoder's.
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"
#include "lpb_common.h"

namespace slate {

namespace {

// ---- the per-block record W writes and D reads (kWpbRecBytes per block)
//   dword 0: flags (bit 0: D decodes this block) | ntags << 16
//   dword 1: decoded length
//   dword 2: pieces | header length << 16 | anchors << 24
//   dword 3: compressed payload length (without the CRC)
//   then anchors, 8 bytes each: input offset | decoded offset << 16, first piece
constexpr uint32_t kWpbD = 1;
constexpr uint32_t kAnchorTags = 8;
constexpr uint32_t kMaxAnchors = 40;
static_assert(kWpbRecBytes == 16 + 8 * kMaxAnchors, "record layout");
constexpr uint32_t kMaxTags = kAnchorTags * kMaxAnchors;
constexpr uint32_t kPiece = 60;       // bytes per piece: 60 + 3 (alignment) fit 16 dwords
constexpr uint32_t kMaxPieces = 320;
// D's staging per wave: input (16-byte phase kept), output, piece records; a 16-byte guard
// before each region keeps the first unit's reads (up to 3 bytes before a source) in range
constexpr uint32_t kWpbInCap = 4240;
constexpr uint32_t kWpbOutCap = 4240;
constexpr uint32_t kGuard = 16;
constexpr uint32_t kMaxGroups = kMaxPieces;
// per wave: guard | IN | guard | OUT | pieces (8 B) | group starts (u16, + 1 sentinel) | junk
// (one dword per lane: where a lane's store goes when it has nothing to store)
constexpr uint32_t kWaveLds =
    kGuard + kWpbInCap + kGuard + kWpbOutCap + kMaxPieces * 8 + ((2 * (kMaxGroups + 1) + 15) & ~15u) + 64 * 4;
constexpr uint32_t kBuildWaves = 2;   // waves per workgroup of the build kernel

// ---- W: lane per block
constexpr uint32_t kWalkThreads = 256;         // 4 waves; three workgroups per CU (VGPRs: 3 waves per SIMD)
constexpr uint32_t kWNS = 8;                   // input ring slots (16 bytes each)
constexpr uint32_t kWIR = kWNS * 16;           // ring bytes
constexpr uint32_t kWStride = kWIR + 8;        // lane records 136 bytes apart (bank spread)
constexpr uint32_t kWSteps = 4;                // tags parsed per iteration
constexpr uint32_t kWChunks = 4;               // CRC chunks absorbed per iteration (= refill rate)

// CRC32 by 6-bit digits.  A 16-byte chunk is 128 message bits; digit k (bits 6k .. 6k+5, 22
// digits) contributes T6[k][digit], the XOR of the slicing-by-16 entries of its bits.  A 64-entry
// table fills the 64 LDS banks exactly once, so 64 lanes reading it never conflict (distinct
// entries sit in distinct banks, equal ones broadcast): the byte tables' random lookups cost the
// walk ~200 bank-conflict cycles per block (SQ_LDS_BANK_CONFLICT).
constexpr uint32_t kCrc6Digits = 22;
struct Crc6Tables {
  uint32_t t[kCrc6Digits][64];
  constexpr Crc6Tables() : t{} {
    uint32_t c8[16][256] = {};
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
      c8[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int q = 1; q < 16; q++) c8[q][i] = (c8[q - 1][i] >> 8) ^ c8[0][c8[q - 1][i] & 0xFF];
    for (uint32_t k = 0; k < kCrc6Digits; k++)
      for (uint32_t v = 0; v < 64; v++) {
        uint32_t r = 0;
        for (uint32_t bt = 0; bt < 6; bt++) {
          const uint32_t b = 6 * k + bt;
          if (b < 128 && ((v >> bt) & 1)) r ^= c8[15 - b / 8][1u << (b % 8)];
        }
        t[k][v] = r;
      }
  }
};
static __constant__ Crc6Tables g_crc6 = Crc6Tables();
constexpr uint32_t kTab6Bytes = kCrc6Digits * 64 * 4;

// the CRC register after the 16 bytes v (little-endian dwords)
__device__ __forceinline__ uint32_t crc6_chunk(const uint32_t* tab, uint32_t c, const v4u& v) {
  const uint32_t x = v.x ^ c, y = v.y, z = v.z, w = v.w;
  const uint32_t xy = __builtin_amdgcn_alignbit(y, x, 30), yz = __builtin_amdgcn_alignbit(z, y, 28);
#define D6(k, src, off) tab[64 * (k) + (((src) >> (off)) & 63u)]
  const uint32_t a = xor3(D6(0, x, 0), D6(1, x, 6), D6(2, x, 12)), b = xor3(D6(3, x, 18), D6(4, x, 24), D6(5, xy, 0));
  const uint32_t e = xor3(D6(6, y, 4), D6(7, y, 10), D6(8, y, 16)), f = xor3(D6(9, y, 22), D6(10, yz, 0), D6(11, z, 2));
  const uint32_t g = xor3(D6(12, z, 8), D6(13, z, 14), D6(14, z, 20)), h = xor3(D6(15, z, 26), D6(16, w, 0), D6(17, w, 6));
  const uint32_t i = xor3(D6(18, w, 12), D6(19, w, 18), D6(20, w, 24));
  const uint32_t j = tab[64 * 21 + (w >> 30)];
#undef D6
  return xor3(xor3(a, b, e), xor3(f, g, h), xor3(i, j, 0u));
}

struct Walk {
  uint32_t sh, clen, last_chunk, dn, s, d, err, dd, hdr;
  int32_t crc_last;
  uint32_t crc, crc_pos;
  uint32_t c_issue, c_commit, n_req;
  uint32_t ntags, pieces, nanch;
  // D's execution groups, decided here in tag order (see "Groups" above): the previous tag
  // (literal-sourced?, its output range), the open group's first output byte and used slots
  uint32_t p_lit, p_d, p_len, g, slots;
  // anchors: the open one (cur), a completed even one waiting for its pair (pend), and one
  // completed in this iteration (fin, index fin_i; fin_v set)
  uint32_t cur_x, cur_y, pend_x, pend_y, fin_x, fin_y, fin_i, fin_v;
};

// CRC32 of the next committed input chunk (bytes outside the block zeroed) -- as decode_lpb2.hip
__device__ __forceinline__ void walk_crc(Walk& L, const uint8_t* in, const uint32_t* tab, bool go) {
  const uint32_t k = L.crc_pos;
  v4u v = rd128(in + (k & (kWNS - 1)) * 16, 0u);
  const bool partial = go && (k == 0 || int32_t(k) == L.crc_last);
  if (__builtin_amdgcn_ballot_w64(partial)) {
    const int32_t lo = int32_t(L.sh) - int32_t(16 * k), hi = int32_t(L.sh + L.clen) - int32_t(16 * k);
    v.x &= keep_mask(lo, hi, 0);
    v.y &= keep_mask(lo, hi, 1);
    v.z &= keep_mask(lo, hi, 2);
    v.w &= keep_mask(lo, hi, 3);
  }
  const uint32_t c = crc6_chunk(tab, L.crc, v);
  L.crc = go ? c : L.crc;
  L.crc_pos += go ? 1u : 0u;
}

// Transposed refill: in load j (0..3), lanes 4i..4i+3 read chunks c_issue..c_issue+3 (one
// 64-byte run) of the block of lane 16j+i; the chunk goes into that block's ring next iteration.
__device__ __forceinline__ void walk_load(uint32_t j, uint32_t lane, uint32_t wave_lane0, uint32_t info, uint32_t rel,
                                          __amdgpu_buffer_rsrc_t rin, v4u& P, uint32_t& slot) {
  const uint32_t o = 16 * j + (lane >> 2), c = lane & 3;
  const uint32_t info_o = __shfl(info, int(o), 64);
  const uint32_t rel_o = __shfl(rel, int(o), 64);
  const uint32_t ci = (info_o >> 4) + c;
  const bool want = c < (info_o & 15);
  P = __builtin_amdgcn_raw_buffer_load_b128(rin, want ? rel_o + 16 * ci : kOOB, 0, 0);
  slot = want ? (wave_lane0 + o) * kWStride + (ci & (kWNS - 1)) * 16 : 0xFFFFFFFFu;
}

}  // namespace

__global__ __launch_bounds__(kWalkThreads) void snappy_walk_kernel(const uint8_t* __restrict__ gin,
                                                                    const uint64_t* __restrict__ in_off, uint32_t n,
                                                                    uint8_t* __restrict__ rec, uint32_t* round_counter) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  {
    const uint32_t* src = &g_crc6.t[0][0];
    for (uint32_t i = threadIdx.x; i < kCrc6Digits * 64; i += blockDim.x) tab[i] = src[i];
    __syncthreads();
  }
  const uint32_t* crc_init = g_crc_lt.init;
  const uint32_t* crc_tail = g_crc_lt.tail;
  uint8_t* rings = smem + kTab6Bytes;
  uint8_t* in = rings + threadIdx.x * kWStride;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_lane0 = threadIdx.x - lane;
  const uint32_t n_rounds = (n + 63) / 64;
  for (uint32_t r = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(round_counter, 1u) : 0u); r < n_rounds;
       r = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(round_counter, 1u) : 0u)) {
    const uint32_t round0 = r * 64, rend = min(round0 + 64, n);
    const uint8_t* in_lo = gin + in_off[round0];
    const uint8_t* in_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(in_lo) & ~uintptr_t(15));
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(in_base, align16(uint64_t((gin + in_off[rend]) - in_base)));
    const __amdgpu_buffer_rsrc_t rrec = make_rsrc(rec + size_t(round0) * kWpbRecBytes, size_t(64) * kWpbRecBytes);
    const uint32_t b = round0 + lane;
    Walk L;
    L.sh = L.clen = L.last_chunk = L.dn = L.s = L.d = L.err = L.hdr = 0;
    L.dd = 1;
    L.crc_last = -1;
    L.crc = 0xFFFFFFFFu;
    L.crc_pos = L.c_issue = L.c_commit = L.n_req = 0;
    L.ntags = L.pieces = L.nanch = 0;
    L.p_lit = L.p_d = L.p_len = L.g = 0;
    L.slots = 4;  // the first tag opens a group
    L.cur_x = L.cur_y = L.pend_x = L.pend_y = L.fin_x = L.fin_y = L.fin_i = L.fin_v = 0;
    uint32_t rel = 0;
    bool have = b < rend;
    if (have) {
      const uint64_t s0 = in_off[b], len = in_off[b + 1] - s0;
      if (len < 6 || len > 0xFFFFFF00ull) {
        have = false;  // block.Decode's size error (or a block W does not stream): the exact decoder reports it
      } else {
        const uint8_t* p = gin + s0;
        L.sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 15);
        rel = uint32_t((p - L.sh) - in_base);
        L.clen = uint32_t(len - 4);
        L.last_chunk = uint32_t((L.sh + len - 1) >> 4);
        L.crc_last = int32_t((L.sh + L.clen - 1) >> 4);
        L.crc = crc_init[L.sh];
      }
    }
    // ---- the first two chunks, then golang/snappy decodedLen (decode.go:20-31)
    {
      const v4u c0 = __builtin_amdgcn_raw_buffer_load_b128(rin, have ? rel : kOOB, 0, 0);
      const v4u c1 = __builtin_amdgcn_raw_buffer_load_b128(rin, (have && L.last_chunk >= 1) ? rel + 16 : kOOB, 0, 0);
      if (have) {
        wr128(in, c0, 0u);
        wr128(in + 16, c1, 0u);
        L.c_commit = L.c_issue = L.last_chunk >= 1 ? 2u : 1u;
        uint64_t x = 0;
        uint32_t sft = 0, hdr = 0;
        bool ok = false, stop = false;
        for (uint32_t i = 0; i < 10 && i < L.clen && !stop; i++) {
          const uint32_t bt = in[L.sh + i];
          if (bt < 0x80) {
            if (!(i == 9 && bt > 1)) {
              x |= uint64_t(bt) << sft;
              ok = x <= 0xffffffffull;
              hdr = i + 1;
            }
            stop = true;
          } else {
            x |= uint64_t(bt & 0x7f) << sft;
            sft += 7;
          }
        }
        if (!ok || x > kSnappyMaxExpansion * uint64_t(L.clen)) {
          L.err = 1;
        } else {
          L.dn = uint32_t(x);
          L.s = L.hdr = hdr;
          L.dd = 0;
        }
      }
    }
    v4u P[4];
    uint32_t S[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      P[j] = v4u{0, 0, 0, 0};
      S[j] = 0xFFFFFFFFu;
    }
    const uint32_t budget = have ? L.clen / 2 + 64 : 0u;
    uint32_t iters = 0;
    auto lane_done = [&]() { return L.dd && int32_t(L.crc_pos) > L.crc_last && L.c_commit > L.last_chunk; };
    while (__ballot(have && !lane_done() && iters < budget)) {
      const bool act = have && !lane_done() && iters < budget;
      // the chunks loaded last iteration go into their rings; ask for up to 4 more
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (S[j] != 0xFFFFFFFFu) wr128(rings + S[j], P[j], 0u);
      L.c_commit += L.n_req;
      const uint32_t lo_chunk = min((L.sh + (L.dd ? L.clen : L.s)) >> 4, L.crc_pos);
      const uint32_t room = lo_chunk + kWNS - L.c_issue, left = L.last_chunk + 1 - L.c_issue;
      const uint32_t nq = act ? min(min(room, left), 4u) : 0u;
      const uint32_t info = (L.c_issue << 4) | nq;
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) walk_load(j, lane, wave_lane0, info, rel, rin, P[j], S[j]);
      L.c_issue += nq;
      L.n_req = nq;
      // CRC of the committed chunks
#pragma unroll
      for (uint32_t k = 0; k < kWChunks; k++)
        walk_crc(L, in, tab, act && L.crc_pos < L.c_commit && int32_t(L.crc_pos) <= L.crc_last);
      // the tags whose header bytes are in (golang/snappy decode_other.go:19-110)
      const int32_t avail = int32_t(16 * L.c_commit) - int32_t(L.sh);
      const uint32_t sn = L.clen;
#pragma unroll
      for (uint32_t k = 0; k < kWSteps; k++) {
        const bool need = act && !L.dd;
        const bool fin = need && L.s >= sn;
        const bool can = need && L.s < sn && avail >= int32_t(min(L.s + 5, sn));
        const v2u w = ring_rd8(in, L.sh + L.s, kWIR - 8);
        const uint32_t c = w.x & 0xff, t = c & 3;
        const uint32_t b14 = (w.x >> 8) | (w.y << 24);
        const uint32_t xl = c >> 2;
        const uint32_t nb = xl >= 60 ? xl - 59 : 0;
        const uint32_t ext = nb >= 4 ? b14 : (b14 & ((1u << (8 * nb)) - 1));
        const uint64_t lit_len = uint64_t(nb ? ext : xl) + 1;
        const uint32_t cp_len = (t == 1) ? 4 + ((c >> 2) & 7) : 1 + (c >> 2);
        const uint32_t off1 = ((c & 0xe0) << 3) | (b14 & 0xff), off2 = b14 & 0xffff;
        const uint32_t cp_off = (t & 2) ? ((t & 1) ? b14 : off2) : off1;
        const uint32_t hl_cp = (t & 2) ? ((t & 1) ? 5u : 3u) : 2u;
        const uint32_t hl = (t == 0) ? 1 + nb : hl_cp;
        const uint32_t s1 = L.s + hl;
        const bool bad_lit = lit_len > uint64_t(L.dn - L.d) || lit_len > uint64_t(sn - min(s1, sn));
        const bool bad_cp = cp_off == 0 || L.d < cp_off || cp_len > L.dn - L.d;
        const bool bad = s1 > sn || (t == 0 ? bad_lit : bad_cp);
        const bool ok = can && !bad;
        L.err |= (can && bad) ? 1u : 0u;
        L.dd |= (fin || (can && bad)) ? 1u : 0u;
        const uint32_t len = t == 0 ? uint32_t(lit_len) : cp_len;
        // ---- D's groups (mirrored exactly by snappy_build_kernel's replay): a tag joins the open
        // group when its source bytes are final before the group's first output byte and a slot is
        // left; a copy whose source lies inside the previous literal-sourced tag reads that tag's
        // input (not across anchors: D's lane starts each anchor without a previous tag)
        const uint32_t tix = L.ntags;
        const bool first_of_anchor = (tix & (kAnchorTags - 1)) == 0;
        const uint32_t so = L.d - cp_off;
        const bool ovl = t != 0 && cp_off < len;
        const bool comp = t != 0 && !ovl && L.p_lit && !first_of_anchor && so >= L.p_d && so + len <= L.p_d + L.p_len;
        const bool lsrc = t == 0 || comp;
        const uint32_t np = (len + kPiece - 1) / kPiece;
        const bool join = !ovl && L.slots < 4 && (lsrc || so + len <= L.g);
        const uint32_t s0 = join ? L.slots : 0u;
        const uint32_t tot = s0 + np;
        const uint32_t nslots = ovl ? 4u : ((tot - 1) & 3) + 1;
        const uint32_t ng = ovl ? L.g : (tot > 4 ? L.d + kPiece * (np - nslots) : (join ? L.g : L.d));
        // every 8th tag opens an anchor (input offset, decoded offset, first piece, open slots);
        // the tags' group-start and slow bits complete it
        const bool opn = ok && first_of_anchor && L.nanch < kMaxAnchors;
        const bool cls = opn && tix > 0;
        L.fin_x = cls ? L.cur_x : L.fin_x;
        L.fin_y = cls ? L.cur_y : L.fin_y;
        L.fin_i = cls ? L.nanch - 1 : L.fin_i;
        L.fin_v |= cls ? 1u : 0u;
        L.cur_x = opn ? ((L.s & 0xffff) | (L.d << 16)) : L.cur_x;
        L.cur_y = opn ? (L.pieces | (L.slots << 10)) : L.cur_y;
        L.nanch += opn ? 1u : 0u;
        const uint32_t bit = tix & (kAnchorTags - 1);
        L.cur_y |= (ok && !join) ? (1u << (16 + bit)) : 0u;
        L.cur_y |= (ok && ovl) ? (1u << (24 + bit)) : 0u;
        L.slots = ok ? nslots : L.slots;
        L.g = ok ? ng : L.g;
        L.p_lit = ok ? uint32_t(lsrc) : L.p_lit;
        L.p_d = ok ? L.d : L.p_d;
        L.p_len = ok ? len : L.p_len;
        L.ntags += ok ? 1u : 0u;
        L.pieces += ok ? np : 0u;
        L.s = ok ? (t == 0 ? s1 + len : s1) : L.s;
        L.d += ok ? len : 0u;
      }
      // an anchor completed in this iteration (at most one: 8 tags per anchor, kWSteps per
      // iteration): an even one waits for its partner, an odd one is stored with it (16 bytes)
      const bool st_pair = L.fin_v && (L.fin_i & 1);
      v4u pr;
      pr.x = L.pend_x;
      pr.y = L.pend_y;
      pr.z = L.fin_x;
      pr.w = L.fin_y;
      __builtin_amdgcn_raw_buffer_store_b128(pr, rrec, st_pair ? lane * kWpbRecBytes + 16 + 8 * (L.fin_i - 1) : kOOB,
                                             0, 0);
      L.pend_x = (L.fin_v && !(L.fin_i & 1)) ? L.fin_x : L.pend_x;
      L.pend_y = (L.fin_v && !(L.fin_i & 1)) ? L.fin_y : L.pend_y;
      L.fin_v = 0;
      iters++;
    }
    if (b < rend) {
      // the block's stored CRC (BE32 after the payload, still in the ring): the register absorbed
      // t zero bytes after the payload, so compare against stored * x^(8t)
      bool okb = have && lane_done() && !L.err && L.d == L.dn && L.s == L.clen;
      if (have && lane_done()) {
        const uint32_t stored = __builtin_bswap32(ring_rd8(in, L.sh + L.clen, kWIR - 8).x);
        const uint32_t t = uint32_t(16 * (L.crc_last + 1)) - (L.sh + L.clen);
        okb = okb && gf2_mulmod(~stored, crc_tail[t]) == L.crc;
      }
      // what D takes: the block and its output fit its LDS staging, the tags its anchors
      okb = okb && L.dn >= 2 && L.sh + L.clen <= kWpbInCap && L.dn + 16 <= kWpbOutCap && L.ntags <= kMaxTags &&
            L.pieces <= kMaxPieces;
      // the last (open) anchor: with its waiting partner, or alone
      const uint32_t li = L.nanch - 1;
      v4u pr;
      pr.x = (li & 1) ? L.pend_x : L.cur_x;
      pr.y = (li & 1) ? L.pend_y : L.cur_y;
      pr.z = L.cur_x;
      pr.w = L.cur_y;
      __builtin_amdgcn_raw_buffer_store_b128(pr, rrec, (okb && L.nanch) ? lane * kWpbRecBytes + 16 + 8 * (li & ~1u)
                                                                       : kOOB, 0, 0);
      v4u h;
      h.x = (okb ? kWpbD : 0u) | (L.ntags << 16);
      h.y = L.dn;
      h.z = L.pieces | (L.hdr << 16) | (L.nanch << 24);
      h.w = L.clen;
      __builtin_amdgcn_raw_buffer_store_b128(h, rrec, lane * kWpbRecBytes, 0, 0);
    }
  }
}

namespace {

// 4 bytes at any byte address of LDS (two naturally aligned dword reads)
__device__ __forceinline__ uint32_t lds_at(const uint8_t* base, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (a & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
}
__device__ __forceinline__ uint32_t bswap16_lo(uint32_t w) { return ((w & 0xff) << 8) | ((w >> 8) & 0xff); }

}  // namespace

// D: one wave per block.
// Piece record (8 bytes): x = output offset | length << 16 | group start << 24 | slow << 25,
// y = LDS address of the source byte (IN for literal-sourced pieces, OUT for copies).
constexpr uint32_t kPieceGs = 1u << 24, kPieceSlow = 1u << 25;

// Stores of a unit that holds bytes [lo, hi) of its dword (lo 0..3, hi 1..4), one nibble per
// (lo, hi) at 4 * (4 lo + hi - 1): bit 0 = a b16 store (at byte 0 when lo == 0, else at 2), bit 1
// = a b8 store, bits 2-3 its byte.  [0,4) is one b32 store.  The b16 of [1,3) also writes byte 3,
// which belongs to a later piece: that piece's first unit is [3, 4), a b8 store, issued after
// every b16 store of the group (or in a later group).
constexpr uint64_t partial_stores_table() {
  uint64_t t = 0;
  for (uint32_t lo = 0; lo < 4; lo++)
    for (uint32_t hi = lo + 1; hi <= 4; hi++) {
      if (lo == 0 && hi == 4) continue;
      const bool pair0 = lo == 0 && hi >= 2;        // bytes 0, 1
      const bool pair2 = lo >= 1 && lo <= 2 && hi >= 3 && !(lo == 2 && hi == 3);  // bytes 2, 3
      const uint32_t b16 = (pair0 || pair2) ? 1u : 0u;
      // the byte a b16 does not cover
      uint32_t a8 = 4;
      if (lo == 0 && hi == 1) a8 = 0;
      else if (lo == 0 && hi == 3) a8 = 2;
      else if (lo == 1) a8 = 1;
      else if (lo == 2 && hi == 3) a8 = 2;
      else if (lo == 3) a8 = 3;
      const uint32_t nib = b16 | (a8 < 4 ? 2u | (a8 << 2) : 0u);
      t |= uint64_t(nib) << (4 * (4 * lo + hi - 1));
    }
  return t;
}
constexpr uint64_t kPartialStores = partial_stores_table();

__global__ __launch_bounds__(64 * kBuildWaves) void snappy_build_kernel(DecodeArgs a, uint8_t* __restrict__ rec,
                                                                         uint32_t* block_counter) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* const lds = smem;  // addresses below are byte offsets from smem
  const uint32_t IN = wave * kWaveLds + kGuard, OUT = IN + kWpbInCap + kGuard, OPS = OUT + kWpbOutCap;
  const uint32_t GRP = OPS + kMaxPieces * 8, JUNK = GRP + ((2 * (kMaxGroups + 1) + 15) & ~15u);
  uint2* const ops = reinterpret_cast<uint2*>(lds + OPS);
  uint16_t* const grp = reinterpret_cast<uint16_t*>(lds + GRP);
  const uint32_t junk = JUNK + 4 * lane;
  // blocks by a static stride: an atomic counter per block serialises on one L2 address (1 M of
  // them took longer than the decode)
  const uint32_t waves_total = gridDim.x * kBuildWaves;
  for (uint32_t b = blockIdx.x * kBuildWaves + __builtin_amdgcn_readfirstlane(wave); b < a.n; b += waves_total) {
    const uint4 h = *reinterpret_cast<const uint4*>(rec + size_t(b) * kWpbRecBytes);
    const uint32_t flags = __builtin_amdgcn_readfirstlane(h.x & 0xffff);
    if (!(flags & kWpbD)) continue;
    const uint32_t ntags = __builtin_amdgcn_readfirstlane(h.x >> 16), dn = __builtin_amdgcn_readfirstlane(h.y);
    const uint32_t npieces = __builtin_amdgcn_readfirstlane(h.z & 0xffff),
                   nanch = __builtin_amdgcn_readfirstlane(h.z >> 24);
    const uint32_t clen = __builtin_amdgcn_readfirstlane(h.w);
    const uint64_t s0 = a.in_off[b];
    const uint32_t sh = uint32_t(s0 & 15);
    // ---- stage the compressed block: chunk c = input bytes [16c, 16c + 16) from the aligned base
    {
      const uint4* g = reinterpret_cast<const uint4*>(a.in + (s0 - sh));
      const uint32_t nch = (sh + clen + 15) >> 4;
      for (uint32_t c = lane; c < nch; c += 64) *reinterpret_cast<uint4*>(lds + IN + 16 * c) = g[c];
    }
    uint2 anc = uint2{0, 0};
    if (lane < nanch) anc = *reinterpret_cast<const uint2*>(rec + size_t(b) * kWpbRecBytes + 16 + 8 * lane);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // ---- pieces: lane a re-parses tags 8a .. 8a+7 (W validated every one of them) and replays
    // W's group decisions from the anchor's group-start / slow bits and open slots
    {
      uint32_t s = anc.x & 0xffff, d = anc.x >> 16, p = anc.y & 0x3ff, slots = (anc.y >> 10) & 7;
      uint32_t pl_dst = 0, pl_len = 0, pl_src = 0;
      bool plit = false;
      const uint32_t t0 = kAnchorTags * lane, t_end = min(ntags, t0 + kAnchorTags);
      for (uint32_t t = t0; t < t_end; t++) {
        // the tag's first bytes: three aligned dwords
        const uint32_t a0 = IN + sh + s;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (a0 & ~3u));
        const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, a0 & 3u), w1 = __builtin_amdgcn_alignbyte(d2, d1, a0 & 3u);
        const uint32_t c = w0 & 0xff, tt = c & 3;
        const uint32_t b14 = (w0 >> 8) | (w1 << 24);
        const uint32_t xl = c >> 2;
        const uint32_t nb = xl >= 60 ? xl - 59 : 0;
        const uint32_t ext = nb >= 4 ? b14 : (b14 & ((1u << (8 * nb)) - 1));
        const uint32_t cp_len = (tt == 1) ? 4 + ((c >> 2) & 7) : 1 + (c >> 2);
        const uint32_t off = (tt & 2) ? ((tt & 1) ? b14 : (b14 & 0xffff)) : (((c & 0xe0) << 3) | (b14 & 0xff));
        const uint32_t hl = tt == 0 ? 1 + nb : ((tt & 2) ? ((tt & 1) ? 5u : 3u) : 2u);
        const uint32_t len = tt == 0 ? (nb ? ext : xl) + 1 : cp_len;
        const uint32_t so = d - off;
        // a copy of bytes the previous (literal-sourced) tag of this anchor produced reads its input
        const bool comp = tt != 0 && plit && so >= pl_dst && so + len <= pl_dst + pl_len;
        const bool lsrc = tt == 0 || comp;
        const uint32_t src = tt == 0 ? IN + sh + s + hl : (comp ? pl_src + (so - pl_dst) : OUT + so);
        const uint32_t bit = t - t0;
        const bool brk = (anc.y >> (16 + bit)) & 1, slow = (anc.y >> (24 + bit)) & 1;
        const uint32_t s0g = brk ? 0u : slots;
        const uint32_t np = (len + kPiece - 1) / kPiece;
        // first piece (every tag has one); more only for tags longer than kPiece
        {
          const bool gs = slow || ((s0g & 3) == 0);
          ops[p] = uint2{d | (min(kPiece, len) << 16) | (gs ? kPieceGs : 0u) | (slow ? kPieceSlow : 0u), src};
        }
        if (__builtin_expect(np > 1, 0)) {
          for (uint32_t q = 1; q < np; q++) {
            const bool gs = slow || (((s0g + q) & 3) == 0);
            ops[p + q] = uint2{(d + kPiece * q) | (min(kPiece, len - kPiece * q) << 16) | (gs ? kPieceGs : 0u) |
                                   (slow ? kPieceSlow : 0u),
                               src + kPiece * q};
          }
        }
        p += np;
        slots = slow ? 4u : ((s0g + np - 1) & 3) + 1;
        plit = lsrc;
        pl_dst = d;
        pl_len = len;
        pl_src = src;
        s += tt == 0 ? hl + len : hl;
        d += len;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // ---- the group list: starts of groups, in piece order, + a sentinel
    uint32_t ngroups = 0;
    for (uint32_t i0 = 0; i0 < npieces; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool gs = i < npieces && (ops[i].x & kPieceGs);
      const uint64_t m = __ballot(gs);
      if (gs) grp[ngroups + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u))] =
          uint16_t(i);
      ngroups += uint32_t(__builtin_popcountll(m));
    }
    if (lane == 0) grp[ngroups] = uint16_t(npieces);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // ---- execute the groups: up to four pieces each, 16 lanes (4 bytes each) per piece; every
    // store is issued by every lane (to its junk dword when it has nothing to store)
    {
      const uint32_t j = lane >> 4, u4 = 4 * (lane & 15);
      for (uint32_t gi = 0; gi < ngroups; gi++) {
        const uint32_t k0 = grp[gi], cnt = grp[gi + 1] - k0;  // uniform reads
        const bool have = j < cnt;
        const uint2 r = ops[k0 + (have ? j : 0u)];
        const uint32_t dst = r.x & 0xffff, len = (r.x >> 16) & 0xff, src = r.y;
        if (__builtin_amdgcn_readfirstlane(r.x) & kPieceSlow) {
          // a copy from itself (offset < length): bytes [dst - off, dst) are final and the pattern
          // repeats with period off; one byte per lane
          const uint32_t dst0 = __builtin_amdgcn_readfirstlane(dst), src0 = __builtin_amdgcn_readfirstlane(src);
          const uint32_t len0 = __builtin_amdgcn_readfirstlane(len);
          const uint32_t off = OUT + dst0 - src0;
          const float rcp = 1.0f / float(off);
          const uint32_t i = lane;
          const uint32_t qq = uint32_t((float(i) + 0.5f) * rcp);
          const uint32_t m = i - qq * off;
          const uint8_t v = lds[src0 + m];
          lds[i < len0 ? OUT + dst0 + i : junk] = v;
          continue;
        }
        const uint32_t ua = (dst & ~3u) + u4;
        const uint32_t lo = u4 == 0 ? (dst & 3u) : 0u;
        const int32_t e = int32_t(dst + len) - int32_t(ua);
        const uint32_t hi = uint32_t(min(max(e, 1), 4));
        // the unit's bytes [lo, hi) of its dword: full, or one b16 and one b8 (kPartialStores)
        const uint32_t idx = (have && int32_t(lo) < e) ? 4 * lo + hi - 1 : 4u;
        const uint32_t code = uint32_t(kPartialStores >> (4 * idx)) & 15u;
        const uint32_t sa = src + u4 - (dst & 3u);  // source of the unit's byte 0 (may precede src by < 4)
        const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (sa & ~3u));
        const uint32_t v = __builtin_amdgcn_alignbyte(w[1], w[0], sa & 3u);
        const uint32_t a16 = lo ? 2u : 0u, a8 = code >> 2;
        *reinterpret_cast<uint32_t*>(lds + (idx == 3 ? OUT + ua : junk)) = v;
        __builtin_amdgcn_wave_barrier();
        *reinterpret_cast<uint16_t*>(lds + ((code & 1) ? OUT + ua + a16 : junk)) = uint16_t(v >> (8 * a16));
        __builtin_amdgcn_wave_barrier();
        lds[(code & 2) ? OUT + ua + a8 : junk] = uint8_t(v >> (8 * a8));
        __builtin_amdgcn_wave_barrier();
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // ---- block.go:95-134 and the rows (row.go:191-261); anything but a clean block goes to the
    // exact decoder (the record's D flag is cleared)
    bool bad = false;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(bswap16_lo(lds_at(lds, OUT + dn - 2)));
    const int32_t osi = int32_t(dn) - 2 - 2 * int32_t(cnt);
    const uint64_t rb0 = a.row_base[b];
    const uint64_t rcap = a.row_base[b + 1] - rb0;
    bad = osi <= 0 || cnt == 0 || cnt > rcap;
    uint32_t kl = 0;
    if (!bad) {
      const uint32_t off0 = bswap16_lo(lds_at(lds, OUT + uint32_t(osi)));
      kl = bswap16_lo(lds_at(lds, OUT + off0));
      const uint32_t lo = (off0 + 2) & 0xffff, hi = (off0 + 2 + kl) & 0xffff;
      bad = off0 > uint32_t(osi) || uint32_t(osi) - off0 < 2 || lo > hi || hi > dn;
    }
    // row 0's suffix length is the first key's length for the prefix check of the others
    uint32_t sl0 = 0;
    if (!bad) sl0 = bswap16_lo(lds_at(lds, OUT + bswap16_lo(lds_at(lds, OUT + uint32_t(osi))) + 2));
    for (uint32_t i0 = 0; i0 < cnt && !bad; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool rbad = false;
      uint4 rw = uint4{0, 0, 0, 0};
      if (i < cnt) {
        const uint32_t ro = bswap16_lo(lds_at(lds, OUT + uint32_t(osi) + 2 * i));
        const uint32_t n = uint32_t(osi) - ro;
        rbad = ro > uint32_t(osi) || n < 13;
        if (!rbad) {
          const uint32_t hw = lds_at(lds, OUT + ro);
          const uint32_t pl = bswap16_lo(hw), sl = bswap16_lo(hw >> 16);
          rbad = (i == 0 ? pl != 0 : pl > sl0) || n - 4 < sl || n - 4 - sl < 9;
          if (!rbad) {
            uint32_t o = 4 + sl;
            const uint32_t fl = lds_at(lds, OUT + ro + o + 8) & 0xff;
            o += 9;
            if (fl & 2) {
              rbad = rbad || n - o < 8;
              o += 8;
            }
            if (fl & 4) {
              rbad = rbad || (o <= n && n - o < 8);
              o += 8;
            }
            uint32_t vl = 0;
            if (!rbad && !(fl & 1)) {
              rbad = o > n || n - o < 4;
              if (!rbad) {
                vl = __builtin_bswap32(lds_at(lds, OUT + ro + o));
                o += 4;
                rbad = n - o < vl;
              }
            }
            rbad = rbad || o > n;
            rw.x = ro;
            rw.y = pl | (sl << 16);
            rw.z = (fl & 1) ? 0u : vl;
            rw.w = (fl & 7) | (((o - 4 - sl) & 0xff) << 8);
          }
        }
      }
      bad = __ballot(rbad) != 0;
      if (!bad && i < cnt) reinterpret_cast<uint4*>(a.rows + rb0)[i] = rw;
    }
    if (bad) {
      if (lane == 0) rec[size_t(b) * kWpbRecBytes] = uint8_t(flags & ~kWpbD);  // the exact decoder takes it
      continue;
    }
    // ---- the decoded block (16-byte chunks; the last one padded inside its slot) and the meta
    {
      uint4* g = reinterpret_cast<uint4*>(a.out + a.out_off[b]);
      const uint32_t nch = (dn + 15) >> 4;
      for (uint32_t c = lane; c < nch; c += 64) g[c] = *reinterpret_cast<const uint4*>(lds + OUT + 16 * c);
    }
    if (lane == 0) {
      slate_block_meta m{};
      m.status = SLATE_OK;
      m.data_len = uint32_t(osi);
      m.n_rows = uint16_t(cnt);
      m.aux = uint16_t(kl);
      a.meta[b] = m;
    }
    // the next block's staging must not overwrite this one's LDS before the stores read it
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

size_t wpb_record_bytes(uint32_t n) { return size_t(n) * kWpbRecBytes; }

hipError_t launch_decode_wpb(hipStream_t st, const DecodeArgs& a_in, uint8_t* rec, uint32_t* counters, int num_cus) {
  DecodeArgs a = a_in;
  if (a.n == 0) return hipGetLastError();
  (void)hipMemsetAsync(counters, 0, 2 * sizeof(uint32_t), st);
  // W: as many 8-wave workgroups as LDS allows (5.5 KiB digit tables + 136 B ring per lane)
  const size_t w_lds = kTab6Bytes + size_t(kWalkThreads) * kWStride;
  static const hipError_t attr_w = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_walk_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(w_lds));
  if (attr_w != hipSuccess) return attr_w;
  const uint32_t rounds = (a.n + 63) / 64;
  const uint32_t w_grid = min((rounds + kWalkThreads / 64 - 1) / (kWalkThreads / 64),
                              uint32_t(num_cus) * uint32_t(163840 / w_lds));
  snappy_walk_kernel<<<w_grid, kWalkThreads, w_lds, st>>>(a.in, a.in_off, a.n, rec, counters);
  // D: workgroups of kBuildWaves waves, as many as LDS allows
  const size_t d_lds = size_t(kBuildWaves) * kWaveLds;
  static const hipError_t attr_d = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_build_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(d_lds));
  if (attr_d != hipSuccess) return attr_d;
  const uint32_t d_grid = min((a.n + kBuildWaves - 1) / kBuildWaves, uint32_t(num_cus) * uint32_t(163840 / d_lds));
  snappy_build_kernel<<<d_grid, 64 * kBuildWaves, d_lds, st>>>(a, rec, counters + 1);
  // F: the exact lane-per-block decoder over whatever D did not complete
  a.wpb = rec;
  return launch_decode_lpb2(st, a, num_cus);
}

}  // namespace slate
