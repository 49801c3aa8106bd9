// Lane-per-block Snappy block decode (the headline kernel).
//
// block.Decode (internal/sstable/block/block.go:78-134) with CodecSnappy:
// CRC32 verify -> golang/snappy v0.0.4 decode (decode_other.go:19-110) ->
// offset checks -> row descriptors (row.go:191-261 as block/iterator.go walks).
//
// One lane owns one block; the 64 lanes of a wave decode 64 consecutive blocks in
// lockstep, so one wave instruction advances 64 independent Snappy tag streams (the
// chain inside one block is serial).  A round (64 blocks) runs as iterations of four
// steps; a step parses a tag if the previous one is used up and moves up to 16 bytes.
//
// Memory.  Every global access is shaped for the number of requests, not bytes
// (tools/scatter_probe.hip measured 16-byte per-lane accesses at 3.5-8x the cost of
// 64-128-byte runs):
//   * input: at the start of each iteration, four transposed loads fetch up to four new
//     16-byte chunks per block: in load j, lanes 4i..4i+3 read four consecutive chunks
//     (one 64-byte run) of block 16j+i.  They land in the block's LDS input ring (8
//     chunks) at the start of the next iteration, so a load has a whole iteration to
//     arrive, and the ring double-buffers a literal stream at full rate;
//   * output: completed aligned 16-byte chunks are flushed at the end of each iteration
//     by four transposed stores (lanes 4i..4i+3 write one block's four chunks);
//   * all buffer loads/stores are always issued (an out-of-range offset drops a lane:
//     tools/buf_probe.hip), so vmcnt bookkeeping is static, and stores come after the
//     loads they could otherwise delay (a vmcnt wait covers every older access);
//   * a copy with offset > 108 (beyond what the 128-byte output ring still holds) and
//     length <= 16 becomes a "hole": its output bytes are reserved, its source is loaded
//     from the flushed output at the end of the iteration, decoding continues, and the
//     bytes are merged into the ring at the start of the next one.  Flush, walker and ring
//     copies wait for a hole that overlaps them.  Longer far copies stream 16 bytes per
//     iteration.
// LDS: every access is naturally aligned (gfx950 serialises misaligned LDS accesses lane
// by lane: tools/lds_cost_probe.hip), see "Rings and natural alignment" below.
// CRC32 is absorbed from the input ring in two of the four steps (slicing-by-16 tables
// shared by the workgroup).  Bytes of a chunk outside the block are zeroed: the register
// starts from a per-alignment state that reaches 0xFFFFFFFF after the leading zeros, and
// the trailing zeros are folded into the stored value (x^(8t) mod P).
// A row walker reads each row's header from the output ring as it is produced and checks
// the key prefix inline; at block end a wave-cooperative pass compares the walked row
// starts with the block's offset array, and mismatches re-derive rows from HBM with the
// exact row.go decoder.
#ifndef SLATE_LPB_OR
#define SLATE_LPB_OR 256
#endif
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"
#include "lpb_common.h"

namespace slate {

namespace {

// ring positions still valid behind d: a step's store reaches 20 bytes past d's dword
// (five dwords), i.e. 109 bytes behind d modulo the ring
// bytes a step moves at most; its store writes kStep/4 + 1 dwords from d's dword (a 32-byte step
// was measured slower in round 5: 4.189 vs 4.151 ms per 1 M blocks, same box, and removed)
constexpr uint32_t kStep = 16;
constexpr uint32_t kStoreReach = kStep + 4;
constexpr uint32_t kReach = kOR - kStoreReach;
// section markers in the assembly (tools/loop_mix.py --marks): reading aid only, they fence the scheduler
#ifdef SLATE_ASM_MARKS
#define LPB_MARK(x) asm volatile("; @@" #x ::: "memory")
#else
#define LPB_MARK(x) ((void)0)
#endif
// CodecLz4 frame constants (LZ4 frame format; decode.hip has the exact path's copies)
constexpr uint32_t kLz4Magic = 0x184D2204u;
constexpr uint32_t kXP1 = 2654435761u, kXP2 = 2246822519u, kXP3 = 3266489917u, kXP4 = 668265263u,
                   kXP5 = 374761393u;
__device__ __forceinline__ uint32_t xrotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// d - 16*fl before a step may advance d (see the throttle): a hole's source ends flushed
// (U <= kReach - 15) and the unflushed bytes plus a step's store stay in the ring (U + kStep +
// kStoreReach <= kOR)
constexpr uint32_t kUnflushed = kOR - 16 - 2 * kStep;
static_assert(kUnflushed + 15 <= kReach && kUnflushed + kStep + kStoreReach <= kOR, "throttle");
// output chunks per block per flush store: lanes kRun*i .. kRun*i + kRun-1 write one run of kRun chunks
// (64-byte runs from the 128-byte ring, 128-byte runs from a 256-byte one); an iteration's
// kFlushStores stores cover 64 / kFlushParts blocks, so with 128-byte runs and 16-byte steps each half
// of the wave flushes every other iteration
constexpr uint32_t kRun = kOR / 32, kFlushStores = kStep / 4;
constexpr uint32_t kFlushBlocks = kFlushStores * (64 / kRun), kFlushParts = 64 / kFlushBlocks;
static_assert(kFlushParts >= 1 && kFlushBlocks * kFlushParts == 64, "flush");
#ifndef SLATE_LPB_NS
#define SLATE_LPB_NS 8
#endif
constexpr uint32_t kNS = SLATE_LPB_NS;  // input ring slots (16 bytes each)
constexpr uint32_t kIR = kNS * 16;
// LDS: output rings, then input rings, no mirrors: every access is naturally aligned and
// wraps per element.  Lane records are 136 bytes apart (34 dwords): blocks of a round
// progress alike, so lanes touch the same ring positions at the same time, and a stride of
// 2 mod 32 dwords spreads them over the banks (a 128-byte stride put all 32 lanes of a
// half-wave on one bank).  Records are therefore 8-byte aligned: 16-byte chunks move as
// two b64 halves.
#ifndef SLATE_LPB_OPAD
#define SLATE_LPB_OPAD 8
#endif
#ifndef SLATE_LPB_IPAD
#define SLATE_LPB_IPAD 8
#endif
constexpr uint32_t kOutStride = kOR + SLATE_LPB_OPAD;
constexpr uint32_t kInStride = kIR + SLATE_LPB_IPAD;
#ifndef SLATE_VERIFY_BATCH
#define SLATE_VERIFY_BATCH 4
#endif
constexpr uint32_t kVerifyBatch = SLATE_VERIFY_BATCH;
// cache policy of the flush and row-descriptor stores (lpb_common.h bstore: sc1 = 16, nt = 2): the
// flush as nt, the rows sc1 (round 6, same-box A/Bs over 1 M blocks: flush nt 3.792 -> 3.752 and
// 3.785 -> 3.751 ms; rows nt 4.263; refills nt 3.758 alone, 3.776 with the flush nt;
// profiles/round6/ab/ab_lpb2_cpol.txt)
#ifndef SLATE_OUT_CPOL
#define SLATE_OUT_CPOL 2
#endif
#ifndef SLATE_ROW_CPOL
#define SLATE_ROW_CPOL 16
#endif
#ifndef SLATE_IN_CPOL  // the refills' loads
#define SLATE_IN_CPOL 0
#endif
constexpr int kOutCpol = SLATE_OUT_CPOL, kRowCpol = SLATE_ROW_CPOL, kInCpol = SLATE_IN_CPOL;
// the previous iteration's hole source is merged before step 1 (measured, configs[1], 1 M blocks,
// round 4: before step 0 4.535 ms, step 1 4.469, step 2 4.524): a step more for the load to arrive
#ifndef SLATE_WALK_LAG
#define SLATE_WALK_LAG 64
#endif
constexpr uint32_t kWalkLag = SLATE_WALK_LAG;  // walker lag (bytes) that calls it a second time in an iteration  // blocks per wait in the cooperative row check

__device__ __forceinline__ v4u pack_row(uint32_t off, uint32_t pl, uint32_t sl, uint32_t vl, uint32_t flags,
                                        uint32_t meta_len, uint32_t status) {
  v4u r;
  r.x = off;
  r.y = (pl & 0xffff) | (sl << 16);
  r.z = vl;
  r.w = (flags & 0xff) | ((meta_len & 0xff) << 8) | ((status & 0xffff) << 16);
  return r;
}

// v0 row decode (row.go:191-261) reading the decoded block from HBM: the exact
// fallback when the streaming walk does not match the offset array.
__device__ v4u row_from_hbm(const uint8_t* data, uint32_t data_len, uint32_t off, int fk, uint32_t* sl_out) {
  *sl_out = 0;
  const uint8_t* p = data + off;
  const uint32_t n = data_len - off;
  uint32_t pl = 0, sl = 0;
  if (n >= 4) {
    pl = out_be16(p);
    sl = out_be16(p + 2);
  }
  if (n < 13) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_TOO_SHORT));
  if (pl > uint32_t(fk < 0 ? 0 : fk)) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_PREFIX));
  uint32_t o = 4;
  if (n - o < sl) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_SUFFIX));
  o += sl;
  if (n - o < 9) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_PANIC));
  const uint32_t flags = out_u8(p + o + 8);
  o += 9;
  if (flags & 2) {
    if (n - o < 8) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_EXPIRE));
    o += 8;
  }
  if (flags & 4) {
    if (n - o < 8) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_CREATE));
    o += 8;
  }
  uint32_t vl = 0;
  if ((flags & 1) == 0) {
    if (n - o < 4) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_VALUE_LEN));
    vl = out_be32(p + o);
    o += 4;
    if (n - o < vl) return pack_row(off, pl, sl, 0, 0, 0, uint32_t(SLATE_E_ROW_VALUE));
  }
  *sl_out = sl;
  return pack_row(off, pl, sl, vl, flags & 7, o - 4 - sl, SLATE_OK);
}

// Per-lane flags as wave masks (one bit per lane; wave-uniform, so they live in SGPR pairs).  Kept
// as bools in the lane's state they lived in VGPRs as 0 / 1: a v_cndmask to write one and a v_cmp
// to read it at every use (~160 of the loop's ~1360 VALU).  As masks they combine with the ballots
// of the step's comparisons by SALU ops, and a select reads them directly (msel).
__device__ __forceinline__ uint64_t bal(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ uint32_t msel(uint64_t m, uint32_t a, uint32_t b);
__device__ __forceinline__ bool mbit(uint64_t m) { return msel(m, 1u, 0u) != 0; }
__device__ __forceinline__ uint32_t msel(uint64_t m, uint32_t a, uint32_t b) {  // this lane's bit of m ? a : b
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}
__device__ __forceinline__ uint32_t sub_sat(uint32_t a, uint32_t b) { return __builtin_elementwise_sub_sat(a, b); }
// a > b (unsigned) as a mask, one v_cmp: a comparison LLVM fuses with a subtraction of the same
// operands becomes the subtraction's borrow, which the ballot then materialises and compares again
__device__ __forceinline__ uint64_t ugt(uint32_t a, uint32_t b) {
  uint64_t m;
  asm("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
  return m;
}

struct Lane {
  // block
  uint32_t in_rel, out_rel, rows_rel;  // offsets of this block in the round's buffer resources
  uint32_t sh, clen, dn, last_chunk, rcap;
  int32_t crc_last;
  uint32_t crc, crc_pos;
  // decode: s = the next tag (payload-relative); src = the current item's source: an input-ring
  // position (sh included) for a literal, an output position for a copy
  uint32_t s, d, rem, src, eff;
  // masks: the current item is a literal (lit), a far copy (far); the decode is done (dd) or failed (err)
  uint64_t mlit, mfar, mdd, merr;
  uint32_t T;  // the output ring's dword at d & ~3 (what the next store merges below d)
  uint32_t z;  // a run-time zero (see rd128)
  uint32_t c_issue, c_commit, n_req, fl;
  uint32_t qoff;  // hole source requested this iteration (loaded once, before the flush)
  // pending hole: up to 16 bytes of a copy with offset > kReach reserve output [hd, hd+hl) and
  // decoding goes on; the source is loaded at the end of the iteration and merged at the start
  // of the next one (mhp's bit is set exactly from a hole's step to the next iteration's start)
  uint64_t mhp;
  uint32_t hd, hl;
  // row walker: phase 0 = header (prefix/suffix lengths), 1 = flags (+ the value length that
  // follows them), 2 = value length after timestamps, 3 = stopped
  uint32_t R, rphase, rneed, rsl, rpl, rflags, ro, nwalk;
  int32_t fk;    // first key length for the prefix check (row.go:203-206), -1 before row 0 decodes
  uint32_t pl0;  // row 0's prefix-length field: block.go's FirstKey length when offsets[0] == 0
  // CodecLz4 (kLz4 instantiation only): the frame's one data block is payload bytes [s0, sn);
  // lph = what the next parse reads (0 a token, 1 a match, 2 nothing: the last literals are
  // out); mtok = the token's match nibble; hb = hand the block to the exact path
  uint32_t sn, lph, mtok, hb;
  // CodecLz4 content checksum: XXH32's four stripe accumulators over output chunks [0, xp)
  uint32_t xp, x0, x1, x2, x3;
};

struct Rsrc {
  __amdgpu_buffer_rsrc_t in, out, rows;
};

// CRC32 of the next committed input chunk (bytes outside the block zeroed).
// slicing-by-8 (SLATE_LPB_CRC8: 8 KiB of tables instead of 16, two dependent lookup rounds per chunk)
#ifndef SLATE_LPB_CRC8
#define SLATE_LPB_CRC8 1
#endif
constexpr uint32_t kLpbTabBytes = SLATE_LPB_CRC8 ? kTab16Bytes / 2 : kTab16Bytes;
__device__ __forceinline__ uint32_t crc_chunk8(const uint8_t* lds, const v4u& v) {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
  lut4<0, 7>(lds, v.x, a0, a1, a2, a3);
  lut4<0, 3>(lds, v.y, b0, b1, b2, b3);
  const uint32_t c = xor3(xor3(a0, a1, a2), xor3(a3, b0, b1), b2) ^ b3;
  lut4<0, 7>(lds, v.z ^ c, a0, a1, a2, a3);
  lut4<0, 3>(lds, v.w, b0, b1, b2, b3);
  return xor3(xor3(a0, a1, a2), xor3(a3, b0, b1), b2) ^ b3;
}

__device__ __forceinline__ void crc_chunk(Lane& L, const uint8_t* in, const uint32_t* tab, bool go) {
  const uint32_t k = L.crc_pos;
  v4u v = rd128(in + (k & (kNS - 1)) * 16, L.z);
  const bool partial = go && (k == 0 || int32_t(k) == L.crc_last);
  if (__builtin_amdgcn_ballot_w64(partial)) {  // wave-uniform branch: first/last chunks only
    const int32_t lo = int32_t(L.sh) - int32_t(16 * k), hi = int32_t(L.sh + L.clen) - int32_t(16 * k);
    v.x &= keep_mask(lo, hi, 0);
    v.y &= keep_mask(lo, hi, 1);
    v.z &= keep_mask(lo, hi, 2);
    v.w &= keep_mask(lo, hi, 3);
  }
  v.x ^= L.crc;
  const uint32_t c = SLATE_LPB_CRC8 ? crc_chunk8(reinterpret_cast<const uint8_t*>(tab), v)
                                    : crc_chunk0(reinterpret_cast<const uint8_t*>(tab), v);
  L.crc = go ? c : L.crc;
  L.crc_pos += go ? 1u : 0u;
}

// ring bytes [p, p+24)
struct W6 {
  uint32_t w[6];
};
__device__ __forceinline__ W6 ring_rd24(const uint8_t* ring, uint32_t p) {
  const uint32_t a = p & (kOR - 8);
  const v2u A = rd64(ring, a), B = rd64(ring, a + 8), C = rd64(ring, a + 16), D = rd64(ring, a + 24);
  const bool q = (p & 4) != 0;
  const uint32_t e[7] = {q ? A.y : A.x, q ? B.x : A.y, q ? B.y : B.x, q ? C.x : B.y,
                         q ? C.y : C.x, q ? D.x : C.y, q ? D.y : D.x};
  const uint32_t b = p & 3;
  W6 r;
#pragma unroll
  for (int k = 0; k < 6; k++) r.w[k] = alignb(e[k + 1], e[k], b);
  return r;
}

// Row walker, one action per call (row.go:191-261 field order), branch-free.  A row whose
// header, flags and value length lie in its first 24 bytes (suffix <= 7 bytes, no
// timestamps: every row of the bench's blocks) is decoded in one action; otherwise phase 0
// reads the key lengths, phase 1 the flags (+ the value length when there are no
// timestamps), phase 2 the value length after the timestamps.
// Returns true with `row`/`ridx` set when the action finished a row.
__device__ __forceinline__ bool walk_step(Lane& L, const uint8_t* ring, bool act, bool hp, v4u& row, uint32_t& ridx) {
  const uint32_t fp = L.R + 4 + L.rsl + 8;
  const bool p0 = L.rphase == 0, p1 = L.rphase == 1;
  const uint32_t rpos = p0 ? L.R : (p1 ? fp : L.R + L.ro);
  const bool in_hole = hp && rpos < L.hd + L.hl && rpos + 8 > L.hd;
  const bool wa = act & (L.rphase < 3) & (L.d >= L.rneed) & !in_hole;
  const bool lost = L.d - rpos > kReach;  // fell behind the ring: the exact fallback takes over
  const W6 q = ring_rd24(ring, rpos);
  // phase 0: prefix / suffix lengths, and the whole row when it fits the first 24 bytes
  const uint32_t pl0 = be16_of(q.w[0]), sl0 = be16_of(q.w[0] >> 16);
  const uint32_t f0 = 12 + sl0;  // flags byte (12..19 when sl0 <= 7)
  const bool hi0 = (f0 & 16) != 0;  // f0 in 16..19 (one-shot rows have f0 in 12..19)
  const uint32_t fw = hi0 ? q.w[4] : q.w[3], fw1 = hi0 ? q.w[5] : q.w[4];
  const uint32_t fl0 = (fw >> (8 * (f0 & 3))) & 0xff;
  const uint32_t vb = (f0 + 1) & 3;  // the value length is bytes f0+1 .. f0+4
  const uint32_t vl0 = __builtin_bswap32(vb == 0 ? fw1 : alignb(fw1, fw, vb));
  const bool tomb0 = (fl0 & 1) != 0;
  const uint32_t rlen0 = 4 + sl0 + 9 + (tomb0 ? 0u : 4u);
  const bool hole0 = hp && rpos < L.hd + L.hl && rpos + rlen0 > L.hd;
  const bool one = p0 & (sl0 <= 7) & !(fl0 & 6) & (L.d >= L.R + rlen0) & !hole0;
  // phase 1: flags, and the value length right after them when there are no timestamps
  const uint32_t fl1 = q.w[0] & 0xff;
  const uint32_t ts = ((fl1 & 2) ? 8u : 0u) + ((fl1 & 4) ? 8u : 0u);
  const uint32_t ro1 = 4 + L.rsl + 9 + ts;
  const bool tomb = (fl1 & 1) != 0;
  const bool done1 = tomb | (ts == 0);
  const uint32_t vl1 = tomb ? 0u : __builtin_bswap32((q.w[0] >> 8) | (q.w[1] << 24));
  // phase 2: value length after the timestamps
  const uint32_t vl2 = __builtin_bswap32(q.w[0]);
  const bool done = wa & !lost & ((p0 & one) | (p1 & done1) | (L.rphase == 2));
  const uint32_t vl_p12 = p1 ? vl1 : vl2;
  const uint32_t vl = p0 ? (tomb0 ? 0u : vl0) : vl_p12;
  const uint32_t fl_p12 = p1 ? fl1 : L.rflags;
  const uint32_t flags = p0 ? fl0 : fl_p12;
  const uint32_t ro = p1 ? ro1 : L.ro;
  const uint32_t rlen_p12 = (p1 & tomb) ? ro1 : ro + 4;
  const uint32_t rlen = p0 ? rlen0 : rlen_p12;
  const uint32_t rpl = p0 ? pl0 : L.rpl, rsl = p0 ? sl0 : L.rsl;
  // row.go:203-206: a prefix longer than the block's first key fails the row, which then
  // keeps only its key lengths; row 0 is decoded against an empty first key
  const bool pfail = rpl > uint32_t(max(L.fk, 0));
  row = pack_row(L.R, rpl, rsl, pfail ? 0u : vl, pfail ? 0u : flags & 7, pfail ? 0u : rlen - 4 - rsl,
                 pfail ? uint32_t(SLATE_E_ROW_PREFIX) : uint32_t(SLATE_OK));
  ridx = L.nwalk;
  L.fk = (done & (L.nwalk == 0) & !pfail) ? int32_t(rsl) : L.fk;
  const bool emit = done & (L.nwalk < L.rcap);
  const uint64_t next = uint64_t(L.R) + rlen + vl;
  // state transitions
  const bool to1 = wa & !lost & p0 & !one;
  const bool to2 = wa & !lost & p1 & !done1;
  L.rpl = to1 ? pl0 : L.rpl;
  L.pl0 = (wa & !lost & p0 & (L.R == 0)) ? pl0 : L.pl0;
  L.rsl = to1 ? sl0 : L.rsl;
  L.rflags = (wa & p1) ? fl1 : L.rflags;
  L.ro = (wa & p1) ? ro1 : L.ro;
  L.nwalk += done ? 1u : 0u;
  const bool stop = (wa & lost) | (done & (next > L.dn));
  const bool adv = done & (next <= L.dn);
  L.R = adv ? uint32_t(next) : L.R;
  // priority stop > adv > to1 > to2, as plain selects (nested ternaries became branches);
  // phase 0 waits for 24 bytes (or the end of the block) so that it can finish the row
  uint32_t rph = L.rphase, rn = L.rneed;
  rph = to2 ? 2u : rph;
  rn = to2 ? L.R + ro1 + 4 : rn;
  rph = to1 ? 1u : rph;
  rn = to1 ? L.R + 4 + sl0 + 13 : rn;
  rph = adv ? 0u : rph;
  rn = adv ? min(uint32_t(next) + 24, L.dn) : rn;
  rph = stop ? 3u : rph;
  rn = stop ? 0xFFFFFFFFu : rn;
  L.rphase = rph;
  L.rneed = rn;
  return emit;
}

// The walker's common case alone (phase 0: a row whose header, flags and value length lie in its
// first 24 bytes, one action), for lanes in phase 0; walk() runs the general walk_step only when
// some lane is in phase 1 or 2 (a suffix over 7 bytes, timestamps).  Same transitions as
// walk_step's phase 0.
__device__ __forceinline__ bool walk_fast(Lane& L, const uint8_t* ring, bool act, bool hp, v4u& row, uint32_t& ridx) {
  const uint32_t rpos = L.R;
  const bool in_hole = hp & (rpos < L.hd + L.hl) & (rpos + 8 > L.hd);
  const bool wa = act & (L.rphase == 0) & (L.d >= L.rneed) & !in_hole;
  const bool lost = L.d - rpos > kReach;  // fell behind the ring: the exact fallback takes over
  const W6 q = ring_rd24(ring, rpos);
  const uint32_t pl0 = be16_of(q.w[0]), sl0 = be16_of(q.w[0] >> 16);
  const uint32_t f0 = 12 + sl0;
  const bool hi0 = (f0 & 16) != 0;
  const uint32_t fw = hi0 ? q.w[4] : q.w[3], fw1 = hi0 ? q.w[5] : q.w[4];
  const uint32_t fl0 = (fw >> (8 * (f0 & 3))) & 0xff;
  const uint32_t vb = (f0 + 1) & 3;
  const uint32_t fa = alignb(fw1, fw, vb);
  const uint32_t vl0 = __builtin_bswap32(vb == 0 ? fw1 : fa);
  const bool tomb0 = (fl0 & 1) != 0;
  const uint32_t rlen0 = 4 + sl0 + 9 + (tomb0 ? 0u : 4u);
  const bool hole0 = hp & (rpos < L.hd + L.hl) & (rpos + rlen0 > L.hd);
  const bool one = (sl0 <= 7) & !(fl0 & 6) & (L.d >= rpos + rlen0) & !hole0;
  const bool done = wa & !lost & one;
  const uint32_t vl = tomb0 ? 0u : vl0;
  const bool pfail = pl0 > uint32_t(max(L.fk, 0));
  row = pack_row(rpos, pl0, sl0, pfail ? 0u : vl, pfail ? 0u : fl0 & 7, pfail ? 0u : rlen0 - 4 - sl0,
                 pfail ? uint32_t(SLATE_E_ROW_PREFIX) : uint32_t(SLATE_OK));
  ridx = L.nwalk;
  L.fk = (done & (L.nwalk == 0) & !pfail) ? int32_t(sl0) : L.fk;
  const bool emit = done & (L.nwalk < L.rcap);
  const uint32_t next = rpos + rlen0 + vl;  // < 2^32: vl0 is checked against dn below first
  const bool vbig = vl > L.dn;
  const bool to1 = wa & !lost & !one;
  L.rpl = to1 ? pl0 : L.rpl;
  L.pl0 = (wa & !lost & (rpos == 0)) ? pl0 : L.pl0;
  L.rsl = to1 ? sl0 : L.rsl;
  L.nwalk += done ? 1u : 0u;
  const bool stop = (wa & lost) | (done & (vbig | (next > L.dn)));
  const bool adv = done & !vbig & (next <= L.dn);
  L.R = adv ? next : L.R;
  uint32_t rph = L.rphase, rn = L.rneed;
  const uint32_t rn1 = rpos + 4 + sl0 + 13, rna = min(next + 24, L.dn);
  rph = to1 ? 1u : rph;
  rn = to1 ? rn1 : rn;
  rph = adv ? 0u : rph;
  rn = adv ? rna : rn;
  rph = stop ? 3u : rph;
  rn = stop ? 0xFFFFFFFFu : rn;
  L.rphase = rph;
  L.rneed = rn;
  return emit;
}

// One walker call: the fast phase-0 action, and the general one for lanes in phase 1 or 2.
__device__ __forceinline__ bool walk(Lane& L, const uint8_t* ring, bool act, v4u& row, uint32_t& ridx) {
  const bool slow = act & ((L.rphase == 1) | (L.rphase == 2));
  const bool slow_go = slow & (L.d >= L.rneed);
  const bool hp = mbit(L.mhp);
  bool emit = walk_fast(L, ring, act, hp, row, ridx);
#ifdef SLATE_COUNT_FAST_ONLY  // static instruction counts of the common path (tools/loop_mix.py)
  if (false) {
#else
  if (__builtin_amdgcn_ballot_w64(slow_go)) {
#endif
    v4u row2;
    uint32_t ridx2;
    const bool e2 = walk_step(L, ring, slow, hp, row2, ridx2);
    row = slow ? row2 : row;
    ridx = slow ? ridx2 : ridx;
    emit = slow ? e2 : emit;
  }
  return emit;
}

// Start of an iteration: (1) the chunks loaded one iteration ago go into their blocks'
// input rings (the loading lane writes them: transposed layout); (2) every block asks for
// up to four more chunks (ring room and payload end permitting); (3) four transposed
// loads fetch them: in load j, lanes 4i..4i+3 read chunks c_issue..c_issue+3 of block 16j+i.
__device__ __forceinline__ void commit_one(uint8_t* ins, uint32_t slot, const v4u& v, uint32_t z) {
  if (slot != 0xFFFFFFFFu) wr128(ins + slot, v, z);  // slot: LDS offset of the ring slot
}

__device__ __forceinline__ void load_one(uint32_t j, uint32_t lane, uint32_t wave_lane0, uint32_t info,
                                         uint32_t rel, const Rsrc& R, v4u& P, uint32_t& slot) {
  const uint32_t o = 16 * j + (lane >> 2), c = lane & 3;
  const uint32_t info_o = __shfl(info, int(o), 64);
  const uint32_t rel_o = __shfl(rel, int(o), 64);
  const uint32_t ci = (info_o >> 3) + c;
  const bool want = c < (info_o & 7);
  P = __builtin_amdgcn_raw_buffer_load_b128(R.in, want ? rel_o + 16 * ci : kOOB, 0, 0);
  slot = want ? (wave_lane0 + o) * kInStride + (ci & (kNS - 1)) * 16 : 0xFFFFFFFFu;
}

// The decode kernel's refill with its loop invariants hoisted: rel_j = the round's input offset of
// the block lane `lane` serves in load j (shuffled once per round), slot_lane = that block's input
// ring in load 0 (LDS offset, fixed for the kernel; load j's is 16 j records further, an immediate);
// S_j = the ring slot's byte offset, or ~0 when the lane loads nothing.
template <uint32_t kJ>
__device__ __forceinline__ void commit_j(uint8_t* ins, uint32_t slot_lane, uint32_t S, const v4u& v, uint32_t z) {
  if (S != 0xFFFFFFFFu) wr128(ins + slot_lane + kJ * 16 * kInStride + S, v, z);
}
template <uint32_t kJ>
__device__ __forceinline__ void load_j(uint32_t lane, uint32_t info, uint32_t rel_j, const Rsrc& R, v4u& P,
                                       uint32_t& S) {
  const uint32_t c = lane & 3;
  const uint32_t info_o = __shfl(info, int(16 * kJ + (lane >> 2)), 64);
  const uint32_t ci = (info_o >> 3) + c;
  const bool want = c < (info_o & 7);
  P = __builtin_amdgcn_raw_buffer_load_b128(R.in, want ? rel_j + 16 * ci : kOOB, 0, kInCpol);
  S = want ? (ci & (kNS - 1)) * 16 : 0xFFFFFFFFu;
}

// Start of an iteration, part 2: how many chunks this block asks for (ring room and
// payload end permitting), then four transposed loads fetch them for the whole wave.
// A block asks only for a whole 64-byte segment of the payload's address (its first and last
// segments excepted): a refill is one run that never straddles a cache line.  Asking for whatever
// was free gave runs of 1-4 chunks at any alignment -- the same bytes in ~twice the runs, and the
// address unit's time goes by runs and lines (round 6, same-box A/Bs on profiling variants, 1 M
// blocks: REFILL_MIN = 1..4 4.230 / 4.150 / 4.138 / 4.130 ms; aligned segments 4.053 ms,
// profiles/round6/ab/).  SLATE_LPB_REFILL_ALIGN=0 restores the unaligned minimum-run rule.
#ifndef SLATE_LPB_REFILL_MIN
#define SLATE_LPB_REFILL_MIN 4
#endif
#ifndef SLATE_LPB_REFILL_ALIGN
#define SLATE_LPB_REFILL_ALIGN 1
#endif
__device__ __forceinline__ uint32_t refill_count(bool act, uint32_t lo_chunk, uint32_t c_issue, uint32_t last_chunk,
                                                 uint32_t phase) {
  const uint32_t room = lo_chunk + kNS - c_issue;
  const uint32_t left = last_chunk + 1 - c_issue;
#if SLATE_LPB_REFILL_ALIGN
  // runs end on 64-byte boundaries of the payload's address (phase = the first chunk's slot in its
  // 64-byte line), so no run straddles a cache line
  const uint32_t seg = min(4u - ((phase + c_issue) & 3u), left);
  return (act && room >= seg) ? seg : 0u;
#else
  const uint32_t n = min(min(room, left), 4u);
  return (act && (n >= SLATE_LPB_REFILL_MIN || n == left)) ? n : 0u;
#endif
}

// Start of an iteration, after the refill: the hole source loaded at the end of the previous
// iteration (Q) fills the pending hole -- a read-modify-write of the five ring dwords around
// [hd, hd+hl): the bytes after the hole were decoded meanwhile.
__device__ __forceinline__ void absorb_hole(Lane& L, const v4u& Q, uint8_t* ring) {
  if (L.mhp) {
    const uint32_t hd = L.hd, b = hd & 3, a4 = hd & ~3u, a = hd & ~7u;
    const v2u A = rd64(ring, a), B = rd64(ring, a + 8), C = rd64(ring, a + 16);
    const bool q = (hd & 4) != 0;
    Win5 o;
    o.y0 = q ? A.y : A.x;
    o.y1 = q ? B.x : A.y;
    o.y2 = q ? B.y : B.x;
    o.y3 = q ? C.x : B.y;
    o.y4 = q ? C.y : C.x;
    const Win5 y = shift_in(Q, o.y0, b);
    // window bytes [b, e) are the hole's: dword j keeps bytes below e - 4j (a 64-bit shift
    // gives 0 for a count of 32), dword 0 also only from b on
    const int32_t e8 = int32_t(8 * (b + L.hl));
    auto upto = [&](int32_t j) -> uint32_t {
      const uint32_t sh = uint32_t(min(max(32 * (j + 1) - e8, 0), 32));
      return uint32_t(0xFFFFFFFFull >> sh);
    };
    const uint32_t m0 = upto(0) & (0xFFFFFFFFu << (8 * b)), m1 = upto(1), m2 = upto(2), m3 = upto(3), m4 = upto(4);
    Win5 n;
    n.y0 = (y.y0 & m0) | (o.y0 & ~m0);
    n.y1 = (y.y1 & m1) | (o.y1 & ~m1);
    n.y2 = (y.y2 & m2) | (o.y2 & ~m2);
    n.y3 = (y.y3 & m3) | (o.y3 & ~m3);
    n.y4 = (y.y4 & m4) | (o.y4 & ~m4);
    if (mbit(L.mhp)) store_win(ring, a4, n);
    // the register copy of d's dword follows a store into that dword
    const uint32_t jd = (((L.d & ~3u) - a4) & (kOR - 1)) >> 2;
    L.T = msel(L.mhp & bal(jd <= 4), pick5(n, jd), L.T);
  }
  L.mhp = 0;
}

// Appends item to list (wave-aggregated: one atomic per wave); every lane of the wave calls it.
__device__ __forceinline__ void lpb_list_append(bool want, uint32_t item, uint32_t* list, uint32_t* count) {
  const uint64_t m = __ballot(want);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == uint32_t(__builtin_ctzll(m))) base = atomicAdd(count, uint32_t(__builtin_popcountll(m)));
  base = __shfl(base, __builtin_ctzll(m), 64);
  if (want) list[base + uint32_t(__builtin_popcountll(m & ((uint64_t(1) << lane) - 1)))] = item;
}

// CodecLz4 content checksum: one XXH32 stripe (output chunk xp, still in the ring) when go.
__device__ __forceinline__ void xxh_absorb(Lane& L, const uint8_t* ring, bool go) {
  const v4u v = rd128(ring + ((L.xp * 16) & (kOR - 1)), L.z);
  L.x0 = go ? xrotl(L.x0 + v.x * kXP2, 13) * kXP1 : L.x0;
  L.x1 = go ? xrotl(L.x1 + v.y * kXP2, 13) * kXP1 : L.x1;
  L.x2 = go ? xrotl(L.x2 + v.z * kXP2, 13) * kXP1 : L.x2;
  L.x3 = go ? xrotl(L.x3 + v.w * kXP2, 13) * kXP1 : L.x3;
  L.xp += go ? 1u : 0u;
}

// CodecLz4: the next sequence half of the frame's data block (LZ4 block format: token,
// literal length extension bytes, literals, little-endian offset, match length extension
// bytes), read from the input ring like a Snappy tag: a token starts a literal run, the
// offset after the literals starts a match.  The checks are the exact path's
// (decode.hip wave_lz4_decode) for one independent block; a run of extension bytes
// longer than the 8-byte window, or any failed check, hands the block to the exact path
// (L.hb), which then decodes and reports it.  A token without literals is parsed with its match.
__device__ __forceinline__ void lz4_parse(Lane& L, bool act, const uint8_t* in, int32_t avail, uint32_t lim_d) {
  const bool need = act && !mbit(L.mdd) && L.rem == 0;
  const bool fin = need && L.lph == 2;
  const bool can = need & (L.lph < 2) & (avail >= int32_t(min(L.s + 8, L.clen))) & (L.d <= lim_d);
  const v2u w = ring_rd8(in, L.sh + L.s, kIR - 8);
  const uint64_t w64 = (uint64_t(w.y) << 32) | w.x;
  const uint32_t tok = w.x & 0xff;
  const bool tokp = L.lph == 0;
  // a token without literals (half of V-half's sequences) is parsed together with its match, so
  // it costs no step of its own; unless it ends the block
  const bool z0 = tokp && (tok >> 4) == 0 && L.s + 1 < L.sn;
  const bool mph = !tokp || z0;           // this step starts a match
  const uint64_t wm = z0 ? w64 >> 8 : w64;  // the window from the match's offset
  const uint32_t n4 = mph ? (tokp ? tok & 15 : L.mtok) : tok >> 4;  // the length nibble
  // extension bytes: 7 after a token, 6 after an offset (5 after a literal-less token's offset);
  // k = how many 255s lead them
  const uint64_t ext = mph ? wm >> 16 : w64 >> 8;
  const uint64_t nz = ~ext & (mph ? (z0 ? 0x000000FFFFFFFFFFull : 0x0000FFFFFFFFFFFFull) : 0x00FFFFFFFFFFFFFFull);
  const uint32_t k = uint32_t(__builtin_ctzll(nz | (uint64_t(1) << 63))) >> 3;
  const uint32_t e = uint32_t(ext >> (8 * k)) & 0xff;
  const bool lng = n4 == 15;
  const uint32_t len = lng ? 15 + 255 * k + e : n4;
  const uint32_t ms = L.s + (z0 ? 1u : 0u);  // where the match's offset starts
  const uint32_t s1 = (mph ? ms + 2 : L.s + 1) + (lng ? k + 1 : 0u);
  const bool ext_bad = lng && nz == 0;  // the run goes on past the window
  const uint32_t room = L.dn - L.d;  // min(plan capacity, block maximum) left; the exact decoder's bounds
  // token: literals [s1, s1 + len); the last sequence's literals end the block exactly
  const uint32_t lit_end = s1 + len;
  const bool bad_tok = lit_end > L.sn || len > room;
  const bool last = lit_end == L.sn;
  // match: offset, then the length (+4); a match may not end the block (a token must follow)
  const uint32_t off = uint32_t(wm) & 0xffff, ml = len + 4;
  const bool bad_m = ms + 2 > L.sn || s1 >= L.sn || off == 0 || off > L.d || ml > room;
  const bool bad = ext_bad || (mph ? bad_m : bad_tok);
  const bool ok = can && !bad;
  L.hb |= (can && bad) ? 1u : 0u;
  L.mdd |= bal(fin || (can && bad));
  const uint64_t okm = bal(ok);
  L.mlit = (okm & bal(!mph)) | (~okm & L.mlit);
  L.rem = ok ? (mph ? ml : len) : L.rem;
  L.src = ok ? (mph ? L.d - off : L.sh + s1) : L.src;
  L.eff = ok ? (mph ? off : kStep) : L.eff;
  L.mfar = (okm & bal(mph && off > kReach)) | (~okm & L.mfar);
  L.s = ok ? (mph ? s1 : lit_end) : L.s;
  L.mtok = (ok && !mph) ? (tok & 15) : L.mtok;
  L.lph = ok ? (mph ? 0u : (last ? 2u : 1u)) : L.lph;
  // the decoded length is known once the last literals are parsed
  const bool fix = ok && !mph && last;
  L.dn = fix ? L.d + len : L.dn;
  L.rneed = fix ? min(L.rneed, L.d + len) : L.rneed;
}

// golang/snappy's tag parse (decode_other.go:19-110) at payload position L.s, in 32-bit
// arithmetic: a literal length that does not fit saturates, and any length beyond the output or
// the payload fails the same checks.
__device__ __forceinline__ void snappy_parse(Lane& L, bool act, const uint8_t* in, int32_t avail, uint32_t lim_d) {
  // written with & | and selects between computed values: short-circuit operators and
  // conditional expressions became divergent branches
  const uint32_t sn = L.clen;
  const bool need = act & !mbit(L.mdd) & (L.rem == 0);
  const bool fin = need & (L.s >= sn);
  // throttle (a hole delays the flush): after any step d - 16*fl <= 96, so the ring keeps every
  // unflushed byte and every far source (offset > kReach) is already flushed
  const uint32_t s5 = min(L.s + 5, sn);
  const bool can = need & (L.s < sn) & (avail >= int32_t(s5)) & (L.d <= lim_d);
  const v2u w = ring_rd8(in, L.sh + L.s, kIR - 8);
  const uint32_t c = w.x & 0xff, t = c & 3, xl = c >> 2;
  const uint32_t b14 = alignb(w.y, w.x, 1);  // bytes s+1 .. s+4
  const uint32_t xl59 = xl - 59;
  const uint32_t nb = xl >= 60 ? xl59 : 0u;  // literal length bytes (1..4)
  const uint32_t ext = b14 & (0xFFFFFFFFu >> ((32 - 8 * nb) & 31));
  const uint32_t lm1 = nb ? ext : xl;
  const uint32_t lm1p = lm1 + 1;
  const uint32_t lit_len = lm1p == 0 ? lm1 : lm1p;  // saturating: fails the bounds below
  const bool tl = t == 0, t1 = t == 1;
  const uint32_t l1 = 4 + (xl & 7), l23 = xl + 1;
  const uint32_t cp_len = t1 ? l1 : l23;
  const uint32_t off1 = ((c >> 5) << 8) | (b14 & 0xff), o16 = b14 & 0xffff;
  const uint32_t off23 = (t & 1) ? b14 : o16;
  const uint32_t cp_off = t1 ? off1 : off23;
  const uint32_t hl_cp = (0x5320u >> (4 * t)) & 15, hl_lit = 1 + nb;  // header bytes: 2, 3, 5 for copies
  const uint32_t hl = tl ? hl_lit : hl_cp;
  const uint32_t len = tl ? lit_len : cp_len;
  const uint32_t s1 = L.s + hl;
  const uint32_t room = L.dn - L.d, left = sn - s1;
  const bool bad_lit = len > left, bad_cp = (cp_off == 0) | (cp_off > L.d);
  const bool bad_t = tl ? bad_lit : bad_cp;
  const bool bad = (s1 > sn) | (len > room) | bad_t;
  const bool ok = can & !bad, fail = can & bad;
  L.merr |= bal(fail);
  L.mdd |= bal(fin | fail);
  const uint32_t src_lit = L.sh + s1, src_cp = L.d - cp_off, s_lit = s1 + len;
  const uint32_t src_new = tl ? src_lit : src_cp, eff_new = tl ? kStep : cp_off, s_new = tl ? s_lit : s1;
  const bool far_new = !tl & (cp_off > kReach);
  const uint64_t okm = bal(ok);
  L.mlit = (okm & bal(tl)) | (~okm & L.mlit);
  L.mfar = (okm & bal(far_new)) | (~okm & L.mfar);
  L.rem = vsel(ok, len, L.rem);
  L.src = vsel(ok, src_new, L.src);
  L.eff = vsel(ok, eff_new, L.eff);
  L.s = vsel(ok, s_new, L.s);
}

// The tag table (SLATE_LPB_TPARSE): per golang/snappy tag byte c (decode_other.go:19-110), the mask
// of the header bytes after c that carry a length (long literals) or an offset (copies), and packed:
// bit 31 literal, bits 24..26 the header length, bits 16..23 the length base (short literal xl + 1,
// long literal 1, copy-1 4 + (xl & 7), copy-2/4 xl + 1), bits 8..10 copy-1's offset high bits.  One
// ds_read_b64 per step replaces the tag's arithmetic.  2 KiB after the CRC tables.
#ifndef SLATE_LPB_TPARSE
#define SLATE_LPB_TPARSE 1
#endif
constexpr uint32_t kTagTabOff = kLpbTabBytes;
constexpr uint32_t kTagTabBytes = SLATE_LPB_TPARSE ? 2048u : 0u;
__device__ __forceinline__ v2u tag_entry(uint32_t c) {
  const uint32_t t = c & 3, xl = c >> 2;
  uint32_t mask, hl, lb, ohi = 0, lit = 0;
  if (t == 0) {
    lit = 1;
    const uint32_t nb = xl >= 60 ? xl - 59 : 0u;
    mask = nb ? 0xFFFFFFFFu >> (32 - 8 * nb) : 0u;
    hl = 1 + nb;
    lb = nb ? 1u : xl + 1;
  } else if (t == 1) {
    mask = 0xffu;
    hl = 2;
    lb = 4 + (xl & 7);
    ohi = (c >> 5) << 8;
  } else {
    mask = t == 2 ? 0xffffu : 0xFFFFFFFFu;
    hl = t == 2 ? 3u : 5u;
    lb = xl + 1;
  }
  v2u e;
  e.x = mask;
  e.y = (lit << 31) | (hl << 24) | (lb << 16) | ohi;
  return e;
}
__device__ __forceinline__ uint32_t rd32a(const uint8_t* ring, uint32_t a) {  // a: 4-byte aligned ring offset
  return *reinterpret_cast<const uint32_t*>(ring + a);
}
// snappy_parse's results by the tag table: the window is the two aligned dwords holding bytes s .. s+4
__device__ __forceinline__ void snappy_parse_t(Lane& L, uint64_t mact, const uint8_t* in, int32_t avail,
                                               uint32_t lim_d) {
  const uint32_t sn = L.clen;
  const uint64_t need = mact & ~L.mdd & bal(L.rem == 0);
  const uint64_t fin = need & bal(L.s >= sn);
  const uint32_t s5 = min(L.s + 5, sn);
  const uint64_t can = need & bal(L.s < sn) & bal(avail >= int32_t(s5)) & bal(L.d <= lim_d);
  // bytes s .. s+4 lie in the two aligned dwords from (sh + s) & ~3: shifted down as one 64-bit value
  const uint32_t p = L.sh + L.s;
  const uint32_t d0 = rd32a(in, p & (kIR - 4)), d1 = rd32a(in, (p + 4) & (kIR - 4));
  const uint64_t w = ((uint64_t(d1) << 32) | d0) >> ((p << 3) & 24);
  const uint32_t c = uint32_t(w) & 0xff;
  const uint32_t b14 = uint32_t(w >> 8);  // bytes s+1 .. s+4
  const v2u e = *(const __attribute__((address_space(3))) v2u*)(kTagTabOff + 8 * c);
  const uint32_t payload = b14 & e.x;
  const uint64_t tl = bal(int32_t(e.y) < 0);
  const uint32_t lb = (e.y >> 16) & 0xff, hl = (e.y >> 24) & 7;
  const uint32_t len = __builtin_elementwise_add_sat(lb, msel(tl, payload, 0u));  // a long literal's length saturates
  const uint32_t cp_off = (e.y & 0x700u) | payload;
  const uint32_t s1 = L.s + hl;
  const uint32_t room = L.dn - L.d, left = sn - s1;
  const uint64_t bad = ugt(s1, sn) | bal(len > room) | (tl & bal(len > left)) | (~tl & (bal(cp_off == 0) | ugt(cp_off, L.d)));
  const uint64_t ok = can & ~bad, fail = can & bad;
  L.merr |= fail;
  L.mdd |= fin | fail;
  const uint32_t src_new = msel(tl, L.sh + s1, L.d - cp_off), eff_new = msel(tl, kStep, cp_off);
  const uint32_t s_new = msel(tl, s1 + len, s1);
  L.mlit = (ok & tl) | (~ok & L.mlit);
  L.mfar = (ok & ~tl & bal(cp_off > kReach)) | (~ok & L.mfar);
  L.rem = msel(ok, len, L.rem);
  L.src = msel(ok, src_new, L.src);
  L.eff = msel(ok, eff_new, L.eff);
  L.s = msel(ok, s_new, L.s);
}

// One step: CRC (two of four steps), parse, a hole or a 16-byte move, and the row walker
// (the other two steps).
// kSlot: 0 and 2 absorb a CRC chunk; 1 and (when needed) 3 run the walker
template <int kSlot, bool kLz4>
__device__ __forceinline__ void lane_step(Lane& L, bool act, uint64_t mact, uint8_t* ring, uint8_t* in,
                                          const uint32_t* tab, const Rsrc& R, uint32_t lim_d, uint32_t cend,
                                          uint32_t dbg) {
#ifdef SLATE_FORCE_DBG  // static instruction-count analysis only (tools/loop_mix.py)
  dbg = SLATE_FORCE_DBG;
#endif
  // ---- CRC32 of one committed chunk (the two steps without the walker)
  LPB_MARK(crc);
  if (kSlot == 0 || kSlot == 2) {
    const bool go = L.crc_pos < L.c_commit && int32_t(L.crc_pos) <= L.crc_last;
    if (dbg & 64) L.crc_pos += go ? 1u : 0u;  // ablation: skip the lookups, keep the ring moving
    else crc_chunk(L, in, tab, go);
  }
  const int32_t avail = int32_t(cend) - int32_t(L.sh);  // committed payload bytes [0, avail)
  LPB_MARK(parse);
  if constexpr (kLz4) lz4_parse(L, act, in, avail, lim_d);
  else if constexpr (SLATE_LPB_TPARSE) snappy_parse_t(L, mact, in, avail, lim_d);
  else snappy_parse(L, act, in, avail, lim_d);
  LPB_MARK(hole);
  // ---- a far copy (offset > kReach: its source left the ring and is flushed) goes on as holes
  // of up to 16 bytes, one pending per lane: reserve the bytes, load the source, go on decoding
  {
    // (a step before the merge of the previous iteration's hole source makes no hole: the merge
    // would take its pending flag for the old one)
    const uint64_t mk = (kSlot >= 1 ? mact : 0) & ~L.mdd & L.mfar & ~L.mhp & bal(L.rem != 0) & bal(L.d <= lim_d);
    const uint32_t n = min(L.rem, 16u);
    L.hd = msel(mk, L.d, L.hd);
    L.hl = msel(mk, n, L.hl);
    L.qoff = msel(mk, L.out_rel + L.src, L.qoff);
    L.mhp |= mk;
    const uint32_t nn = msel(mk, n, 0u);
    L.d += nn;
    L.rem -= nn;
    L.src += nn;
  }
  // ---- move up to 16 bytes of a literal or a near copy into the output ring
  LPB_MARK(move);
  {
    const uint64_t cp = mact & ~L.mdd & ~L.mfar & bal(L.rem != 0) & bal(L.d <= lim_d);
    const uint32_t k16 = min(L.rem, kStep);
    const uint32_t k_lit = min(k16, sub_sat(cend, L.src)), k_near = min(k16, L.eff);
    uint32_t k = msel(L.mlit, k_lit, k_near);
    // a ring copy stops short of the pending hole's bytes
    const uint32_t k_hole = sub_sat(L.hd, L.src);
    const uint64_t cut = ~L.mlit & L.mhp & bal(L.src < L.hd + L.hl) & bal(L.src + k > L.hd);
    k = msel(cut, k_hole, k);
    k = msel(cp, k, 0u);
    // bytes from d on are not yet output: storing them when k == 0 is harmless; the first
    // dword keeps the bytes below d (L.T)
    const uint32_t b = L.d & 3;
    const uint32_t m8 = kOR == kIR ? kOR - 8 : msel(L.mlit, kIR - 8, kOR - 8);
    {
      // the source ring: the input ring for a literal, the output ring for a copy (LDS offsets)
      extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
      const uint32_t srb = msel(L.mlit, uint32_t(in - smem), uint32_t(ring - smem));
      const v4u v = ring_rd16(smem + srb, L.src, m8);
      const Win5 y = shift_in(v, L.T, b);
      store_win(ring, L.d & ~3u, y);
      L.T = pick5(y, (b + k) >> 2);
    }
    L.d += k;
    L.rem -= k;
    // periodic output: once a whole period was copied, the pattern can be read twice as far back
    const uint64_t step_cp = ~L.mlit & bal(k != 0) & bal(k == L.eff) & bal(L.eff < kStep);
    const uint32_t eff2 = msel(step_cp, 2 * L.eff, L.eff);
    L.src = msel(L.mlit, L.src + k, L.d - eff2);
    L.eff = eff2;
  }
  LPB_MARK(walk);
  // ---- the walker: every iteration once, and a second time only when some lane's walker has
  // fallen more than 64 bytes behind (rows shorter than the iteration's output)
  if (kSlot == 1 ||
      (kSlot == 3 && __builtin_amdgcn_ballot_w64(act & (L.rphase < 3) & (L.d >= L.rneed) & (L.d - L.R > kWalkLag)))) {
    v4u row;
    uint32_t ridx;
    const bool have_row = walk(L, ring, act && !(dbg & 128), row, ridx);
    const uint32_t off = (have_row && !(dbg & 16384)) ? L.rows_rel + 16 * ridx : kOOB;
    __builtin_amdgcn_raw_buffer_store_b128(row, R.rows, off, 0, kRowCpol);
  }
}

// End of a four-step iteration: every completed aligned 16-byte output chunk (at most four:
// a step adds at most 16 bytes; the ring keeps them, since unflushed bytes stay within 79 of
// d and the ring holds 112) and the rows the walker finished, as always-issued stores.
// The chunks are written transposed: in store j, lanes 4i..4i+3 write chunks 0..3 of the
// block of lane 16j+i, so every store instruction writes 16 runs of 64 contiguous bytes
// instead of 64 scattered 16-byte pieces (tools/scatter_probe.hip: ~3.5x cheaper).
// The same for the output: until a block's decode is done its flush run ends at the last 64-byte
// boundary of the output's address it reaches, so the stores are whole 64-byte segments (round 6,
// same-box A/B with aligned refills: 4.053 ms -> 3.790 ms at 4-chunk segments, 3.840 ms at 8;
// profiles/round6/ab/).  The throttle (lim_d) holds the ring's bound whatever the flush keeps back.
#ifndef SLATE_LPB_FLUSH_SEG
#define SLATE_LPB_FLUSH_SEG 4
#endif
__device__ __forceinline__ void flush_iteration(Lane& L, bool act, uint8_t* outs, uint32_t lane, const Rsrc& R,
                                                uint32_t dbg, uint32_t part, uint32_t flush_lane, uint32_t ophase) {
  const bool mine = kFlushParts == 1 || (lane / kFlushBlocks) == part;
  uint32_t done = (act && mine) ? min(L.d >> 4, msel(L.mhp, L.hd >> 4, 0xFFFFFFFFu)) - L.fl : 0u;
#if SLATE_LPB_FLUSH_SEG > 1
  // until the block's decode is done, a run stops at the last SLATE_LPB_FLUSH_SEG-chunk boundary
  // of the output's address it reaches (the chunks after it wait for the next flush)
  {
    const uint32_t n = min(done, kRun), keep = (ophase + L.fl + n) & (SLATE_LPB_FLUSH_SEG - 1);
    done = msel(L.mdd, done, n > keep ? n - keep : 0u);
  }
#else
  (void)ophase;
#endif
  const uint32_t base = L.out_rel + 16 * L.fl;       // where this lane's next chunk goes
  const uint32_t info = (done << 7) | ((L.fl * 16) & (kOR - 1)) >> 4;  // count | ring slot of fl
  // the served block's ring: flush_lane (the kernel's constant for part 0, store 0) + the part's and
  // the store's record offsets (the latter an immediate)
  const uint8_t* ring_p = outs + flush_lane + part * (kFlushBlocks * kOutStride);
#pragma unroll
  for (uint32_t j = 0; j < kFlushStores; j++) {
    const uint32_t o = part * kFlushBlocks + (64 / kRun) * j + lane / kRun, c = lane % kRun;
    const uint32_t info_o = __shfl(info, int(o), 64);
    const uint32_t base_o = __shfl(base, int(o), 64);
    const uint8_t* ring_o = ring_p + (64 / kRun) * j * kOutStride;
    const v4u v = rd128(ring_o + ((((info_o & 127) + c) * 16) & (kOR - 1)), L.z);
    __builtin_amdgcn_raw_buffer_store_b128(v, R.out, (c < (info_o >> 7) && !(dbg & 1024)) ? base_o + 16 * c : kOOB, 0,
                                           kOutCpol);
  }
  L.fl += min(done, kRun);
}

}  // namespace

// The LZ4 frame descriptor check (HC = second byte of XXH32(FLG .. DictID), seed 0) for the two
// descriptor lengths the fast path takes: 2 bytes (FLG, BD) or 10 (+ content size).
__device__ __forceinline__ uint32_t lz4_xxh_avalanche(uint32_t h) {
  h ^= h >> 15;
  h *= kXP2;
  h ^= h >> 13;
  h *= kXP3;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t lz4_xxh_byte(uint32_t h, uint32_t b) { return xrotl(h + b * kXP5, 11) * kXP1; }
__device__ __forceinline__ uint32_t lz4_xxh_word(uint32_t h, uint32_t w) { return xrotl(h + w * kXP3, 17) * kXP4; }

// One LZ4 frame per block on the fast path: magic, FLG/BD as lz4_header, no dictionary, no block
// checksums, the descriptor checksum, then exactly one compressed data block followed by the
// EndMark and (FLG bit 2) the content checksum, ending the payload.  payload bytes 0..23 are
// dwords d[0..5] (from the first three committed chunks).  On success the lane's parse state is
// set and the function returns true; anything else goes to the exact path.
__device__ __forceinline__ bool lz4_frame_head(Lane& L, const uint32_t* d, uint32_t cap, uint32_t& want_size) {
  auto byte = [&](uint32_t i) { return (d[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  const uint32_t flg = byte(4), bd = byte(5);
  const bool csize = (flg & 8) != 0;
  bool ok = d[0] == kLz4Magic && (flg >> 6) == 1 && !(flg & 2) && !(bd & 0x8F) && ((bd >> 4) & 7) >= 4 &&
            !(flg & 1) && !(flg & 0x10);
  const uint32_t bmax = 1u << (8 + 2 * ((bd >> 4) & 7));
  // descriptor checksum: XXH32 of bytes 4..5 or 4..13
  uint32_t h2 = lz4_xxh_byte(lz4_xxh_byte(kXP5 + 2, flg), bd);
  uint32_t h10 = lz4_xxh_word(lz4_xxh_word(kXP5 + 10, d[1]), d[2]);  // bytes 4..7, 8..11
  h10 = lz4_xxh_byte(lz4_xxh_byte(h10, byte(12)), byte(13));
  const uint32_t hc = csize ? byte(14) : byte(6);
  ok = ok && hc == ((lz4_xxh_avalanche(csize ? h10 : h2) >> 8) & 0xff);
  // the content size (8 bytes LE after BD) must fit 32 bits; compared with the output at the end
  want_size = csize ? d[1] >> 16 | d[2] << 16 : 0xFFFFFFFFu;
  ok = ok && (!csize || ((d[2] >> 16 | d[3] << 16) == 0 && want_size != 0xFFFFFFFFu));
  const uint32_t p = csize ? 15u : 7u;  // the first block size
  const uint32_t bs = csize ? (d[3] >> 24 | d[4] << 8) : (d[1] >> 24 | d[2] << 8);
  const uint32_t tail = (flg & 4) ? 8u : 4u;  // EndMark (+ content checksum)
  ok = ok && bs != 0 && !(bs >> 31) && bs <= bmax && uint64_t(p) + 4 + bs + tail == L.clen;
  L.s = p + 4;
  L.sn = p + 4 + bs;
  L.lph = 0;
  L.dn = min(cap, bmax);
  return ok;
}

template <bool kLz4>
__global__ __launch_bounds__(kLpb2Threads) void decode_lpb2_kernel(DecodeArgs a, ZsFastArgs z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  {
    const uint32_t* src = &g_crc16.t[0][0];
    for (uint32_t i = threadIdx.x; i < kLpbTabBytes / 4; i += blockDim.x) tab[i] = src[i];
    if constexpr (kTagTabBytes != 0)
      for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x)
        reinterpret_cast<v2u*>(smem + kTagTabOff)[i] = tag_entry(i);
    __syncthreads();
  }
  const uint32_t* crc_init = g_crc_lt.init;  // used once per round: constant memory
  const uint32_t* crc_tail = g_crc_lt.tail;
  uint8_t* outs = smem + kLpbTabBytes + kTagTabBytes;
  uint8_t* ins = outs + kLpb2Threads * kOutStride;
  uint8_t* ring = outs + threadIdx.x * kOutStride;
  uint8_t* in = ins + threadIdx.x * kInStride;
  // wave-uniform by construction: the buffer resources derived from it must live in SGPRs
  const uint32_t waves_total = gridDim.x * (kLpb2Threads / 64);
  const uint32_t wave_g = blockIdx.x * (kLpb2Threads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  // loop invariants of the transposed refill and flush (LDS offsets of the served blocks' rings)
  const uint32_t slot_lane = (threadIdx.x - lane + (lane >> 2)) * kInStride;
  const uint32_t flush_lane = (threadIdx.x - lane + lane / kRun) * kOutStride;

  // Rounds are handed out by an atomic counter (one dequeue per round, lane 0): waves that
  // finish early take more, so the launch ends when the work does, not when the unluckiest
  // wave's static share does (1 M blocks = 15,625 rounds over 2,048 waves).  Without a counter
  // (raw index/filter payloads from api_sst.cpp) the split is static.
  const uint32_t n_rounds = (a.n + 63) / 64;
  uint32_t r = a.round_counter ? __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(a.round_counter, 1u) : 0u)
                               : wave_g;
  for (; r < n_rounds;
       r = a.round_counter ? __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(a.round_counter, 1u) : 0u)
                           : r + waves_total) {
    const uint32_t round0 = r * 64;
    // ---- the round's buffer resources (wave-uniform)
    const uint32_t rend = min(round0 + 64, a.n);
    const uint8_t* in_lo = a.in + a.in_off[round0];
    const uint8_t* in_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(in_lo) & ~uintptr_t(15));
    const uint8_t* in_hi = a.in + a.in_off[rend];
    Rsrc R;
    R.in = make_rsrc(in_base, align16(uint64_t(in_hi - in_base)));
    uint8_t* out_base = a.out + a.out_off[round0];
    R.out = make_rsrc(out_base, a.out_off[rend] - a.out_off[round0]);
    slate_row* rows_base = a.rows + a.row_base[round0];
    R.rows = make_rsrc(rows_base, 16 * (a.row_base[rend] - a.row_base[round0]));

    Lane L;
    const v4u zero = {0, 0, 0, 0};
    v4u Q = zero;
    v4u P0 = zero, P1 = zero, P2 = zero, P3 = zero;
    uint32_t S0 = 0xFFFFFFFFu, S1 = 0xFFFFFFFFu, S2 = 0xFFFFFFFFu, S3 = 0xFFFFFFFFu;
    const uint32_t b = round0 + lane;
    slate_block_meta m{};
    bool have = b < rend;
    L.in_rel = L.out_rel = L.rows_rel = 0;
    L.sh = L.clen = L.dn = L.last_chunk = L.rcap = 0;
    L.crc_last = -1;
    L.crc = 0xFFFFFFFFu;
    L.crc_pos = 0;
    L.s = L.d = L.rem = L.src = L.T = 0;
    L.mlit = L.mfar = 0;
    bool dd0 = true, err0 = false;  // the masks L.mdd / L.merr once every lane has set up
    L.z = a.rt_zero;
    L.eff = 16;

    L.c_issue = L.c_commit = L.n_req = L.fl = 0;
    L.qoff = kOOB;
    L.mhp = 0;
    L.hd = L.hl = 0;
    L.R = 0;
    L.rphase = 0;
    L.rneed = 4;
    L.rsl = L.rpl = L.rflags = L.ro = L.nwalk = 0;
    L.fk = -1;
    L.pl0 = 0xFFFFFFFFu;
    L.sn = L.lph = L.mtok = L.hb = 0;
    L.xp = 0;
    L.x0 = kXP1 + kXP2;
    L.x1 = kXP2;
    L.x2 = 0;
    L.x3 = 0u - kXP1;
    uint32_t want_size = 0xFFFFFFFFu;  // CodecLz4: the frame's content size (0xFFFFFFFF: none)
    if (have) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      if (len < (a.raw ? 4u : 6u)) {
        m.status = SLATE_E_BLOCK_TOO_SMALL;
        a.meta[b] = m;
        have = false;
      } else {
        const uint8_t* gin = a.in + s0;
        L.sh = uint32_t(reinterpret_cast<uintptr_t>(gin) & 15);
        L.in_rel = uint32_t((gin - L.sh) - in_base);
        L.clen = uint32_t(len - 4);
        L.last_chunk = uint32_t((L.sh + len - 1) >> 4);  // includes the stored CRC
        L.crc_last = L.clen ? int32_t((L.sh + L.clen - 1) >> 4) : -1;
        L.crc = L.clen ? crc_init[L.sh] : 0xFFFFFFFFu;
        L.out_rel = uint32_t(a.out_off[b] - a.out_off[round0]);
        const uint64_t rb = a.row_base[b];
        L.rows_rel = uint32_t(16 * (rb - a.row_base[round0]));
        L.rcap = uint32_t(min<uint64_t>(a.row_base[b + 1] - rb, 0xFFFFFFFFull));
      }
    }
    // ---- the block's first two chunks (aligned, inside the block's chunk range), then
    // golang/snappy decodedLen (decode.go:20-31) over the committed ring
    {
      const v4u c0 = __builtin_amdgcn_raw_buffer_load_b128(R.in, have ? L.in_rel : kOOB, 0, 0);
      const v4u c1 = __builtin_amdgcn_raw_buffer_load_b128(R.in, (have && L.last_chunk >= 1) ? L.in_rel + 16 : kOOB, 0, 0);
      if constexpr (kLz4) {
        // CodecLz4: three chunks hold the frame head at any alignment (sh + 19 <= 34 bytes)
        const v4u c2 = __builtin_amdgcn_raw_buffer_load_b128(R.in, (have && L.last_chunk >= 2) ? L.in_rel + 32 : kOOB, 0, 0);
        if (have) {
          wr128(in, c0, L.z);
          wr128(in + 16, c1, L.z);
          wr128(in + 32, c2, L.z);
          L.c_commit = min(L.last_chunk + 1, 3u);
          L.c_issue = L.c_commit;
          const v2u q0 = ring_rd8(in, L.sh, kIR - 8), q1 = ring_rd8(in, L.sh + 8, kIR - 8),
                    q2 = ring_rd8(in, L.sh + 16, kIR - 8);
          const uint32_t dw[6] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y};
          const uint32_t cap = uint32_t(min<uint64_t>(a.out_off[b + 1] - a.out_off[b], 0xFFFFFFF0ull));
          if (lz4_frame_head(L, dw, cap, want_size)) dd0 = false;
          else L.hb = 1;
        }
      } else if (have) {
        wr128(in, c0, L.z);
        wr128(in + 16, c1, L.z);
        L.c_commit = L.last_chunk >= 1 ? 2u : 1u;
        L.c_issue = L.c_commit;
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
          err0 = true;
        } else {
          L.dn = uint32_t(x);
          L.s = hdr;
          dd0 = false;
        }
      }
    }

    L.mdd = bal(dd0);
    L.merr = bal(err0);
    // the refill's per-round invariant: the input offset of the block each lane serves in load j
    const uint32_t rel0 = __shfl(L.in_rel, int(lane >> 2), 64), rel1 = __shfl(L.in_rel, int(16 + (lane >> 2)), 64),
                   rel2 = __shfl(L.in_rel, int(32 + (lane >> 2)), 64), rel3 = __shfl(L.in_rel, int(48 + (lane >> 2)), 64);
    // ---------------- streaming decode, 64 blocks in lockstep
    uint32_t iters = 0, fin_iter = 0;
    const uint32_t phase = uint32_t((reinterpret_cast<uintptr_t>(in_base) >> 4) + (L.in_rel >> 4)) & 3u;
    const uint32_t ophase = uint32_t((reinterpret_cast<uintptr_t>(out_base) >> 4) + (L.out_rel >> 4)) & 7u;
    const uint64_t t_round = (dbg_bits(a) & 512) ? __builtin_amdgcn_s_memtime() : 0;
    // a lane is done when its decode is finished, no hole is pending, and every chunk
    // is committed and in the CRC.  Every step consumes input, produces output or waits
    // on a load issued at most one iteration earlier, so a block needs far fewer than
    // `budget` iterations; the budget only guarantees that the loop ends (an exhausted
    // lane reports SLATE_E_HIP, never a wrong result).
    const uint32_t budget = have ? (L.clen + L.dn) / 2 + 1024 : 0u;
    for (;;) {
      const uint64_t mact =
          bal(have) & bal(iters < budget) & ~(L.mdd & ~L.mhp & bal(int32_t(L.crc_pos) > L.crc_last) & bal(L.c_commit > L.last_chunk));
      if (!mact) break;
      const bool act = mbit(mact);
      LPB_MARK(refill);
      commit_j<0>(ins, slot_lane, S0, P0, L.z);
      commit_j<1>(ins, slot_lane, S1, P1, L.z);
      commit_j<2>(ins, slot_lane, S2, P2, L.z);
      commit_j<3>(ins, slot_lane, S3, P3, L.z);
      L.c_commit += L.n_req;
      // the next chunks' loads (committed at the next iteration's start)
      {
        // the ring keeps every chunk from the oldest byte still to be read or CRC'd
        const uint32_t lo_pos = msel(L.mdd, L.sh + L.clen, msel(L.mlit & bal(L.rem != 0), L.src, L.sh + L.s));
        const uint32_t lo_chunk = min(lo_pos >> 4, L.crc_pos);
        const uint32_t n = refill_count(act, lo_chunk, L.c_issue, L.last_chunk, phase);
        const uint32_t info = (L.c_issue << 3) | n;
        load_j<0>(lane, info, rel0, R, P0, S0);
        load_j<1>(lane, info, rel1, R, P1, S1);
        load_j<2>(lane, info, rel2, R, P2, S2);
        load_j<3>(lane, info, rel3, R, P3, S3);
        L.c_issue += n;
        L.n_req = n;
      }
      // per iteration: the throttle's limit on d, and the end of the committed input (ring positions)
      const uint32_t lim_d = 16 * L.fl + kUnflushed, cend = 16 * L.c_commit;
      LPB_MARK(absorb);
      lane_step<0, kLz4>(L, act, mact, ring, in, tab, R, lim_d, cend, dbg_bits(a));
      absorb_hole(L, Q, ring);
      lane_step<1, kLz4>(L, act, mact, ring, in, tab, R, lim_d, cend, dbg_bits(a));
      lane_step<2, kLz4>(L, act, mact, ring, in, tab, R, lim_d, cend, dbg_bits(a));
      lane_step<3, kLz4>(L, act, mact, ring, in, tab, R, lim_d, cend, dbg_bits(a));
      // the hole source requested in this iteration (at most one per lane; sc1: L1 bypass),
      // before the flush stores so that vmcnt waits stay static; it is merged at the start of
      // the next iteration
      LPB_MARK(flush);
      Q = __builtin_amdgcn_raw_buffer_load_b128(R.out, (dbg_bits(a) & 32768) ? kOOB : L.qoff, 0, 16);
      L.qoff = kOOB;
      flush_iteration(L, act, outs, lane, R, dbg_bits(a), iters % kFlushParts, flush_lane, ophase);
      if constexpr (kLz4) {
        // the content checksum's stripes: the chunks completed so far (up to kStep / 4), still in the ring
#pragma unroll
        for (uint32_t j = 0; j < kStep / 4; j++) xxh_absorb(L, ring, L.xp < min(L.d >> 4, msel(L.mhp, L.hd >> 4, 0xFFFFFFFFu)));
      }
      iters++;
      fin_iter = act ? iters : fin_iter;  // profiling (debug 131072): the lane's last active iteration
    }
    const uint32_t round_cycles = (dbg_bits(a) & 512) ? uint32_t(__builtin_amdgcn_s_memtime() - t_round) : 0u;

    // ---------------- finalise the round's blocks (SIMD across lanes)
    // iters counts the wave's iterations: a lane that finished early is not exhausted
    if (have && !(mbit(L.mdd) && !mbit(L.mhp) && int32_t(L.crc_pos) > L.crc_last && L.c_commit > L.last_chunk)) {
      m.status = SLATE_E_HIP;  // step budget exhausted (see above): a kernel defect, reported loudly
      a.meta[b] = m;
      have = false;
    }
    uint8_t* gout = out_base + L.out_rel;
    slate_row* grows = reinterpret_cast<slate_row*>(reinterpret_cast<uint8_t*>(rows_base) + L.rows_rel);
    // rows stage: 0 = no rows to produce, 1 = walked rows to verify, 2 = re-derive from HBM
    uint32_t rows_stage = 0, nr = 0, osi_u = 0;
    bool hand_back = false;  // CodecLz4: the exact path decodes this block
    if (have) {
      const uint32_t stored = __builtin_bswap32(ring_rd8(in, L.sh + L.clen, kIR - 8).x);
      // the register absorbed t zero bytes after the payload: compare against stored * x^(8t)
      const uint32_t t = L.clen ? uint32_t(16 * (L.crc_last + 1)) - (L.sh + L.clen) : 0u;
      const bool crc_ok = gf2_mulmod(~stored, crc_tail[t]) == L.crc;
      bool dec_ok;
      if constexpr (kLz4) {
        // the data block ended on its last literals, then the EndMark; the content size if any
        const uint32_t endmark = ring_rd8(in, L.sh + L.sn, kIR - 8).x;
        dec_ok = !L.hb && L.lph == 2 && L.rem == 0 && L.s == L.sn && L.d == L.dn && endmark == 0 &&
                 (want_size == 0xFFFFFFFFu || want_size == L.d);
        hand_back = crc_ok && !dec_ok;
        if (crc_ok && dec_ok && L.clen - L.sn == 8) {
          // FLG bit 2: XXH32 of the decoded block, the rest of its stripes and its tail from the ring
          const uint32_t dn = L.dn;
          while (L.xp < dn / 16) xxh_absorb(L, ring, true);
          uint32_t h = dn >= 16 ? xrotl(L.x0, 1) + xrotl(L.x1, 7) + xrotl(L.x2, 12) + xrotl(L.x3, 18) : kXP5;
          h += dn;
          const v4u tv = rd128(ring + ((dn & ~15u) & (kOR - 1)), L.z);
          const uint32_t tb = dn & 15, tw[4] = {tv.x, tv.y, tv.z, tv.w};
          for (uint32_t i = 0; 4 * (i + 1) <= tb; i++) h = lz4_xxh_word(h, tw[i]);
          for (uint32_t i = tb & ~3u; i < tb; i++) h = lz4_xxh_byte(h, (tw[i >> 2] >> (8 * (i & 3))) & 0xff);
          hand_back = lz4_xxh_avalanche(h) != ring_rd8(in, L.sh + L.sn + 4, kIR - 8).x;
          dec_ok = !hand_back;  // a mismatch: the exact path reports it
        }
      } else {
        dec_ok = !mbit(L.merr) && L.d == L.dn && L.s == L.clen && L.rem == 0;
      }
      const uint32_t dn = L.dn;
      if (!crc_ok) {
        m.status = SLATE_E_BLOCK_CHECKSUM;
      } else if (!dec_ok) {
        m.status = SLATE_E_SNAPPY_CORRUPT;  // (CodecLz4: handed back, not written)
      } else {
        // remaining output chunks (the last one is padded inside its 16-byte slot)
        while (L.fl * 16 < dn) {
          const v4u o = rd128(ring + ((L.fl * 16) & (kOR - 1)), L.z);
          reinterpret_cast<v4u*>(gout)[L.fl] = o;
          L.fl++;
        }
        // let the row walker catch up on the block's last bytes (still in the ring)
        for (int i = 0; i < 16 && L.rphase < 3 && L.d >= L.rneed; i++) {
          v4u row;
          uint32_t ridx;
          if (walk_step(L, ring, true, mbit(L.mhp), row, ridx)) reinterpret_cast<v4u*>(grows)[ridx] = row;
        }
        if (a.raw) {
          m.data_len = dn;  // a decompressed index / filter buffer
        } else if (dn < 2) {
          m.status = SLATE_E_BLOCK_UNCOMP_SMALL;
        } else {
          // block.go:101-134 over the decoded block.  The tail (offsets, count) is read
          // from the output ring when it is still there, else from HBM.
          const uint32_t cnt = be16_of(ring_rd8(ring, dn - 2).x);
          const int64_t osi = int64_t(dn) - 2 - 2 * int64_t(cnt);
          if (osi <= 0) {
            m.status = SLATE_E_BLOCK_INDEX_OFFSET;
            m.detail = int32_t(osi);
          } else {
            const bool tail_in_ring = dn - uint32_t(osi) <= kReach;
            auto off_at = [&](uint32_t i) -> uint32_t {
              const uint32_t p = uint32_t(osi) + 2 * i;
              if (tail_in_ring) return be16_of(ring_rd8(ring, p).x);
              return out_be16(gout + p);
            };
            const uint16_t osi16 = uint16_t(osi);
            uint32_t bad = 0xFFFFFFFFu;
            for (uint32_t i = 0; i < cnt; i++) {
              if (off_at(i) > osi16) {
                bad = i;
                break;
              }
            }
            if (bad != 0xFFFFFFFFu) {
              m.status = SLATE_E_BLOCK_OFFSET_BOUNDS;
              m.aux = uint16_t(bad);
              m.detail = int32_t(off_at(bad));
            } else {
              m.data_len = uint32_t(osi);
              m.n_rows = uint16_t(cnt);
              if (cnt == 0) {
                m.status = SLATE_E_BLOCK_NO_OFFSETS;
              } else {
                const uint32_t off0 = off_at(0);
                if (uint64_t(osi) - off0 < 2) {
                  m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
                } else {
                  // FirstKey quirk (block.go:130-131): the BE16 at Data[off0]; the walker read
                  // it already when off0 is the first row's start
                  const uint16_t kl = uint16_t((off0 == 0 && L.pl0 != 0xFFFFFFFFu) ? L.pl0 : out_be16(gout + off0));
                  const uint16_t lo = uint16_t(off0 + 2), hi = uint16_t(off0 + 2 + kl);
                  if (lo > hi || hi > dn) {
                    m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
                  } else {
                    m.aux = kl;
                    if (cnt > L.rcap) m.flags |= SLATE_BLKF_ROWS_TRUNCATED;
                    nr = cnt < L.rcap ? cnt : L.rcap;
                    osi_u = uint32_t(osi);
                    // walked rows are usable when at least nr rows were walked and the walk
                    // stays inside Data; their starts are then compared with the offsets below
                    bool walk_ok = L.nwalk >= nr;
                    if (walk_ok) {
                      if (L.nwalk > nr) walk_ok = nr < L.rcap;  // row nr's start is in the rows array
                      else walk_ok = L.rphase != 3 && L.R <= osi_u;
                    }
                    rows_stage = walk_ok ? 1u : 2u;
                  }
                }
              }
            }
          }
        }
      }
    }
    if constexpr (kLz4) {
      lpb_list_append(hand_back, b, z.list, z.count);
      if (hand_back) {
        have = false;
        rows_stage = 0;
      }
    }
    // ---- wave-cooperative check of the walked row starts against offsets[] (block.go:107-118):
    // per block, coalesced loads of its offsets and row descriptors; eight blocks per wait
    {
      uint64_t todo = (dbg_bits(a) & 65536) ? 0 : __ballot(rows_stage == 1);  // 65536: profiling only
      uint64_t mism = 0;
      while (todo) {
        uint32_t js[kVerifyBatch], nrs[kVerifyBatch], osis[kVerifyBatch], outs[kVerifyBatch], rws[kVerifyBatch],
            nws[kVerifyBatch], Rs[kVerifyBatch], ends[kVerifyBatch];
        uint32_t ob[kVerifyBatch], wr[kVerifyBatch];
        uint32_t nb = 0;
#pragma unroll
        for (uint32_t q = 0; q < kVerifyBatch; q++) {
          const bool v = todo != 0;
          const uint32_t j = v ? uint32_t(__builtin_ctzll(todo)) : 0u;
          todo &= v ? todo - 1 : todo;
          nb += v ? 1u : 0u;
          js[q] = j;
          nrs[q] = v ? __builtin_amdgcn_readlane(nr, j) : 0u;
          osis[q] = __builtin_amdgcn_readlane(osi_u, j);
          outs[q] = __builtin_amdgcn_readlane(L.out_rel, j);
          rws[q] = __builtin_amdgcn_readlane(L.rows_rel, j);
          nws[q] = __builtin_amdgcn_readlane(L.nwalk, j);
          Rs[q] = __builtin_amdgcn_readlane(L.R, j);
          const uint32_t i = lane;
          const bool in = i < min(nrs[q], 64u);
          ob[q] = __builtin_amdgcn_raw_buffer_load_b16(R.out, in ? outs[q] + osis[q] + 2 * i : kOOB, 0, 16);
          wr[q] = __builtin_amdgcn_raw_buffer_load_b32(R.rows, in ? rws[q] + 16 * i : kOOB, 0, 16);
          ends[q] = __builtin_amdgcn_raw_buffer_load_b32(
              R.rows, (lane == 0 && nws[q] > nrs[q]) ? rws[q] + 16 * nrs[q] : kOOB, 0, 16);
        }
#pragma unroll
        for (uint32_t q = 0; q < kVerifyBatch; q++) {
          if (q < nb) {
          const uint32_t o = ((ob[q] & 0xff) << 8) | ((ob[q] >> 8) & 0xff);
          bool bad = lane < min(nrs[q], 64u) && o != wr[q];
          // blocks with more than 64 rows: the remaining rows, one group of 64 at a time
          for (uint32_t i0 = 64; i0 < nrs[q]; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool in = i < nrs[q];
            const uint32_t b2 = __builtin_amdgcn_raw_buffer_load_b16(R.out, in ? outs[q] + osis[q] + 2 * i : kOOB, 0, 16);
            const uint32_t w2 = __builtin_amdgcn_raw_buffer_load_b32(R.rows, in ? rws[q] + 16 * i : kOOB, 0, 16);
            bad = bad || (in && (((b2 & 0xff) << 8) | ((b2 >> 8) & 0xff)) != w2);
          }
          // the walk must also end inside Data: the start of row nr (recorded when more rows
          // were walked) or the walker's position
          const uint32_t end_last = nws[q] > nrs[q] ? __builtin_amdgcn_readfirstlane(ends[q]) : Rs[q];
          bad = bad || end_last > osis[q];
          if (__ballot(bad)) mism |= uint64_t(1) << js[q];
          }
        }
      }
      if (rows_stage == 1 && ((mism >> lane) & 1)) rows_stage = 2;
    }
    // ---- exact fallback: rows re-derived from HBM with the row.go decoder (corrupt blocks only)
    if (rows_stage == 2) {
      int fk = -1;
      for (uint32_t i = 0; i < nr; i++) {
        uint32_t sl;
        const uint32_t off = out_be16(gout + osi_u + 2 * i);
        const v4u r = row_from_hbm(gout, osi_u, off, fk, &sl);
        if (i == 0 && (r.w >> 16) == SLATE_OK) fk = int(sl);
        reinterpret_cast<v4u*>(grows)[i] = r;
      }
    }
    if (dbg_bits(a) & 131072) m.detail = int32_t(fin_iter);  // profiling only: results are wrong by design
    if (have) a.meta[b] = m;
    if ((dbg_bits(a) & 512) && lane == 0 && round0 + 1 < a.n) {
      // profiling only: loop iterations and cycles of this round, in meta.detail of its first two blocks
      a.meta[round0].detail = int32_t(iters);
      a.meta[round0 + 1].detail = int32_t(round_cycles);
    }
  }
}


size_t lpb2_lds_bytes() {
  return kLpbTabBytes + kTagTabBytes + size_t(kLpb2Threads) * (kOutStride + kInStride);
}

// CodecLz4 plan, lane per block: oracle lz4_frame_len's decoded size (the bytes the in-order
// decoder writes before its first structural error; decode.hip lz4_frame_len) for frames whose
// first data block is followed by the EndMark or by nothing: the header checks, then the
// token / match structure of that block walked without copying (literals are skipped).  The
// block streams through the lane's 128-byte input ring by the decoder's transposed refills (64
// bytes per block per iteration), and up to eight sequence halves are parsed per iteration.  A
// frame with a second data block, or a length extension longer than the 8-byte window, is
// appended to `list` for the serial plan.
constexpr uint32_t kLz4PlanThreads = 256;
constexpr uint32_t kLz4PlanSteps = 8;
__global__ __launch_bounds__(kLz4PlanThreads) void plan_lz4_lane_kernel(const uint8_t* __restrict__ gin,
                                                                        const uint64_t* __restrict__ in_off, uint32_t n,
                                                                        uint64_t* __restrict__ out_sz,
                                                                        uint64_t* __restrict__ row_sz, uint32_t* list,
                                                                        uint32_t* count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave_lane0 = threadIdx.x - lane;
  uint8_t* in = smem + threadIdx.x * kInStride;
  const uint32_t stride = gridDim.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the scans turn the trailing zero into the totals
    out_sz[n] = 0;
    row_sz[n] = 0;
  }
  for (uint32_t r0 = blockIdx.x * blockDim.x + wave_lane0; r0 < n; r0 += stride) {
    const uint32_t b = r0 + lane;
    const uint32_t rend = min(r0 + 64, n);
    const uint8_t* in_lo = gin + in_off[r0];
    const uint8_t* in_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(in_lo) & ~uintptr_t(15));
    Rsrc R;
    R.in = make_rsrc(in_base, align16(uint64_t((gin + in_off[rend]) - in_base)));
    const uint32_t z = 0;
    uint32_t sh = 0, rel = 0, clen = 0, last_chunk = 0;
    bool have = b < rend, fb = false;
    if (have) {
      const uint64_t s0 = in_off[b], len = in_off[b + 1] - s0;
      const uint8_t* p = gin + s0;
      sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 15);
      rel = uint32_t((p - sh) - in_base);
      have = len >= 6;  // decoded_len: a shorter block decodes nothing
      clen = have ? uint32_t(len - 4) : 0u;
      last_chunk = have ? uint32_t((sh + clen - 1) >> 4) : 0u;  // the frame's chunks (not the CRC)
    }
    // the frame head: three chunks
    const v4u c0 = __builtin_amdgcn_raw_buffer_load_b128(R.in, have ? rel : kOOB, 0, 0);
    const v4u c1 = __builtin_amdgcn_raw_buffer_load_b128(R.in, (have && last_chunk >= 1) ? rel + 16 : kOOB, 0, 0);
    const v4u c2 = __builtin_amdgcn_raw_buffer_load_b128(R.in, (have && last_chunk >= 2) ? rel + 32 : kOOB, 0, 0);
    wr128(in, c0, z);
    wr128(in + 16, c1, z);
    wr128(in + 32, c2, z);
    uint32_t c_commit = min(last_chunk + 1, 3u), c_issue = c_commit, n_req = 0;
    // lz4_header: magic, FLG / BD, the descriptor in the buffer; no dictionary
    const v2u q0 = ring_rd8(in, sh, kIR - 8), q1 = ring_rd8(in, sh + 8, kIR - 8), q2 = ring_rd8(in, sh + 16, kIR - 8);
    const uint32_t flg = q0.y & 0xff, bd = (q0.y >> 8) & 0xff;
    const bool csize = (flg & 8) != 0, bcheck = (flg & 0x10) != 0;
    const uint32_t pos = csize ? 15u : 7u;  // the first block size word (after HC)
    const bool hdr_ok = have && clen >= 7 && q0.x == kLz4Magic && (flg >> 6) == 1 && !(flg & 2) && !(bd & 0x8F) &&
                        ((bd >> 4) & 7) >= 4 && clen >= pos && !(flg & 1);
    const uint32_t bmax = 1u << (8 + 2 * ((bd >> 4) & 7));
    const uint32_t bs = csize ? (q1.y >> 24 | q2.x << 8) : (q0.y >> 24 | q1.x << 8);
    const uint32_t sz = bs & 0x7FFFFFFFu;
    // a block size word, not the EndMark, the block (and its checksum) inside the frame
    const bool blk = hdr_ok && clen >= pos + 4 && bs != 0 && sz <= bmax &&
                     uint64_t(clen) - pos - 4 >= uint64_t(sz) + (bcheck ? 4u : 0u);
    const bool stored = (bs >> 31) != 0;
    const uint32_t sn = pos + 4 + sz, tail = sn + (bcheck ? 4u : 0u);  // the next block size word
    uint32_t s = stored ? sn : pos + 4;  // a stored block is not walked
    uint32_t dl = blk && stored ? sz : 0u, lph = 0, mtok = 0;
    // ph: 0 walking the block, 1 waiting for the word after it, 2 done
    uint32_t ph = !blk ? 2u : (stored ? 1u : 0u);
    v4u P0 = c0, P1 = c0, P2 = c0, P3 = c0;
    uint32_t S0 = 0xFFFFFFFFu, S1 = 0xFFFFFFFFu, S2 = 0xFFFFFFFFu, S3 = 0xFFFFFFFFu;
    const uint32_t budget = (clen + 63) / 64 + (clen + 3) / 4 + 8;  // > chunks / 4 + halves / 8: never hit
    uint32_t it = 0;
    for (; __ballot(ph < 2 && it < budget); it++) {
      const bool act = ph < 2 && it < budget;
      commit_one(smem, S0, P0, z);
      commit_one(smem, S1, P1, z);
      commit_one(smem, S2, P2, z);
      commit_one(smem, S3, P3, z);
      c_commit += n_req;
      const uint32_t lo_chunk = (sh + min(s, tail)) >> 4;
      const uint32_t nq = refill_count(act, lo_chunk, c_issue, last_chunk,
                                        uint32_t((reinterpret_cast<uintptr_t>(in_base) >> 4) + (rel >> 4)) & 3u);
      const uint32_t info = (c_issue << 3) | nq;
      load_one(0, lane, wave_lane0, info, rel, R, P0, S0);
      load_one(1, lane, wave_lane0, info, rel, R, P1, S1);
      load_one(2, lane, wave_lane0, info, rel, R, P2, S2);
      load_one(3, lane, wave_lane0, info, rel, R, P3, S3);
      c_issue += nq;
      n_req = nq;
      const int32_t avail = int32_t(16 * c_commit) - int32_t(sh);
#pragma unroll
      for (uint32_t k = 0; k < kLz4PlanSteps; k++) {
        const bool can = act && ph == 0 && avail >= int32_t(min(s + 8, clen));
        const v2u w = ring_rd8(in, sh + s, kIR - 8);
        const uint64_t w64 = (uint64_t(w.y) << 32) | w.x;
        const uint32_t tok = w.x & 0xff;
        const bool tokp = lph == 0;
        // a token without literals is walked together with its match (as lz4_parse)
        const bool z0 = tokp && (tok >> 4) == 0 && s + 1 < sn;
        const bool mph = !tokp || z0;
        const uint64_t wm = z0 ? w64 >> 8 : w64;
        const uint32_t n4 = mph ? (tokp ? tok & 15 : mtok) : tok >> 4;
        const uint64_t ext = mph ? wm >> 16 : w64 >> 8;
        const uint64_t nz =
            ~ext & (mph ? (z0 ? 0x000000FFFFFFFFFFull : 0x0000FFFFFFFFFFFFull) : 0x00FFFFFFFFFFFFFFull);
        const uint32_t kk = uint32_t(__builtin_ctzll(nz | (uint64_t(1) << 63))) >> 3;
        const bool lng = n4 == 15;
        const uint32_t len = lng ? 15 + 255 * kk + (uint32_t(ext >> (8 * kk)) & 0xff) : n4;
        const uint32_t ms = s + (z0 ? 1u : 0u);
        const uint32_t s1 = (mph ? ms + 2 : s + 1) + (lng ? kk + 1 : 0u);
        const bool to_list = lng && nz == 0;  // the run goes on past the window
        // lz4_frame_len: the token at s < sz, its literals inside the block and the block maximum
        const uint32_t lit_end = s1 + len;
        const bool err_t = s >= sn || lit_end > sn || len > bmax - dl;
        // the offset (2 bytes), 0 < offset <= output so far, the length, and a token after it
        const uint32_t off = uint32_t(wm) & 0xffff, ml = len + 4;
        const bool err_m = ms + 2 > sn || s1 >= sn || off == 0 || off > dl || ml > bmax - dl;
        const bool err = mph ? err_m : err_t;
        const bool good = can && !to_list && !err;
        fb = fb || (can && to_list);
        const bool last = !mph && lit_end == sn;
        // an error leaves the bytes of the blocks before this one: none
        dl = (can && !to_list && err) ? 0u : (good ? dl + (mph ? ml : len) : dl);
        ph = (can && (to_list || err)) ? 2u : ((good && last) ? 1u : ph);
        s = good ? (mph ? s1 : lit_end) : s;
        mtok = (good && !mph) ? (tok & 15) : mtok;
        lph = good ? (mph ? 0u : 1u) : lph;
      }
      // the word after the block: a second data block goes to the serial plan
      const bool tail_in = act && ph == 1 && avail >= int32_t(min(tail + 4, clen));
      if (tail_in) {
        const uint32_t next = tail + 4 <= clen ? ring_rd8(in, sh + tail, kIR - 8).x : 0u;
        fb = fb || next != 0;
        ph = 2;
      }
    }
    fb = fb || (have && ph < 2);  // (budget: never reached)
    if (b < rend && !fb) {
      out_sz[b] = align16(dl);
      row_sz[b] = row_capacity(dl);
    }
    lpb_list_append(b < rend && fb, b, list, count);
  }
}

template <bool kLz4>
hipError_t launch_lpb(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus) {
  const size_t lds = lpb2_lds_bytes();
  const uint32_t waves_needed = (a.n + 63) / 64;
  uint32_t grid = (waves_needed + kLpb2Threads / 64 - 1) / (kLpb2Threads / 64);
  grid = min(grid, uint32_t(num_cus) * uint32_t(163840 / lds));
  // one workgroup takes (nearly) the whole 160 KiB LDS of a CU
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_lpb2_kernel<kLz4>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  decode_lpb2_kernel<kLz4><<<grid, kLpb2Threads, lds, st>>>(a, z);
  return hipGetLastError();
}

hipError_t launch_decode_lpb2(hipStream_t st, const DecodeArgs& a, int num_cus) {
  if (a.n == 0) return hipGetLastError();
  return launch_lpb<false>(st, a, ZsFastArgs{}, num_cus);
}

hipError_t launch_lz4_plan(hipStream_t st, const uint8_t* in, const uint64_t* in_off, uint32_t n, uint64_t* out_sz,
                           uint64_t* row_sz, uint32_t* list, uint32_t* count) {
  if (n == 0) {
    (void)hipMemsetAsync(out_sz, 0, 8, st);
    (void)hipMemsetAsync(row_sz, 0, 8, st);
    return hipGetLastError();
  }
  const uint32_t grid = min((n + kLz4PlanThreads - 1) / kLz4PlanThreads, 8192u);
  plan_lz4_lane_kernel<<<grid, kLz4PlanThreads, size_t(kLz4PlanThreads) * kInStride, st>>>(in, in_off, n, out_sz,
                                                                                            row_sz, list, count);
  return hipGetLastError();
}

hipError_t launch_lz4_fast(hipStream_t st, const DecodeArgs& a, const ZsFastArgs& z, int num_cus) {
  if (a.n == 0) return hipGetLastError();
#ifdef SLATE_LPB_NO_LZ4  // experiment builds of the Snappy kernel alone (LZ4 frames take the exact path)
  (void)st, (void)z, (void)num_cus;
  return hipErrorNotSupported;
#else
  return launch_lpb<true>(st, a, z, num_cus);
#endif
}

}  // namespace slate
