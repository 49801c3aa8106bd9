// Snappy block decode in two phases per round of 64 blocks (the headline kernel).
//
// block.Decode (internal/sstable/block/block.go:78-134) with CodecSnappy: CRC32 verify ->
// golang/snappy v0.0.4 decode (decode_other.go:19-110) -> offset checks -> row descriptors
// (row.go:191-261 as block/iterator.go walks).
//
// A Snappy tag stream is a serial chain inside a block, but the bytes it describes are not:
// once every tag's output position and source are known, a block's output is a gather.  So
// each wave takes 64 blocks at a time ("a round") and:
//
//   P (parse, lane per block): lane l walks block l's tag chain and CRC32s its bytes.  The
//     compressed bytes stream through a small LDS ring per lane, filled by transposed loads
//     (four lanes read one block's 64-byte run, tools/scatter_probe.hip).  Every tag becomes
//     one 32-bit op -- a literal (input position, length) or a copy (offset, length) -- and a
//     copy whose source lies inside one of the last kH ops is rewritten against that op: a
//     copy of a literal's bytes becomes a literal of the input bytes, a copy of a copy takes
//     the sum of the offsets.  Rows repeat their neighbours' bytes (V-half: the seq/flags/
//     value-length bytes and the value halves), so almost every copy ends as a literal and
//     the rest point at the block's first occurrences.  Ops collect in an LDS ring and are
//     flushed 64 bytes per block (transposed stores) into the block's own output slot, which
//     the output overwrites later.
//
//   M (materialize, wave per block): for each block of the round, the wave stages the
//     compressed block in LDS, reads its ops 64 at a time (one per lane), places them by a
//     wave prefix sum of their lengths, and copies every op whose source bytes are ready --
//     all literals and copies of earlier batches in the first round, the remaining copies in
//     later rounds once the ops overlapping their sources are done (a 64-bit mask per lane).
//     Then the block.go offset checks, the FirstKey quirk and the row descriptors run lane-
//     parallel over the decoded block in LDS, and the block is written with 16-byte stores.
//
// Blocks whose compressed or decoded size exceeds the M staging (8 KiB), or whose ops do not
// fit their output slot, are queued for the wave-per-block decoder (decode.hip), which
// handles any block.  Every ablation branch of the shipped library folds away (dbg_bits).
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"
#include "lpb_common.h"
#include "rows.h"

namespace slate {

namespace {

constexpr uint32_t kNS = 8;                       // input ring slots (16 bytes each)
constexpr uint32_t kIR = kNS * 16;
constexpr uint32_t kInStride = kIR + 8;           // 136 B lane records: bank spread (decode_lpb2.hip)
constexpr uint32_t kOpSlots = 32;                 // op staging ring per lane (one dword per op)
constexpr uint32_t kOpStride = kOpSlots * 4 + 8;  // 136 B (the dword after the ring is the lane's junk slot)
constexpr uint32_t kGroup = 16;                   // ops per flushed group (64 bytes)
constexpr int kH = 6;                             // ops a copy is resolved against
constexpr uint32_t kMCap = 8192;                  // M staging per block: compressed and decoded
constexpr uint32_t kMSlack = 64;                  // window reads run up to 24 bytes past a position
constexpr uint32_t kPBytes = 64 * (kInStride + kOpStride);
constexpr uint32_t kMBytes = 2 * (kMCap + kMSlack) + 256;  // + a junk word per lane
constexpr uint32_t kWaveBytes = kPBytes > kMBytes ? kPBytes : kMBytes;
constexpr uint32_t kCrcSteps = 3;                 // CRC chunk steps per iteration
constexpr uint32_t kTagSteps = 4;                 // tag steps per iteration
// op word: [31] copy, [30:17] length - 1, [16:0] literal: input position in the M staging
// (alignment shift included); copy: offset back from the op's output position
constexpr uint32_t kOpCopy = 0x80000000u;
constexpr uint32_t kLenShift = 17;
constexpr uint32_t kSrcMask = (1u << 17) - 1;
constexpr uint32_t kLitF = 0x80000000u;           // history: literal-sourced entry
// lane status after P
constexpr uint32_t kStNone = 0, kStDecode = 1, kStDone = 2, kStFallback = 3;

// Cache policy bits (gfx950 CPol): 16 = sc1 (around the CU's L1: ops this wave just stored).
constexpr int kSc1 = 16;

struct Rsrc {
  __amdgpu_buffer_rsrc_t in, out;
};

struct PLane {
  uint32_t in_rel, out_rel, sh, clen, last_chunk, dn, cap_ops;
  int32_t crc_last;
  uint32_t crc, crc_pos, c_issue, c_commit, n_req;
  uint32_t s, d, err, fin, fb;
  uint32_t nop, nfl;
  uint32_t hy[kH], hl[kH], hs[kH];
  uint32_t z;
};

__device__ __forceinline__ void commit_one(uint8_t* rings, uint32_t slot, const v4u& v, uint32_t z) {
  if (slot != 0xFFFFFFFFu) wr128(rings + slot, v, z);
}

// Transposed refill: in load j, lanes 4i..4i+3 read chunks c_issue..c_issue+3 of block 16j+i;
// slot = LDS byte offset (from smem) of the owner's ring slot, written at the next commit.
__device__ __forceinline__ void load_one(uint32_t j, uint32_t lane, uint32_t rbase, uint32_t info, uint32_t rel,
                                         const Rsrc& R, v4u& P, uint32_t& slot) {
  const uint32_t o = 16 * j + (lane >> 2), c = lane & 3;
  const uint32_t info_o = __shfl(info, int(o), 64);
  const uint32_t rel_o = __shfl(rel, int(o), 64);
  const uint32_t ci = (info_o >> 3) + c;
  const bool want = c < (info_o & 7);
  P = __builtin_amdgcn_raw_buffer_load_b128(R.in, want ? rel_o + 16 * ci : kOOB, 0, 0);
  slot = want ? rbase + o * kInStride + (ci & (kNS - 1)) * 16 : 0xFFFFFFFFu;
}

// CRC32 of the next committed chunk (bytes outside the payload zeroed; decode_lpb2.hip).
__device__ __forceinline__ void crc_step(PLane& L, const uint8_t* ring, const uint32_t* tab, bool act) {
  const bool go = act && L.crc_pos < L.c_commit && int32_t(L.crc_pos) <= L.crc_last;
  const uint32_t k = L.crc_pos;
  v4u v = rd128(ring + (k & (kNS - 1)) * 16, L.z);
  const bool partial = go && (k == 0 || int32_t(k) == L.crc_last);
  if (__builtin_amdgcn_ballot_w64(partial)) {
    const int32_t lo = int32_t(L.sh) - int32_t(16 * k), hi = int32_t(L.sh + L.clen) - int32_t(16 * k);
    v.x &= keep_mask(lo, hi, 0);
    v.y &= keep_mask(lo, hi, 1);
    v.z &= keep_mask(lo, hi, 2);
    v.w &= keep_mask(lo, hi, 3);
  }
  const uint32_t c = crc16_chunk(tab, L.crc, v);
  L.crc = go ? c : L.crc;
  L.crc_pos += go ? 1u : 0u;
}

// One tag (golang/snappy decode_other.go:19-110, same checks in the same order as
// decode_lpb2.hip) -> one op in the lane's staging ring.  Straight-line code: every choice is
// a select on data, so the 64 lanes never split into exec-masked branches.
__device__ __forceinline__ void tag_step(PLane& L, const uint8_t* ring, uint8_t* opr, bool act) {
  const int32_t avail = int32_t(16 * L.c_commit) - int32_t(L.sh);  // committed payload bytes [0, avail)
  const uint32_t sn = L.clen;
  const bool need = act && !L.fin;
  const bool end = need && L.s >= sn;
  const bool can = need && L.s < sn && avail >= int32_t(min(L.s + 5, sn)) && L.nop - L.nfl < kOpSlots;
  const v2u w = ring_rd8(ring, L.sh + L.s, kIR - 8);
  const uint32_t c = w.x & 0xff, t = c & 3;
  const uint32_t b14 = (w.x >> 8) | (w.y << 24);  // bytes s+1 .. s+4
  const uint32_t xl = c >> 2;
  const uint32_t nb = xl >= 60 ? xl - 59 : 0;
  const uint32_t ext = nb >= 4 ? b14 : (b14 & ((1u << (8 * nb)) - 1));
  const uint32_t lit_m1 = nb ? ext : xl;  // literal length - 1 (the +1 cannot wrap below)
  const uint32_t cp_len = (t == 1) ? 4 + ((c >> 2) & 7) : 1 + (c >> 2);
  const uint32_t off1 = ((c & 0xe0) << 3) | (b14 & 0xff), off2 = b14 & 0xffff;
  const uint32_t cp_off = (t & 2) ? ((t & 1) ? b14 : off2) : off1;
  const uint32_t hl_cp = (t & 2) ? ((t & 1) ? 5u : 3u) : 2u;
  const bool lit = t == 0;
  const uint32_t hdr = lit ? 1 + nb : hl_cp;
  const uint32_t s1 = L.s + hdr;
  const uint32_t room_out = L.dn - L.d;
  const bool bad_lit = lit_m1 >= room_out || lit_m1 >= sn - min(s1, sn);
  const bool bad_cp = cp_off == 0 || L.d < cp_off || cp_len > room_out;
  const bool bad = s1 > sn || (lit ? bad_lit : bad_cp);
  const bool ok = can && !bad;
  L.err |= (can && bad) ? 1u : 0u;
  L.fin |= (end || (can && bad)) ? 1u : 0u;
  const uint32_t len = lit ? lit_m1 + 1 : cp_len;
  // a copy inside one of the last kH ops takes that op's source
  const uint32_t a = L.d - cp_off;
  uint32_t src = lit ? L.sh + s1 : cp_off;
  uint32_t cpy = lit ? 0u : 1u;
#pragma unroll
  for (int h = 0; h < kH; h++) {
    const uint32_t x = a - L.hy[h];                              // a's place in entry h (wraps below it)
    const bool hit = !lit && x < L.hl[h] && L.hl[h] - x >= len;  // [a, a+len) inside entry h
    const uint32_t hs = L.hs[h];
    const uint32_t cand = (hs & kLitF) ? (hs & ~kLitF) + x : cp_off + hs;
    src = hit ? cand : src;
    cpy = hit ? (hs >> 31) ^ 1u : cpy;
  }
  const uint32_t op = (cpy << 31) | ((len - 1) << kLenShift) | (src & kSrcMask);
  // history: shift in the new op when there is one
#pragma unroll
  for (int h = 0; h < kH - 1; h++) {
    L.hy[h] = ok ? L.hy[h + 1] : L.hy[h];
    L.hl[h] = ok ? L.hl[h + 1] : L.hl[h];
    L.hs[h] = ok ? L.hs[h + 1] : L.hs[h];
  }
  L.hy[kH - 1] = ok ? L.d : L.hy[kH - 1];
  L.hl[kH - 1] = ok ? len : L.hl[kH - 1];
  L.hs[kH - 1] = ok ? (cpy ? src : (kLitF | src)) : L.hs[kH - 1];
  // the op goes to its staging slot, or (no op) to the lane's junk dword after the ring
  *reinterpret_cast<uint32_t*>(opr + (ok ? (L.nop & (kOpSlots - 1)) * 4 : kOpSlots * 4)) = op;
  L.nop += ok ? 1u : 0u;
  L.s = ok ? (lit ? s1 + len : s1) : L.s;
  L.d += ok ? len : 0u;
  // ops that no longer fit the block's output slot: the wave-per-block decoder takes it
  const bool over = ok && L.nop > L.cap_ops;
  L.fb |= over ? 1u : 0u;
  L.fin |= over ? 1u : 0u;
}

// Complete 16-op groups (64 bytes) of every lane that has one, as four transposed stores
// (lanes 4i..4i+3 write one block's group); with `all`, every lane's last partial group.
__device__ __forceinline__ void flush_ops(PLane& L, bool all, uint8_t* oprs, uint32_t lane, const Rsrc& R) {
  // a lane that left for the wave-per-block decoder stores nothing more (its ops may exceed its slot)
  const bool ready = !L.fb && (all ? L.nop > L.nfl : L.nop - L.nfl >= kGroup);
  const uint32_t info = (ready ? 1u : 0u) | (L.nfl & kGroup);
  const uint32_t base = L.out_rel + 4 * L.nfl;
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t o = 16 * j + (lane >> 2), c = lane & 3;
    const uint32_t info_o = __shfl(info, int(o), 64);
    const uint32_t base_o = __shfl(base, int(o), 64);
    const uint8_t* r = oprs + o * kOpStride + (info_o & kGroup) * 4 + 16 * c;  // this wave's op rings
    const v4u v = rd128(r, L.z);
    __builtin_amdgcn_raw_buffer_store_b128(v, R.out, (info_o & 1) ? base_o + 16 * c : kOOB, 0, 0);
  }
  L.nfl += ready ? kGroup : 0u;
}

// ---------------------------------------------------------------- M helpers
// Inclusive wave prefix sum with DPP row shifts and row broadcasts (no LDS round trips).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
  (void)lane;
  int x = int(v);
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return uint32_t(x);
}

// 16 bytes at any position of an LDS buffer, from naturally aligned b64 reads.
__device__ __forceinline__ v4u lds_rd16(const uint8_t* base, uint32_t p, uint32_t z) {
  const uint32_t a = p & ~7u;
  const v2u A = *reinterpret_cast<const v2u*>(base + a);
  const v2u B = *reinterpret_cast<const v2u*>(base + a + 8 + z);
  const v2u C = *reinterpret_cast<const v2u*>(base + a + 16);
  const bool q = (p & 4) != 0;
  const uint32_t e0 = q ? A.y : A.x, e1 = q ? B.x : A.y, e2 = q ? B.y : B.x, e3 = q ? C.x : B.y, e4 = q ? C.y : C.x;
  const uint32_t b = p & 3;
  v4u r;
  r.x = alignb(e1, e0, b);
  r.y = alignb(e2, e1, b);
  r.z = alignb(e3, e2, b);
  r.w = alignb(e4, e3, b);
  return r;
}

// Copy `len` bytes from sb[q..] to out[y..] on this lane, in 64-byte steps: the four 16-byte
// source windows of a step (and the source of the op's last dword) are read first -- one LDS
// round trip -- then the 16 output dwords are written: whole dwords with b32 stores, the op's
// first and last dword byte by byte (a neighbouring op may own the rest of them).  A store
// that is not wanted goes to the lane's junk word, so the wave never branches on data.
// `ordered` (an overlapping copy with offset >= 16) takes 16 bytes per step, so every byte it
// reads was written by an earlier step (LDS keeps a wave's accesses in order).
__device__ __forceinline__ void lane_copy(bool run, bool ordered, const uint8_t* sb, uint32_t q, uint8_t* out,
                                          uint32_t y, uint32_t len, uint8_t* junk, uint32_t z) {
  const uint32_t hb = y & 3u;                    // the op starts hb bytes into its first dword
  const uint32_t span = run ? hb + len : 0u;     // bytes from the first dword's start to the op's end
  uint32_t maxs = span;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) maxs = max(maxs, uint32_t(__shfl_xor(int(maxs), o, 64)));
  const uint32_t step = __ballot(run && ordered) ? 16u : 64u;
  const uint32_t y4 = y - hb, q4 = q - hb;       // source of the first dword's byte 0 (may precede q)
  const uint32_t olast = (span - 1) & ~3u;       // offset of the op's last dword from y4
  for (uint32_t t = 0; t < maxs; t += step) {
    v4u w[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) w[u] = lds_rd16(sb, q4 + t + 16 * (step == 64u ? u : 0u), z);
    const bool last_here = span && olast >= t && olast < t + step;
    const uint32_t wl = lds_rd16(sb, q4 + olast, z).x;  // the op's last dword (when it is partial)
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t wv[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t o = t + 16 * u + 4 * k;   // dword offset from y4
        const bool in_step = u == 0 || step == 64u;
        const bool whole = in_step && o + 4 <= span && (o != 0 || hb == 0);
        *reinterpret_cast<uint32_t*>(whole ? out + y4 + o : junk) = wv[k];
      }
    }
    // partial first dword (bytes hb .. min(4, span)) and partial last dword (bytes 0 .. span - olast)
    const bool first_part = t == 0 && span && (hb != 0 || span < 4);
    const uint32_t w0 = w[0].x;
#pragma unroll
    for (uint32_t i = 1; i < 4; i++) {
      const bool want = first_part && i >= hb && i < span;
      out[want ? y4 + i : uint32_t(junk - out)] = uint8_t(w0 >> (8 * i));
    }
    if (hb == 0) out[(first_part) ? y4 : uint32_t(junk - out)] = uint8_t(w0);
    const bool last_part = last_here && olast != 0 && span - olast < 4;
#pragma unroll
    for (uint32_t i = 0; i < 3; i++) {
      const bool want = last_part && i < span - olast;
      out[want ? y4 + olast + i : uint32_t(junk - out)] = uint8_t(wl >> (8 * i));
    }
    __asm__ volatile("" ::: "memory");
  }
}

}  // namespace

__global__ __launch_bounds__(kLpb3Threads) void decode_lpb3_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  {
    const uint32_t* src = &g_crc16.t[0][0];
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = src[i];
    __syncthreads();
  }
  const uint32_t* crc_init = g_crc_lt.init;
  const uint32_t* crc_tail = g_crc_lt.tail;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  uint8_t* wbase = smem + kTab16Bytes + wave * kWaveBytes;
  // P: input rings then op rings; M: staged input then decoded output
  uint8_t* rings = wbase;            // rings of this wave's lanes (absolute slots below use smem)
  uint8_t* ring = wbase + lane * kInStride;
  uint8_t* oprs = wbase + 64 * kInStride;
  uint8_t* opr = oprs + lane * kOpStride;
  uint8_t* m_in = wbase;
  uint8_t* m_out = wbase + kMCap + kMSlack;
  uint8_t* m_junk = wbase + 2 * (kMCap + kMSlack);  // one junk word per lane for unwanted stores
  const uint32_t waves_total = gridDim.x * (kLpb3Threads / 64);
  const uint32_t wave_g = blockIdx.x * (kLpb3Threads / 64) + wave;
  const uint32_t z = a.rt_zero;

  for (uint32_t round0 = wave_g * 64; round0 < a.n; round0 += waves_total * 64) {
    const uint32_t rend = min(round0 + 64, a.n);
    const uint8_t* in_lo = a.in + a.in_off[round0];
    const uint8_t* in_base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(in_lo) & ~uintptr_t(15));
    const uint8_t* in_hi = a.in + a.in_off[rend];
    Rsrc R;
    R.in = make_rsrc(in_base, align16(uint64_t(in_hi - in_base)));
    uint8_t* out_base = a.out + a.out_off[round0];
    R.out = make_rsrc(out_base, a.out_off[rend] - a.out_off[round0]);

    const uint32_t dbg = dbg_bits(a);
    const uint64_t t_p0 = (dbg & 512) ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t m_rounds = 0, p_iters = 0;
    // ---------------- P: lane l parses block round0 + l
    PLane L;
    const uint32_t b = round0 + lane;
    uint32_t st = b < a.n ? kStDecode : kStNone;
    L.in_rel = L.out_rel = L.sh = L.clen = L.last_chunk = L.dn = L.cap_ops = 0;
    L.crc_last = -1;
    L.crc = 0xFFFFFFFFu;
    L.crc_pos = L.c_issue = L.c_commit = L.n_req = 0;
    L.s = L.d = L.err = L.fb = L.nop = L.nfl = 0;
    L.fin = 1;
    L.z = z;
#pragma unroll
    for (int h = 0; h < kH; h++) {
      L.hy[h] = 0;
      L.hl[h] = 0;
      L.hs[h] = 0;
    }
    if (st == kStDecode) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      const uint64_t region = a.out_off[b + 1] - a.out_off[b];
      if (len < 6) {
        slate_block_meta m{};
        m.status = SLATE_E_BLOCK_TOO_SMALL;
        a.meta[b] = m;
        st = kStDone;
      } else {
        const uint8_t* gin = a.in + s0;
        L.sh = uint32_t(reinterpret_cast<uintptr_t>(gin) & 15);
        if (L.sh + len + 16 > kMCap || region > kMCap - 16) {
          st = kStFallback;
        } else {
          L.in_rel = uint32_t((gin - L.sh) - in_base);
          L.clen = uint32_t(len - 4);
          L.last_chunk = uint32_t((L.sh + len - 1) >> 4);
          L.crc_last = L.clen ? int32_t((L.sh + L.clen - 1) >> 4) : -1;
          L.crc = L.clen ? crc_init[L.sh] : 0xFFFFFFFFu;
          L.out_rel = uint32_t(a.out_off[b] - a.out_off[round0]);
          L.cap_ops = uint32_t(region / 64) * kGroup;
        }
      }
    }
    const bool have = st == kStDecode;
    // the block's first two chunks, then golang/snappy decodedLen (decode.go:20-31)
    {
      const v4u c0 = __builtin_amdgcn_raw_buffer_load_b128(R.in, have ? L.in_rel : kOOB, 0, 0);
      const v4u c1 = __builtin_amdgcn_raw_buffer_load_b128(R.in, (have && L.last_chunk >= 1) ? L.in_rel + 16 : kOOB, 0, 0);
      if (have) {
        wr128(ring, c0, L.z);
        wr128(ring + 16, c1, L.z);
        L.c_commit = L.last_chunk >= 1 ? 2u : 1u;
        L.c_issue = L.c_commit;
        uint64_t x = 0;
        uint32_t sft = 0, hdr = 0;
        bool ok = false, stop = false;
        for (uint32_t i = 0; i < 10 && i < L.clen && !stop; i++) {
          const uint32_t bt = ring[L.sh + i];
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
          L.s = hdr;
          L.fin = 0;
        }
      }
    }
    {
      v4u P0 = {0, 0, 0, 0}, P1 = P0, P2 = P0, P3 = P0;
      uint32_t S0 = 0xFFFFFFFFu, S1 = S0, S2 = S0, S3 = S0;
      const uint32_t rbase = uint32_t(rings - smem);
      uint32_t iters = 0;
      // every iteration commits a chunk, CRCs one or parses a tag while any remain, so a
      // block needs far fewer than `budget` iterations; the budget only bounds the loop
      // (an exhausted lane reports SLATE_E_HIP, never a wrong result)
      const uint32_t budget = have ? L.clen + 1024 : 0u;
      while (__ballot(have && !(L.fin && int32_t(L.crc_pos) > L.crc_last && L.c_commit > L.last_chunk) &&
                      iters < budget)) {
        const bool act =
            have && !(L.fin && int32_t(L.crc_pos) > L.crc_last && L.c_commit > L.last_chunk) && iters < budget;
        commit_one(smem, S0, P0, L.z);
        commit_one(smem, S1, P1, L.z);
        commit_one(smem, S2, P2, L.z);
        commit_one(smem, S3, P3, L.z);
        L.c_commit += L.n_req;
        {
          const uint32_t lo_pos = L.fin ? L.clen : L.s;
          const uint32_t lo_chunk = min((L.sh + lo_pos) >> 4, L.crc_pos);
          const uint32_t room = lo_chunk + kNS - L.c_issue, left = L.last_chunk + 1 - L.c_issue;
          const uint32_t n = act ? min(min(room, left), 4u) : 0u;
          const uint32_t info = (L.c_issue << 3) | n;
          load_one(0, lane, rbase, info, L.in_rel, R, P0, S0);
          load_one(1, lane, rbase, info, L.in_rel, R, P1, S1);
          load_one(2, lane, rbase, info, L.in_rel, R, P2, S2);
          load_one(3, lane, rbase, info, L.in_rel, R, P3, S3);
          L.c_issue += n;
          L.n_req = n;
        }
#pragma unroll
        for (uint32_t k = 0; k < kCrcSteps; k++) crc_step(L, ring, tab, act);
#pragma unroll
        for (uint32_t k = 0; k < kTagSteps; k++) tag_step(L, ring, opr, act);
        if (__ballot(L.nop - L.nfl >= kGroup)) flush_ops(L, false, oprs, lane, R);
        iters++;
      }
      p_iters = iters;
      if (have && !(L.fin && int32_t(L.crc_pos) > L.crc_last && L.c_commit > L.last_chunk)) {
        slate_block_meta m{};
        m.status = SLATE_E_HIP;  // iteration budget exhausted: a kernel defect, reported loudly
        a.meta[b] = m;
        st = kStDone;
      }
    }
    flush_ops(L, true, oprs, lane, R);
    __builtin_amdgcn_s_waitcnt(0);  // the op stores are in L2 before M reads them (sc1)
    // P verdict: checksum first (block.go:84-88), then the Snappy stream (compression.go:132)
    if (st == kStDecode) {
      if (L.fb) {
        st = kStFallback;
      } else {
        const uint32_t stored = __builtin_bswap32(ring_rd8(ring, L.sh + L.clen, kIR - 8).x);
        const uint32_t t = L.clen ? uint32_t(16 * (L.crc_last + 1)) - (L.sh + L.clen) : 0u;
        const bool crc_ok = gf2_mulmod(~stored, crc_tail[t]) == L.crc;
        const bool snappy_ok = !L.err && L.d == L.dn && L.s == L.clen;
        if (!crc_ok || !snappy_ok) {
          slate_block_meta m{};
          m.status = !crc_ok ? SLATE_E_BLOCK_CHECKSUM : SLATE_E_SNAPPY_CORRUPT;
          a.meta[b] = m;
          st = kStDone;
        }
      }
    }
    if (st == kStFallback) a.fb_list[atomicAdd(a.fb_count, 1u)] = b;
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");

    const uint64_t t_p1 = (dbg & 512) ? __builtin_amdgcn_s_memtime() : 0;
    // ---------------- M: the wave materializes each decodable block of the round.  The next
    // block's first 4 KiB of input and first 192 ops are loaded while this one is decoded.
    uint64_t todo = (dbg & (1u << 22)) ? 0 : __ballot(st == kStDecode);  // 1 << 22: P only (profiling)
    v4u pin[4];
    uint32_t pop[3];
    auto prefetch = [&](uint32_t j) {
      const uint32_t sh = __builtin_amdgcn_readlane(L.sh, j), clen = __builtin_amdgcn_readlane(L.clen, j);
      const uint32_t in_rel = __builtin_amdgcn_readlane(L.in_rel, j), out_rel = __builtin_amdgcn_readlane(L.out_rel, j);
      const uint32_t nop = __builtin_amdgcn_readlane(L.nop, j);
      const uint32_t nch = (sh + clen + 15) >> 4;
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t c = u * 64 + lane;
        pin[u] = __builtin_amdgcn_raw_buffer_load_b128(R.in, c < nch ? in_rel + 16 * c : kOOB, 0, 0);
      }
#pragma unroll
      for (uint32_t u = 0; u < 3; u++) {
        const uint32_t k = u * 64 + lane;
        pop[u] = __builtin_amdgcn_raw_buffer_load_b32(R.out, k < nop ? out_rel + 4 * k : kOOB, 0, kSc1);
      }
    };
    if (todo) prefetch(uint32_t(__builtin_ctzll(todo)));
    while (todo) {
      const uint32_t j = uint32_t(__builtin_ctzll(todo));
      todo &= todo - 1;
      const uint32_t bj = round0 + j;
      const uint32_t sh = __builtin_amdgcn_readlane(L.sh, j);
      const uint32_t clen = __builtin_amdgcn_readlane(L.clen, j);
      const uint32_t dn = __builtin_amdgcn_readlane(L.dn, j);
      const uint32_t in_rel = __builtin_amdgcn_readlane(L.in_rel, j);
      const uint32_t out_rel = __builtin_amdgcn_readlane(L.out_rel, j);
      const uint32_t nop = __builtin_amdgcn_readlane(L.nop, j);
      // stage the compressed block: the prefetched first 256 chunks, then any rest
      const uint32_t nch = (sh + clen + 15) >> 4;
      uint32_t cur_op[3];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t c = u * 64 + lane;
        if (c < nch) *reinterpret_cast<v4u*>(m_in + 16 * c) = pin[u];
      }
#pragma unroll
      for (uint32_t u = 0; u < 3; u++) cur_op[u] = pop[u];
      for (uint32_t c = 256 + lane; c < nch; c += 64)
        *reinterpret_cast<v4u*>(m_in + 16 * c) = __builtin_amdgcn_raw_buffer_load_b128(R.in, in_rel + 16 * c, 0, 0);
      if (todo) prefetch(uint32_t(__builtin_ctzll(todo)));
      __asm__ volatile("" ::: "memory");
      // ops in batches of 64, one per lane
      uint32_t yb = 0;
      bool stuck = false;  // a batch that needs more rounds than it has ops: a kernel defect
      for (uint32_t k0 = 0; k0 < nop; k0 += 64) {
        const bool valid = k0 + lane < nop;
        const uint32_t op = k0 < 192 ? (k0 == 0 ? cur_op[0] : (k0 == 64 ? cur_op[1] : cur_op[2]))
                                     : __builtin_amdgcn_raw_buffer_load_b32(
                                           R.out, valid ? out_rel + 4 * (k0 + lane) : kOOB, 0, kSc1);
        const uint32_t len = valid ? ((op >> kLenShift) & 0x3fffu) + 1 : 0u;
        const bool copy = valid && (op & kOpCopy) != 0;
        const uint32_t srcf = op & kSrcMask;
        const uint32_t incl = wave_incl_scan(len, lane);
        const uint32_t y = yb + incl - len;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t q = copy ? y - srcf : srcf;  // source position (decoded output / staged input)
        const bool coop = copy && srcf < 16 && srcf < len;  // overlapping copy with a short period
        const bool ordered = copy && srcf < len;            // overlapping copy with a period >= 16
        const uint32_t need_end = copy ? q + min(len, srcf) : 0u;
        bool pending = valid;
        bool run = valid && (!copy || need_end <= yb);
        uint64_t done = 0, dep = 0;
        bool deps_known = false;
        for (uint32_t rounds = 0;; rounds++) {
          m_rounds++;
          if (rounds > 64) {
            stuck = true;
            break;
          }
          // copies with a short period: the wave writes one at a time, lane i byte i
          const uint64_t cm = __ballot(run && coop);
          lane_copy(run && !coop, ordered, copy ? m_out : m_in, q, m_out, y, len, m_junk + 4 * lane, z);
          for (uint64_t r = cm; r; r &= r - 1) {
            const uint32_t qq = uint32_t(__builtin_ctzll(r));
            const uint32_t yy = __builtin_amdgcn_readlane(y, qq), ll = __builtin_amdgcn_readlane(len, qq);
            const uint32_t ff = __builtin_amdgcn_readlane(srcf, qq);
            if (lane < ll) m_out[yy + lane] = m_out[yy - ff + lane % ff];
            __asm__ volatile("" ::: "memory");
          }
          done |= __ballot(run);
          pending = pending && !run;
          if (!__ballot(pending)) break;
          if (!deps_known) {
            // ops whose output overlaps a pending copy's source bytes [q, need_end)
            for (uint64_t r = __ballot(pending); r; r &= r - 1) {
              const uint32_t qq = uint32_t(__builtin_ctzll(r));
              const uint32_t qs = __builtin_amdgcn_readlane(q, qq), qe = __builtin_amdgcn_readlane(need_end, qq);
              const uint64_t hi = __ballot(valid && y < qe), lo = __ballot(valid && y + len <= qs);
              dep = lane == qq ? (hi & ~lo) : dep;
            }
            deps_known = true;
          }
          __asm__ volatile("" ::: "memory");
          run = pending && (dep & ~done) == 0;
        }
        yb += total;
      }
      __builtin_amdgcn_wave_barrier();
      __asm__ volatile("" ::: "memory");
      // block.Decode structure checks (block.go:95-131) over the decoded block in LDS
      slate_block_meta m{};
      if (stuck || yb != dn) {
        m.status = SLATE_E_HIP;  // reported loudly, never a wrong result
        if (lane == 0) a.meta[bj] = m;
        continue;
      }
      const uint8_t* buf = m_out;
      const uint32_t n = dn;
      {
        const uint32_t chunks = (n + 15) / 16;
        for (uint32_t c = lane; c < chunks; c += 64)
          __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u*>(buf + 16 * c), R.out, out_rel + 16 * c,
                                                 0, 0);
      }
      bool rows_go = false;
      uint32_t cnt = 0, osi_u = 0;
      if (n < 2) {
        m.status = SLATE_E_BLOCK_UNCOMP_SMALL;
      } else {
        cnt = ld_be16(buf + n - 2);
        const int64_t osi = int64_t(n) - 2 - 2 * int64_t(cnt);
        if (osi <= 0) {
          m.status = SLATE_E_BLOCK_INDEX_OFFSET;
          m.detail = int32_t(osi);
        } else {
          const uint16_t osi16 = uint16_t(osi);
          uint32_t bad = 0xFFFFFFFFu;
          for (uint32_t i = lane; i < cnt; i += 64)
            if (ld_be16(buf + osi + 2 * i) > osi16 && i < bad) bad = i;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) bad = min(bad, uint32_t(__shfl_xor(int(bad), o, 64)));
          if (bad != 0xFFFFFFFFu) {
            m.status = SLATE_E_BLOCK_OFFSET_BOUNDS;
            m.aux = uint16_t(bad);
            m.detail = ld_be16(buf + osi + 2 * bad);
          } else {
            m.data_len = uint32_t(osi);
            m.n_rows = uint16_t(cnt);
            if (cnt == 0) {
              m.status = SLATE_E_BLOCK_NO_OFFSETS;
            } else {
              const uint32_t off0 = ld_be16(buf + osi);
              if (uint64_t(osi) - off0 < 2) {
                m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
              } else {
                const uint16_t kl = ld_be16(buf + off0);
                const uint16_t lo = uint16_t(off0 + 2), hi = uint16_t(off0 + 2 + kl);
                if (lo > hi || hi > n) {
                  m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
                } else {
                  m.aux = kl;
                  rows_go = true;
                  osi_u = uint32_t(osi);
                }
              }
            }
          }
        }
      }
      if (rows_go && !(dbg & (1u << 23))) {  // 1 << 23: no row descriptors (profiling)
        // row descriptors: row 0 against firstKey = nil, the others against row 0's key
        const uint64_t rb = a.row_base[bj];
        const uint32_t rcap = uint32_t(min(uint64_t(0xFFFFFFFFu), a.row_base[bj + 1] - rb));
        uint32_t nr = cnt;
        if (nr > rcap) {
          nr = rcap;
          m.flags |= SLATE_BLKF_ROWS_TRUNCATED;
        }
        int fk = -1;
        {
          slate_row r0;
          uint32_t sl0;
          decode_row(buf, osi_u, ld_be16(buf + osi_u), -1, r0, &sl0);
          if (r0.status == SLATE_OK) fk = int(sl0);
        }
        slate_row* grows = a.rows + rb;
        for (uint32_t i = lane; i < nr; i += 64) {
          slate_row r;
          uint32_t sl;
          decode_row(buf, osi_u, ld_be16(buf + osi_u + 2 * i), i == 0 ? -1 : fk, r, &sl);
          grows[i] = r;
        }
      }
      if (lane == 0) a.meta[bj] = m;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this block's LDS reads are done before the next staging
      __builtin_amdgcn_wave_barrier();
      __asm__ volatile("" ::: "memory");
    }
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
    if ((dbg & 512) && lane == 0 && round0 + 3 < a.n) {
      // profiling only: P cycles, M cycles, M rounds and P iterations of this round, in meta.detail
      const uint64_t t_m1 = __builtin_amdgcn_s_memtime();
      a.meta[round0].detail = int32_t(t_p1 - t_p0);
      a.meta[round0 + 1].detail = int32_t(t_m1 - t_p1);
      a.meta[round0 + 2].detail = int32_t(m_rounds);
      a.meta[round0 + 3].detail = int32_t(p_iters);
    }
  }
}

size_t lpb3_lds_bytes() { return kTab16Bytes + size_t(kLpb3Threads / 64) * kWaveBytes; }

hipError_t launch_decode_lpb3(hipStream_t st, const DecodeArgs& a, int num_cus) {
  if (a.n == 0) return hipGetLastError();
  const size_t lds = lpb3_lds_bytes();
  const uint32_t waves_needed = (a.n + 63) / 64;
  uint32_t grid = (waves_needed + kLpb3Threads / 64 - 1) / (kLpb3Threads / 64);
  grid = min(grid, uint32_t(num_cus) * uint32_t(163840 / lds));
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_lpb3_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
  if (attr != hipSuccess) return attr;
  decode_lpb3_kernel<<<grid, kLpb3Threads, lds, st>>>(a);
  return hipGetLastError();
}

}  // namespace slate
