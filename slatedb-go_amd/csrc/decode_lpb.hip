// Lane-per-block Snappy block decode (the headline kernel).
//
// block.Decode (internal/sstable/block/block.go:78-134) with CodecSnappy:
// CRC32 verify -> golang/snappy v0.0.4 decode (decode_other.go semantics) ->
// offset checks -> row descriptors (row.go:191-261 as block/iterator.go walks).
//
// Why lane-per-block: the Snappy tag stream is a serial chain inside a block,
// so a wavefront working on ONE block pays a whole wave instruction per tag.
// Here each of the 64 lanes decodes its own block, so one wave instruction
// advances 64 tag streams.  Per lane, LDS holds
//   * an input ring (8 x 16-byte chunks + mirror).  The encoded block streams in
//     with one global_load_dwordx4 per 16 bytes, issued kPf steps before it is
//     committed to LDS (software pipeline over a wave-uniform step counter, so
//     the s_waitcnt for a chunk never waits on a younger load); the CRC32 is
//     absorbed chunk by chunk at commit (slicing-by-4 tables shared in LDS);
//   * an output ring (256 bytes + mirrors).  Copies with offset <= 236 read it
//     with unaligned ds_read_b32 (correct and fast on gfx950, tools/lds_probe.hip);
//     longer offsets read the already-flushed output in HBM.
// Each completed 16-byte output chunk is flushed with one global_store_dwordx4
// (output is 16-byte aligned per block, see the plan kernel).  A row walker reads
// each row's header fields from the output ring as soon as they are produced, so
// row descriptors need no second pass; they are checked against the block's
// offset array when the block completes (exact fallback re-derives descriptors
// from HBM if the walk and the offsets disagree).
// The 64 lanes of a wave run their blocks in lockstep rounds so the per-block
// finalisation (offset checks, row verification) runs SIMD-parallel.
#include "common.h"
#include "kernels.h"
#include "wave_crc.h"

namespace slate {

typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) v4u gv4u;  // global-memory view

namespace {

constexpr uint32_t kRing = 256;                  // output ring bytes
constexpr uint32_t kReach = kRing - 20;          // copies with off <= kReach read the ring
constexpr uint32_t kSlots = 8;                   // input ring chunks
constexpr uint32_t kInBytes = kSlots * 16;
// per-lane LDS: [pre 16 | out ring 256 | post 16 | in ring 128 | in mirror 16]
constexpr uint32_t kOutOff = 16;
constexpr uint32_t kInOff = 16 + kRing + 16;
constexpr uint32_t kLaneStride = kInOff + kInBytes + 16;  // 432

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<u32u*>(p) = v; }
__device__ __forceinline__ uint32_t be16_of(uint32_t w) { return ((w & 0xff) << 8) | ((w >> 8) & 0xff); }

// dword write at ring position x (0..255) keeping the mirrors coherent: bytes
// that spill past 255 also land at 0..2, and writes near 0 are copied past 255
// so that a 4-byte read at any position <= 255 sees the current bytes.
__device__ __forceinline__ void ring_st32(uint8_t* ring, uint32_t x, uint32_t v) {
  st32(ring + x, v);
  if (x < 3) st32(ring + kRing + x, v);
  if (x > kRing - 4) st32(ring + x - kRing, v);
}

enum : uint32_t { kHeader = 0, kDecoding = 1, kTail = 2, kDone = 3 };
enum : uint32_t { kLit = 0, kRingCopy = 1, kHbmCopy = 2, kShortCopy = 3 };

struct Lane {
  const uint8_t* gin;   // block bytes
  uint8_t* gout;        // decoded block (16-byte aligned)
  slate_row* grows;
  uint32_t sh, clen, dn, last_chunk;
  uint32_t s, c_issue, c_commit, pend, crc;
  uint32_t rem, src, off, kind;
  uint32_t d, fl, err, phase;
  uint32_t R, rphase, rneed, rsl, ro, rflags, rpl, nwalk, rcap;
};

// commit the 16-byte chunk c_commit (loaded kPf steps ago) into the input ring and
// absorb its message bytes into the CRC
__device__ __forceinline__ void commit_chunk(Lane& L, uint8_t* in, const uint32_t* tab, const v4u v) {
  const uint32_t k = L.c_commit++;
  uint8_t* slot = in + (k & (kSlots - 1)) * 16;
  *reinterpret_cast<v4u*>(slot) = v;
  if ((k & (kSlots - 1)) == 0) *reinterpret_cast<v4u*>(in + kInBytes) = v;
  const int32_t lo = int32_t(16 * k) - int32_t(L.sh), hi = lo + 16;
  const int32_t mlo = lo < 0 ? 0 : lo, mhi = hi > int32_t(L.clen) ? int32_t(L.clen) : hi;
  uint32_t c = L.crc;
  if (mlo == lo && mhi == hi) {
    c = crc_word(tab, c, v.x);
    c = crc_word(tab, c, v.y);
    c = crc_word(tab, c, v.z);
    c = crc_word(tab, c, v.w);
  } else {
    for (int32_t i = mlo; i < mhi; i++) c = tab[(c ^ slot[i - lo]) & 0xff] ^ (c >> 8);
  }
  L.crc = c;
}

// v0 row decode (row.go:191-261) reading the decoded block from HBM: the exact
// fallback when the streaming walk does not match the offset array.
__device__ void row_from_hbm(const uint8_t* data, uint32_t data_len, uint32_t off, int fk, slate_row& r,
                             uint32_t* sl_out) {
  r.row_off = off;
  r.key_prefix_len = 0;
  r.key_suffix_len = 0;
  r.value_len = 0;
  r.flags = 0;
  r.meta_len = 0;
  *sl_out = 0;
  const uint8_t* p = data + off;
  const uint32_t n = data_len - off;
  if (n >= 4) {
    r.key_prefix_len = ld_be16(p);
    r.key_suffix_len = ld_be16(p + 2);
  }
  if (n < 13) { r.status = SLATE_E_ROW_TOO_SHORT; return; }
  const uint16_t pl = r.key_prefix_len, sl = r.key_suffix_len;
  if (pl > uint16_t(fk < 0 ? 0 : fk)) { r.status = SLATE_E_ROW_PREFIX; return; }
  uint32_t o = 4;
  if (n - o < sl) { r.status = SLATE_E_ROW_SUFFIX; return; }
  o += sl;
  if (n - o < 9) { r.status = SLATE_E_ROW_PANIC; return; }
  const uint8_t flags = p[o + 8];
  o += 9;
  if (flags & 2) {
    if (n - o < 8) { r.status = SLATE_E_ROW_EXPIRE; return; }
    o += 8;
  }
  if (flags & 4) {
    if (n - o < 8) { r.status = SLATE_E_ROW_CREATE; return; }
    o += 8;
  }
  if ((flags & 1) == 0) {
    if (n - o < 4) { r.status = SLATE_E_ROW_VALUE_LEN; return; }
    const uint32_t vl = ld_be32(p + o);
    o += 4;
    if (n - o < vl) { r.status = SLATE_E_ROW_VALUE; return; }
    r.value_len = vl;
  }
  r.flags = flags & 7;
  r.meta_len = uint8_t(o - 4 - sl);
  r.status = SLATE_OK;
  *sl_out = sl;
}

// golang/snappy decodedLen (decode.go:20-31) over the committed input ring
__device__ __forceinline__ void parse_header(Lane& L, const uint8_t* in) {
  uint64_t x = 0;
  uint32_t sft = 0, hdr = 0;
  bool ok = false;
  for (uint32_t i = 0; i < L.clen && i < 10; i++) {
    const uint32_t bt = in[(L.sh + i) & (kInBytes - 1)];
    if (bt < 0x80) {
      if (i == 9 && bt > 1) break;
      x |= uint64_t(bt) << sft;
      ok = x <= 0xffffffffull;
      hdr = i + 1;
      break;
    }
    x |= uint64_t(bt & 0x7f) << sft;
    sft += 7;
  }
  if (!ok || x > kSnappyMaxExpansion * uint64_t(L.clen)) {
    L.err = 1;
    L.phase = kTail;
  } else {
    L.dn = uint32_t(x);
    L.s = hdr;
    L.phase = kDecoding;
  }
}

// Row walker: read the header fields of the row at R from the output ring as soon
// as they are complete (row.go:191-261 field order).
__device__ __forceinline__ void walk_rows(Lane& L, const uint8_t* ring) {
  for (int step = 0; step < 4 && L.d >= L.rneed; step++) {
    if (L.rphase == 0) {
      if (L.d - L.R > kReach) { L.rphase = 4; L.rneed = 0xFFFFFFFFu; break; }
      const uint32_t w = ld32(ring + (L.R & (kRing - 1)));
      L.rpl = be16_of(w);
      L.rsl = be16_of(w >> 16);
      L.rneed = L.R + 4 + L.rsl + 9;
      L.rphase = 1;
    } else if (L.rphase == 1) {
      const uint32_t fp = L.R + 4 + L.rsl + 8;
      if (L.d - fp > kReach) { L.rphase = 4; L.rneed = 0xFFFFFFFFu; break; }
      L.rflags = ring[fp & (kRing - 1)];
      L.ro = 4 + L.rsl + 9 + ((L.rflags & 2) ? 8 : 0) + ((L.rflags & 4) ? 8 : 0);
      if (L.rflags & 1) {
        L.rphase = 3;  // tombstone: the row ends after the metadata
        L.rneed = L.R + L.ro;
      } else {
        L.rneed = L.R + L.ro + 4;
        L.rphase = 2;
      }
    } else {
      uint32_t vl = 0, rlen = L.ro;
      if (L.rphase == 2) {
        const uint32_t vp = L.R + L.ro;
        if (L.d - vp > kReach) { L.rphase = 4; L.rneed = 0xFFFFFFFFu; break; }
        vl = __builtin_bswap32(ld32(ring + (vp & (kRing - 1))));
        rlen = L.ro + 4;
      }
      if (L.nwalk < L.rcap) {
        slate_row r;
        r.row_off = L.R;
        r.key_prefix_len = uint16_t(L.rpl);
        r.key_suffix_len = uint16_t(L.rsl);
        r.value_len = vl;
        r.flags = uint8_t(L.rflags & 7);
        r.meta_len = uint8_t(rlen - 4 - L.rsl);
        r.status = SLATE_OK;
        L.grows[L.nwalk] = r;
      }
      L.nwalk++;
      const uint64_t next = uint64_t(L.R) + rlen + vl;
      if (next > L.dn) {
        L.rphase = 4;  // ran past the block: stop walking
        L.rneed = 0xFFFFFFFFu;
      } else {
        L.R = uint32_t(next);
        L.rphase = 0;
        L.rneed = L.R + 4;
      }
    }
  }
}

// One pipeline step: commit the chunk that landed in P, issue the next chunk
// load into P, then advance the lane's decode by up to 16 output bytes.
__device__ __forceinline__ void lane_step(Lane& L, v4u& P, uint32_t bit, bool have, uint8_t* ring, uint8_t* in,
                                          const uint32_t* tab, const v4u* dummy) {
  if (L.pend & bit) {
    commit_chunk(L, in, tab, P);
    L.pend &= ~bit;
  }
  // keep the next load below the commit: the old and new P then share registers
  // and the loop-carried value needs no copy (a copy would wait on the load)
  __asm__ volatile("" ::: "memory");
  {
    // window of chunks the ring must keep: from the oldest byte still to be read
    const uint32_t lo_pos = L.phase == kHeader ? 0u
                            : L.phase == kTail ? L.clen
                            : (L.rem && L.kind == kLit) ? L.src : L.s;
    const uint32_t lo_chunk = (L.sh + lo_pos) >> 4;
    const bool room = have && L.c_issue <= L.last_chunk && L.c_issue < lo_chunk + kSlots;
    const uint64_t real = reinterpret_cast<uint64_t>(L.gin - L.sh) + 16 * uint64_t(L.c_issue);
    gv4u* ap = reinterpret_cast<gv4u*>(room ? real : reinterpret_cast<uint64_t>(dummy));
    // always issued (one dwordx4, read-once data): keeps the wave's load order, and so
    // s_waitcnt, static
    P = __builtin_nontemporal_load(ap);
    if (room) {
      L.pend |= bit;
      L.c_issue++;
    }
  }
  if (!have) return;
  const int32_t avail = int32_t(16 * L.c_commit) - int32_t(L.sh);  // committed input bytes [0, avail)
  if (L.phase == kHeader) {
    if (avail >= int32_t(L.clen < 10 ? L.clen : 10)) parse_header(L, in);
    return;
  }
  if (L.phase == kTail) {
    if (L.c_commit > L.last_chunk) L.phase = kDone;
    return;
  }
  if (L.phase != kDecoding) return;
  const uint32_t sn = L.clen;
  // ---- parse the next tag (golang/snappy decode_other.go:19-110)
  if (L.rem == 0) {
    if (L.err || L.s >= sn) {
      L.phase = kTail;
      return;
    }
    if (avail < int32_t(min(L.s + 5, sn))) return;  // tag bytes still in flight
    const uint32_t q = (L.sh + L.s) & (kInBytes - 1);
    const uint32_t w0 = ld32(in + q), w1 = ld32(in + q + 4);
    const uint32_t c = w0 & 0xff, t = c & 3;
    if (t == 0) {
      uint32_t xl = c >> 2, hl = 1;
      if (xl >= 60) {
        const uint32_t nb = xl - 59;
        hl = 1 + nb;
        const uint32_t tail = (w0 >> 8) | (w1 << 24);  // bytes s+1 .. s+4
        xl = nb == 4 ? tail : (tail & ((1u << (8 * nb)) - 1));
      }
      if (L.s + hl > sn) { L.err = 1; return; }
      L.s += hl;
      const uint64_t len = uint64_t(xl) + 1;
      if (len > uint64_t(L.dn - L.d) || len > uint64_t(sn - L.s)) { L.err = 1; return; }
      L.kind = kLit;
      L.src = L.s;
      L.rem = uint32_t(len);
      L.s += uint32_t(len);
    } else {
      uint32_t hl, len, off;
      if (t == 1) {
        hl = 2;
        len = 4 + ((c >> 2) & 7);
        off = ((c & 0xe0) << 3) | ((w0 >> 8) & 0xff);
      } else if (t == 2) {
        hl = 3;
        len = 1 + (c >> 2);
        off = (w0 >> 8) & 0xffff;
      } else {
        hl = 5;
        len = 1 + (c >> 2);
        off = (w0 >> 8) | (w1 << 24);
      }
      if (L.s + hl > sn) { L.err = 1; return; }
      L.s += hl;
      if (off == 0 || L.d < off || len > L.dn - L.d) { L.err = 1; return; }
      L.src = L.d - off;
      L.off = off;
      L.rem = len;
      L.kind = off < 4 ? kShortCopy : (off <= kReach ? kRingCopy : kHbmCopy);
    }
  }
  // ---- emit up to 16 bytes of the current tag into the output ring
  uint32_t k = L.rem < 16 ? L.rem : 16;
  const uint32_t x = L.d & (kRing - 1);
  if (L.kind == kLit) {
    const int32_t have_in = avail - int32_t(L.src);
    if (have_in <= 0) return;  // literal bytes still in flight
    if (int32_t(k) > have_in) k = uint32_t(have_in);
    const uint32_t q0 = L.sh + L.src;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
      ring_st32(ring, (x + 4 * j) & (kRing - 1), ld32(in + ((q0 + 4 * j) & (kInBytes - 1))));
  } else if (L.kind == kRingCopy) {
    if (k > L.off) k = L.off;  // read only bytes already written
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
      ring_st32(ring, (x + 4 * j) & (kRing - 1), ld32(ring + ((L.src + 4 * j) & (kRing - 1))));
  } else if (L.kind == kShortCopy) {
    // offset 1..3: the output is periodic; build the pattern from the last off bytes
    const uint32_t v = ld32(ring + ((L.d - L.off) & (kRing - 1)));
    uint32_t p0, p1, p2;
    if (L.off == 1) {
      p0 = p1 = p2 = (v & 0xff) * 0x01010101u;
    } else if (L.off == 2) {
      p0 = p1 = p2 = (v & 0xffff) * 0x00010001u;
    } else {
      const uint32_t tt = v & 0xffffff;
      p0 = tt | (tt << 24);
      p1 = (tt >> 8) | (tt << 16);
      p2 = (tt >> 16) | (tt << 8);
    }
    // dword j starts at phase (4j) mod off of the pattern
    ring_st32(ring, x, p0);
    ring_st32(ring, (x + 4) & (kRing - 1), p1);
    ring_st32(ring, (x + 8) & (kRing - 1), p2);
    ring_st32(ring, (x + 12) & (kRing - 1), p0);
  } else {
    // the source was flushed to HBM long ago (off > kReach): aligned loads + funnel shift
    const uint32_t a0 = L.src & ~3u, sb = (L.src & 3u) * 8;
    const uint32_t* g = reinterpret_cast<const uint32_t*>(L.gout + a0);
    uint32_t w[5];
#pragma unroll
    for (int j = 0; j < 5; j++) w[j] = g[j];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t val = sb ? ((w[j] >> sb) | (w[j + 1] << (32 - sb))) : w[j];
      ring_st32(ring, (x + 4 * j) & (kRing - 1), val);
    }
  }
  L.d += k;
  L.src += k;
  L.rem -= k;
  // ---- flush the completed 16-byte chunk (at most one per step)
  if ((L.d >> 4) > L.fl) {
    const uint4 v = *reinterpret_cast<const uint4*>(ring + ((L.fl * 16) & (kRing - 1)));
    reinterpret_cast<uint4*>(L.gout)[L.fl] = v;
    L.fl++;
  }
  walk_rows(L, ring);
}

}  // namespace

__global__ __launch_bounds__(kLpbThreads) void decode_lpb_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(smem);
  load_crc_tables(tab);
  uint8_t* region = smem + kTabBytes + threadIdx.x * kLaneStride;
  uint8_t* ring = region + kOutOff;
  uint8_t* in = region + kInOff;
  const v4u* dummy = reinterpret_cast<const v4u*>(a.large_count);  // 16 readable scratch bytes
  const uint32_t waves_total = gridDim.x * (kLpbThreads / 64);
  const uint32_t wave_g = blockIdx.x * (kLpbThreads / 64) + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;

  for (uint32_t round0 = wave_g * 64; round0 < a.n; round0 += waves_total * 64) {
    Lane L;
    v4u P0 = {0, 0, 0, 0}, P1 = P0, P2 = P0, P3 = P0;
    const uint32_t b = round0 + lane;
    slate_block_meta m{};
    bool have = b < a.n;
    L.pend = 0;
    L.phase = kDone;
    L.gin = nullptr;
    L.sh = 0;
    L.c_issue = L.c_commit = 0;
    L.last_chunk = 0;
    if (have) {
      const uint64_t s0 = a.in_off[b], len = a.in_off[b + 1] - s0;
      if (len < (a.raw ? 4u : 6u)) {
        m.status = SLATE_E_BLOCK_TOO_SMALL;
        a.meta[b] = m;
        have = false;
      } else {
        L.gin = a.in + s0;
        L.sh = uint32_t(reinterpret_cast<uintptr_t>(L.gin) & 15);
        L.clen = uint32_t(len - 4);
        L.last_chunk = uint32_t((L.sh + len - 1) >> 4);
        L.gout = a.out + a.out_off[b];
        const uint64_t rb = a.row_base[b];
        L.grows = a.rows + rb;
        L.rcap = uint32_t(min<uint64_t>(a.row_base[b + 1] - rb, 0xFFFFFFFFull));
        L.crc = 0xFFFFFFFFu;
        L.dn = 0;
        L.s = 0;
        L.d = L.fl = L.err = 0;
        L.rem = L.src = L.off = L.kind = 0;
        L.phase = kHeader;
        L.R = 0;
        L.rphase = 0;
        L.rneed = 4;
        L.nwalk = 0;
        L.rsl = L.ro = L.rflags = L.rpl = 0;
      }
    }

    // ---------------- streaming decode, 64 blocks in lockstep, 4-deep load pipeline
    while (__ballot(have && L.phase != kDone)) {
      const bool act = have && L.phase != kDone;
      lane_step(L, P0, 1u, act, ring, in, tab, dummy);
      lane_step(L, P1, 2u, act, ring, in, tab, dummy);
      lane_step(L, P2, 4u, act, ring, in, tab, dummy);
      lane_step(L, P3, 8u, act, ring, in, tab, dummy);
    }

    // ---------------- finalise the round's blocks (SIMD across lanes)
    if (have) {
      const uint32_t stored = __builtin_bswap32(ld32(in + ((L.sh + L.clen) & (kInBytes - 1))));
      const bool snappy_ok = !L.err && L.d == L.dn && L.s == L.clen && L.rem == 0;
      const uint32_t dn = L.dn;
      if (stored != ~L.crc) {
        m.status = SLATE_E_BLOCK_CHECKSUM;
      } else if (!snappy_ok) {
        m.status = SLATE_E_SNAPPY_CORRUPT;
      } else {
        // remaining output chunks (the last one is padded inside its 16-byte slot)
        while (L.fl * 16 < dn) {
          const uint4 v = *reinterpret_cast<const uint4*>(ring + ((L.fl * 16) & (kRing - 1)));
          reinterpret_cast<uint4*>(L.gout)[L.fl] = v;
          L.fl++;
        }
        // let the row walker catch up on the block's last bytes (still in the ring)
        for (int i = 0; i < 16 && L.d >= L.rneed; i++) walk_rows(L, ring);
        if (a.raw) {
          m.data_len = dn;  // a decompressed index / filter buffer
        } else if (dn < 2) {
          m.status = SLATE_E_BLOCK_UNCOMP_SMALL;
        } else {
          // block.go:101-134 over the decoded block, now in HBM (this lane's own stores)
          const uint8_t* buf = L.gout;
          const uint32_t cnt = ld_be16(buf + dn - 2);
          const int64_t osi = int64_t(dn) - 2 - 2 * int64_t(cnt);
          if (osi <= 0) {
            m.status = SLATE_E_BLOCK_INDEX_OFFSET;
            m.detail = int32_t(osi);
          } else {
            const uint16_t osi16 = uint16_t(osi);
            uint32_t bad = 0xFFFFFFFFu;
            const uint32_t nr = cnt < L.rcap ? cnt : L.rcap;
            bool walk_ok = L.nwalk >= nr;
            for (uint32_t i = 0; i < cnt; i++) {
              const uint16_t ofs = ld_be16(buf + osi + 2 * i);
              if (ofs > osi16) {
                bad = i;
                break;
              }
              if (i < nr && walk_ok && L.grows[i].row_off != ofs) walk_ok = false;
            }
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
                  if (lo > hi || hi > dn) {
                    m.status = SLATE_E_BLOCK_FIRSTKEY_PANIC;
                  } else {
                    m.aux = kl;
                    if (cnt > L.rcap) m.flags |= SLATE_BLKF_ROWS_TRUNCATED;
                    // walked rows are exact when they start where the offsets say and
                    // the last one ends inside Data; prefixes are checked against row 0
                    if (walk_ok) {
                      uint32_t end_last = 0;
                      if (L.nwalk > nr) {
                        if (nr >= L.rcap) walk_ok = false;  // the next start was not recorded
                        else end_last = L.grows[nr].row_off;
                      } else {
                        if (L.rphase == 4) walk_ok = false;
                        end_last = L.R;
                      }
                      if (walk_ok && end_last > uint32_t(osi)) walk_ok = false;
                    }
                    if (walk_ok) {
                      // a row failing the prefix check keeps only its key lengths (row.go:203-206)
                      const uint32_t fk0 = L.grows[0].key_suffix_len;
                      const bool fk_nil = L.grows[0].key_prefix_len != 0;  // row 0 itself fails
                      for (uint32_t i = 0; i < nr; i++) {
                        const uint32_t pl = L.grows[i].key_prefix_len;
                        if (i == 0 ? fk_nil : (fk_nil ? pl != 0 : pl > fk0)) {
                          slate_row r = L.grows[i];
                          r.value_len = 0;
                          r.flags = 0;
                          r.meta_len = 0;
                          r.status = SLATE_E_ROW_PREFIX;
                          L.grows[i] = r;
                        }
                      }
                    } else {
                      int fk = -1;
                      for (uint32_t i = 0; i < nr; i++) {
                        slate_row r;
                        uint32_t sl;
                        row_from_hbm(buf, uint32_t(osi), ld_be16(buf + osi + 2 * i), fk, r, &sl);
                        if (i == 0 && r.status == SLATE_OK) fk = int(sl);
                        L.grows[i] = r;
                      }
                    }
                  }
                }
              }
            }
          }
        }
      }
      a.meta[b] = m;
    }
  }
}

hipError_t launch_decode_lpb(hipStream_t st, const DecodeArgs& a, int num_cus) {
  if (a.n == 0) return hipGetLastError();
  const size_t lds = kTabBytes + size_t(kLpbThreads) * kLaneStride;
  const uint32_t waves_needed = (a.n + 63) / 64;
  uint32_t grid = (waves_needed + kLpbThreads / 64 - 1) / (kLpbThreads / 64);
  grid = min(grid, uint32_t(num_cus) * kLpbWgPerCu);
  decode_lpb_kernel<<<grid, kLpbThreads, lds, st>>>(a);
  return hipGetLastError();
}

}  // namespace slate
