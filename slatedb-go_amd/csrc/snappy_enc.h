// golang/snappy v0.0.4 block-format encoder (encode.go Encode + encode_other.go
// encodeBlock/emitLiteral/emitCopy), one wavefront per buffer, byte-exact.
//
// The match finder's probe loop is serial in Go: probe t at position s_t reads
// table[hash(s_t)] and then writes s_t there.  The positions themselves do not
// depend on the table: s_{t+1} = s_t + (skip_t >> 5) with skip starting at 32
// (kProbe.cum).  So the wave evaluates 64 consecutive probes at once:
//   * each lane hashes its position;
//   * a lane's candidate is the table entry, or, when an earlier lane of the
//     batch hashed to the same slot, that lane's position (positions increase, so
//     the latest earlier writer is the one Go would see).  Collisions are
//     detected through an LDS owner array; the rare colliding batch takes a
//     64-step shuffle scan;
//   * the first lane whose 4 bytes match ends the batch; only lanes up to it
//     commit their table writes (the last writer per slot).
// Match extension compares 64 bytes per step with a ballot; literals are copied
// by all lanes.  Table bookkeeping after each copy is done by lane 0 in Go order.
#pragma once
#include "common.h"

namespace slate {


constexpr uint32_t kSnapMaxBlock = 65536;    // encode.go maxBlockSize
constexpr uint32_t kSnapMinNonLiteral = 17;  // 1 + 1 + inputMargin
constexpr uint32_t kSnapInputMargin = 15;
constexpr uint32_t kSnapMaxTable = 1u << 14;
constexpr uint32_t kProbeSlots = 320;        // cum[] reaches past 65536 at t = 266
#ifndef SLATE_SNAP_CUMREG  // the probe schedule in registers (1) or read per batch from constant memory (0)
#define SLATE_SNAP_CUMREG 1
#endif
#ifndef SLATE_SNAP_ALWAYS_SORT  // A/B: sort every probe batch instead of the owner-array duplicate check
#define SLATE_SNAP_ALWAYS_SORT 0
#endif

struct SnapProbe {
  uint32_t cum[kProbeSlots + 1];
  constexpr SnapProbe() : cum{} {
    uint32_t skip = 32, c = 0;
    for (uint32_t t = 0; t <= kProbeSlots; t++) {
      cum[t] = c;
      c += skip >> 5;
      skip += skip >> 5;
      if (c > 0x7FFFFFFFu) c = 0x7FFFFFFFu;
    }
  }
};
static __constant__ SnapProbe g_snap_probe = SnapProbe();
constexpr SnapProbe kSnapProbeConst{};  // the same schedule as compile-time constants (serial probes)

__host__ __device__ constexpr uint64_t snappy_max_encoded_len(uint64_t n) { return 32 + n + n / 6; }

// table slots used for a chunk of n bytes (encode_other.go:206-210)
__device__ inline uint32_t snappy_table_size(uint32_t n, uint32_t* shift) {
  uint32_t sh = 24, ts = 256;
  while (ts < kSnapMaxTable && ts < n) {
    ts <<= 1;
    sh--;
  }
  *shift = sh;
  return ts;
}

// 4 unaligned bytes as two aligned dword reads (gfx950 serialises a misaligned LDS access lane by
// lane); the buffers keep at least 4 readable bytes past their end
// The aligned address is formed from p by pointer arithmetic, not an integer round trip, so the
// compiler still knows an LDS pointer is one: a generic (flat) load also counts in vmcnt, and its
// wait then drains every outstanding global store of the encoded output first.
__device__ inline uint32_t snap_ld32(const uint8_t* p) {
  const uint32_t m = uint32_t(reinterpret_cast<uintptr_t>(p)) & 3u;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - m);
  return __builtin_amdgcn_alignbyte(w[1], w[0], m);
}
__device__ inline uint32_t snap_hash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

// emitLiteral (encode_other.go:12-38): header by lane 0, bytes by all lanes
__device__ inline uint32_t snap_emit_literal(uint8_t* dst, uint32_t d, const uint8_t* lit, uint32_t len, int lane) {
  const uint32_t n = len - 1;
  uint32_t hl;
  if (n < 60) {
    hl = 1;
    if (lane == 0) dst[d] = uint8_t(n << 2);
  } else if (n < 256) {
    hl = 2;
    if (lane == 0) {
      dst[d] = 60 << 2;
      dst[d + 1] = uint8_t(n);
    }
  } else {
    hl = 3;
    if (lane == 0) {
      dst[d] = 61 << 2;
      dst[d + 1] = uint8_t(n);
      dst[d + 2] = uint8_t(n >> 8);
    }
  }
  uint8_t* o = dst + d + hl;
  for (uint32_t k = lane; k < len; k += kWave) o[k] = lit[k];
  return d + hl + len;
}

// emitCopy (encode_other.go:40-76)
__device__ inline uint32_t snap_emit_copy(uint8_t* dst, uint32_t d, uint32_t offset, uint32_t length, int lane) {
  while (length >= 68) {
    if (lane == 0) {
      dst[d] = 63 << 2 | 2;
      dst[d + 1] = uint8_t(offset);
      dst[d + 2] = uint8_t(offset >> 8);
    }
    d += 3;
    length -= 64;
  }
  if (length > 64) {
    if (lane == 0) {
      dst[d] = 59 << 2 | 2;
      dst[d + 1] = uint8_t(offset);
      dst[d + 2] = uint8_t(offset >> 8);
    }
    d += 3;
    length -= 60;
  }
  if (length >= 12 || offset >= 2048) {
    if (lane == 0) {
      dst[d] = uint8_t((length - 1) << 2 | 2);
      dst[d + 1] = uint8_t(offset);
      dst[d + 2] = uint8_t(offset >> 8);
    }
    return d + 3;
  }
  if (lane == 0) {
    dst[d] = uint8_t((offset >> 8) << 5 | (length - 4) << 2 | 1);
    dst[d + 1] = uint8_t(offset);
  }
  return d + 2;
}

// first s' >= s with src[i + (s'-s)] != src[s'] or s' == n (encode_other.go:176)
__device__ inline uint32_t snap_extend(const uint8_t* src, uint32_t n, uint32_t i, uint32_t s, int lane) {
  for (;;) {
    const uint32_t p = s + lane;
    const bool stop = p >= n || src[i + lane] != src[p];
    const uint64_t m = __ballot(stop);
    if (m) return s + uint32_t(__builtin_ctzll(m));
    s += kWave;
    i += kWave;
  }
}

__device__ inline void snap_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v from lane (lane ^ J), in VALU cross-lane operations (DPP, gfx950 permlane swaps) rather than
// LDS-crossbar shuffles: the sort below is one serial chain of 21 of these per probe batch.
template <uint32_t J>
__device__ __forceinline__ uint32_t snap_xor(uint32_t v, int lane) {
  if constexpr (J == 1) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const int m = __builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xf, 0xf, false);  // row_half_mirror: lane ^ 7
    return uint32_t(__builtin_amdgcn_update_dpp(0, m, 0x1B, 0xf, 0xf, false));      // quad_perm [3,2,1,0]: ^ 3
  } else if constexpr (J == 8) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  } else if constexpr (J == 16) {
    // odd rows of the first operand swap with even rows of the second: {r0 r0 r2 r2}, {r1 r1 r3 r3}
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else {
    // upper half of the first operand swaps with the lower half of the second: {lo lo}, {hi hi}
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? r[0] : r[1];
  }
}
template <uint32_t K, uint32_t J>
__device__ __forceinline__ uint32_t snap_bitonic_step(uint32_t v, int lane) {
  const uint32_t o = snap_xor<J>(v, lane);
  const bool up = (uint32_t(lane) & K) == 0 || K == 64;
  const bool lower = (uint32_t(lane) & J) == 0;
  return (lower == up) ? min(v, o) : max(v, o);
}
template <uint32_t K, uint32_t J>
__device__ __forceinline__ uint32_t snap_bitonic_merge(uint32_t v, int lane) {
  v = snap_bitonic_step<K, J>(v, lane);
  if constexpr (J > 1) v = snap_bitonic_merge<K, J / 2>(v, lane);
  return v;
}

// For each valid lane: the latest earlier (*prev) and the earliest later (*next) valid lane of the
// wave with the same hash slot h (< 2^14), or 64.  Bitonic sort of (h, lane) keys across the wave;
// invalid lanes get unique keys above every slot.  Results go back to their lanes by ds_permute.
__device__ inline void snap_slot_neighbours(uint32_t h, bool valid, int lane, int32_t* prev, int32_t* next) {
  uint32_t v = ((valid ? h : (1u << 14) + uint32_t(lane)) << 6) | uint32_t(lane);
  v = snap_bitonic_merge<2, 1>(v, lane);
  v = snap_bitonic_merge<4, 2>(v, lane);
  v = snap_bitonic_merge<8, 4>(v, lane);
  v = snap_bitonic_merge<16, 8>(v, lane);
  v = snap_bitonic_merge<32, 16>(v, lane);
  v = snap_bitonic_merge<64, 32>(v, lane);
  const uint32_t pv = uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x138, 0xf, 0xf, false));  // wave_shr:1
  const uint32_t nv = uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x130, 0xf, 0xf, false));  // wave_shl:1
  const bool vv = (v >> 6) < (1u << 14);
  const uint32_t p_lane = (lane > 0 && vv && (pv >> 6) == (v >> 6)) ? (pv & 63) : 64u;
  const uint32_t n_lane = (lane < 63 && vv && (nv >> 6) == (v >> 6)) ? (nv & 63) : 64u;
  // sorted position `lane` holds original lane (v & 63): send the answers there
  *prev = __builtin_amdgcn_ds_permute(int((v & 63) * 4), int(p_lane));
  *next = __builtin_amdgcn_ds_permute(int((v & 63) * 4), int(n_lane));
}

// encodeBlock (encode_other.go:165-238) for kSnapMinNonLiteral <= n <= 65536.
// table: kSnapMaxTable u16 slots (LDS); owner: kSnapMaxTable bytes (LDS).
// owner_mask: the owner array has owner_mask + 1 bytes (a power of two); slots that share an owner
// byte only make the duplicate check fire for nothing (the sort then finds the true neighbours)
// K > 0: each search for the next match first probes K positions one at a time (wave-uniform, one
// lane writing the table; golang's order exactly), then goes on with 64-probe batches from probe K.
// Short literal runs (a bloom filter's bits: ~3 bytes between matches) then cost a few dependent LDS
// reads instead of a whole batch with its duplicate-slot sort.
template <uint32_t K = 0>
__device__ __forceinline__ uint32_t snappy_encode_block_wave(const uint8_t* src, uint32_t n, uint8_t* dst, uint16_t* table,
                                             uint8_t* owner, int lane, uint32_t owner_mask = kSnapMaxTable - 1) {
  uint32_t shift;
  const uint32_t ts = snappy_table_size(n, &shift);
  for (uint32_t i = lane; i < ts; i += kWave) table[i] = 0;
  snap_sync();
  const int32_t s_limit = int32_t(n) - int32_t(kSnapInputMargin);
  uint32_t d = 0, next_emit = 0;
  int32_t s = 1;
#if SLATE_SNAP_CUMREG
  // the probe schedule held in registers: cum[64 k + lane] and cum[64 k + lane + 1], k = 0..4
  uint32_t cu[5], cn[5];
#pragma unroll
  for (uint32_t k = 0; k < 5; k++) {
    cu[k] = g_snap_probe.cum[min(64 * k + uint32_t(lane) + K, kProbeSlots)];
    cn[k] = g_snap_probe.cum[min(64 * k + uint32_t(lane) + K + 1, kProbeSlots)];
  }
#endif
  for (;;) {
    // ---------------- probe loop, 64 probes per batch
    int32_t cand = 0;
    bool found = false, remainder = false;
#pragma unroll
    for (uint32_t t = 0; t < K; t++) {
      const int32_t st = s + int32_t(kSnapProbeConst.cum[t]);
      if (s + int32_t(kSnapProbeConst.cum[t + 1]) > s_limit) {  // nextS > sLimit: emitRemainder
        remainder = true;
        break;
      }
      const uint32_t cur = snap_ld32(src + st);
      const uint32_t h = snap_hash(cur, shift);
      const int32_t c = int32_t(table[h]);
      if (lane == 0) table[h] = uint16_t(st);  // (LDS accesses of a wave stay in order)
      if (cur == snap_ld32(src + c)) {
        s = st;
        cand = c;
        found = true;
        break;
      }
    }
    for (uint32_t t0 = 0; !found && !remainder; t0 += kWave) {
      const uint32_t t = K + t0 + lane;
      const bool in_sched = t + 1 <= kProbeSlots;
#if SLATE_SNAP_CUMREG
      const uint32_t kb = t0 >> 6;  // wave-uniform
      const uint32_t ct = kb == 0 ? cu[0] : kb == 1 ? cu[1] : kb == 2 ? cu[2] : kb == 3 ? cu[3] : cu[4];
      const uint32_t ctn = kb == 0 ? cn[0] : kb == 1 ? cn[1] : kb == 2 ? cn[2] : kb == 3 ? cn[3] : cn[4];
      const int32_t st = in_sched ? s + int32_t(ct) : 0x7FFFFFFF;
      const int32_t snext = in_sched ? s + int32_t(ctn) : 0x7FFFFFFF;
#else
      const int32_t st = in_sched ? s + int32_t(g_snap_probe.cum[t]) : 0x7FFFFFFF;
      const int32_t snext = in_sched ? s + int32_t(g_snap_probe.cum[t + 1]) : 0x7FFFFFFF;
#endif
      const bool valid = in_sched && snext <= s_limit;
      uint32_t cur = 0, h = 0;
      if (valid) {
        cur = snap_ld32(src + st);
        h = snap_hash(cur, shift);
        if (!SLATE_SNAP_ALWAYS_SORT) owner[h & owner_mask] = uint8_t(lane);
      }
      snap_sync();
      const bool dup = valid && (SLATE_SNAP_ALWAYS_SORT || owner[h & owner_mask] != uint8_t(lane));
      const uint64_t dupmask = __ballot(dup);
      const uint64_t validmask = __ballot(valid);
      int32_t c = valid ? int32_t(table[h]) : 0;
      // Lanes of this batch that share a table slot: each takes its candidate from the latest
      // earlier lane with that slot (the serial encoder's table would hold that position), and
      // only the latest lane that ran writes the slot.  The lanes are sorted by (slot, lane)
      // with a 64-wide bitonic network, so the neighbours in sorted order are exactly those
      // lanes (21 exchange steps, instead of two 63-step shuffle scans).
      int32_t prev = 64, next = 64;
      if (dupmask) {  // (wave-uniform: every lane takes part in the cross-lane operations)
        snap_slot_neighbours(h, valid, lane, &prev, &next);
        const int32_t sp = __shfl(st, prev < 64 ? prev : lane, 64);
        if (valid && prev < 64) c = sp;
      }
      const bool match = valid && cur == snap_ld32(src + c);
      const uint64_t mm = __ballot(match);
      const uint32_t istar = mm ? uint32_t(__builtin_ctzll(mm)) : 64u;
      const bool ran = valid && uint32_t(lane) <= istar;
      const bool last = !(next < 64 && uint32_t(next) <= istar);
      if (ran && last) table[h] = uint16_t(st);
      snap_sync();
      if (mm) {
        s = __builtin_amdgcn_readlane(st, int(istar));  // istar is wave-uniform
        cand = __builtin_amdgcn_readlane(c, int(istar));
        found = true;
        break;
      }
      if (validmask != ~0ull) break;  // nextS > sLimit: emitRemainder
    }
    if (!found) break;
    // ---------------- emit literal + copies (encode_other.go:194-235)
    d = snap_emit_literal(dst, d, src + next_emit, uint32_t(s) - next_emit, lane);
    bool done = false;
    for (;;) {
      const int32_t base = s;
      s = int32_t(snap_extend(src, n, uint32_t(cand) + 4, uint32_t(s) + 4, lane));
      d = snap_emit_copy(dst, d, uint32_t(base - cand), uint32_t(s - base), lane);
      next_emit = uint32_t(s);
      if (s >= s_limit) {
        done = true;
        break;
      }
      const uint32_t lo = snap_ld32(src + s - 1), hi = snap_ld32(src + s + 3);
      const uint32_t prev_hash = snap_hash(lo, shift);
      const uint32_t x1 = (lo >> 8) | (hi << 24);
      const uint32_t curr_hash = snap_hash(x1, shift);
      // table[prevHash] = s-1; candidate = table[currHash]; table[currHash] = s (encode_other.go:
      // 226-231) with one wave barrier instead of three: the read is taken before either write,
      // and the write of prevHash is forwarded when the two slots coincide
      const int32_t old = int32_t(table[curr_hash]);
      snap_sync();
      cand = prev_hash == curr_hash ? s - 1 : old;
      if (lane == 0) {
        table[prev_hash] = uint16_t(s - 1);
        table[curr_hash] = uint16_t(s);
      }
      // (the next table reads come after the probe batch's barrier, or after this one's)
      if (x1 != snap_ld32(src + cand)) {
        s++;
        break;
      }
    }
    if (done) break;
  }
  if (next_emit < n) d = snap_emit_literal(dst, d, src + next_emit, n - next_emit, lane);
  snap_sync();
  return d;
}

// snappy.Encode (encode.go:17-42): uvarint length, then 64 KiB blocks.
template <uint32_t K = 0>
__device__ __forceinline__ uint32_t snappy_encode_wave(const uint8_t* src, uint32_t n, uint8_t* dst, uint16_t* table, uint8_t* owner,
                                       int lane, uint32_t owner_mask = kSnapMaxTable - 1) {
  uint32_t d = 0;
  {
    uint64_t v = n;
    while (v >= 0x80) {
      if (lane == 0) dst[d] = uint8_t(v) | 0x80;
      d++;
      v >>= 7;
    }
    if (lane == 0) dst[d] = uint8_t(v);
    d++;
  }
  for (uint32_t p = 0; p < n;) {
    const uint32_t pn = min(n - p, kSnapMaxBlock);
    if (pn < kSnapMinNonLiteral) d = snap_emit_literal(dst, d, src + p, pn, lane);
    else d += snappy_encode_block_wave<K>(src + p, pn, dst + d, table, owner, lane, owner_mask);
    p += pn;
  }
  snap_sync();
  return d;
}

}  // namespace slate
