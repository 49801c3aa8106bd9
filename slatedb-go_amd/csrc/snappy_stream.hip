// Streaming Snappy decode of one large buffer (an SST's index or bloom filter, decode.go:83-100,
// bloom.go:70-91), one wavefront: golang/snappy v0.0.4 decode (decode_other.go:19-110) with the
// same control flow and error checks as wave_snappy_decode (decode.hip), but the input is staged
// through a 32 KiB LDS window and the last 64 KiB of output stay in an LDS ring, so the tag walk
// pays LDS latency instead of global-memory latency.  A buffer like this is a single serial tag
// stream: the lane-per-block decoder would run it on one lane (~0.1 s for a 2.5 MB index).
// Copies reaching further back than the ring read the output already written to HBM.
#include <utility>

#include "common.h"
#include "kernels.h"

namespace slate {
namespace {

constexpr uint32_t kInWin = 32768;   // input window bytes
constexpr uint32_t kRing = 65536;    // output ring bytes
constexpr uint32_t kW = 64;

struct Stream {
  const uint8_t* in;
  uint32_t sn;       // payload bytes
  uint32_t wb;       // window base (input offset of win[0])
  uint8_t* win;
  uint8_t* ring;
  uint8_t* out;
};

// window := input [base, base + kInWin) (16-byte aligned base); wave-synchronous
__device__ void refill(Stream& S, uint32_t s, int lane) {
  const uint32_t base = s & ~15u;
  __syncthreads();  // earlier reads of the window are done
  for (uint32_t j = uint32_t(lane); j < kInWin / 16; j += kW) {
    const uint32_t o = base + 16 * j;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (o + 16 <= S.sn) {
      v = *reinterpret_cast<const uint4*>(S.in + o);
    } else if (o < S.sn) {
      uint8_t b[16] = {};
      for (uint32_t k = 0; k < 16 && o + k < S.sn; k++) b[k] = S.in[o + k];
      v = *reinterpret_cast<const uint4*>(b);
    }
    *reinterpret_cast<uint4*>(S.win + 16 * j) = v;
  }
  S.wb = base;
  __syncthreads();
}

__device__ __forceinline__ uint32_t in_byte(const Stream& S, uint32_t s) { return S.win[s - S.wb]; }

}  // namespace

// in: payload (header varint at [0, hdr)), sn payload bytes; out: dn decoded bytes.
// fallback: when not null, the kernel runs only if the fragment-parallel path (below) gave up
// (*fallback != 0); otherwise it reports that path's success.
__global__ __launch_bounds__(64) void snappy_stream_kernel(const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                                           uint32_t dn, int32_t* status, const uint32_t* fallback) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x;
  if (fallback && *fallback == 0) {
    if (lane == 0) *status = SLATE_OK;
    return;
  }
  Stream S{in, sn, 0, smem, smem + kInWin, out};
  uint32_t s = hdr, d = 0;
  refill(S, s, lane);
  int st = SLATE_OK;
  // the tag and up to four more bytes, one LDS round trip: lane k reads byte s + k.  After a copy
  // tag the next tag's bytes are read before the copy moves its bytes (both LDS round trips
  // overlap); `have` says that `mine` already holds them.
  uint32_t mine = 0;
  bool have = false;
  while (s < sn) {
    if (!have) {
      if (s + 5 > S.wb + kInWin) refill(S, s, lane);
      mine = (uint32_t(lane) < 5 && s + lane < S.wb + kInWin) ? in_byte(S, s + lane) : 0u;
    }
    have = false;
    const uint32_t c = __builtin_amdgcn_readlane(mine, 0);
    const uint32_t b1 = __builtin_amdgcn_readlane(mine, 1), b2 = __builtin_amdgcn_readlane(mine, 2),
                   b3 = __builtin_amdgcn_readlane(mine, 3), b4 = __builtin_amdgcn_readlane(mine, 4);
    const uint32_t t = c & 3;
    if (t == 0) {
      uint32_t x = c >> 2;
      if (x < 60) {
        s += 1;
      } else {
        const uint32_t nb = x - 59;
        s += 1 + nb;
        if (s > sn) {
          st = SLATE_E_SNAPPY_CORRUPT;
          break;
        }
        const uint32_t all = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
        x = nb >= 4 ? all : (all & ((1u << (8 * nb)) - 1));
      }
      const uint64_t len = uint64_t(x) + 1;
      if (len > uint64_t(dn - d) || len > uint64_t(sn - s)) {
        st = SLATE_E_SNAPPY_CORRUPT;
        break;
      }
      const uint32_t L = uint32_t(len);
      if (s + L > S.wb + kInWin && L + 16 <= kInWin) refill(S, s, lane);
      const bool from_win = s + L <= S.wb + kInWin;
      for (uint32_t j = uint32_t(lane); j < L; j += kW) {
        const uint8_t v = from_win ? S.win[s + j - S.wb] : in[s + j];
        out[d + j] = v;
        S.ring[(d + j) & (kRing - 1)] = v;
      }
      d += L;
      s += L;
      continue;
    }
    uint32_t len, off;
    if (t == 1) {
      s += 2;
      len = 4 + ((c >> 2) & 7);
      off = ((c & 0xe0) << 3) | b1;
    } else if (t == 2) {
      s += 3;
      len = 1 + (c >> 2);
      off = b1 | (b2 << 8);
    } else {
      s += 5;
      len = 1 + (c >> 2);
      off = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
    }
    if (s > sn) {
      st = SLATE_E_SNAPPY_CORRUPT;
      break;
    }
    if (off == 0 || d < off || len > dn - d) {
      st = SLATE_E_SNAPPY_CORRUPT;
      break;
    }
    if (s < sn && s + 5 <= S.wb + kInWin) {
      mine = (uint32_t(lane) < 5) ? in_byte(S, s + lane) : 0u;
      have = true;
    }
    // len <= 64: one lane per byte; byte j repeats the off-byte pattern when off < len
    const uint32_t j = uint32_t(lane);
    const uint32_t src = d - off + (off >= len ? j : j % off);
    uint8_t v = 0;
    if (off <= kRing) {
      if (j < len) v = S.ring[src & (kRing - 1)];
    } else {
      __threadfence();  // the bytes were stored to HBM by this wave earlier
      if (j < len) v = __builtin_nontemporal_load(out + src);
    }
    if (j < len) {
      out[d + j] = v;
      S.ring[(d + j) & (kRing - 1)] = v;
    }
    d += len;
  }
  if (st == SLATE_OK && d != dn) st = SLATE_E_SNAPPY_CORRUPT;
  if (lane == 0) *status = st;
}

size_t snappy_stream_lds_bytes() { return kInWin + kRing; }

hipError_t launch_snappy_stream(hipStream_t st, const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                uint32_t dn, int32_t* status) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_stream_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     int(snappy_stream_lds_bytes()));
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(snappy_stream_kernel, dim3(1), dim3(64), snappy_stream_lds_bytes(), st, in, sn, hdr, out, dn,
                     status, static_cast<const uint32_t*>(nullptr));
  return hipGetLastError();
}

// ------------------------------------------------------------------ tag-parallel decode
// The whole stream decoded with parallel passes; the only serial work is following the tag
// chain in strides (about 3 x cbrt(tags) dependent loads instead of one per tag):
//   1. sp_next: for every byte position p, where the tag after a tag starting at p begins and
//      that tag's decoded length (a tag running past the payload jumps to ERR = sn + 1);
//   2. sp_jump x 2 kLog: pointer doubling: 2^kLog and 2^(2 kLog) tags ahead and the decoded
//      bytes in between;
//   3. sp_hops: one lane follows the true chain from the header in strides of 2^(2 kLog) tags,
//      then one lane per such stride in strides of 2^kLog tags (sp_subhops);
//   4. sp_walk: one lane per small stride lists its tags (position, decoded offset): every tag;
//   5. sp_check: per tag, decode_other.go's copy checks (offset 0, offset beyond the output);
//   6. sp_bytes: per decoded byte, its tag by binary search: a literal byte is final (value
//      from the input), a copied byte points at the byte it copies;
//   7. sp_ptr x ceil(log2 dn): pointer doubling until every byte points at a literal byte;
//   8. sp_gather: out[x] = value of the literal byte x points at.
// A failed check (an invalid tag on the chain, a bad copy, a wrong total length) sets
// *fallback and the serial stream kernel decodes the buffer instead, so the result -- bytes
// and status -- is always the serial decoder's; success here implies its success with the
// same bytes (every check it makes is made, on the same values).
namespace {
constexpr uint32_t kLog = 7;  // small stride: 128 tags; large stride: 16384 tags
constexpr uint32_t kStride = 1u << kLog;

struct ParScratch {
  uint32_t *j0, *d0, *ja, *da, *jb, *db, *j1, *d1, *Hp, *Hd, *hp, *hd, *tp, *td, *pa, *pb, *flag, *changed;
  uint8_t* val;
  uint32_t n_pos, n_big, n_hops, n_tags_cap, dn;
};

__host__ __device__ inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline ParScratch par_carve(void* base, uint32_t sn, uint32_t dn, size_t* bytes) {
  ParScratch p;
  p.n_pos = sn + 2;
  p.n_big = (sn >> (2 * kLog)) + 4;
  p.n_hops = p.n_big * kStride + 8;
  p.n_tags_cap = sn + 1;
  p.dn = dn;
  uint8_t* q = static_cast<uint8_t*>(base);
  auto take = [&](size_t words) {
    uint32_t* r = reinterpret_cast<uint32_t*>(q);
    q += al256(words * 4);
    return r;
  };
  p.j0 = take(p.n_pos);
  p.d0 = take(p.n_pos);
  p.ja = take(p.n_pos);
  p.da = take(p.n_pos);
  p.jb = take(p.n_pos);
  p.db = take(p.n_pos);
  p.j1 = take(p.n_pos);
  p.d1 = take(p.n_pos);
  p.Hp = take(p.n_big + 1);
  p.Hd = take(p.n_big + 1);
  p.hp = take(p.n_hops + 1);
  p.hd = take(p.n_hops + 1);
  p.tp = take(p.n_tags_cap);
  p.td = take(p.n_tags_cap);
  p.pa = take(size_t(dn) + 1);
  p.pb = take(size_t(dn) + 1);
  p.flag = take(8);  // [0] give up, [1] small strides, [2] tags, [3] large hops, [4] LZ4: decoded length
  p.changed = take(64);
  p.val = reinterpret_cast<uint8_t*>(q);
  q += al256(size_t(dn) + 16);
  if (bytes) *bytes = size_t(q - static_cast<uint8_t*>(base));
  return p;
}

// the tag at p (golang/snappy decode_other.go:19-110 field layout): header length, decoded
// length, copy offset (0 for a literal), literal bytes start; false when it runs past sn
__device__ __forceinline__ bool tag_at(const uint8_t* in, uint32_t sn, uint32_t p, uint32_t* next, uint32_t* len,
                                       uint32_t* off, uint32_t* lit) {
  auto b = [&](uint32_t k) -> uint32_t { return p + k < sn ? uint32_t(in[p + k]) : 0u; };
  const uint32_t c = in[p], t = c & 3;
  if (t == 0) {
    const uint32_t x = c >> 2;
    const uint32_t nb = x < 60 ? 0u : x - 59;
    const uint64_t s1 = uint64_t(p) + 1 + nb;
    uint32_t v = x;
    if (nb) v = b(1) | (nb > 1 ? b(2) << 8 : 0u) | (nb > 2 ? b(3) << 16 : 0u) | (nb > 3 ? b(4) << 24 : 0u);
    const uint64_t l = uint64_t(v) + 1;
    *off = 0;
    *lit = uint32_t(s1);
    if (s1 > sn || l > sn - s1) return false;
    *next = uint32_t(s1 + l);
    *len = uint32_t(l);
    return true;
  }
  const uint32_t hl = t == 1 ? 2u : (t == 2 ? 3u : 5u);
  *len = t == 1 ? 4 + ((c >> 2) & 7) : 1 + (c >> 2);
  *off = t == 1 ? (((c & 0xe0) << 3) | b(1)) : (t == 2 ? (b(1) | (b(2) << 8)) : (b(1) | (b(2) << 8) | (b(3) << 16) | (b(4) << 24)));
  *lit = 0;
  if (uint64_t(p) + hl > sn) return false;
  *next = p + hl;
  return true;
}

__global__ void sp_next_kernel(const uint8_t* __restrict__ in, uint32_t sn, uint32_t hdr, ParScratch P) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.n_pos) return;
  uint32_t nx = sn + 1, dl = 0;  // ERR
  if (p >= sn) {
    nx = p;  // END and ERR stay where they are
  } else if (p >= hdr) {
    uint32_t n, l, o, lt;
    if (tag_at(in, sn, p, &n, &l, &o, &lt)) {
      nx = n;
      dl = l;
    }
  }
  P.j0[p] = nx;
  P.d0[p] = dl;
  P.ja[p] = nx;
  P.da[p] = dl;
}

__global__ void sp_jump_kernel(uint32_t n, const uint32_t* __restrict__ js, const uint32_t* __restrict__ ds,
                               uint32_t* __restrict__ jd, uint32_t* __restrict__ dd) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t q = js[p];
  const uint64_t s = uint64_t(ds[p]) + ds[q];
  jd[p] = js[q];
  dd[p] = s > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(s);
}

// the true chain from the header in strides of kStride^2 tags (one lane; the loads are its path)
__global__ void sp_hops_kernel(uint32_t sn, uint32_t hdr, ParScratch P, const uint32_t* __restrict__ jk,
                               const uint32_t* __restrict__ dk) {
  if (threadIdx.x != 0) return;
  uint32_t p = hdr, i = 0;
  uint64_t d = 0;
  bool bad = false;
  while (true) {
    if (i >= P.n_big) {
      bad = true;
      break;
    }
    P.Hp[i] = p;
    P.Hd[i] = uint32_t(d > 0xFFFFFFFFull ? 0xFFFFFFFFull : d);
    i++;
    if (p >= sn) break;
    d += dk[p];
    p = jk[p];
  }
  if (bad || p != sn || d != P.dn) P.flag[0] = 1;  // an invalid tag on the chain, or the wrong length
  P.flag[3] = i;
}

// large stride I in strides of kStride tags: small stride index I * kStride + k
__global__ void sp_subhops_kernel(uint32_t sn, ParScratch P) {
  const uint32_t I = blockIdx.x * blockDim.x + threadIdx.x;
  if (P.flag[0]) return;
  const uint32_t nH = P.flag[3];  // large strides 0 .. nH-2, the last one ends at END
  if (I + 1 >= nH) return;
  uint32_t p = P.Hp[I], d = P.Hd[I], k = 0;
  for (; k < kStride && p < sn; k++) {
    P.hp[I * kStride + k] = p;
    P.hd[I * kStride + k] = d;
    d += P.d1[p];
    p = P.j1[p];
  }
  if (I + 2 == nH) {  // the end of the chain closes the list of small strides
    P.hp[I * kStride + k] = p;
    P.hd[I * kStride + k] = d;
    P.flag[1] = I * kStride + k + 1;
  }
}

// small stride i lists its tags: positions and decoded offsets, densely (tag i * kStride + k)
__global__ void sp_walk_kernel(uint32_t sn, ParScratch P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (P.flag[0]) return;
  const uint32_t nh = P.flag[1];  // hops: strides 0 .. nh-2, the last one ends at END
  if (i + 1 >= nh) return;
  uint32_t p = P.hp[i], d = P.hd[i], k = 0;
  const uint32_t base = i * kStride;
  for (; k < kStride && p < sn; k++) {
    P.tp[base + k] = p;
    P.td[base + k] = d;
    d += P.d0[p];
    p = P.j0[p];
  }
  if (i + 2 == nh) P.flag[2] = base + k;
}

// decode_other.go's copy checks per tag: offset 0 or beyond the bytes decoded so far
__global__ void sp_check_kernel(const uint8_t* __restrict__ in, uint32_t sn, ParScratch P) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (P.flag[0] || t >= P.flag[2]) return;
  uint32_t n, l, o, lt;
  const bool ok = tag_at(in, sn, P.tp[t], &n, &l, &o, &lt);
  const bool is_copy = (in[P.tp[t]] & 3) != 0;
  if (!ok || (is_copy && (o == 0 || o > P.td[t]))) atomicOr(P.flag, 1u);
}

// decoded byte x: its tag, then either its final value (literal) or the byte it copies
__global__ void sp_bytes_kernel(const uint8_t* __restrict__ in, uint32_t sn, ParScratch P) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= P.dn || P.flag[0]) return;
  uint32_t lo = 0, hi = P.flag[2];  // last tag with td <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.td[mid] <= x) lo = mid;
    else hi = mid;
  }
  uint32_t n, l, o, lt;
  tag_at(in, sn, P.tp[lo], &n, &l, &o, &lt);
  const uint32_t k = x - P.td[lo];
  if (o == 0) {
    P.val[x] = in[lt + k];
    P.pa[x] = x;
  } else {
    P.pa[x] = x - o;  // forward copy semantics: byte x repeats byte x - off (checked: off <= td)
  }
}

// one doubling round; changed[r] records whether any pointer moved, and a round after one
// where none moved has nothing left to do (its output buffer is the same as its input's)
__global__ void sp_ptr_kernel(uint32_t n, const uint32_t* __restrict__ ps, uint32_t* __restrict__ pd,
                              const uint32_t* __restrict__ flag, uint32_t* __restrict__ changed, uint32_t r) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n || flag[0]) return;
  if (r > 0 && changed[r - 1] == 0) {
    pd[x] = ps[x];
    return;
  }
  const uint32_t a = ps[x], b = ps[a];
  pd[x] = b;
  if (__ballot(a != b) && (threadIdx.x & 63) == 0) changed[r] = 1u;
}

__global__ void sp_gather_kernel(const ParScratch P, const uint32_t* __restrict__ ps, uint8_t* __restrict__ out) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= P.dn || P.flag[0]) return;
  out[x] = P.val[ps[x]];
}

// ----------------------------------------------------------------- LZ4 blocks, same passes
// One LZ4 data block (the lz4 block format: sequences of literals then a match, the last one
// literals only) decoded with the passes above, a "tag" being one sequence.  The exact decoder
// is decode.hip wave_lz4_decode's sequence loop (oracle/slate_oracle.c lz4_frame, pierrec/lz4
// v4 decoder): every check it makes on a block is made here on the same values, and any that
// fails sets flag[0], so the caller hands the payload to it.  `cap` (the frame's block maximum)
// bounds the decoded length, which the chain pass finds (flag[4]).  A match reaches back at most
// `prior` bytes before the block: 0 for independent blocks, the frame's bytes decoded so far for
// linked ones (whose earlier blocks are final in out[-prior, 0) by then).
//
// the sequence at p: next sequence, decoded length, literals [lit, lit + ll), match offset;
// last = the literals end the block (no match).  false when it runs past the block.
__device__ __forceinline__ bool lz_seq_at(const uint8_t* in, uint32_t sz, uint32_t p, uint32_t* next, uint32_t* len,
                                          uint32_t* lit, uint32_t* ll_out, uint32_t* mo, bool* last) {
  uint32_t s = p + 1;
  const uint32_t tok = in[p];
  uint32_t ll = tok >> 4;  // sz <= 4 MiB: the 255-runs cannot overflow
  if (ll == 15) {
    uint32_t b;
    do {
      if (s >= sz) return false;
      b = in[s++];
      ll += b;
    } while (b == 255);
  }
  if (ll > sz - s) return false;
  *lit = s;
  *ll_out = ll;
  s += ll;
  *mo = 0;
  *last = s == sz;
  if (s == sz) {
    *next = sz;
    *len = ll;
    return true;
  }
  if (sz - s < 2) return false;
  *mo = uint32_t(in[s]) | uint32_t(in[s + 1]) << 8;
  s += 2;
  uint32_t ml = tok & 15;
  if (ml == 15) {
    uint32_t b;
    do {
      if (s >= sz) return false;
      b = in[s++];
      ml += b;
    } while (b == 255);
  }
  *next = s;
  *len = ll + ml + 4;
  return true;
}

__global__ void lz_next_kernel(const uint8_t* __restrict__ in, uint32_t sz, ParScratch P) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.n_pos) return;
  uint32_t nx = sz + 1, dl = 0;  // ERR
  if (p >= sz) {
    nx = p;  // END and ERR stay where they are
  } else {
    uint32_t n, l, lt, ll, o;
    bool last;
    if (lz_seq_at(in, sz, p, &n, &l, &lt, &ll, &o, &last)) {
      nx = n;
      dl = l;
    }
  }
  P.j0[p] = nx;
  P.d0[p] = dl;
  P.ja[p] = nx;
  P.da[p] = dl;
}

// sp_hops_kernel for a block of unknown decoded length: the chain must end at the block's end
// with at most P.dn (the cap) bytes decoded; the length goes to flag[4]
__global__ void lz_hops_kernel(uint32_t sz, ParScratch P, const uint32_t* __restrict__ jk,
                               const uint32_t* __restrict__ dk) {
  if (threadIdx.x != 0) return;
  uint32_t p = 0, i = 0;
  uint64_t d = 0;
  bool bad = sz == 0;  // a compressed block holds at least one sequence
  while (!bad) {
    if (i >= P.n_big) {
      bad = true;
      break;
    }
    P.Hp[i] = p;
    P.Hd[i] = uint32_t(d > 0xFFFFFFFFull ? 0xFFFFFFFFull : d);
    i++;
    if (p >= sz) break;
    d += dk[p];
    p = jk[p];
  }
  if (bad || p != sz || d > P.dn) P.flag[0] = 1;
  P.flag[3] = i;
  P.flag[4] = uint32_t(d > P.dn ? 0 : d);
}

// the exact decoder's per-sequence checks: a match offset of 0 or reaching before the frame's
// window, and a sequence with a match ending the block (the decoder then wants another token)
__global__ void lz_check_kernel(const uint8_t* __restrict__ in, uint32_t sz, uint32_t prior, ParScratch P) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (P.flag[0] || t >= P.flag[2]) return;
  uint32_t n, l, lt, ll, o;
  bool last;
  const bool ok = lz_seq_at(in, sz, P.tp[t], &n, &l, &lt, &ll, &o, &last);
  if (!ok || (!last && (o == 0 || uint64_t(o) > uint64_t(P.td[t]) + ll + prior || n >= sz))) atomicOr(P.flag, 1u);
}

// decoded byte x: its sequence, then its literal value or the byte its match copies
__global__ void lz_bytes_kernel(const uint8_t* __restrict__ in, uint32_t sz, ParScratch P,
                                const uint8_t* __restrict__ out) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= P.dn || P.flag[0]) return;
  uint32_t lo = 0, hi = P.flag[2];  // last sequence with td <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P.td[mid] <= x) lo = mid;
    else hi = mid;
  }
  uint32_t n, l, lt, ll, o;
  bool last;
  lz_seq_at(in, sz, P.tp[lo], &n, &l, &lt, &ll, &o, &last);
  const uint32_t k = x - P.td[lo];
  if (k < ll) {
    P.val[x] = in[lt + k];
    P.pa[x] = x;
  } else if (x < o) {  // a linked block's match into the blocks before it (checked: o <= x + prior)
    P.val[x] = out[int64_t(x) - int64_t(o)];
    P.pa[x] = x;
  } else {
    P.pa[x] = x - o;
  }
}
}  // namespace

size_t lz4_par_scratch_bytes(uint32_t sz, uint32_t cap) {
  size_t bytes = 0;
  par_carve(nullptr, sz, cap, &bytes);
  return bytes + 256;
}

const uint32_t* lz4_par_result(const void* scratch, uint32_t sz, uint32_t cap) {
  return par_carve(const_cast<void*>(scratch), sz, cap, nullptr).flag;
}

hipError_t launch_lz4_par_chain(hipStream_t st, const uint8_t* in, uint32_t sz, uint32_t cap, void* scratch) {
  if (sz >= 0xFFFFFF00u || cap >= 0xFFFFFF00u) return hipErrorInvalidValue;
  const ParScratch P = par_carve(scratch, sz, cap, nullptr);
  hipError_t e = hipMemsetAsync(P.flag, 0, 32, st);
  if (e != hipSuccess) return e;
  const uint32_t g = (P.n_pos + 255) / 256;
  lz_next_kernel<<<g, 256, 0, st>>>(in, sz, P);
  uint32_t* bj[2] = {P.ja, P.jb};
  uint32_t* bd[2] = {P.da, P.db};
  uint32_t *js = P.ja, *ds = P.da;
  int nxt = 1;
  for (uint32_t k = 0; k < 2 * kLog; k++) {
    const bool keep = k + 1 == kLog;
    uint32_t* jt = keep ? P.j1 : bj[nxt];
    uint32_t* dt = keep ? P.d1 : bd[nxt];
    sp_jump_kernel<<<g, 256, 0, st>>>(P.n_pos, js, ds, jt, dt);
    if (!keep) nxt ^= 1;
    js = jt;
    ds = dt;
  }
  lz_hops_kernel<<<1, 64, 0, st>>>(sz, P, js, ds);
  return hipGetLastError();
}

hipError_t launch_lz4_par_bytes(hipStream_t st, const uint8_t* in, uint32_t sz, uint32_t cap, uint32_t dn,
                                uint32_t prior, void* scratch, uint8_t* out) {
  if (dn > cap) return hipErrorInvalidValue;
  ParScratch P = par_carve(scratch, sz, cap, nullptr);  // the chain pass's layout
  P.dn = dn;
  sp_subhops_kernel<<<(P.n_big + 63) / 64, 64, 0, st>>>(sz, P);
  sp_walk_kernel<<<(P.n_hops + 63) / 64, 64, 0, st>>>(sz, P);
  lz_check_kernel<<<(P.n_tags_cap + 255) / 256, 256, 0, st>>>(in, sz, prior, P);
  if (dn) {
    const uint32_t gb = (dn + 255) / 256;
    lz_bytes_kernel<<<gb, 256, 0, st>>>(in, sz, P, out);
    uint32_t *ps = P.pa, *pd = P.pb;
    hipError_t e = hipMemsetAsync(P.changed, 0, 64 * 4, st);
    if (e != hipSuccess) return e;
    for (uint32_t r = 0; (1ull << r) < uint64_t(dn); r++) {
      sp_ptr_kernel<<<gb, 256, 0, st>>>(dn, ps, pd, P.flag, P.changed, r);
      std::swap(ps, pd);
    }
    sp_gather_kernel<<<gb, 256, 0, st>>>(P, ps, out);
  }
  return hipGetLastError();
}

size_t snappy_par_scratch_bytes(uint32_t sn, uint32_t dn) {
  size_t bytes = 0;
  par_carve(nullptr, sn, dn, &bytes);
  return bytes + 256;
}

hipError_t launch_snappy_decode_par(hipStream_t st, const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                    uint32_t dn, void* scratch, int32_t* status) {
  if (sn >= 0xFFFFFF00u || dn >= 0xFFFFFF00u) return hipErrorInvalidValue;
  static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_stream_kernel),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   int(snappy_stream_lds_bytes()));
  if (a1 != hipSuccess) return a1;
  const ParScratch P = par_carve(scratch, sn, dn, nullptr);
  hipError_t e = hipMemsetAsync(P.flag, 0, 16, st);
  if (e != hipSuccess) return e;
  const uint32_t g = (P.n_pos + 255) / 256;
  sp_next_kernel<<<g, 256, 0, st>>>(in, sn, hdr, P);
  // level k+1 from level k; level kLog (stride kStride) is kept in j1/d1, the others ping-pong
  uint32_t* bj[2] = {P.ja, P.jb};
  uint32_t* bd[2] = {P.da, P.db};
  uint32_t *js = P.ja, *ds = P.da;
  int nxt = 1;
  for (uint32_t k = 0; k < 2 * kLog; k++) {
    const bool keep = k + 1 == kLog;
    uint32_t* jt = keep ? P.j1 : bj[nxt];
    uint32_t* dt = keep ? P.d1 : bd[nxt];
    sp_jump_kernel<<<g, 256, 0, st>>>(P.n_pos, js, ds, jt, dt);
    if (!keep) nxt ^= 1;
    js = jt;
    ds = dt;
  }
  sp_hops_kernel<<<1, 64, 0, st>>>(sn, hdr, P, js, ds);
  sp_subhops_kernel<<<(P.n_big + 63) / 64, 64, 0, st>>>(sn, P);
  sp_walk_kernel<<<(P.n_hops + 63) / 64, 64, 0, st>>>(sn, P);
  sp_check_kernel<<<(P.n_tags_cap + 255) / 256, 256, 0, st>>>(in, sn, P);
  const uint32_t gb = (dn + 255) / 256;
  if (dn) {
    sp_bytes_kernel<<<gb, 256, 0, st>>>(in, sn, P);
    uint32_t *ps = P.pa, *pd = P.pb;
    uint32_t* changed = P.changed;  // one word per round
    e = hipMemsetAsync(changed, 0, 64 * 4, st);
    if (e != hipSuccess) return e;
    for (uint32_t r = 0; (1ull << r) < uint64_t(dn); r++) {  // chains are shorter than dn
      sp_ptr_kernel<<<gb, 256, 0, st>>>(dn, ps, pd, P.flag, changed, r);
      std::swap(ps, pd);
    }
    sp_gather_kernel<<<gb, 256, 0, st>>>(P, ps, out);
  }
  hipLaunchKernelGGL(snappy_stream_kernel, dim3(1), dim3(64), snappy_stream_lds_bytes(), st, in, sn, hdr, out, dn,
                     status, static_cast<const uint32_t*>(P.flag));
  return hipGetLastError();
}

}  // namespace slate
