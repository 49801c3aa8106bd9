// Streaming Snappy decode of one large buffer (an SST's index or bloom filter, decode.go:83-100,
// bloom.go:70-91), one wavefront: golang/snappy v0.0.4 decode (decode_other.go:19-110) with the
// same control flow and error checks as wave_snappy_decode (decode.hip), but the input is staged
// through a 32 KiB LDS window and the last 64 KiB of output stay in an LDS ring, so the tag walk
// pays LDS latency instead of global-memory latency.  A buffer like this is a single serial tag
// stream: the lane-per-block decoder would run it on one lane (~0.1 s for a 2.5 MB index).
// Copies reaching further back than the ring read the output already written to HBM.
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
__global__ __launch_bounds__(64) void snappy_stream_kernel(const uint8_t* in, uint32_t sn, uint32_t hdr, uint8_t* out,
                                                           uint32_t dn, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x;
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
                     status);
  return hipGetLastError();
}

}  // namespace slate
