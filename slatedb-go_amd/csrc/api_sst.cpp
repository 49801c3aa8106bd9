// C-ABI: SST builder (builder.go), table (flatbuf.go:143 EncodeTable), reader
// (decode.go), bloom (bloom.go) and single-block encode (block.go:54).
// Compute runs in the encode/decode kernels; this file does queueing and the
// flatbuffer footer framing only.
#include <algorithm>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <sys/mman.h>
#include <memory>
#include <vector>

#include "encode.h"
#include "flatbuf.h"
#include "host_ctx.h"

using namespace slate;

namespace {

inline uint64_t bloom_filter_bytes(uint32_t nk, uint32_t bpk) {  // bloom.go:135-139 (uint32 math)
  uint32_t bits = nk * bpk;
  return uint64_t(uint32_t(bits + 7) / 8);
}
inline uint16_t bloom_num_probes(uint32_t bpk) {  // bloom.go:174-178
  volatile float f = float(bpk) * 0.69f;
  return uint16_t(f);
}
inline void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24));
  v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}

}  // namespace

// ------------------------------------------------------------- GPU CRC helpers
int ctx_crc32_device(slate_ctx* ctx, const uint8_t* d_data, size_t n, uint32_t* crc) {
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(ctx->e_j.ensure(crc_scratch_bytes(n) + 16));
  uint32_t* scratch = ctx->e_j.as<uint32_t>();
  uint32_t* out = scratch + (crc_scratch_bytes(n) / 4);
  {
    GpuSpan gs(ctx, ctx->stream);
    SLATE_HIP(launch_crc32(ctx->stream, d_data, n, scratch, out, ctx->num_cus));
  }
  SLATE_HIP(hipMemcpyAsync(crc, out, 4, hipMemcpyDeviceToHost, ctx->stream));
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  return SLATE_OK;
}

int ctx_crc32_host_buffer(slate_ctx* ctx, const uint8_t* data, size_t n, uint32_t* crc) {
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(ctx->e_i.ensure(n + 16));
  // through the context's page-locked staging (a pageable copy of a 10 MB index ran at a few GB/s)
  const int s = ctx_h2d(ctx, ctx->e_i.p, data, n, ctx->stream);
  if (s) return s;
  return ctx_crc32_device(ctx, ctx->e_i.as<uint8_t>(), n, crc);
}

// ---------------------------------------------------------- Snappy helpers
// snappy.Encode (golang/snappy encode.go:17-42) of a device buffer: one wave per
// 64 KiB chunk on the GPU; the host only concatenates varint ‖ chunk outputs.
int ctx_snappy_encode_device(slate_ctx* ctx, const uint8_t* d_src, size_t n, std::vector<uint8_t>& out) {
  SLATE_HIP(ctx_bind(ctx));
  const uint64_t nch = (uint64_t(n) + kSnapMaxChunk - 1) / kSnapMaxChunk;
  SLATE_HIP(ctx->e_h.ensure(nch * kSnapChunkSlot + nch * 4 + 64));
  uint8_t* slots = ctx->e_h.as<uint8_t>();
  uint32_t* lens = reinterpret_cast<uint32_t*>(slots + nch * kSnapChunkSlot);
  SLATE_HIP(launch_snappy_chunks(ctx->stream, d_src, n, slots, lens, ctx->num_cus));
  std::vector<uint32_t> hl(nch);
  if (nch) SLATE_HIP(hipMemcpyAsync(hl.data(), lens, nch * 4, hipMemcpyDeviceToHost, ctx->stream));
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  out.clear();
  uint64_t v = n;
  while (v >= 0x80) {
    out.push_back(uint8_t(v) | 0x80);
    v >>= 7;
  }
  out.push_back(uint8_t(v));
  size_t o = out.size(), total = out.size();
  for (uint64_t c = 0; c < nch; c++) total += hl[c];
  out.resize(total);
  for (uint64_t c = 0; c < nch; c++) {
    if (hl[c]) SLATE_HIP(hipMemcpyAsync(out.data() + o, slots + c * kSnapChunkSlot, hl[c], hipMemcpyDeviceToHost,
                                        ctx->stream));
    o += hl[c];
  }
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  return SLATE_OK;
}

// The same encoding assembled on the device: varint header and the chunks' encodings back to back
// in `asmb` (device-to-device copies on stream st), then its CRC32 on the device, so the encoded
// payload crosses the link once (into `out` after `out`'s current bytes), with its BE32 CRC
// appended (bloom.Encode / encodeIndex framing).  slots / asmb / crcb: the buffers it may use;
// lanes: large copies through the context's page-locked lanes (only from the context's own thread).
static int snappy_encode_crc_on(slate_ctx* ctx, hipStream_t st, DevBuf& slotb, DevBuf& asmb, DevBuf& crcb,
                                const uint8_t* d_src, size_t n, std::vector<uint8_t>& out, bool lanes,
                                const std::function<void()>* launched = nullptr) {
  SLATE_HIP(ctx_bind(ctx));
  const uint64_t nch = (uint64_t(n) + kSnapMaxChunk - 1) / kSnapMaxChunk;
  SLATE_HIP(slotb.ensure(nch * kSnapChunkSlot + nch * 12 + 64));
  uint8_t* slots = slotb.as<uint8_t>();
  uint32_t* lens = reinterpret_cast<uint32_t*>(slots + nch * kSnapChunkSlot);
  uint64_t* d_off = reinterpret_cast<uint64_t*>(slots + nch * kSnapChunkSlot + ((nch * 4 + 7) & ~uint64_t(7)));
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_snappy_chunks(st, d_src, n, slots, lens, ctx->num_cus));
    gs.stop();
    if (launched) (*launched)();  // (before the span's destructor waits for the kernel, timing on)
  }
  std::vector<uint32_t> hl(nch);
  if (nch) SLATE_HIP(hipMemcpyAsync(hl.data(), lens, nch * 4, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  uint8_t hdr[10];
  size_t hn = 0;
  for (uint64_t v = n; ; v >>= 7) {
    hdr[hn++] = uint8_t(v & 0x7f) | (v >= 0x80 ? 0x80 : 0);
    if (v < 0x80) break;
  }
  size_t total = hn;
  for (uint64_t c = 0; c < nch; c++) total += hl[c];
  SLATE_HIP(asmb.ensure(total + 64));
  uint8_t* d = asmb.as<uint8_t>();
  SLATE_HIP(hipMemcpyAsync(d, hdr, hn, hipMemcpyHostToDevice, st));
  // the chunks back to back after the length header: one gather launch (offsets from the host)
  std::vector<uint64_t> ho(nch);
  size_t o = hn;
  for (uint64_t c = 0; c < nch; c++) {
    ho[c] = o;
    o += hl[c];
  }
  if (nch) SLATE_HIP(hipMemcpyAsync(d_off, ho.data(), nch * 8, hipMemcpyHostToDevice, st));
  SLATE_HIP(crcb.ensure(crc_scratch_bytes(total) + 16));
  uint32_t* scratch = crcb.as<uint32_t>();
  uint32_t* cout = scratch + (crc_scratch_bytes(total) / 4);
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_snappy_gather(st, slots, lens, d_off, nch, d));
    SLATE_HIP(launch_crc32(st, d, total, scratch, cout, ctx->num_cus));
  }
  uint32_t crc = 0;
  SLATE_HIP(hipMemcpyAsync(&crc, cout, 4, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const size_t base = out.size();
  out.resize(base + total + 4);
  if (lanes) {
    const int s2 = ctx_d2h(ctx, out.data() + base, d, total, st);
    if (s2) return s2;
  } else if (total) {
    SLATE_HIP(hipMemcpyAsync(out.data() + base, d, total, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
  }
  out[base + total] = uint8_t(crc >> 24);
  out[base + total + 1] = uint8_t(crc >> 16);
  out[base + total + 2] = uint8_t(crc >> 8);
  out[base + total + 3] = uint8_t(crc);
  return SLATE_OK;
}

int ctx_snappy_encode_crc_device(slate_ctx* ctx, const uint8_t* d_src, size_t n, std::vector<uint8_t>& out) {
  return snappy_encode_crc_on(ctx, ctx->stream, ctx->e_h, ctx->e_k, ctx->e_j, d_src, n, out, true);
}

int ctx_snappy_encode_host(slate_ctx* ctx, const uint8_t* data, size_t n, std::vector<uint8_t>& out) {
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(ctx->e_i.ensure(n + 16));
  if (n) SLATE_HIP(hipMemcpyAsync(ctx->e_i.p, data, n, hipMemcpyHostToDevice, ctx->stream));
  return ctx_snappy_encode_device(ctx, ctx->e_i.as<uint8_t>(), n, out);
}

// compress.Encode (compression.go:80-116) with CodecLz4 / CodecZlib / CodecZstd of n payloads
// already on the device (payload i: raw_len[i] bytes at d_raw + raw_start[i]): frames back to back
// at codec_frames(ctx) (ctx->c_out after kFramePad bytes: the frame CRC reads the aligned dword
// before a frame), each followed by its BE32 CRC32 when with_crc (block.Encode, bloom.Encode,
// encodeIndex framing); out_off (n + 1) on the host.  encode_codecs.hip does the work.
constexpr size_t kFramePad = 16;
static uint8_t* codec_frames(slate_ctx* ctx) { return ctx->c_out.as<uint8_t>() + kFramePad; }
static int ctx_codec_frames(slate_ctx* ctx, int codec, const uint8_t* d_raw, const uint64_t* raw_start,
                            const uint64_t* raw_len, uint64_t n, bool with_crc, std::vector<uint64_t>& out_off) {
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx_bind(ctx));
  std::vector<CodecPiece> pieces;
  std::vector<CodecPayload> pay(n);
  std::vector<uint32_t> small, big;
  uint64_t tags = 0, bodies = 0, seqs = 0;
  for (uint64_t p = 0; p < n; p++) {
    const uint64_t len = raw_len[p];
    if (len > 0xFFFFFF00ull) return SLATE_E_INVALID_ARG;
    const uint32_t np = len ? uint32_t((len + kCodecPieceMax - 1) / kCodecPieceMax) : 1u;
    pay[p] = CodecPayload{raw_start[p], uint32_t(len), uint32_t(pieces.size()), np, 0};
    for (uint32_t k = 0; k < np; k++) {
      const uint32_t l = uint32_t(std::min<uint64_t>(kCodecPieceMax, len - uint64_t(k) * kCodecPieceMax));
      CodecPiece c{raw_start[p] + uint64_t(k) * kCodecPieceMax, tags, bodies, seqs, l,
                   (k == 0 ? 1u : 0u) | (k + 1 == np ? 2u : 0u)};
      tags += codec_piece_tags_bytes(l);
      bodies += codec_piece_body_bytes(l);
      if (l > kCodecSmallPiece) {
        seqs += l / 3 + 2;
        big.push_back(uint32_t(pieces.size()));
      } else {
        small.push_back(uint32_t(pieces.size()));
      }
      pieces.push_back(c);
    }
  }
  const uint64_t np = pieces.size();
  // device tables: pieces | payloads | small list | big list | tag_len | body_len | out_off
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_pc = carve(np * sizeof(CodecPiece)), o_pay = carve(n * sizeof(CodecPayload)),
               o_sl = carve(small.size() * 4 + 4), o_bl = carve(big.size() * 4 + 4), o_tl = carve(np * 4),
               o_bo = carve(np * 4), o_oo = carve((n + 1) * 8);
  SLATE_HIP(ctx->c_meta.ensure(off));
  SLATE_HIP(ctx->c_tags.ensure(tags + 64));
  SLATE_HIP(ctx->c_bodies.ensure(bodies + 64));
  SLATE_HIP(ctx->c_seqs.ensure(seqs * kCodecSeqBytes + 64));
  uint8_t* m = ctx->c_meta.as<uint8_t>();
  auto* d_pc = reinterpret_cast<CodecPiece*>(m + o_pc);
  auto* d_pay = reinterpret_cast<CodecPayload*>(m + o_pay);
  auto* d_sl = reinterpret_cast<uint32_t*>(m + o_sl);
  auto* d_bl = reinterpret_cast<uint32_t*>(m + o_bl);
  auto* d_tl = reinterpret_cast<uint32_t*>(m + o_tl);
  auto* d_bo = reinterpret_cast<uint32_t*>(m + o_bo);
  auto* d_oo = reinterpret_cast<uint64_t*>(m + o_oo);
  int s = ctx_h2d(ctx, d_pc, pieces.data(), np * sizeof(CodecPiece), st);
  if (!s) s = ctx_h2d(ctx, d_pay, pay.data(), n * sizeof(CodecPayload), st);
  if (!s && !small.empty()) s = ctx_h2d(ctx, d_sl, small.data(), small.size() * 4, st);
  if (!s && !big.empty()) s = ctx_h2d(ctx, d_bl, big.data(), big.size() * 4, st);
  if (s) return s;
  SLATE_HIP(launch_codec_encode(st, codec, d_raw, d_pc, d_sl, uint32_t(small.size()), d_bl, uint32_t(big.size()),
                                ctx->c_tags.as<uint8_t>(), d_tl, ctx->c_bodies.as<uint8_t>(), d_bo, ctx->c_seqs.p,
                                ctx->num_cus));
  std::vector<uint32_t> bl(np);
  s = ctx_d2h(ctx, bl.data(), d_bo, np * 4, st);
  if (s) return s;
  // frame sizes (pc_frame_kernel's layout)
  out_off.assign(n + 1, 0);
  for (uint64_t p = 0; p < n; p++) {
    uint64_t f = 0;
    const uint32_t L = pay[p].len;
    if (codec == SLATE_CODEC_LZ4) f = 7 + 8;
    else if (codec == SLATE_CODEC_ZLIB) f = 2 + 4;
    else f = 4 + 1 + (L < 256 ? 1 : (L < 65536 + 256 ? 2 : 4)) + 4;
    for (uint32_t k = 0; k < pay[p].npieces; k++) {
      const CodecPiece& c = pieces[pay[p].first + k];
      const uint32_t b = bl[pay[p].first + k];
      if (codec == SLATE_CODEC_ZLIB && b == kBodyRaw) return SLATE_E_HIP;  // deflate always fits its slot
      const uint64_t body = b == kBodyRaw ? c.len : b;
      if (codec == SLATE_CODEC_LZ4) f += c.len ? 4 + body : 0;
      else if (codec == SLATE_CODEC_ZSTD) f += 3 + body;
      else f += body;
    }
    out_off[p + 1] = out_off[p] + f + (with_crc ? 4 : 0);
  }
  SLATE_HIP(ctx->c_out.ensure(out_off[n] + kFramePad + 64));
  s = ctx_h2d(ctx, d_oo, out_off.data(), (n + 1) * 8, st);
  if (s) return s;
  SLATE_HIP(launch_codec_frames(st, codec, d_raw, d_pay, uint32_t(n), d_pc, ctx->c_bodies.as<uint8_t>(), d_bo, d_oo,
                                codec_frames(ctx), with_crc, ctx->num_cus));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

// compress.Encode (compression.go:80-116) of a host buffer.
static int codec_encode_host(slate_ctx* ctx, int codec, const uint8_t* data, size_t n, std::vector<uint8_t>& out) {
  if (codec == SLATE_CODEC_NONE) {
    out.assign(data, data + n);
    return SLATE_OK;
  }
  if (codec == SLATE_CODEC_SNAPPY) return ctx_snappy_encode_host(ctx, data, n, out);
  if (codec != SLATE_CODEC_LZ4 && codec != SLATE_CODEC_ZLIB && codec != SLATE_CODEC_ZSTD) return SLATE_E_INVALID_CODEC;
  SLATE_HIP(ctx_bind(ctx));
  SLATE_HIP(ctx->c_in.ensure(n + 64));
  int s = ctx_h2d(ctx, ctx->c_in.p, data, n, ctx->stream);
  if (s) return s;
  const uint64_t start = 0, len = n;
  std::vector<uint64_t> fo;
  s = ctx_codec_frames(ctx, codec, ctx->c_in.as<uint8_t>(), &start, &len, 1, false, fo);
  if (s) return s;
  out.resize(fo[1]);
  return ctx_d2h(ctx, out.data(), codec_frames(ctx), fo[1], ctx->stream);
}

// CRC32 verify + snappy.Decode of one `payload ‖ BE32 CRC` buffer (index,
// filter) on the GPU: the lane-per-block decoder in raw mode.  *bstatus gets
// SLATE_OK, SLATE_E_BLOCK_CHECKSUM or SLATE_E_SNAPPY_CORRUPT.
int ctx_snappy_decode_buffer(slate_ctx* ctx, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                             int* bstatus) {
  if (len < 4) return SLATE_E_INVALID_ARG;
  const size_t clen = len - 4;
  uint64_t dl = 0;
  uint32_t hdr_len = 0;
  // above this decoded size the lane-per-block decoder would walk the stream on one lane
  constexpr uint64_t kStreamMin = 16384;
  {
    uint64_t x = 0;
    uint32_t sft = 0;
    bool ok = false;
    for (size_t i = 0; i < clen && i < 10; i++) {
      uint32_t bt = buf[i];
      if (bt < 0x80) {
        if (i == 9 && bt > 1) break;
        x |= uint64_t(bt) << sft;
        ok = x <= 0xffffffffull;
        break;
      }
      x |= uint64_t(bt & 0x7f) << sft;
      sft += 7;
    }
    if (ok && x <= kSnappyMaxExpansion * uint64_t(clen)) {
      dl = x;  // else the kernel reports it
      hdr_len = 0;
      while (buf[hdr_len] >= 0x80) hdr_len++;
      hdr_len++;
    }
  }
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  if (dl > kStreamMin && dl <= 0xFFFFFFF0ull && clen <= 0xFFFFFFF0ull) {
    // one long serial tag stream (an index or filter): the one-wave streaming decoder after
    // a GPU CRC (block.go / bloom.go order: checksum first, then decode)
    uint32_t crc = 0;
    int cs = ctx_crc32_host_buffer(ctx, buf, clen, &crc);
    if (cs != SLATE_OK) return cs;
    const uint32_t want = (uint32_t(buf[clen]) << 24) | (uint32_t(buf[clen + 1]) << 16) |
                          (uint32_t(buf[clen + 2]) << 8) | uint32_t(buf[clen + 3]);
    if (crc != want) {
      *bstatus = SLATE_E_BLOCK_CHECKSUM;
      return SLATE_OK;
    }
    SLATE_HIP(ctx->d_in.ensure(len + 64));
    SLATE_HIP(ctx->d_out.ensure(align16(dl) + 32));
    SLATE_HIP(ctx->d_scratch.ensure(256 + snappy_par_scratch_bytes(uint32_t(clen), uint32_t(dl))));
    int32_t* d_st = ctx->d_scratch.as<int32_t>();
    SLATE_HIP(hipMemcpyAsync(ctx->d_in.p, buf, clen, hipMemcpyHostToDevice, st));
    // the tag-parallel decoder; the serial streaming decoder runs instead (on the device, same
    // launch sequence) when the stream fails one of its checks
    SLATE_HIP(launch_snappy_decode_par(st, ctx->d_in.as<uint8_t>(), uint32_t(clen), hdr_len, ctx->d_out.as<uint8_t>(),
                                       uint32_t(dl), ctx->d_scratch.as<uint8_t>() + 256, d_st));
    int32_t h_st = 0;
    SLATE_HIP(hipMemcpyAsync(&h_st, d_st, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    *bstatus = h_st;
    if (h_st == SLATE_OK) {
      out.resize(dl);
      SLATE_HIP(hipMemcpyAsync(out.data(), ctx->d_out.p, dl, hipMemcpyDeviceToHost, st));
      SLATE_HIP(hipStreamSynchronize(st));
    }
    return SLATE_OK;
  }
  SLATE_HIP(ctx->d_in.ensure(len + 16));
  SLATE_HIP(ctx->d_out.ensure(align16(dl) + 32));
  SLATE_HIP(ctx->d_scratch.ensure(128));
  uint64_t* u = ctx->d_scratch.as<uint64_t>();  // in_off[2] | out_off[2] | row_base[2] | meta(16) | rows(16)
  const uint64_t hv[6] = {0, len, 0, align16(dl), 0, 0};
  SLATE_HIP(hipMemcpyAsync(ctx->d_in.p, buf, len, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(u, hv, sizeof(hv), hipMemcpyHostToDevice, st));
  DecodeArgs a{SLATE_CODEC_SNAPPY, ctx->d_in.as<uint8_t>(), u, 1, ctx->d_out.as<uint8_t>(), u + 2,
               reinterpret_cast<slate_block_meta*>(u + 6), reinterpret_cast<slate_row*>(u + 8), u + 4,
               reinterpret_cast<uint32_t*>(u + 11), reinterpret_cast<uint32_t*>(u + 10), 0};
  a.raw = 1;
  SLATE_HIP(launch_decode_lpb2(st, a, ctx->num_cus));
  slate_block_meta m;
  SLATE_HIP(hipMemcpyAsync(&m, u + 6, sizeof(m), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  *bstatus = m.status;
  if (m.status == SLATE_OK) {
    out.resize(m.data_len);
    if (m.data_len) {
      SLATE_HIP(hipMemcpyAsync(out.data(), ctx->d_out.p, m.data_len, hipMemcpyDeviceToHost, st));
      SLATE_HIP(hipStreamSynchronize(st));
    }
  }
  return SLATE_OK;
}

// Any codec: Snappy through the function above; LZ4 / Zlib / Zstd through the plan kernels
// (decoded capacity) and one wave per payload reading and writing HBM (decode_payload_kernel).
// payloads from this size on take the split paths (smaller ones: one wave, no set-up)
constexpr size_t kSplitMin = 32 * 1024;

// XXH32 (seed 0) of a few host bytes (the LZ4 frame descriptor's checksum byte).
static uint32_t xxh32_small(const uint8_t* p, size_t n) {
  constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  uint32_t h = P5 + uint32_t(n);  // n < 16
  size_t i = 0;
  for (; i + 4 <= n; i += 4) h = rotl(h + (uint32_t(p[i]) | uint32_t(p[i + 1]) << 8 | uint32_t(p[i + 2]) << 16 |
                                           uint32_t(p[i + 3]) << 24) * P3, 17) * P4;
  for (; i < n; i++) h = rotl(h + uint32_t(p[i]) * P5, 11) * P1;
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

// Adler-32 (RFC 1950) of n device bytes: a = 1 + sum x, b = n + sum (n - j) x, from 4 KiB slices'
// partial sums (stream-synchronous).
static int device_adler32(slate_ctx* ctx, const uint8_t* d, uint32_t n, uint32_t* adler) {
  hipStream_t st = ctx->stream;
  const uint32_t nsl = (n + 4095) / 4096;
  SLATE_HIP(ctx->e_k.ensure(size_t(nsl) * 16 + 64));
  if (nsl) SLATE_HIP(launch_adler_slices(st, d, n, ctx->e_k.as<uint64_t>()));
  std::vector<uint64_t> part(2 * size_t(nsl));
  if (nsl) SLATE_HIP(hipMemcpyAsync(part.data(), ctx->e_k.p, part.size() * 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  uint64_t a = 1, b = n % 65521;
  for (uint32_t t = 0; t < nsl; t++) {
    const uint64_t end = std::min<uint64_t>(n, 4096ull * (t + 1));
    a = (a + part[2 * t]) % 65521;
    b = (b + part[2 * t + 1] % 65521 + (part[2 * t] % 65521) * ((n - end) % 65521)) % 65521;
  }
  *adler = uint32_t((b << 16) | a);
  return SLATE_OK;
}

// The GPU part of the split payload paths: the payload's CRC, then its blocks (blk = offset /
// header word pairs) one wave each into 64 KiB slots, their outputs concatenated, the content size
// and checksum (LZ4: XXH32; Zstd: XXH64's low half), and the decoded bytes back into `out`.
static int payload_split_run(slate_ctx* ctx, const uint8_t* buf, size_t len, const std::vector<uint32_t>& blk,
                             uint32_t bmax, int codec, bool has_size, uint64_t content, bool has_sum, uint32_t want,
                             std::vector<uint8_t>& out, int* bstatus, int* handled) {
  const size_t clen = len - 4;
  const uint32_t nblk = uint32_t(blk.size() / 2);
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx->d_in.ensure(len + 64));
  int s = ctx_h2d(ctx, ctx->d_in.p, buf, len, st);
  if (s) return s;
  uint32_t crc = 0;
  s = ctx_crc32_device(ctx, ctx->d_in.as<uint8_t>(), clen, &crc);
  if (s) return s;
  if (crc != ld_be32(buf + clen)) {
    *bstatus = SLATE_E_BLOCK_CHECKSUM;  // block.Decode / bloom.Decode / DecodeIndex check it first
    *handled = 1;
    return SLATE_OK;
  }
  SLATE_HIP(ctx->d_scratch.ensure(size_t(nblk) * 12 + 64));
  uint32_t* d_blk = ctx->d_scratch.as<uint32_t>();
  uint32_t* d_sizes = d_blk + 2 * size_t(nblk);
  SLATE_HIP(ctx->d_rows.ensure(size_t(nblk) * kLz4PayloadSlot + 64));  // the blocks' output slots
  if (nblk) SLATE_HIP(hipMemcpyAsync(d_blk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, st));
  if (codec == SLATE_CODEC_LZ4)
    SLATE_HIP(launch_lz4_payload_blocks(st, ctx->d_in.as<uint8_t>(), d_blk, nblk, bmax, ctx->d_rows.as<uint8_t>(),
                                        d_sizes, ctx->num_cus));
  else if (codec == SLATE_CODEC_ZSTD)
    SLATE_HIP(launch_zstd_payload_blocks(st, ctx->d_in.as<uint8_t>(), d_blk, nblk, bmax, ctx->d_rows.as<uint8_t>(),
                                         d_sizes, ctx->num_cus));
  else
    SLATE_HIP(launch_zlib_payload_segs(st, ctx->d_in.as<uint8_t>(), d_blk, nblk, ctx->d_rows.as<uint8_t>(), d_sizes,
                                       ctx->num_cus));
  std::vector<uint32_t> sizes(nblk);
  if (nblk) SLATE_HIP(hipMemcpyAsync(sizes.data(), d_sizes, size_t(nblk) * 4, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  uint64_t total = 0;
  for (uint32_t k = 0; k < nblk; k++) {
    if (sizes[k] == ~0u) return SLATE_OK;  // the serial path decodes (and reports) it
    total += sizes[k];
  }
  if (total > 0xFFFFFF00ull || (has_size && content != total)) return SLATE_OK;
  SLATE_HIP(ctx->d_out.ensure(total + 64));
  uint8_t* d_out = ctx->d_out.as<uint8_t>();
  uint64_t o = 0;
  for (uint32_t k = 0; k < nblk; k++) {
    if (sizes[k])
      SLATE_HIP(hipMemcpyAsync(d_out + o, ctx->d_rows.as<uint8_t>() + size_t(k) * kLz4PayloadSlot, sizes[k],
                               hipMemcpyDeviceToDevice, st));
    o += sizes[k];
  }
  if (has_sum && codec == SLATE_CODEC_ZLIB) {
    uint32_t got = 0;
    s = device_adler32(ctx, d_out, uint32_t(total), &got);
    if (s) return s;
    if (got != want) return SLATE_OK;  // the serial path reports the checksum
  } else if (has_sum) {
    if (codec == SLATE_CODEC_LZ4) SLATE_HIP(launch_xxh32(st, d_out, uint32_t(total), d_sizes));
    else SLATE_HIP(launch_xxh64_lo(st, d_out, uint32_t(total), d_sizes));
    uint32_t got = 0;
    SLATE_HIP(hipMemcpyAsync(&got, d_sizes, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    if (got != want) return SLATE_OK;  // the serial path reports the checksum
  }
  out.resize(total);
  s = ctx_d2h(ctx, out.data(), d_out, total, st);
  if (s) return s;
  *bstatus = SLATE_OK;
  *handled = 1;
  return SLATE_OK;
}

// LZ4 frames with larger data blocks -- pierrec/lz4 v4's writer defaults: 4 MiB blocks, a content
// checksum -- or linked blocks have each compressed block decoded by the tag-parallel passes
// (snappy_stream.hip launch_lz4_par_chain / _bytes) over the whole GPU, one block after another
// (a linked block's matches may reach into the blocks before it); stored blocks are copied.  Same
// contract as lz4_payload_split.
static int lz4_payload_par_run(slate_ctx* ctx, const uint8_t* buf, size_t len, const std::vector<uint32_t>& blk,
                               uint32_t bmax, bool indep, bool has_size, uint64_t content, bool has_sum, uint32_t want,
                               std::vector<uint8_t>& out, int* bstatus, int* handled) {
  const size_t clen = len - 4;
  const uint32_t nblk = uint32_t(blk.size() / 2);
  // a block decodes to at most bmax bytes, and to at most 255 per encoded byte (+ the last
  // literals): cap[k] bounds block k, their sum the output buffer
  auto cap_of = [&](uint32_t k) -> uint32_t {
    const uint32_t bs = blk[2 * k + 1], sz = bs & 0x7FFFFFFFu;
    return (bs >> 31) ? sz : uint32_t(std::min<uint64_t>(bmax, 256ull * sz + 64));
  };
  uint64_t out_bound = 0;
  uint32_t smax = 0, cmax = 0;
  for (uint32_t k = 0; k < nblk; k++) {
    out_bound += cap_of(k);
    smax = std::max(smax, blk[2 * k + 1] & 0x7FFFFFFFu);
    cmax = std::max(cmax, cap_of(k));
  }
  if (out_bound > (1ull << 31)) return SLATE_OK;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx->d_in.ensure(len + 64));
  int s = ctx_h2d(ctx, ctx->d_in.p, buf, len, st);
  if (s) return s;
  uint32_t crc = 0;
  s = ctx_crc32_device(ctx, ctx->d_in.as<uint8_t>(), clen, &crc);
  if (s) return s;
  if (crc != ld_be32(buf + clen)) {
    *bstatus = SLATE_E_BLOCK_CHECKSUM;  // block.Decode / bloom.Decode / DecodeIndex check it first
    *handled = 1;
    return SLATE_OK;
  }
  SLATE_HIP(ctx->d_scratch.ensure(lz4_par_scratch_bytes(smax, cmax) + 64));
  SLATE_HIP(ctx->d_out.ensure(out_bound + 64));
  SLATE_HIP(ctx->e_k.ensure(64));
  uint8_t* d_in = ctx->d_in.as<uint8_t>();
  uint8_t* d_out = ctx->d_out.as<uint8_t>();
  void* scratch = ctx->d_scratch.p;
  uint64_t total = 0;
  for (uint32_t k = 0; k < nblk; k++) {
    const uint32_t off = blk[2 * k], bs = blk[2 * k + 1], sz = bs & 0x7FFFFFFFu;
    if (bs >> 31) {  // stored
      if (sz) SLATE_HIP(hipMemcpyAsync(d_out + total, d_in + off, sz, hipMemcpyDeviceToDevice, st));
      total += sz;
      continue;
    }
    uint32_t res[5] = {1, 0, 0, 0, 0};
    const uint32_t cap = cap_of(k);  // = bmax whenever a block could reach it
    const uint32_t* d_res = lz4_par_result(scratch, sz, cap);
    SLATE_HIP(launch_lz4_par_chain(st, d_in + off, sz, cap, scratch));
    SLATE_HIP(hipMemcpyAsync(res, d_res, sizeof(res), hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    if (res[0]) return SLATE_OK;  // the serial path decodes (and reports) it
    const uint32_t dn = res[4];
    SLATE_HIP(launch_lz4_par_bytes(st, d_in + off, sz, cap, dn, indep ? 0u : uint32_t(total), scratch,
                                   d_out + total));
    SLATE_HIP(hipMemcpyAsync(res, d_res, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    if (res[0]) return SLATE_OK;
    total += dn;
  }
  if (total > 0xFFFFFF00ull || (has_size && content != total)) return SLATE_OK;
  if (has_sum) {
    SLATE_HIP(launch_xxh32(st, d_out, uint32_t(total), ctx->e_k.as<uint32_t>()));
    uint32_t got = 0;
    SLATE_HIP(hipMemcpyAsync(&got, ctx->e_k.p, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    if (got != want) return SLATE_OK;  // the serial path reports the checksum
  }
  out.resize(total);
  s = ctx_d2h(ctx, out.data(), d_out, total, st);
  if (s) return s;
  *bstatus = SLATE_OK;
  *handled = 1;
  return SLATE_OK;
}

// A large CodecLz4 index / filter (`frame || BE32 CRC`) decoded block by block in parallel when
// its frame has no block checksums and no dictionary: independent blocks of at most 64 KiB (the
// shape this builder writes) one wave each, larger or linked ones (pierrec's 4 MiB blocks)
// through lz4_payload_par_run.  The frame header and the
// block list are read here (structure only, as the plan does); the CRC, the blocks and the
// content checksum are computed on the GPU.  Returns 1 with *bstatus and `out` set, or 0 when
// the serial path must decode the payload (another shape, or any check failing: that path then
// reports it exactly); < 0 never (HIP errors are returned as their status).
static int lz4_payload_split(slate_ctx* ctx, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                             int* bstatus, int* handled) {
  *handled = 0;
  const size_t clen = len - 4;
  const uint8_t* f = buf;
  auto le32 = [&](size_t i) {
    return uint32_t(f[i]) | uint32_t(f[i + 1]) << 8 | uint32_t(f[i + 2]) << 16 | uint32_t(f[i + 3]) << 24;
  };
  if (clen < 7 || le32(0) != 0x184D2204u) return SLATE_OK;
  const uint32_t flg = f[4], bd = f[5];
  if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8F) || ((bd >> 4) & 7) < 4 || (flg & 1) || (flg & 0x10))
    return SLATE_OK;
  const bool indep = (flg & 0x20) != 0;
  const uint32_t bmax = 1u << (8 + 2 * ((bd >> 4) & 7));
  const size_t hl = 2 + ((flg & 8) ? 8 : 0);
  if (clen < 4 + hl + 1 || f[4 + hl] != ((xxh32_small(f + 4, hl) >> 8) & 0xFF)) return SLATE_OK;
  uint64_t content = 0;
  if (flg & 8)
    for (int k = 7; k >= 0; k--) content = (content << 8) | f[6 + k];
  std::vector<uint32_t> blk;
  size_t pos = 4 + hl + 1;
  for (;;) {
    if (clen - pos < 4) return SLATE_OK;
    const uint32_t bs = le32(pos);
    if (bs == 0) {
      pos += 4;
      break;
    }
    const uint32_t sz = bs & 0x7FFFFFFFu;
    if (sz > bmax || clen - pos - 4 < sz || pos + 4 > 0xFFFFFFFFull) return SLATE_OK;
    blk.push_back(uint32_t(pos + 4));
    blk.push_back(bs);
    pos += 4 + sz;
  }
  uint32_t want = 0;
  const bool ccheck = (flg & 4) != 0;
  if (ccheck) {
    if (clen - pos < 4) return SLATE_OK;
    want = le32(pos);
    pos += 4;
  }
  if (pos != clen) return SLATE_OK;
  if (bmax > kLz4PayloadSlot || !indep)
    return lz4_payload_par_run(ctx, buf, len, blk, bmax, indep, (flg & 8) != 0, content, ccheck, want, out, bstatus, handled);
  return payload_split_run(ctx, buf, len, blk, bmax, SLATE_CODEC_LZ4, (flg & 8) != 0, content, ccheck, want, out,
                           bstatus, handled);
}

// A large CodecZstd index / filter that is one frame whose blocks depend on each other -- repeat
// offsets, treeless literals and repeat tables across blocks, the frames klauspost/compress's
// streaming writer (compression.go:105-118) and libzstd write -- through the block-parallel decoder
// (zstd_par.hip): headers and entropy state first, then literals, sequences and bytes per block;
// the content size and XXH64 last.  Same contract as lz4_payload_split.
static int zstd_payload_par_run(slate_ctx* ctx, const uint8_t* buf, size_t len, const std::vector<uint32_t>& blk,
                                uint32_t bmax, bool has_size, uint64_t content, bool has_sum, uint32_t want,
                                std::vector<uint8_t>& out, int* bstatus, int* handled) {
  *handled = 0;
  const size_t clen = len - 4;
  const uint32_t nblk = uint32_t(blk.size() / 2);
  if (nblk == 0 || nblk > (1u << 16) || clen >= (1u << 28)) return SLATE_OK;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx->d_in.ensure(len + 64));
  int s = ctx_h2d(ctx, ctx->d_in.p, buf, len, st);
  if (s) return s;
  uint32_t crc = 0;
  s = ctx_crc32_device(ctx, ctx->d_in.as<uint8_t>(), clen, &crc);
  if (s) return s;
  if (crc != ld_be32(buf + clen)) {
    *bstatus = SLATE_E_BLOCK_CHECKSUM;  // block.Decode / bloom.Decode / DecodeIndex check it first
    *handled = 1;
    return SLATE_OK;
  }
  const double t0 = host_trace() ? now_ms() : 0.0;
  const uint8_t* d_in = ctx->d_in.as<uint8_t>();
  SLATE_HIP(ctx->d_scratch.ensure(zstd_par_scratch_bytes(nblk) + 64));
  SLATE_HIP(ctx->e_b.ensure(blk.size() * 4 + 64));
  void* scratch = ctx->d_scratch.p;
  SLATE_HIP(hipMemcpyAsync(ctx->e_b.p, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, st));
  SLATE_HIP(launch_zstd_par_headers(st, d_in, ctx->e_b.as<uint32_t>(), nblk, bmax, scratch, ctx->num_cus));
  uint32_t res[4] = {1, 0, 0, 0};
  SLATE_HIP(hipMemcpyAsync(res, zstd_par_result(scratch), sizeof(res), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  if (res[0]) {
    if (host_trace()) fprintf(stderr, "[slate zstd-par] %u blocks: headers refused\n", nblk);
    return SLATE_OK;  // the serial path decodes (and reports) it
  }
  const uint32_t nseq = res[1], nlit = res[2];
  SLATE_HIP(ctx->d_rows.ensure(size_t(nlit) + 64));                        // literals
  SLATE_HIP(ctx->e_c.ensure(3 * (size_t(nseq) + 64) * 4 + 256));           // ll | ml | offset
  uint32_t* sll = ctx->e_c.as<uint32_t>();
  uint32_t* sml = sll + nseq + 64;
  uint32_t* sof = sml + nseq + 64;
  SLATE_HIP(launch_zstd_par_body(st, d_in, nblk, bmax, scratch, ctx->d_rows.as<uint8_t>(), sll, sml, sof,
                                 ctx->num_cus));
  SLATE_HIP(hipMemcpyAsync(res, zstd_par_result(scratch), sizeof(res), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const double t1 = host_trace() ? now_ms() : 0.0;
  if (host_trace())
    fprintf(stderr, "[slate zstd-par] %u blocks, %u sequences, %u literals, %u B out, fail %u: headers+body %.2f ms\n",
            nblk, nseq, nlit, res[3], res[0], t1 - t0);
  if (res[0]) return SLATE_OK;
  const uint32_t total = res[3];
  if (has_size && content != total) return SLATE_OK;  // the serial path reports the frame size
  SLATE_HIP(ctx->d_out.ensure(size_t(total) + 64));
  SLATE_HIP(ctx->e_a.ensure(2 * (size_t(total) + 1) * 4 + 64 * 4 + 256));  // pa | pb | changed
  SLATE_HIP(ctx->e_d.ensure(size_t(total) + 64));                          // val
  uint32_t* pa = ctx->e_a.as<uint32_t>();
  uint32_t* pb = pa + total + 1;
  uint32_t* changed = pb + total + 1;
  uint8_t* d_out = ctx->d_out.as<uint8_t>();
  SLATE_HIP(launch_zstd_par_bytes(st, d_in, nblk, total, scratch, ctx->d_rows.as<uint8_t>(), sll, sml, sof,
                                  ctx->e_d.as<uint8_t>(), pa, pb, changed, d_out, ctx->num_cus));
  if (has_sum) SLATE_HIP(launch_xxh64_lo(st, d_out, total, ctx->e_b.as<uint32_t>()));
  uint32_t tail[2] = {1, 0};
  SLATE_HIP(hipMemcpyAsync(tail, zstd_par_result(scratch), 4, hipMemcpyDeviceToHost, st));
  if (has_sum) SLATE_HIP(hipMemcpyAsync(tail + 1, ctx->e_b.p, 4, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  if (host_trace()) fprintf(stderr, "[slate zstd-par] bytes + checksum %.2f ms, fail %u\n", now_ms() - t1, tail[0]);
  if (tail[0] || (has_sum && tail[1] != want)) return SLATE_OK;  // the serial path reports it
  out.resize(total);
  s = ctx_d2h(ctx, out.data(), d_out, total, st);
  if (s) return s;
  *bstatus = SLATE_OK;
  *handled = 1;
  return SLATE_OK;
}

// A large CodecZstd index / filter decoded block by block in parallel when it is one frame whose
// compressed blocks decode on their own (the frames this builder writes; decode.hip
// zstd_payload_blocks_kernel checks it block by block).  Same contract as lz4_payload_split.
static int zstd_payload_split(slate_ctx* ctx, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                              int* bstatus, int* handled) {
  *handled = 0;
  const size_t clen = len - 4;
  const uint8_t* f = buf;
  auto le32 = [&](size_t i) {
    return uint32_t(f[i]) | uint32_t(f[i + 1]) << 8 | uint32_t(f[i + 2]) << 16 | uint32_t(f[i + 3]) << 24;
  };
  if (clen < 6 || le32(0) != 0xFD2FB528u) return SLATE_OK;
  const uint32_t fhd = f[4], fcsf = fhd >> 6, ss = (fhd >> 5) & 1, dif = fhd & 3;
  if (fhd & 8) return SLATE_OK;
  const uint32_t dsz = dif == 3 ? 4 : dif, fl = fcsf == 0 ? ss : (2u << (fcsf - 1));
  const size_t hsize = 1 + (ss ? 0 : 1) + dsz + fl;
  if (clen < 4 + hsize) return SLATE_OK;
  size_t q = 5;
  uint64_t window = 0;
  if (!ss) {
    const uint32_t wd = f[q++], wl = 10 + (wd >> 3);
    window = (1ull << wl) + ((1ull << wl) >> 3) * (wd & 7);
  }
  uint32_t dict = 0;
  for (uint32_t i = 0; i < dsz; i++) dict |= uint32_t(f[q++]) << (8 * i);
  if (dict) return SLATE_OK;
  uint64_t fcs = 0;
  for (uint32_t i = 0; i < fl; i++) fcs |= uint64_t(f[q + i]) << (8 * i);
  if (fl == 2) fcs += 256;
  if (ss) window = fcs;
  if (window > (1ull << 29)) return SLATE_OK;
  const uint32_t bmax = uint32_t(window < 128 * 1024 ? window : 128 * 1024);
  std::vector<uint32_t> blk;
  size_t pos = 4 + hsize;
  for (;;) {
    if (clen - pos < 3) return SLATE_OK;
    const uint32_t bh = uint32_t(f[pos]) | uint32_t(f[pos + 1]) << 8 | uint32_t(f[pos + 2]) << 16;
    const uint32_t bt = (bh >> 1) & 3, bs = bh >> 3;
    if (bt == 3 || bs > bmax) return SLATE_OK;
    const size_t body = bt == 1 ? 1 : bs;
    if (clen - pos - 3 < body || pos + 3 > 0xFFFFFFFFull) return SLATE_OK;
    blk.push_back(uint32_t(pos + 3));
    blk.push_back(bh);
    pos += 3 + body;
    if (bh & 1) break;
  }
  const bool has_sum = (fhd >> 2) & 1;
  uint32_t want = 0;
  if (has_sum) {
    if (clen - pos < 4) return SLATE_OK;
    want = le32(pos);
    pos += 4;
  }
  if (pos != clen) return SLATE_OK;  // one frame, nothing after it
  if (bmax <= kLz4PayloadSlot) {  // this builder's frames: 64 KiB pieces (larger blocks never fit the slots)
    const int s = payload_split_run(ctx, buf, len, blk, bmax, SLATE_CODEC_ZSTD, fl != 0, fcs, has_sum, want, out,
                                    bstatus, handled);
    if (s || *handled) return s;
  }
  // blocks that do not decode on their own (or larger than the split path's slots)
  return zstd_payload_par_run(ctx, buf, len, blk, bmax, fl != 0, fcs, has_sum, want, out, bstatus, handled);
}

// A large CodecZlib index / filter whose stream has no flush points -- the shape compress/zlib's
// writer (compression.go:96-103) and zlib produce -- through the speculative block-parallel inflate
// (zlib_par.hip): block starts found and decoded speculatively, the true chain walked, every byte
// resolved by pointer doubling; then the Adler-32 on the GPU.  Same contract as lz4_payload_split
// (a FDICT header, or any failed check: the serial path decodes and reports it).
static int zlib_payload_par_run(slate_ctx* ctx, const uint8_t* buf, size_t len, uint32_t want,
                                std::vector<uint8_t>& out, int* bstatus, int* handled) {
  *handled = 0;
  const size_t clen = len - 4;
  if (clen < 6 + 4 || clen >= (1u << 28) || (buf[1] & 0x20)) return SLATE_OK;
  const uint32_t dend = uint32_t(clen - 4);
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx->d_in.ensure(len + 64));
  int s = ctx_h2d(ctx, ctx->d_in.p, buf, len, st);
  if (s) return s;
  uint32_t crc = 0;
  s = ctx_crc32_device(ctx, ctx->d_in.as<uint8_t>(), clen, &crc);
  if (s) return s;
  if (crc != ld_be32(buf + clen)) {
    *bstatus = SLATE_E_BLOCK_CHECKSUM;  // block.Decode / bloom.Decode / DecodeIndex check it first
    *handled = 1;
    return SLATE_OK;
  }
  const double t0 = host_trace() ? now_ms() : 0.0;
  SLATE_HIP(ctx->d_scratch.ensure(zlib_par_scratch_bytes(uint32_t(clen)) + 64));
  void* scratch = ctx->d_scratch.p;
  const uint8_t* d_in = ctx->d_in.as<uint8_t>();
  SLATE_HIP(launch_zlib_par_chain(st, d_in, uint32_t(clen), 16, dend, scratch, ctx->num_cus));
  uint32_t res[5] = {1, 0, 0, 0, 0};
  SLATE_HIP(hipMemcpyAsync(res, zlib_par_result(scratch), sizeof(res), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const double t1 = host_trace() ? now_ms() : 0.0;
  if (host_trace())
    fprintf(stderr, "[slate zlib-par] %zu B: %u survivors, %u candidates, %u blocks, %u B out, fail %u: chain %.2f ms\n",
            clen, res[1], res[2], res[3], res[4], res[0], t1 - t0);
  if (res[0]) return SLATE_OK;  // the serial path decodes (and reports) it
  const uint32_t total = res[4];
  SLATE_HIP(ctx->d_rows.ensure(size_t(total) + 64));                       // val
  SLATE_HIP(ctx->e_a.ensure(2 * (size_t(total) + 1) * 4 + 64 * 4 + 256));  // pa | pb | changed
  SLATE_HIP(ctx->d_out.ensure(size_t(total) + 64));
  uint32_t* pa = ctx->e_a.as<uint32_t>();
  uint32_t* pb = pa + total + 1;
  uint32_t* changed = pb + total + 1;
  uint8_t* d_out = ctx->d_out.as<uint8_t>();
  SLATE_HIP(launch_zlib_par_bytes(st, d_in, uint32_t(clen), total, scratch, ctx->d_rows.as<uint8_t>(), pa, pb, changed,
                                  d_out, ctx->num_cus));
  SLATE_HIP(hipMemcpyAsync(res, zlib_par_result(scratch), 4, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  if (res[0]) return SLATE_OK;
  uint32_t got = 0;
  s = device_adler32(ctx, d_out, total, &got);
  if (s) return s;
  if (host_trace()) fprintf(stderr, "[slate zlib-par] bytes + adler %.2f ms\n", now_ms() - t1);
  if (got != want) return SLATE_OK;  // the serial path reports the checksum (read at dend by the caller)
  out.resize(total);
  s = ctx_d2h(ctx, out.data(), d_out, total, st);
  if (s) return s;
  *bstatus = SLATE_OK;
  *handled = 1;
  return SLATE_OK;
}

// A large CodecZlib index / filter (`zlib stream || BE32 CRC`) inflated piece by piece in parallel:
// this builder ends every piece but the last with an empty stored block, so the stream is cut
// after each `00 00 FF FF` (decode.hip zlib_payload_segs_kernel checks that every segment is a
// whole piece).  Same contract as lz4_payload_split.
static int zlib_payload_split(slate_ctx* ctx, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                              int* bstatus, int* handled) {
  *handled = 0;
  const size_t clen = len - 4;
  const uint8_t* f = buf;
  if (clen < 2 + 4) return SLATE_OK;
  const uint32_t b0 = f[0], b1 = f[1];
  if ((b0 & 0x0f) != 8 || (b0 >> 4) > 7 || ((b0 << 8) | b1) % 31 != 0 || (b1 & 0x20)) return SLATE_OK;
  const size_t dend = clen - 4;  // the Adler-32 trailer (big-endian) follows the deflate stream
  const uint32_t want = uint32_t(f[dend]) << 24 | uint32_t(f[dend + 1]) << 16 | uint32_t(f[dend + 2]) << 8 | f[dend + 3];
  std::vector<uint32_t> seg;
  size_t s0 = 2;
  for (size_t i = 2; i + 4 <= dend; i++) {
    if (f[i] == 0 && f[i + 1] == 0 && f[i + 2] == 0xFF && f[i + 3] == 0xFF) {
      seg.push_back(uint32_t(s0));
      seg.push_back(uint32_t(i + 4 - s0));
      s0 = i + 4;
      i += 3;
    }
  }
  if (s0 >= dend || dend > 0xFFFFFFFFull) return zlib_payload_par_run(ctx, buf, len, want, out, bstatus, handled);
  seg.push_back(uint32_t(s0));
  seg.push_back(uint32_t(dend - s0));
  // this builder's pieces hold at most 64 KiB each; a longer segment means the `00 00 FF FF` were
  // ordinary bytes of another writer's stream
  bool pieces = seg.size() > 2;
  for (size_t k = 1; k < seg.size() && pieces; k += 2) pieces = seg[k] <= 2 * kLz4PayloadSlot;
  if (pieces) {
    const int s = payload_split_run(ctx, buf, len, seg, 0, SLATE_CODEC_ZLIB, false, 0, true, want, out, bstatus, handled);
    if (s || *handled) return s;
  }
  // no piece ends (compress/zlib's and zlib's own streams), or `00 00 FF FF` inside a block's data
  return zlib_payload_par_run(ctx, buf, len, want, out, bstatus, handled);
}

int ctx_payload_decode_buffer(slate_ctx* ctx, int codec, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                              int* bstatus) {
  if (codec == SLATE_CODEC_SNAPPY) return ctx_snappy_decode_buffer(ctx, buf, len, out, bstatus);
  if ((codec == SLATE_CODEC_LZ4 || codec == SLATE_CODEC_ZSTD || codec == SLATE_CODEC_ZLIB) && len >= kSplitMin &&
      len <= 0xFFFFFF00ull) {
    int handled = 0;
    const int s = codec == SLATE_CODEC_LZ4    ? lz4_payload_split(ctx, buf, len, out, bstatus, &handled)
                  : codec == SLATE_CODEC_ZSTD ? zstd_payload_split(ctx, buf, len, out, bstatus, &handled)
                                              : zlib_payload_split(ctx, buf, len, out, bstatus, &handled);
    if (s || handled) return s;
  }
  if (codec != SLATE_CODEC_LZ4 && codec != SLATE_CODEC_ZLIB && codec != SLATE_CODEC_ZSTD) return SLATE_E_INVALID_CODEC;
  if (len < 4 || len > 0xFFFFFF00ull) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  // in_off[2] | out_off[2] | row_base[2] | meta (16 B) | rows (16 B) | plan scratch
  constexpr size_t kHead = 10 * sizeof(uint64_t);
  SLATE_HIP(ctx->d_scratch.ensure(kHead + decode_scratch_bytes(1) + 64));
  // 16 bytes of headroom: the payload kernel's CRC (wave_crc32) reads the aligned dword before it
  SLATE_HIP(ctx->d_in.ensure(len + 16 + 64));
  uint64_t* u = ctx->d_scratch.as<uint64_t>();
  const uint64_t hv[2] = {16, 16 + len};
  SLATE_HIP(hipMemcpyAsync(ctx->d_in.as<uint8_t>() + 16, buf, len, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(u, hv, sizeof(hv), hipMemcpyHostToDevice, st));
  SLATE_HIP(launch_decode_plan(st, codec, ctx->d_in.as<uint8_t>(), u, 1, u + 2, u + 4,
                               reinterpret_cast<uint8_t*>(u) + kHead));
  uint64_t cap[2] = {0, 0};
  SLATE_HIP(hipMemcpyAsync(cap, u + 2, sizeof(cap), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  SLATE_HIP(ctx->d_out.ensure(cap[1] + 64));
  DecodeArgs a{codec, ctx->d_in.as<uint8_t>(), u, 1, ctx->d_out.as<uint8_t>(), u + 2,
               reinterpret_cast<slate_block_meta*>(u + 6), reinterpret_cast<slate_row*>(u + 8), u + 4, nullptr, nullptr,
               0};
  a.raw = 1;
  SLATE_HIP(launch_decode_payload(st, a, ctx->num_cus));
  slate_block_meta m;
  SLATE_HIP(hipMemcpyAsync(&m, u + 6, sizeof(m), hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  *bstatus = m.status;
  if (m.status == SLATE_OK) {
    out.resize(m.data_len);
    if (m.data_len) {
      SLATE_HIP(hipMemcpyAsync(out.data(), ctx->d_out.p, m.data_len, hipMemcpyDeviceToHost, st));
      SLATE_HIP(hipStreamSynchronize(st));
    }
  }
  return SLATE_OK;
}

// --------------------------------------------------------------- SST builder
void SegPool::close() {
  std::lock_guard<std::mutex> g(mu);
  open = false;
  for (auto& f : free_list) {
    if (f.pinned) (void)hipHostUnregister(f.p);
    munmap(f.p, f.cap);
  }
  free_list.clear();
}

// Encoded bytes on the host: one allocation per GPU pass (uninitialised), blocks are views into
// it; the table keeps the allocations alive.
// Large ones are 2 MiB-aligned anonymous mappings advised for transparent huge pages (a fresh
// 1 GB buffer otherwise costs ~260 k page faults on first touch, more than its PCIe transfer),
// and go back to the context's pool when released, so that repeated builds reuse them.
struct HostBytes {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  bool mapped = false, pinned = false;
  std::shared_ptr<SegPool> pool;
  explicit HostBytes(size_t len, std::shared_ptr<SegPool> pl = nullptr) : n(len), pool(std::move(pl)) {
    if (pool && pool->take(len, &p, &cap, &pinned)) {
      mapped = true;
      return;
    }
    if (len >= kSegHuge) {
      cap = (len + kSegHuge - 1) & ~(kSegHuge - 1);
      void* q = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (q != MAP_FAILED) {
        (void)madvise(q, cap, MADV_HUGEPAGE);
        p = static_cast<uint8_t*>(q);
        mapped = true;
        return;
      }
    }
    cap = len ? len : 1;
    p = static_cast<uint8_t*>(malloc(cap));
    if (!p) cap = 0;  // callers check ok(): a host OOM becomes SLATE_E_OOM, not a fault
  }
  bool ok() const { return p != nullptr; }
  // a pooled mapping registered once (kept registered in the pool): the GPU writes it directly
  bool pin() {
    if (!pinned && mapped && pool) pinned = hipHostRegister(p, cap, hipHostRegisterDefault) == hipSuccess;
    if (!pinned) (void)hipGetLastError();
    return pinned;
  }
  ~HostBytes() {
    if (!mapped) {
      free(p);
    } else if (!pool || !pool->give(p, cap, pinned)) {
      if (pinned) (void)hipHostUnregister(p);
      munmap(p, cap);
    }
  }
  HostBytes(const HostBytes&) = delete;
  HostBytes& operator=(const HostBytes&) = delete;
};
struct ByteView {
  std::shared_ptr<HostBytes> seg;
  size_t off = 0, len = 0;
  const uint8_t* data() const { return seg ? seg->p + off : nullptr; }
};

struct slate_sst_table {
  slate_sst_info info{};
  std::vector<uint8_t> first_key;
  std::vector<ByteView> chunks;  // Table.Blocks: one per finished block, then the final chunk
  bool has_bloom = false;
  uint16_t num_probes = 0;
  std::vector<uint8_t> bloom_bits;
};

struct slate_sst_builder {
  slate_ctx* ctx;
  slate_sst_config cfg;
  // Snappy filter beside the final flush: 1 while its chunk encode is not yet queued (the flush then
  // holds its pack launch, so the filter's serial chains get CUs before the pack fills them), 2 after
  std::atomic<int> filter_gate{0};
  uint32_t gate_timeouts = 0;  // final flushes whose pack stopped waiting for the filter (host trace)
  // pending KVs (not yet in a finished block), on the device: key / value bytes, n+1 offsets
  // into them, tombstone flags
  DevBuf d_keys, d_vals, d_koff, d_voff, d_tomb, d_tmp;
  uint64_t n_pend = 0, kbytes = 0, vbytes = 0;
  // single-KV adds (slate_sst_builder_add) gathered on the host, moved to the device in one go
  std::vector<uint8_t> hk, hv, ht;
  std::vector<uint64_t> hko{0}, hvo{0};
  uint64_t pending_lower = 2;  // lower bound of the pending KVs' encoded size
  bool dirty = false;
  // Go's block.Builder for the single-add path (builder.go:160-176, block.go:162-182), replayed on
  // the host so that NextBlock hands out a block after the very Add that finished it: the open
  // block's first key and curBlockSize, and whether a block was finished since the last GPU pass.
  // A batch add leaves the open block unknown here (track = false: the lower bound decides).
  bool track = true;
  std::vector<uint8_t> open_first;
  uint64_t open_size = 0;
  bool boundary = false;
  std::deque<ByteView> blocks;  // finished, not yet popped
  std::vector<uint64_t> meta_off;
  std::vector<uint8_t> meta_keys;
  std::vector<uint64_t> meta_key_off{0};
  std::vector<uint8_t> first_key;
  bool has_first_key = false;
  uint64_t current_len = 0;
  uint32_t num_keys = 0;  // builder.go:111 (uint32)
  DevBuf d_hashes;        // FNV-1 hashes of every key added (bloom input)
  uint64_t n_hashes = 0;
  ByteView last_block;    // the final block (Build keeps it in the last chunk)
  int sticky = SLATE_OK;
  bool built = false;
  // a non-final flush's blocks on their way to the host (ctx_d2h_side on a worker thread): joined
  // before anything reads them or the device buffers they come from (builder_join_d2h)
  std::future<int> d2h_job;
};

static int builder_join_d2h(slate_sst_builder* b) {
  if (!b->d2h_job.valid()) return SLATE_OK;
  const int s = b->d2h_job.get();
  if (s && !b->sticky) b->sticky = s;
  return s;
}

// Append n KVs (offsets relative to their byte arrays, key_off[0] / value_off[0] need not be 0)
// to the device-resident pending set.  dev: the arrays are device pointers.  tomb may be null
// (empty value = tombstone).
static int pending_append(slate_sst_builder* b, const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals,
                          const uint64_t* val_off, const uint8_t* tomb, uint64_t n, bool dev, uint64_t k0, uint64_t k1,
                          uint64_t v0, uint64_t v1) {
  if (n == 0) return SLATE_OK;
  slate_ctx* ctx = b->ctx;
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx_bind(ctx));
  const uint64_t kb = k1 - k0, vb = v1 - v0;
  SLATE_HIP(b->d_keys.grow_keep(b->kbytes + kb + 16, b->kbytes, st));
  SLATE_HIP(b->d_vals.grow_keep(b->vbytes + vb + 16, b->vbytes, st));
  SLATE_HIP(b->d_koff.grow_keep((b->n_pend + n + 1) * 8, (b->n_pend + 1) * 8, st));
  SLATE_HIP(b->d_voff.grow_keep((b->n_pend + n + 1) * 8, (b->n_pend + 1) * 8, st));
  SLATE_HIP(b->d_tomb.grow_keep(b->n_pend + n + 16, b->n_pend, st));
  uint8_t* dk = b->d_keys.as<uint8_t>() + b->kbytes;
  uint8_t* dv = b->d_vals.as<uint8_t>() + b->vbytes;
  uint64_t* dko = b->d_koff.as<uint64_t>() + b->n_pend;  // entry n_pend (== kbytes) is rewritten
  uint64_t* dvo = b->d_voff.as<uint64_t>() + b->n_pend;
  uint8_t* dt = b->d_tomb.as<uint8_t>() + b->n_pend;
  std::unique_ptr<GpuSpan> g_add;  // the device passes (a host batch's uploads are not in it)
  if (dev) {
    g_add.reset(new GpuSpan(ctx, st));
    if (kb) SLATE_HIP(hipMemcpyAsync(dk, keys + k0, kb, hipMemcpyDeviceToDevice, st));
    if (vb) SLATE_HIP(hipMemcpyAsync(dv, vals + v0, vb, hipMemcpyDeviceToDevice, st));
    SLATE_HIP(launch_kv_rebase(st, key_off, n, dko, b->kbytes));
    SLATE_HIP(launch_kv_rebase(st, val_off, n, dvo, b->vbytes));
    if (tomb) SLATE_HIP(hipMemcpyAsync(dt, tomb, n, hipMemcpyDeviceToDevice, st));
  } else {
    int s = ctx_h2d(ctx, dk, keys + k0, kb, st);
    if (!s) s = ctx_h2d(ctx, dv, vals + v0, vb, st);
    // raw offsets to scratch, rebased on the device
    SLATE_HIP(b->d_tmp.ensure((n + 1) * 16 + 16));
    uint64_t* t0 = b->d_tmp.as<uint64_t>();
    if (!s) s = ctx_h2d(ctx, t0, key_off, (n + 1) * 8, st);
    if (!s) s = ctx_h2d(ctx, t0 + n + 1, val_off, (n + 1) * 8, st);
    if (!s && tomb) s = ctx_h2d(ctx, dt, tomb, n, st);
    if (s) return s;
    g_add.reset(new GpuSpan(ctx, st));
    SLATE_HIP(launch_kv_rebase(st, t0, n, dko, b->kbytes));
    SLATE_HIP(launch_kv_rebase(st, t0 + n + 1, n, dvo, b->vbytes));
  }
  if (!tomb) SLATE_HIP(launch_kv_tomb_from_values(st, dvo, n, dt));
  b->n_pend += n;
  b->kbytes += kb;
  b->vbytes += vb;
  b->num_keys += uint32_t(n);
  b->dirty = true;
  return SLATE_OK;
}

// the single adds gathered on the host join the device-resident pending set
static int pending_push_host(slate_sst_builder* b) {
  const uint64_t n = b->hko.size() - 1;
  if (n == 0) return SLATE_OK;
  const uint32_t nk = b->num_keys;
  int st = pending_append(b, b->hk.data(), b->hko.data(), b->hv.data(), b->hvo.data(), b->ht.data(), n, false, 0,
                          b->hk.size(), 0, b->hv.size());
  b->num_keys = nk;  // counted when they were added
  b->hk.clear();
  b->hv.clear();
  b->ht.clear();
  b->hko.assign(1, 0);
  b->hvo.assign(1, 0);
  return st;
}

// async_d2h (non-final flushes of a chunked host batch, slate_sst_builder_add_batch): the finished
// blocks leave through the context's second download pipe on a worker thread, and the call returns
// once they are packed, so the caller's next upload overlaps their transfer.
static int builder_flush(slate_sst_builder* b, bool final, const std::function<void(uint64_t)>* after_hashes = nullptr,
                         const std::function<void()>* after_meta = nullptr, bool async_d2h = false) {
  slate_ctx* ctx = b->ctx;
  hipStream_t st = ctx->stream;
  {
    const int js = builder_join_d2h(b);  // (the pack below rewrites the buffer it reads)
    if (js) return js;
  }
  int pst = pending_push_host(b);
  if (pst) return pst;
  const uint64_t n64 = b->n_pend;
  b->dirty = false;
  if (n64 == 0) return SLATE_OK;
  if (n64 >= 0xFFFFFFF0ull) return SLATE_E_INVALID_ARG;
  const uint32_t n = uint32_t(n64);
  SLATE_HIP(ctx_bind(ctx));
  uint8_t* d_keys = b->d_keys.as<uint8_t>();
  uint8_t* d_vals = b->d_vals.as<uint8_t>();
  uint64_t* d_key_off = b->d_koff.as<uint64_t>();
  uint64_t* d_val_off = b->d_voff.as<uint64_t>();
  uint8_t* d_tomb = b->d_tomb.as<uint8_t>();
  SLATE_HIP(b->d_hashes.grow_keep((b->n_hashes + n64) * 8 + 64, b->n_hashes * 8, st));
  // ---- work buffers
  const uint64_t chunks = (n64 + 4095) / 4096;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  size_t o_adj = carve(n64 * 4), o_next = carve(n64 * 4), o_bytes = carve(n64 * 8), o_exit = carve(n64 * 4),
         o_entry = carve(chunks * 4), o_starts = carve(n64 * 4), o_counts = carve((chunks + 1) * 8),
         o_bstart = carve(n64 * 4), o_bsize = carve((n64 + 1) * 8), o_big = carve(n64 * 4), o_flags = carve(64),
         o_scan = carve(scan_scratch_bytes(uint32_t(n64 + 1))), o_fko = carve((n64 + 1) * 8),
         o_pick = carve(kv_pick_scratch_bytes(n64));
  SLATE_HIP(ctx->e_d.ensure(off));
  uint8_t* base = ctx->e_d.as<uint8_t>();
  EncodeBufs w;
  w.hashes = b->d_hashes.as<uint64_t>() + b->n_hashes;
  w.adj = reinterpret_cast<uint32_t*>(base + o_adj);
  w.next = reinterpret_cast<uint32_t*>(base + o_next);
  w.bytes = reinterpret_cast<uint64_t*>(base + o_bytes);
  w.exit_pos = reinterpret_cast<uint32_t*>(base + o_exit);
  w.entry = reinterpret_cast<uint32_t*>(base + o_entry);
  w.starts_tmp = reinterpret_cast<uint32_t*>(base + o_starts);
  w.counts = reinterpret_cast<uint64_t*>(base + o_counts);
  w.chunk_base = w.counts;
  w.block_start = reinterpret_cast<uint32_t*>(base + o_bstart);
  w.block_size = reinterpret_cast<uint64_t*>(base + o_bsize);
  w.big_list = reinterpret_cast<uint32_t*>(base + o_big);
  w.flags = reinterpret_cast<uint32_t*>(base + o_flags);
  w.maxlen = w.flags + 1;
  w.big_count = w.flags + 2;
  w.status = w.flags + 3;
  void* scan_scratch = base + o_scan;
  EncodeArgs a{d_keys, d_key_off, d_vals, d_val_off, d_tomb, n, b->cfg.block_size, b->cfg.codec};
  const bool trace = host_trace();
  double tp = trace ? now_ms() : 0.0;
  auto mark = [&](const char* what) {
    if (!trace) return;
    const double t = now_ms();
    fprintf(stderr, "[slate build]   %s %.2f ms\n", what, t - tp);
    tp = t;
  };
  GpuSpan g_seg(ctx, st);
  SLATE_HIP(launch_encode(st, a, w, ctx->num_cus));
  SLATE_HIP(hipMemsetAsync(w.counts + chunks, 0, 8, st));
  SLATE_HIP(launch_scan_u64(st, w.counts, uint32_t(chunks + 1), scan_scratch));
  g_seg.stop();
  uint64_t nb_total = 0;
  SLATE_HIP(hipMemcpyAsync(&nb_total, w.counts + chunks, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  // every key's hash is in d_hashes now (the final flush consumes all pending keys)
  if (final && after_hashes) (*after_hashes)(b->n_hashes + n64);
  GpuSpan g_blocks(ctx, st);
  SLATE_HIP(launch_encode_blocks(st, a, w));
  g_blocks.stop();
  // the last block is still open unless this is the final flush (Build)
  const uint64_t nb = final ? nb_total : nb_total - 1;
  std::vector<uint32_t> starts(nb_total);
  SLATE_HIP(hipMemcpyAsync(starts.data(), w.block_start, nb_total * 4, hipMemcpyDeviceToHost, st));
  // the finished blocks' first keys (the index's BlockMeta keys), gathered on the device
  uint64_t* fko = reinterpret_cast<uint64_t*>(base + o_fko);
  SLATE_HIP(ctx->e_h.ensure(b->kbytes + 16));
  GpuSpan g_pick(ctx, st);
  SLATE_HIP(launch_kv_pick_keys(st, w.block_start, nb, d_keys, d_key_off, fko, base + o_pick, ctx->e_h.as<uint8_t>()));
  g_pick.stop();
  std::vector<uint64_t> fk_off(nb + 1);
  SLATE_HIP(hipMemcpyAsync(fk_off.data(), fko, (nb + 1) * 8, hipMemcpyDeviceToHost, st));
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(hipMemsetAsync(w.block_size + nb, 0, 8, st));
    SLATE_HIP(launch_scan_u64(st, w.block_size, uint32_t(nb + 1), scan_scratch));
  }
  std::vector<uint64_t> out_off(nb + 1);
  SLATE_HIP(hipMemcpyAsync(out_off.data(), w.block_size, (nb + 1) * 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  mark("segment + first keys");
  {
    const size_t mk = b->meta_keys.size();
    b->meta_keys.resize(mk + fk_off[nb]);
    int s = ctx_d2h(ctx, b->meta_keys.data() + mk, ctx->e_h.p, fk_off[nb], st);
    if (s) return s;
  }
  // the index entries of the finished blocks (builder.go:169-176) are known once their final sizes
  // are: queued before the blocks' D2H, so the Build's index flatbuffer can start beside it
  auto queue_meta = [&](const std::vector<uint64_t>& oo) {
    uint64_t cl = b->current_len;
    for (uint64_t k = 0; k < nb; k++) {
      b->meta_off.push_back(cl);
      b->meta_key_off.push_back(b->meta_key_off.back() + (fk_off[k + 1] - fk_off[k]));
      if (!(final && k + 1 == nb)) cl += oo[k + 1] - oo[k];
    }
    if (final && after_meta) (*after_meta)();
  };
  std::shared_ptr<HostBytes> seg;
  static const bool pin_segs = [] {  // SLATE_PIN_SEGS=0: blocks through the staging pipe (A/B runs)
    const char* e = getenv("SLATE_PIN_SEGS");
    return !(e && *e == '0');
  }();
  auto blocks_d2h = [&](const std::shared_ptr<HostBytes>& sg, const void* src, size_t len) -> int {
    if (len >= (8u << 20) && pin_segs && sg->pin()) {
      // straight into the registered segment: no staging copy on the host's cores (they are busy
      // with the next piece's upload); async: the caller joins the copy's event
      if (!async_d2h || final) {
        SLATE_HIP(hipMemcpyAsync(sg->p, src, len, hipMemcpyDeviceToHost, st));
        SLATE_HIP(hipStreamSynchronize(st));
        return SLATE_OK;
      }
      if (!ctx->d2h_after) SLATE_HIP(hipEventCreateWithFlags(&ctx->d2h_after, hipEventDisableTiming));
      SLATE_HIP(hipEventRecord(ctx->d2h_after, st));
      b->d2h_job = std::async(std::launch::async, [ctx, sg, src, len]() -> int {
        SLATE_HIP(ctx_bind(ctx));
        PipeLane& L0 = ctx->d2h_lanes[0];
        SLATE_HIP(lane_init(L0));
        SLATE_HIP(hipStreamWaitEvent(L0.stream, ctx->d2h_after, 0));
        SLATE_HIP(hipMemcpyAsync(sg->p, src, len, hipMemcpyDeviceToHost, L0.stream));
        SLATE_HIP(hipStreamSynchronize(L0.stream));
        return SLATE_OK;
      });
      return SLATE_OK;
    }
    if (!async_d2h || final || len == 0) return ctx_d2h(ctx, sg->p, src, len, st);
    if (!ctx->d2h_after) SLATE_HIP(hipEventCreateWithFlags(&ctx->d2h_after, hipEventDisableTiming));
    SLATE_HIP(hipEventRecord(ctx->d2h_after, st));
    // (the job holds the segment; src stays valid until the join at the next flush)
    b->d2h_job = std::async(std::launch::async, [ctx, sg, src, len] {
      return ctx_d2h_side(ctx, sg->p, src, len, ctx->d2h_after);
    });
    return SLATE_OK;
  };
  if (nb && b->cfg.codec == SLATE_CODEC_SNAPPY) {
    // raw sizes -> per-block slots; golang/snappy + CRC per block; scan of the
    // compressed sizes; compaction into back-to-back blocks
    const uint64_t raw_total = out_off[nb];
    // 16 guard bytes in front: the wave CRC of a slot reads the aligned dword around its first
    // byte, i.e. up to 3 bytes before block 0's slot (outside a fresh allocation: a fault)
    SLATE_HIP(ctx->s_slots.ensure(snappy_slots_bytes(raw_total, nb) + 16));
    SLATE_HIP(ctx->s_aux.ensure((nb + 1) * 8 + 64));
    uint8_t* slots = ctx->s_slots.as<uint8_t>() + 16;
    uint64_t* csize = ctx->s_aux.as<uint64_t>();
    // the filter's chunk encode queued first (it holds one CU per 64 KiB piece for its serial
    // chains; launched after the pack it would wait for the whole pack): at most 20 ms
    for (int spin = 0; final && b->filter_gate.load() == 1 && spin < 1000; spin++)
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    if (final && b->filter_gate.load() == 1) b->gate_timeouts++;
    GpuSpan g_pack(ctx, st);
    SLATE_HIP(hipMemsetAsync(csize + nb, 0, 8, st));
    SLATE_HIP(launch_pack_snappy(st, a, w, uint32_t(nb), w.block_size, slots, csize, ctx->num_cus));
    g_pack.stop();
    uint32_t big = 0;
    SLATE_HIP(hipMemcpyAsync(&big, w.big_count, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    GpuSpan g_big(ctx, st);
    if (big) {
      SLATE_HIP(ctx->s_raw.ensure(raw_total + 64));
      SLATE_HIP(launch_pack_snappy_big(st, a, w, w.block_size, ctx->s_raw.as<uint8_t>(), slots, csize, big,
                                       ctx->num_cus));
    }
    SLATE_HIP(launch_scan_u64(st, csize, uint32_t(nb + 1), scan_scratch));
    g_big.stop();
    std::vector<uint64_t> fin(nb + 1);
    SLATE_HIP(hipMemcpyAsync(fin.data(), csize, (nb + 1) * 8, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    SLATE_HIP(ctx->e_e.ensure(fin[nb] + 16));
    {
      GpuSpan gs(ctx, st);
      SLATE_HIP(launch_compact(st, slots, w.block_size, csize, uint32_t(nb), ctx->e_e.as<uint8_t>(), ctx->num_cus));
    }
    mark("pack snappy");
    out_off.swap(fin);
    seg = std::make_shared<HostBytes>(out_off[nb], ctx->seg_pool);
    if (!seg->ok()) return SLATE_E_OOM;
    queue_meta(out_off);
    int s = blocks_d2h(seg, ctx->e_e.p, out_off[nb]);
    mark("blocks D2H");
    if (s) return s;
  } else if (nb) {
    const uint64_t total = out_off[nb];
    SLATE_HIP(ctx->e_e.ensure(total + 16));
    {
      GpuSpan gs(ctx, st);
      SLATE_HIP(launch_pack(st, a, w, uint32_t(nb), w.block_size, ctx->e_e.as<uint8_t>(), ctx->num_cus));
    }
    uint32_t status = 0;
    SLATE_HIP(hipMemcpyAsync(&status, w.status, 4, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    if (status) return SLATE_E_CAPACITY;
    mark("pack");
    const uint8_t* src = ctx->e_e.as<uint8_t>();
    if (b->cfg.codec != SLATE_CODEC_NONE) {
      // LZ4 / Zlib / Zstd: the raw blocks (Data || offsets || count, before their CRC) framed
      std::vector<uint64_t> rs(nb), rl(nb), fo;
      for (uint64_t k = 0; k < nb; k++) {
        rs[k] = out_off[k];
        rl[k] = out_off[k + 1] - out_off[k] - 4;
      }
      int s = ctx_codec_frames(ctx, b->cfg.codec, src, rs.data(), rl.data(), nb, true, fo);
      if (s) return s;
      out_off.swap(fo);
      src = codec_frames(ctx);
      mark("codec frames");
    }
    seg = std::make_shared<HostBytes>(out_off[nb], ctx->seg_pool);
    if (!seg->ok()) return SLATE_E_OOM;
    queue_meta(out_off);
    int s = blocks_d2h(seg, src, out_off[nb]);
    mark("blocks D2H");
    if (s) return s;
  }
  // ---- queue the finished blocks (builder.go:169-176, finishBlock :192-213; their index
  // entries went in before the D2H)
  // (views moved, not copied: ~270 k blocks per 10 M-KV build, each copy of the segment's
  // shared_ptr an atomic round trip on one cache line)
  for (uint64_t k = 0; k < nb; k++) {
    ByteView v{seg, out_off[k], out_off[k + 1] - out_off[k]};
    if (final && k + 1 == nb) {
      b->last_block = std::move(v);  // Build: the last block opens the final chunk
    } else {
      b->current_len += v.len;
      b->blocks.push_back(std::move(v));
    }
  }
  const uint64_t consumed = final ? n64 : starts[nb_total - 1];
  b->n_hashes += consumed;
  if (final || consumed == n64) {
    b->n_pend = b->kbytes = b->vbytes = 0;
    b->pending_lower = 2;
    return SLATE_OK;
  }
  if (consumed == 0) return SLATE_OK;  // nothing finished: the pending set stays as it is
  // keep the open block's KVs pending: move them to the front (through scratch: may overlap)
  uint64_t cut[2] = {0, 0};
  SLATE_HIP(hipMemcpyAsync(&cut[0], d_key_off + consumed, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(&cut[1], d_val_off + consumed, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const uint64_t r = n64 - consumed, rk = b->kbytes - cut[0], rv = b->vbytes - cut[1];
  SLATE_HIP(b->d_tmp.ensure(rk + rv + r + 2 * (r + 1) * 8 + 64));
  uint8_t* t = b->d_tmp.as<uint8_t>();
  uint64_t* to = reinterpret_cast<uint64_t*>(t);
  uint8_t* tk = t + 2 * (r + 1) * 8;
  uint8_t* tv = tk + rk;
  uint8_t* tt = tv + rv;
  SLATE_HIP(launch_kv_rebase(st, d_key_off + consumed, r, to, 0));
  SLATE_HIP(launch_kv_rebase(st, d_val_off + consumed, r, to + r + 1, 0));
  if (rk) SLATE_HIP(hipMemcpyAsync(tk, d_keys + cut[0], rk, hipMemcpyDeviceToDevice, st));
  if (rv) SLATE_HIP(hipMemcpyAsync(tv, d_vals + cut[1], rv, hipMemcpyDeviceToDevice, st));
  SLATE_HIP(hipMemcpyAsync(tt, d_tomb + consumed, r, hipMemcpyDeviceToDevice, st));
  SLATE_HIP(hipMemcpyAsync(d_key_off, to, (r + 1) * 8, hipMemcpyDeviceToDevice, st));
  SLATE_HIP(hipMemcpyAsync(d_val_off, to + r + 1, (r + 1) * 8, hipMemcpyDeviceToDevice, st));
  if (rk) SLATE_HIP(hipMemcpyAsync(d_keys, tk, rk, hipMemcpyDeviceToDevice, st));
  if (rv) SLATE_HIP(hipMemcpyAsync(d_vals, tv, rv, hipMemcpyDeviceToDevice, st));
  SLATE_HIP(hipMemcpyAsync(d_tomb, tt, r, hipMemcpyDeviceToDevice, st));
  SLATE_HIP(hipStreamSynchronize(st));
  b->n_pend = r;
  b->kbytes = rk;
  b->vbytes = rv;
  b->pending_lower = 2 + 15 * r + rv;  // a lower bound (row.go:95-107 without the value lengths)
  return SLATE_OK;
}

extern "C" {

slate_sst_builder* slate_sst_builder_new(slate_ctx* ctx, const slate_sst_config* cfg, int* status) {
  int dummy;
  if (!status) status = &dummy;
  if (!ctx || !cfg) {
    *status = SLATE_E_INVALID_ARG;
    return nullptr;
  }
  if (cfg->codec < SLATE_CODEC_NONE || cfg->codec > SLATE_CODEC_ZSTD) {
    *status = SLATE_E_INVALID_CODEC;
    return nullptr;
  }
  slate_sst_builder* b = new slate_sst_builder();
  b->ctx = ctx;
  b->cfg = *cfg;
  *status = SLATE_OK;
  return b;
}

void slate_sst_builder_free(slate_sst_builder* b) {
  if (!b) return;
  (void)builder_join_d2h(b);
  (void)hipSetDevice(b->ctx->device);
  for (DevBuf* d : {&b->d_hashes, &b->d_keys, &b->d_vals, &b->d_koff, &b->d_voff, &b->d_tomb, &b->d_tmp})
    d->release();
  delete b;
}

int slate_sst_builder_add(slate_sst_builder* b, const uint8_t* key, size_t key_len, const uint8_t* value,
                          size_t value_len, int kind) {
  if (!b || (!key && key_len)) return SLATE_E_INVALID_ARG;
  if (b->built) return SLATE_E_INVALID_ARG;
  if (key_len == 0) return SLATE_E_INVALID_ARG;  // block.go:163 assert (panic in Go)
  b->num_keys += 1;
  bool tomb = kind == 1;
  b->hk.insert(b->hk.end(), key, key + key_len);
  b->hko.push_back(b->hk.size());
  if (!tomb && value_len) b->hv.insert(b->hv.end(), value, value + value_len);
  b->hvo.push_back(b->hv.size());
  b->ht.push_back(tomb ? 1 : 0);
  b->pending_lower += 2 + 13 + (tomb ? 0 : 4 + value_len);
  b->dirty = true;
  if (b->track) {
    // v0Size (row.go:95-107) + the offset, the key prefix against the block's first key
    // (computePrefixLen, row.go:292-318: a uint16)
    auto entry = [&](uint64_t prefix) { return 2 + 2 + 2 + (key_len - prefix) + 8 + 1 + (tomb ? 0 : 4 + value_len); };
    if (b->open_first.empty()) {
      b->open_first.assign(key, key + key_len);
      b->open_size = 2 + entry(0);
    } else {
      const size_t m = std::min(key_len, b->open_first.size());
      size_t lcp = 0;
      while (lcp < m && b->open_first[lcp] == key[lcp]) lcp++;
      const uint64_t sz = b->open_size + entry(uint16_t(lcp));
      if (sz > b->cfg.block_size) {  // block.Builder.Add refuses it: the block is finished
        b->boundary = true;
        b->open_first.assign(key, key + key_len);
        b->open_size = 2 + entry(0);
      } else {
        b->open_size = sz;
      }
    }
  }
  if (!b->has_first_key) {  // builder.go:178-180
    b->first_key.assign(key, key + key_len);
    b->has_first_key = true;
  }
  return SLATE_OK;
}

int slate_sst_builder_add_value(slate_sst_builder* b, const uint8_t* key, size_t key_len, const uint8_t* value,
                                size_t value_len) {
  return slate_sst_builder_add(b, key, key_len, value, value_len, value_len == 0 ? 1 : 0);
}

int slate_sst_builder_add_batch(slate_sst_builder* b, const uint8_t* keys, const uint64_t* key_off,
                                const uint8_t* values, const uint64_t* value_off, const uint8_t* is_tomb, uint64_t n) {
  if (!b || (n && (!keys || !key_off || !value_off))) return SLATE_E_INVALID_ARG;
  if (b->built) return SLATE_E_INVALID_ARG;
  if (n == 0) return SLATE_OK;
  // the same effect as n calls of slate_sst_builder_add, up to the first empty key
  // (block.go:163), which fails; a tombstone's value bytes are not kept.  The scan for that key and
  // the encoded size's lower bound runs in pieces on the context's copy threads (one core takes
  // ~10 ms over 10 M offsets, all of it before the upload starts): piece k stops at its first
  // empty key, and the first piece that stopped early sets m.
  uint64_t m = n, lower = 0;
  {
    const size_t T = n >= (1u << 20) ? std::min<size_t>(b->ctx->pool()->size(), 64) : 1;
    std::vector<uint64_t> stop(T), part(T);
    auto piece = [&](size_t k) {
      const uint64_t lo = n * k / T, hi = n * (k + 1) / T;
      uint64_t i = lo, low = 0;
      for (; i < hi && key_off[i + 1] > key_off[i]; i++) {
        const uint64_t vl = value_off[i + 1] - value_off[i];
        const bool tomb = is_tomb ? is_tomb[i] != 0 : vl == 0;
        low += 2 + 13 + (tomb ? 0 : 4 + vl);
      }
      stop[k] = i;
      part[k] = low;
    };
    if (T == 1) {
      piece(0);
    } else {
      b->ctx->pool()->run(T, piece);
    }
    for (size_t k = 0; k < T; k++) {
      lower += part[k];
      if (stop[k] < n * (k + 1) / T) {
        m = stop[k];
        break;
      }
    }
  }
  if (m) {
    b->track = false;
    int st = pending_push_host(b);  // keep the order of earlier single adds
    if (st) return b->sticky = st;
    if (is_tomb) {
      // tombstones with value bytes: take the per-KV path so that those bytes are dropped
      bool dropped = false;
      for (uint64_t i = 0; i < m && !dropped; i++) dropped = is_tomb[i] && value_off[i + 1] > value_off[i];
      if (dropped) {
        for (uint64_t i = 0; i < m; i++) {
          st = slate_sst_builder_add(b, keys + key_off[i], key_off[i + 1] - key_off[i], values + value_off[i],
                                     value_off[i + 1] - value_off[i], is_tomb[i] ? 1 : 0);
          if (st) return st;
        }
        return m == n ? SLATE_OK : SLATE_E_INVALID_ARG;
      }
    }
    if (!b->has_first_key) {  // builder.go:178-180
      b->first_key.assign(keys + key_off[0], keys + key_off[1]);
      b->has_first_key = true;
    }
    // SLATE_ADD_PIECE (KVs per piece; unset or 0 = one piece): a large batch goes up in pieces, each
    // followed by a flush of the blocks it finished, whose download (the context's second pipe, a
    // worker thread) overlaps the next piece's upload; the last piece stays pending for Build's
    // final flush.  Off by default: on the MI355X boxes the two directions at once ran slower than
    // one after the other (10 M KV CodecNone: add 25 -> 53-56 ms for build 33 -> 19-22 ms;
    // profiles/round6/ab/ab_encode_pieces_pin.txt).  (read per call: tests set it)
    const char* piece_env = getenv("SLATE_ADD_PIECE");
    const uint64_t piece_kv = piece_env ? uint64_t(strtoull(piece_env, nullptr, 10)) : uint64_t(0);
    const bool pieces = piece_kv && m >= 2 * piece_kv &&
                        (b->cfg.codec == SLATE_CODEC_NONE || b->cfg.codec == SLATE_CODEC_SNAPPY);
    const uint64_t np = pieces ? (m + piece_kv - 1) / piece_kv : 1;
    for (uint64_t k = 0; k < np; k++) {
      const uint64_t a = m * k / np, e = m * (k + 1) / np;
      st = pending_append(b, keys, key_off + a, values, value_off + a, is_tomb ? is_tomb + a : nullptr, e - a, false,
                          key_off[a], key_off[e], value_off[a], value_off[e]);
      if (st) {
        (void)builder_join_d2h(b);
        return b->sticky = st;
      }
      if (k + 1 < np) {
        st = builder_flush(b, false, nullptr, nullptr, true);  // (it resets pending_lower to its remainder)
        if (st) {
          (void)builder_join_d2h(b);
          return b->sticky = st;
        }
      }
    }
    st = builder_join_d2h(b);
    if (st) return st;
    if (np > 1) {
      // the last piece's lower bound without a second scan: 15 bytes per row, plus the value bytes
      // when no tombstone flags are given (an empty value is then the only tombstone)
      const uint64_t a = m * (np - 1) / np;
      b->pending_lower += 15 * (m - a) + (is_tomb ? 0 : value_off[m] - value_off[a]);
    } else {
      b->pending_lower += lower;
    }
  }
  return m == n ? SLATE_OK : SLATE_E_INVALID_ARG;
}

// Device-resident KVs (compaction's merged output): keys / values / offsets / tombstones in
// device memory of the builder's context, the same effect as slate_sst_builder_add_batch.
int slate_sst_builder_add_batch_device(slate_sst_builder* b, const uint8_t* d_keys, const uint64_t* d_key_off,
                                       const uint8_t* d_values, const uint64_t* d_value_off, const uint8_t* d_is_tomb,
                                       uint64_t n) {
  if (!b || (n && (!d_keys || !d_key_off || !d_value_off))) return SLATE_E_INVALID_ARG;
  if (b->built) return SLATE_E_INVALID_ARG;
  if (n == 0) return SLATE_OK;
  slate_ctx* ctx = b->ctx;
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx_bind(ctx));
  b->track = false;
  int s = pending_push_host(b);
  if (s) return b->sticky = s;
  // the first empty key ends the batch (block.go:163); the range and the first key
  SLATE_HIP(b->d_tmp.ensure(64));
  uint64_t* q = b->d_tmp.as<uint64_t>();
  SLATE_HIP(launch_kv_first_empty(st, d_key_off, n, q));
  uint64_t h[5];
  SLATE_HIP(hipMemcpyAsync(&h[0], q, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(&h[1], d_key_off, 16, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(&h[3], d_value_off, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  const uint64_t m = std::min<uint64_t>(h[0], n);
  if (m == 0) return SLATE_E_INVALID_ARG;
  uint64_t ends[2];
  SLATE_HIP(hipMemcpyAsync(&ends[0], d_key_off + m, 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipMemcpyAsync(&ends[1], d_value_off + m, 8, hipMemcpyDeviceToHost, st));
  if (!b->has_first_key) {
    b->first_key.resize(h[2] - h[1]);
    SLATE_HIP(hipMemcpyAsync(b->first_key.data(), d_keys + h[1], h[2] - h[1], hipMemcpyDeviceToHost, st));
    b->has_first_key = true;
  }
  SLATE_HIP(hipStreamSynchronize(st));
  s = pending_append(b, d_keys, d_key_off, d_values, d_value_off, d_is_tomb, m, true, h[1], ends[0], h[3], ends[1]);
  if (s) return b->sticky = s;
  b->pending_lower += 15 * m;  // a lower bound: every row is at least 15 bytes with its offset
  return m == n ? SLATE_OK : SLATE_E_INVALID_ARG;
}

int slate_sst_builder_next_block(slate_sst_builder* b, uint8_t* out, size_t out_cap, size_t* len, int* present) {
  if (!b || !present) return SLATE_E_INVALID_ARG;
  *present = 0;
  (void)builder_join_d2h(b);
  if (b->sticky) return b->sticky;
  // A finished block exists only once the pending KVs overflow one block: single adds know exactly
  // when Go finished one (the replayed block.Builder); after batch adds, the lower bound avoids a
  // GPU pass while they certainly fit.
  const bool due = b->track ? b->boundary : b->pending_lower > b->cfg.block_size;
  if (b->blocks.empty() && b->dirty && due) {
    int st = builder_flush(b, false);
    if (st) return b->sticky = st;
    b->boundary = false;
  }
  if (b->blocks.empty()) return SLATE_OK;
  const ByteView& blk = b->blocks.front();
  if (len) *len = blk.len;
  if (blk.len > out_cap || (!out && blk.len)) return SLATE_E_CAPACITY;
  if (blk.len) memcpy(out, blk.data(), blk.len);
  b->blocks.pop_front();
  *present = 1;
  return SLATE_OK;
}

}  // extern "C"

// The SST filter of every key added (builder.go:225-235: bloom.go:112-133 Build, :52-67 Encode)
// for CodecNone / CodecSnappy, computed on the context's second stream by a host thread of its own
// while the final flush encodes the blocks on the main stream (the flush touches none of these
// buffers, and nothing here goes through the context's page-locked lanes).
struct FilterOut {
  int st = SLATE_OK;
  uint16_t np = 0;
  std::vector<uint8_t> section;  // compress(BE16 numProbes || bits) || BE32 CRC
  std::vector<uint8_t> bits;
};

// SLATE_FILTER_FIRST=0: the flush does not hold its pack for the filter's chunk launch (A/B runs)
static bool filter_first() {
  static const bool on = [] {
    const char* e = getenv("SLATE_FILTER_FIRST");
    return !(e && *e == '0');
  }();
  return on;
}

// The filter's device buffers sized before the flush holds its pack for the filter (the gate): an
// ensure() that has to grow a buffer frees the old one, and hipFree waits for the device, so growing
// them on the filter's thread while the flush waits would stretch the wait.  Failures are left to
// build_filter_aux, which makes the same calls and reports them.
static void filter_prealloc(slate_sst_builder* b, uint64_t n_hashes) {
  slate_ctx* ctx = b->ctx;
  if (b->num_keys == 0) return;
  const uint32_t np = bloom_num_probes(b->cfg.filter_bits_per_key);
  const uint64_t nb = bloom_filter_bytes(b->num_keys, b->cfg.filter_bits_per_key);
  if (nb * 8 == 0 || nb * 8 > 0xFFFFFFFFull) return;
  (void)ctx->x_words.ensure(((nb + 3) & ~uint64_t(3)) + 16);
  (void)ctx->x_enc.ensure(nb + 2 + 16);
  (void)ctx->x_bkt.ensure(bloom_bucket_scratch_bytes(n_hashes, np, uint32_t(nb * 8)));
  const uint64_t nch = (nb + 2 + kSnapMaxChunk - 1) / kSnapMaxChunk;
  (void)ctx->x_slots.ensure(nch * kSnapChunkSlot + nch * 12 + 64);
}

static FilterOut build_filter_aux(slate_sst_builder* b, uint64_t n_hashes) {
  struct GateOpen {
    slate_sst_builder* b;
    ~GateOpen() { b->filter_gate.store(2); }
  } gate_open{b};
  FilterOut f;
  slate_ctx* ctx = b->ctx;
  auto fail = [&](int st) {
    f.st = st;
    return f;
  };
  if (ctx_bind(ctx) != hipSuccess) return fail(SLATE_E_NO_DEVICE);
  if (!ctx->aux) {
    const hipError_t e = hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking);
    if (e != hipSuccess) return fail(hip_status(e));
  }
  hipStream_t st = ctx->aux;
  uint64_t nb = 0;
  if (b->num_keys > 0) {
    f.np = bloom_num_probes(b->cfg.filter_bits_per_key);
    nb = bloom_filter_bytes(b->num_keys, b->cfg.filter_bits_per_key);
    if (nb * 8 == 0 || nb * 8 > 0xFFFFFFFFull) return fail(SLATE_E_INVALID_ARG);  // Go: divide by zero / uint32 bits
  }
  auto hip = [&](hipError_t e) {
    if (e != hipSuccess) fprintf(stderr, "[slate hip] %s in the filter job\n", hipGetErrorString(e));
    return e == hipSuccess ? SLATE_OK : hip_status(e);
  };
  int s = hip(ctx->x_words.ensure(((nb + 3) & ~uint64_t(3)) + 16));
  if (!s) s = hip(ctx->x_enc.ensure(nb + 2 + 16));
  const size_t bkt = nb ? bloom_bucket_scratch_bytes(n_hashes, f.np, uint32_t(nb * 8)) : 0;
  if (!s && bkt) s = hip(ctx->x_bkt.ensure(bkt));
  if (s) return fail(s);
  uint32_t* words = ctx->x_words.as<uint32_t>();
  uint8_t* enc = ctx->x_enc.as<uint8_t>();
  const uint8_t hdr[2] = {uint8_t(f.np >> 8), uint8_t(f.np)};
  if (nb) {
    s = hip(hipMemsetAsync(words, 0, (nb + 3) & ~uint64_t(3), st));
    if (!s) {
      GpuSpan gs(ctx, st);
      s = hip(launch_bloom_build_bucketed(st, b->d_hashes.as<uint64_t>(), n_hashes, f.np, uint32_t(nb * 8), words,
                                          bkt ? ctx->x_bkt.p : nullptr));
    }
  }
  // the BE16 header by two device memsets (a pageable host-to-device copy would hold this thread until
  // the stream drains, delaying the launches queued behind it)
  if (!s) s = hip(hipMemsetAsync(enc, hdr[0], 1, st));
  if (!s) s = hip(hipMemsetAsync(enc + 1, hdr[1], 1, st));
  if (!s && nb) s = hip(hipMemcpyAsync(enc + 2, words, nb, hipMemcpyDeviceToDevice, st));
  f.bits.resize(nb);
  if (b->cfg.codec == SLATE_CODEC_SNAPPY) {
    // the Snappy chunks are queued right behind the bloom build, ahead of the bits' copy to the host:
    // launched before the flush's pack kernel takes every CU's LDS, the filter's serial chains run
    // beside the pack instead of after it
    if (s) return fail(s);
    const std::function<void()> launched = [b] { b->filter_gate.store(2); };
    s = snappy_encode_crc_on(ctx, st, ctx->x_slots, ctx->x_asm, ctx->x_crc, enc, nb + 2, f.section, false, &launched);
    if (!s && nb) s = hip(hipMemcpyAsync(f.bits.data(), words, nb, hipMemcpyDeviceToHost, st));
    if (!s) s = hip(hipStreamSynchronize(st));
    if (s) return fail(s);
    return f;
  }
  if (!s && nb) s = hip(hipMemcpyAsync(f.bits.data(), words, nb, hipMemcpyDeviceToHost, st));
  if (!s) s = hip(hipStreamSynchronize(st));
  if (s) return fail(s);
  // CodecNone: BE16 numProbes || bits || BE32 CRC (the CRC on the device)
  s = hip(ctx->x_crc.ensure(crc_scratch_bytes(nb + 2) + 16));
  if (s) return fail(s);
  uint32_t* scratch = ctx->x_crc.as<uint32_t>();
  uint32_t* cout = scratch + crc_scratch_bytes(nb + 2) / 4;
  uint32_t crc = 0;
  {
    GpuSpan gs(ctx, st);
    s = hip(launch_crc32(st, enc, nb + 2, scratch, cout, ctx->num_cus));
  }
  if (!s) s = hip(hipMemcpyAsync(&crc, cout, 4, hipMemcpyDeviceToHost, st));
  if (!s) s = hip(hipStreamSynchronize(st));
  if (s) return fail(s);
  f.section.reserve(nb + 6);
  f.section.push_back(hdr[0]);
  f.section.push_back(hdr[1]);
  f.section.insert(f.section.end(), f.bits.begin(), f.bits.end());
  put_be32(f.section, crc);
  return f;
}

extern "C" {

int slate_sst_builder_build(slate_sst_builder* b, slate_sst_table** table) {
  if (!b || !table || b->built) return SLATE_E_INVALID_ARG;
  if (b->sticky) return b->sticky;
  slate_ctx* ctx = b->ctx;
  const double t0 = host_trace() ? now_ms() : 0.0;
  // None / Snappy: the filter is built beside the final flush (its GPU work overlaps the blocks'
  // encode and their transfer); other codecs' filter encoders share the flush's buffers
  static const bool side_ok = [] {  // SLATE_SIDE_FILTER=0: the filter after the flush (A/B runs)
    const char* e = getenv("SLATE_SIDE_FILTER");
    return !(e && *e == '0');
  }();
  const bool side_filter = side_ok && (b->cfg.codec == SLATE_CODEC_NONE || b->cfg.codec == SLATE_CODEC_SNAPPY) &&
                           b->num_keys >= b->cfg.min_filter_keys;
  std::future<FilterOut> fjob;
  const std::function<void(uint64_t)> start_filter = [&](uint64_t nh) {
    if (b->cfg.codec == SLATE_CODEC_SNAPPY && filter_first()) {
      filter_prealloc(b, nh);
      b->filter_gate.store(1);
    }
    fjob = std::async(std::launch::async, build_filter_aux, b, nh);
  };
  // the index flatbuffer (host work) is built beside the last blocks' D2H and the filter's encode:
  // the final flush starts it once every index entry is queued (b->meta_* are not touched after)
  // (CodecNone: the thread also takes the payload's CRC, which then needs no GPU round trip)
  struct IndexFb {
    std::vector<uint8_t> fb;
    uint32_t crc = 0;
  };
  std::future<IndexFb> fb_job;
  const std::function<void()> start_index = [&] {
    fb_job = std::async(std::launch::async, [b] {
      IndexFb r;
      r.fb = fb_encode_index(b->meta_off, b->meta_keys, b->meta_key_off);
      if (b->cfg.codec == SLATE_CODEC_NONE) r.crc = crc32_host16(r.fb.data(), r.fb.size());
      return r;
    });
  };
  int st = builder_flush(b, true, side_filter ? &start_filter : nullptr, &start_index);
  if (side_filter && !fjob.valid() && !st) start_filter(b->n_hashes);  // nothing was pending
  // a failed final flush may have queued index entries of blocks it never delivered: the builder
  // keeps the error instead of letting a retry push them twice (started filter / index jobs are
  // joined by their futures)
  if (st) return b->sticky = st;
  if (!fb_job.valid()) start_index();  // no block was finished by the final flush
  const double t1 = host_trace() ? now_ms() : 0.0;
  b->built = true;
  slate_sst_table* t = new slate_sst_table();
  std::vector<uint8_t> buf(b->last_block.data(), b->last_block.data() + b->last_block.len);
  const uint64_t filter_off = b->current_len + buf.size();
  uint64_t filter_len = 0;
  // ---- bloom filter (builder.go:225-235, bloom.go:112-133 Build, :52-67 Encode)
  if (side_filter) {
    FilterOut f = fjob.get();
    if (f.st) {
      fb_job.wait();
      delete t;
      return b->sticky = f.st;
    }
    buf.reserve(buf.size() + f.section.size() + 16);  // (one copy of the section, no regrowth)
    buf.insert(buf.end(), f.section.begin(), f.section.end());
    t->bloom_bits.swap(f.bits);
    t->has_bloom = true;
    t->num_probes = f.np;
    filter_len = f.section.size();
  } else if (b->num_keys >= b->cfg.min_filter_keys) {
    uint16_t np = 0;
    uint64_t nb = 0;
    if (b->num_keys > 0) {
      np = bloom_num_probes(b->cfg.filter_bits_per_key);
      nb = bloom_filter_bytes(b->num_keys, b->cfg.filter_bits_per_key);
      if (nb * 8 == 0 || nb * 8 > 0xFFFFFFFFull) {  // Go: divide by zero panic / uint32 bits
        fb_job.wait();
        delete t;
        return SLATE_E_INVALID_ARG;
      }
    }
    SLATE_HIP(ctx_bind(ctx));
    SLATE_HIP(ctx->e_f.ensure(((nb + 3) & ~uint64_t(3)) + 16));
    SLATE_HIP(ctx->e_g.ensure(nb + 2 + 16));
    uint32_t* words = ctx->e_f.as<uint32_t>();
    if (nb) {
      SLATE_HIP(hipMemsetAsync(words, 0, (nb + 3) & ~uint64_t(3), ctx->stream));
      {
        GpuSpan gs(ctx, ctx->stream);
        SLATE_HIP(launch_bloom_build(ctx->stream, b->d_hashes.as<uint64_t>(), b->n_hashes, np, uint32_t(nb * 8), words));
      }
    }
    // encoded filter = compress(BE16 numProbes || bits) || BE32 CRC (bloom.go:52-67)
    uint8_t hdr[2] = {uint8_t(np >> 8), uint8_t(np)};
    uint8_t* enc = ctx->e_g.as<uint8_t>();
    SLATE_HIP(hipMemcpyAsync(enc, hdr, 2, hipMemcpyHostToDevice, ctx->stream));
    if (nb) SLATE_HIP(hipMemcpyAsync(enc + 2, words, nb, hipMemcpyDeviceToDevice, ctx->stream));
    t->bloom_bits.resize(nb);
    if (nb) SLATE_HIP(hipMemcpyAsync(t->bloom_bits.data(), words, nb, hipMemcpyDeviceToHost, ctx->stream));
    SLATE_HIP(hipStreamSynchronize(ctx->stream));
    uint32_t crc = 0;
    const size_t f0 = buf.size();
    if (b->cfg.codec == SLATE_CODEC_SNAPPY) {
      st = ctx_snappy_encode_crc_device(ctx, enc, nb + 2, buf);  // payload || BE32 CRC
      if (st) { delete t; return st; }
      crc = ld_be32(buf.data() + buf.size() - 4);
      buf.resize(buf.size() - 4);  // appended again below
    } else if (b->cfg.codec != SLATE_CODEC_NONE) {
      const uint64_t start = 0, len = nb + 2;
      std::vector<uint64_t> fo;
      st = ctx_codec_frames(ctx, b->cfg.codec, enc, &start, &len, 1, true, fo);
      if (st) { delete t; return st; }
      const size_t o = buf.size();
      buf.resize(o + fo[1]);
      st = ctx_d2h(ctx, buf.data() + o, codec_frames(ctx), fo[1], ctx->stream);
      if (st) { delete t; return st; }
      crc = ld_be32(buf.data() + buf.size() - 4);
      buf.resize(buf.size() - 4);  // appended again below
    } else {
      st = ctx_crc32_device(ctx, enc, nb + 2, &crc);
      if (st) { delete t; return st; }
      buf.push_back(hdr[0]);
      buf.push_back(hdr[1]);
      buf.insert(buf.end(), t->bloom_bits.begin(), t->bloom_bits.end());
    }
    t->has_bloom = true;
    t->num_probes = np;
    put_be32(buf, crc);
    filter_len = buf.size() - f0;
  }
  const double t2 = host_trace() ? now_ms() : 0.0;
  // ---- index (builder.go:238-244, flatbuf.go:126-139)
  std::vector<uint8_t> index;
  double t_fb = 0.0;
  {
    IndexFb job = fb_job.get();
    std::vector<uint8_t>& fb = job.fb;
    t_fb = host_trace() ? now_ms() : 0.0;
    if (b->cfg.codec == SLATE_CODEC_SNAPPY) {
      // encoded and CRC'd on the device: the payload comes back once, with its CRC
      SLATE_HIP(ctx_bind(ctx));
      SLATE_HIP(ctx->e_i.ensure(fb.size() + 16));
      st = ctx_h2d(ctx, ctx->e_i.p, fb.data(), fb.size(), ctx->stream);
      if (!st) st = ctx_snappy_encode_crc_device(ctx, ctx->e_i.as<uint8_t>(), fb.size(), index);
      if (st) { delete t; return st; }
    } else if (b->cfg.codec == SLATE_CODEC_NONE) {
      index.swap(fb);  // (the payload as built: no copy; its CRC from the index thread)
      put_be32(index, job.crc);
    } else {
      st = codec_encode_host(ctx, b->cfg.codec, fb.data(), fb.size(), index);
      if (st) { delete t; return st; }
      uint32_t icrc = 0;
      st = ctx_crc32_host_buffer(ctx, index.data(), index.size(), &icrc);
      if (st) { delete t; return st; }
      put_be32(index, icrc);
    }
  }
  const uint64_t index_off = b->current_len + buf.size();
  const uint64_t meta_off = index_off + index.size();
  // ---- info (builder.go:246-258, flatbuf.go:62-81)
  InfoFields inf;
  inf.index_offset = index_off;
  inf.index_len = index.size();
  inf.filter_offset = filter_off;
  inf.filter_len = filter_len;
  inf.codec = b->cfg.codec;
  inf.has_first_key = b->has_first_key;
  inf.first_key = b->first_key;
  std::vector<uint8_t> info = fb_encode_info(inf);
  uint32_t fcrc = 0;
  st = ctx_crc32_host_buffer(ctx, info.data(), info.size(), &fcrc);
  if (st) { delete t; return st; }
  put_be32(info, fcrc);
  put_be32(info, uint32_t(meta_off));  // builder.go:260 uint32(metaOffset)
  t->info.index_offset = index_off;
  t->info.index_len = index.size();
  t->info.filter_offset = filter_off;
  t->info.filter_len = filter_len;
  t->info.codec = b->cfg.codec;
  t->info.first_key_len = uint32_t(b->first_key.size());
  t->first_key = b->first_key;
  // the final chunk: last block and filter (buf), index, info and the meta offset, each copied once
  PoolScope pool(ctx);
  const size_t fin_len = buf.size() + index.size() + info.size();
  // (from the context's pool of released SST buffers: a reused mapping has its pages already, where
  // a fresh one faults them in during the copies below -- ~20 MB at 10 M KV)
  auto fin = std::make_shared<HostBytes>(fin_len, ctx->seg_pool);
  if (!fin->ok()) {
    delete t;
    return SLATE_E_OOM;
  }
  t->chunks.reserve(b->blocks.size() + 1);
  t->chunks.assign(std::make_move_iterator(b->blocks.begin()), std::make_move_iterator(b->blocks.end()));
  b->blocks.clear();
  if (!buf.empty()) par_memcpy(fin->p, buf.data(), buf.size());
  if (!index.empty()) par_memcpy(fin->p + buf.size(), index.data(), index.size());
  memcpy(fin->p + buf.size() + index.size(), info.data(), info.size());
  t->chunks.push_back(ByteView{fin, 0, fin_len});
  *table = t;
  if (host_trace())
    fprintf(stderr,
            "[slate build] flush %.2f ms, filter %.2f ms, index + info %.2f ms (index flatbuffer wait %.2f ms), "
            "filter gate timeouts %u\n",
            t1 - t0, t2 - t1, now_ms() - t2, t_fb - t2, b->gate_timeouts);
  return SLATE_OK;
}

void slate_sst_table_free(slate_sst_table* t) { delete t; }

int slate_sst_table_info(const slate_sst_table* t, slate_sst_info* info, uint8_t* first_key, size_t first_key_cap) {
  if (!t || !info) return SLATE_E_INVALID_ARG;
  *info = t->info;
  if (t->first_key.size() > first_key_cap) return SLATE_E_CAPACITY;
  if (!t->first_key.empty() && first_key) memcpy(first_key, t->first_key.data(), t->first_key.size());
  return SLATE_OK;
}

size_t slate_sst_table_num_chunks(const slate_sst_table* t) { return t ? t->chunks.size() : 0; }

int slate_sst_table_chunk(const slate_sst_table* t, size_t i, const uint8_t** data, size_t* len) {
  if (!t || i >= t->chunks.size() || !data || !len) return SLATE_E_INVALID_ARG;
  *data = t->chunks[i].data();
  *len = t->chunks[i].len;
  return SLATE_OK;
}

size_t slate_sst_table_encoded_len(const slate_sst_table* t) {
  size_t n = 0;
  if (t)
    for (auto& c : t->chunks) n += c.len;
  return n;
}

// Runs of chunks adjacent in one host allocation are copied as one piece (the blocks of one
// GPU pass are back to back), split over threads.
int slate_sst_table_encode(const slate_sst_table* t, uint8_t* out, size_t out_cap) {
  if (!t) return SLATE_E_INVALID_ARG;
  if (slate_sst_table_encoded_len(t) > out_cap || (!out && slate_sst_table_encoded_len(t))) return SLATE_E_CAPACITY;
  CopyPool threads(slate_sst_table_encoded_len(t) >= (64u << 20) ? kCopyThreads : 1);  // no context here
  PoolScope scope(&threads);
  size_t o = 0, i = 0;
  while (i < t->chunks.size()) {
    const ByteView& c = t->chunks[i];
    size_t j = i + 1, len = c.len;
    while (j < t->chunks.size() && t->chunks[j].seg == c.seg && t->chunks[j].off == c.off + len) len += t->chunks[j++].len;
    if (len) par_memcpy(out + o, c.data(), len);
    o += len;
    i = j;
  }
  return SLATE_OK;
}

int slate_sst_table_bloom(const slate_sst_table* t, int* present, uint16_t* num_probes, uint8_t* bits,
                          size_t bits_cap, size_t* bits_len) {
  if (!t || !present) return SLATE_E_INVALID_ARG;
  *present = t->has_bloom;
  if (num_probes) *num_probes = t->num_probes;
  if (bits_len) *bits_len = t->bloom_bits.size();
  if (!t->has_bloom) return SLATE_OK;
  if (t->bloom_bits.size() > bits_cap) return SLATE_E_CAPACITY;
  if (!t->bloom_bits.empty() && bits) memcpy(bits, t->bloom_bits.data(), t->bloom_bits.size());
  return SLATE_OK;
}

// ---------------------------------------------------------------- reader side
// DecodeInfo (flatbuf.go:102-124).  The info footer is ~80 bytes of host framing:
// its CRC is checked on the host.
int slate_decode_info(const uint8_t* buf, size_t len, slate_sst_info* info, uint8_t* first_key,
                      size_t first_key_cap) {
  if (!info || (len && !buf)) return SLATE_E_INVALID_ARG;
  if (len <= 4) return SLATE_E_INFO_TOO_SHORT;
  size_t ci = len - 4;
  if (ld_be32(buf + ci) != crc32_host(buf, ci)) return SLATE_E_INFO_CHECKSUM;
  InfoFields f;
  if (!fb_decode_info(buf, len, &f)) return SLATE_E_FLATBUF;
  info->index_offset = f.index_offset;
  info->index_len = f.index_len;
  info->filter_offset = f.filter_offset;
  info->filter_len = f.filter_len;
  info->codec = f.codec;  // unchecked cast (flatbuf.go:121)
  info->first_key_len = uint32_t(f.first_key.size());
  if (f.first_key.size() > first_key_cap) return SLATE_E_CAPACITY;
  if (!f.first_key.empty() && first_key) memcpy(first_key, f.first_key.data(), f.first_key.size());
  return SLATE_OK;
}

int slate_encode_info(const slate_sst_info* info, const uint8_t* first_key, uint8_t* out, size_t out_cap,
                      size_t* out_len) {
  if (!info) return SLATE_E_INVALID_ARG;
  InfoFields f;
  f.index_offset = info->index_offset;
  f.index_len = info->index_len;
  f.filter_offset = info->filter_offset;
  f.filter_len = info->filter_len;
  f.codec = info->codec;
  f.has_first_key = first_key != nullptr;
  if (first_key) f.first_key.assign(first_key, first_key + info->first_key_len);
  std::vector<uint8_t> v = fb_encode_info(f);
  put_be32(v, crc32_host(v.data(), v.size()));
  if (out_len) *out_len = v.size();
  if (v.size() > out_cap || !out) return SLATE_E_CAPACITY;
  memcpy(out, v.data(), v.size());
  return SLATE_OK;
}

// ReadInfo (decode.go:25-48) over the whole object.
int slate_sst_read_info(const uint8_t* sst, size_t sst_len, slate_sst_info* info, uint8_t* first_key,
                        size_t first_key_cap) {
  if (!info || (sst_len && !sst)) return SLATE_E_INVALID_ARG;
  if (sst_len <= 4) return SLATE_E_SST_TOO_SHORT;
  uint64_t oi = sst_len - 4;
  uint32_t mo = ld_be32(sst + oi);
  if (mo > oi) return SLATE_E_BLOB_RANGE;  // bytesBlob.ReadRange (blob.go:24)
  return slate_decode_info(sst + mo, size_t(oi - mo), info, first_key, first_key_cap);
}

}  // extern "C"

struct slate_index {
  std::vector<uint64_t> offsets;
  std::vector<uint8_t> keys;
  std::vector<uint64_t> key_off;
  std::vector<uint8_t> data;  // decoded flatbuffer bytes (Index.Data)
};

extern "C" {

int slate_crc32_device(slate_ctx* ctx, const uint8_t* d_data, size_t n, uint32_t* crc) {
  if (!ctx || !crc || (n && !d_data)) return SLATE_E_INVALID_ARG;
  return ctx_crc32_device(ctx, d_data, n, crc);
}

// DecodeIndex (flatbuf.go:83-100) + Index.BlockMeta() (flatbuf.go:22-31).
int slate_decode_index(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec, slate_index** index) {
  if (!ctx || !index || (len && !buf)) return SLATE_E_INVALID_ARG;
  if (len <= 4) return SLATE_E_INDEX_TOO_SHORT;
  size_t ci = len - 4;
  uint32_t crc = 0;
  int st = ctx_crc32_host_buffer(ctx, buf, ci, &crc);
  if (st) return st;
  if (crc != ld_be32(buf + ci)) return SLATE_E_INDEX_CHECKSUM;
  if (codec < SLATE_CODEC_NONE || codec > SLATE_CODEC_ZSTD) return SLATE_E_INVALID_CODEC;
  slate_index* x = new slate_index();
  if (codec != SLATE_CODEC_NONE) {
    int bst = 0;
    st = ctx_payload_decode_buffer(ctx, codec, buf, len, x->data, &bst);
    if (st || bst) {
      delete x;
      return st ? st : (bst == SLATE_E_BLOCK_CHECKSUM ? SLATE_E_INDEX_CHECKSUM : bst);
    }
  } else {
    x->data.assign(buf, buf + ci);
  }
  if (!fb_decode_index(x->data.data(), x->data.size(), &x->offsets, &x->keys, &x->key_off)) {
    delete x;
    return SLATE_E_FLATBUF;
  }
  *index = x;
  return SLATE_OK;
}

void slate_index_free(slate_index* index) { delete index; }

int slate_index_seek(slate_ctx* ctx, const slate_index* index, const uint8_t* keys, const uint64_t* key_off,
                     uint64_t n, uint64_t* block_out) {
  if (!ctx || !index || (n && (!key_off || !block_out))) return SLATE_E_INVALID_ARG;
  if (n == 0) return SLATE_OK;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  const uint64_t nb = index->offsets.size(), ib = index->keys.size(), kb = key_off[n] - key_off[0];
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_ik = carve(ib + 16), o_iko = carve((nb + 1) * 8), o_q = carve(kb + 16), o_qo = carve((n + 1) * 8),
               o_out = carve(n * 8);
  SLATE_HIP(ctx->e_h.ensure(off));
  uint8_t* base = ctx->e_h.as<uint8_t>();
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = key_off[i] - key_off[0];
  if (ib) SLATE_HIP(hipMemcpyAsync(base + o_ik, index->keys.data(), ib, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(base + o_iko, index->key_off.data(), (nb + 1) * 8, hipMemcpyHostToDevice, st));
  if (kb) SLATE_HIP(hipMemcpyAsync(base + o_q, keys + key_off[0], kb, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(base + o_qo, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  SLATE_HIP(launch_index_seek(st, base + o_ik, reinterpret_cast<const uint64_t*>(base + o_iko), nb, base + o_q,
                              reinterpret_cast<const uint64_t*>(base + o_qo), n, reinterpret_cast<uint64_t*>(base + o_out)));
  SLATE_HIP(hipMemcpyAsync(block_out, base + o_out, n * 8, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

size_t slate_index_num_blocks(const slate_index* index) { return index ? index->offsets.size() : 0; }

int slate_index_block_meta(const slate_index* index, size_t i, uint64_t* offset, const uint8_t** first_key,
                           size_t* first_key_len) {
  if (!index || i >= index->offsets.size()) return SLATE_E_INVALID_ARG;
  if (offset) *offset = index->offsets[i];
  if (first_key) *first_key = index->keys.data() + index->key_off[i];
  if (first_key_len) *first_key_len = index->key_off[i + 1] - index->key_off[i];
  return SLATE_OK;
}

int slate_index_block_offsets(const slate_index* index, uint64_t* offsets, size_t cap) {
  if (!index || (index->offsets.size() && !offsets)) return SLATE_E_INVALID_ARG;
  if (cap < index->offsets.size()) return SLATE_E_CAPACITY;
  if (index->offsets.size()) memcpy(offsets, index->offsets.data(), 8 * index->offsets.size());
  return SLATE_OK;
}

// getBlockRange (decode.go:93-103).
int slate_read_blocks_range(const slate_sst_info* info, const slate_index* index, uint64_t start, uint64_t end,
                            uint64_t* range_start, uint64_t* range_end) {
  if (!info || !index || !range_start || !range_end) return SLATE_E_INVALID_ARG;
  if (start >= end) return SLATE_E_RANGE_START;
  if (end > index->offsets.size()) return SLATE_E_RANGE_END;
  *range_start = index->offsets[start];
  *range_end = end < index->offsets.size() ? index->offsets[end] : info->filter_offset;
  return SLATE_OK;
}

// ReadBlocks (decode.go:107-149): one GPU batch for the whole range.
int slate_read_blocks(slate_ctx* ctx, const slate_sst_info* info, const slate_index* index, uint64_t start,
                      uint64_t end, const uint8_t* data, size_t data_len, uint8_t* out, uint64_t out_cap,
                      uint64_t* out_off, slate_block_meta* meta, slate_row* rows, uint64_t rows_cap,
                      uint64_t* row_base, uint64_t* failed_block) {
  uint64_t rs, re;
  int st = slate_read_blocks_range(info, index, start, end, &rs, &re);
  if (st) return st;
  if (re < rs || data_len != re - rs) return SLATE_E_BLOB_RANGE;
  const uint64_t n = end - start;
  std::vector<uint64_t> in_off(n + 1);
  for (uint64_t i = 0; i < n; i++) {
    uint64_t s = index->offsets[start + i] - rs;
    // the last block of the index runs to the end of the range (decode.go:132-133)
    uint64_t e = (start + i + 1 == index->offsets.size()) ? data_len : index->offsets[start + i + 1] - rs;
    if (s > data_len || e > data_len || s > e) return SLATE_E_BLOB_RANGE;
    in_off[i] = s;
    in_off[i + 1] = e;
  }
  // blocks are contiguous in the range; in_off[i+1] of one block is in_off of the next
  st = slate_block_decode_batch(ctx, info->codec, data, in_off.data(), uint32_t(n), out, out_cap, out_off, meta, rows,
                                rows_cap, row_base);
  if (st) return st;
  if (failed_block) {
    *failed_block = UINT64_MAX;
    for (uint64_t i = 0; i < n; i++)
      if (meta[i].status != SLATE_OK) {
        *failed_block = start + i;
        break;
      }
  }
  return SLATE_OK;
}

// ---------------------------------------------------------------------- read-ahead block reader
}  // extern "C"

// sstable.Iterator.nextBlockIter (iterator.go:92-118) with read-ahead and multiple buffering:
// batches of read_ahead blocks, up to kReaderSlots held.  Each batch is decoded into a slot while
// the caller walks an earlier one: next() asks for the following batch's bytes (NEED_DATA) as soon
// as a slot is free, before it serves the current batch, so the GPU decodes batches k+1 and k+2
// while the caller consumes batch k.  CodecNone / CodecSnappy batches are planned on the host (the varint header)
// and decoded by one launch, one workgroup per block, reading the staged bytes and writing decoded
// bytes, meta and rows through host-mapped page-locked memory (launch_decode_small); other codecs
// take slate_read_blocks into buffers grown from the plan (kept across batches).
struct ReaderSlot {
  uint64_t b0 = 0, b1 = 0;      // blocks [b0, b1)
  uint64_t fail = UINT64_MAX;   // the first failing block (known once synced)
  bool fed = false, synced = false, fast = false;
  hipEvent_t done = nullptr;
  PinBuf h_in, h_out, h_meta, h_rows, h_desc;  // fast path: host-mapped staging and results
  DevBuf d_scr;                                // fast path, one-wave blocks: device staging
  std::vector<uint64_t> out_off, row_base;     // per block, into the slot's outputs
  std::vector<uint8_t> out;                    // other codecs (slate_read_blocks)
  std::vector<slate_block_meta> meta;
  std::vector<slate_row> rows;
  const uint8_t* out_p = nullptr;
  const slate_block_meta* meta_p = nullptr;
  const slate_row* rows_p = nullptr;
};

// Batches the reader holds: the one being served and up to two decoding behind it (with one, a
// batch's launch-to-completion latency was exposed: 2.0-2.8 us per block at read-ahead 64, against
// ~0.5 us of kernel time per block)
constexpr int kReaderSlots = 3;

struct slate_block_reader {
  slate_ctx* ctx;
  slate_sst_info info;
  const slate_index* index;
  uint64_t next = 0, nblocks = 0;
  uint32_t ahead = 64;
  uint64_t fed_end = 0;          // blocks before it were fed
  uint64_t w0 = 0, w1 = 0;       // the batch the next feed decodes
  bool ended = false;
  hipStream_t stream = nullptr;  // the reader's own stream (its batches queue behind each other)
  ReaderSlot slot[kReaderSlots];
  ~slate_block_reader() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& x : slot) {
      if (x.done) (void)hipEventDestroy(x.done);
      x.h_in.release();
      x.h_out.release();
      x.h_meta.release();
      x.h_rows.release();
      x.h_desc.release();
      x.d_scr.release();
    }
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// the SST byte range of block i alone (getBlockRange for [i, i+1))
inline void block_range(const slate_block_reader* r, uint64_t i, uint64_t* s, uint64_t* e) {
  *s = r->index->offsets[i];
  *e = i + 1 < r->nblocks ? r->index->offsets[i + 1] : r->info.filter_offset;
}

// the next window from fed_end: up to read_ahead blocks, cut before the first block whose own range
// is inverted (Go reads one block per call and fails only at that block, serving those before it);
// such a block is a window of its own, whose want() range then fails as Go's ReadRange does
void reader_window(slate_block_reader* r) {
  const uint64_t w0 = r->fed_end, lim = std::min<uint64_t>(w0 + r->ahead, r->nblocks);
  uint64_t s, e;
  block_range(r, w0, &s, &e);
  uint64_t w1 = w0 + 1;
  if (e >= s)
    for (; w1 < lim; w1++) {
      block_range(r, w1, &s, &e);
      if (e < s) break;
    }
  r->w0 = w0;
  r->w1 = w1;
}

ReaderSlot* reader_holding(slate_block_reader* r, uint64_t b) {
  for (auto& x : r->slot)
    if (x.fed && b >= x.b0 && b < x.b1) return &x;
  return nullptr;
}

ReaderSlot* reader_free_slot(slate_block_reader* r) {
  for (auto& x : r->slot)
    if (!x.fed || x.b1 <= r->next) return &x;
  return nullptr;
}

int reader_sync(slate_block_reader* r, ReaderSlot& x) {
  if (x.synced) return SLATE_OK;
  if (x.fast) {
    SLATE_HIP(hipEventSynchronize(x.done));
    const slate_block_meta* m = x.h_meta.as<slate_block_meta>();
    for (uint64_t i = 0; i < x.b1 - x.b0; i++)
      if (m[i].status != SLATE_OK) {
        x.fail = x.b0 + i;
        break;
      }
  }
  x.synced = true;
  return SLATE_OK;
}

// the fast path: CodecNone / CodecSnappy, every block within the small kernels' LDS windows
int reader_feed_fast(slate_block_reader* r, ReaderSlot& x, const uint8_t* data, const std::vector<uint64_t>& in_off,
                     bool* taken) {
  *taken = false;
  const int codec = r->info.codec;
  if (!host_plannable(codec)) return SLATE_OK;
  const uint64_t n = in_off.size() - 1;
  std::vector<SmallDesc> par, wave;
  par.reserve(n);
  uint64_t in_tot = 0, out_tot = 0, rows_tot = 0;
  x.out_off.resize(n + 1);
  x.row_base.resize(n + 1);
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t len = in_off[i + 1] - in_off[i];
    const uint64_t dl = host_decoded_len(codec, data + in_off[i], len);
    const uint64_t osz = align16(dl), rsz = row_capacity(dl);
    SmallDesc d{uint32_t(i), uint32_t(len), in_tot, out_tot, osz, rows_tot, rsz, 0};
    if (small_par_fits(codec, len, osz)) par.push_back(d);
    else if (small_wave_fits(len, osz) && len < 0xFFFFFFF0ull) wave.push_back(d);
    else return SLATE_OK;  // a block beyond the windows: the batch path
    x.out_off[i] = out_tot;
    x.row_base[i] = rows_tot;
    in_tot += align16(len) + 16;
    out_tot += osz;
    rows_tot += rsz;
  }
  x.out_off[n] = out_tot;
  x.row_base[n] = rows_tot;
  // the one-wave blocks' decoded bytes in the device scratch after every input
  const uint64_t dev_out0 = align16(in_tot) + 256;
  for (auto& d : wave) d.dev_out = dev_out0 + d.out_off;
  SLATE_HIP(x.h_in.ensure(in_tot + 64));
  SLATE_HIP(x.h_out.ensure(out_tot + 64));
  SLATE_HIP(x.h_meta.ensure(n * sizeof(slate_block_meta) + 64));
  SLATE_HIP(x.h_rows.ensure((rows_tot + 1) * sizeof(slate_row) + 64));
  SLATE_HIP(x.h_desc.ensure((n + 1) * sizeof(SmallDesc)));
  if (!wave.empty()) SLATE_HIP(x.d_scr.ensure(dev_out0 + out_tot + 64));
  uint8_t* hin = x.h_in.as<uint8_t>();
  for (const auto* v : {&par, &wave})
    for (const SmallDesc& d : *v) memcpy(hin + d.in_off, data + in_off[d.block], d.in_len);
  SmallDesc* hd = x.h_desc.as<SmallDesc>();
  std::copy(par.begin(), par.end(), hd);
  std::copy(wave.begin(), wave.end(), hd + par.size());
  auto* hin_d = static_cast<uint8_t*>(mapped_ptr(x.h_in.p));
  auto* hout_d = static_cast<uint8_t*>(mapped_ptr(x.h_out.p));
  auto* meta_d = static_cast<slate_block_meta*>(mapped_ptr(x.h_meta.p));
  auto* rows_d = static_cast<slate_row*>(mapped_ptr(x.h_rows.p));
  auto* desc_d = static_cast<SmallDesc*>(mapped_ptr(x.h_desc.p));
  if (!hin_d || !hout_d || !meta_d || !rows_d || !desc_d) return SLATE_OK;
  DecodeArgs a{codec, nullptr, nullptr, 1, nullptr, nullptr, meta_d, rows_d, nullptr, nullptr, nullptr, 0};
  SLATE_HIP(launch_decode_small(r->stream, a, desc_d, uint32_t(par.size()), uint32_t(n), hin_d, hout_d,
                                wave.empty() ? nullptr : x.d_scr.as<uint8_t>()));
  if (!x.done) SLATE_HIP(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
  SLATE_HIP(hipEventRecord(x.done, r->stream));
  x.out_p = x.h_out.as<uint8_t>();
  x.meta_p = x.h_meta.as<slate_block_meta>();
  x.rows_p = x.h_rows.as<slate_row>();
  x.fast = true;
  x.synced = false;
  *taken = true;
  return SLATE_OK;
}

}  // namespace

extern "C" {

int slate_block_reader_create(slate_ctx* ctx, const slate_sst_info* info, const slate_index* index,
                              uint64_t first_block, uint32_t read_ahead, slate_block_reader** reader) {
  if (!ctx || !info || !index || !reader || read_ahead == 0) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  slate_block_reader* r = new (std::nothrow) slate_block_reader();
  if (!r) return SLATE_E_OOM;
  r->ctx = ctx;
  r->info = *info;
  r->index = index;
  r->next = first_block;
  r->fed_end = first_block;
  r->nblocks = index->offsets.size();
  r->ahead = read_ahead;
  if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
    r->stream = nullptr;
    delete r;
    return SLATE_E_HIP;
  }
  *reader = r;
  return SLATE_OK;
}

void slate_block_reader_free(slate_block_reader* reader) {
  if (reader) (void)ctx_bind(reader->ctx);
  delete reader;
}

int slate_block_reader_next(slate_block_reader* r, slate_block_view* view) {
  if (!r || !view) return SLATE_E_INVALID_ARG;
  if (r->ended || r->next >= r->nblocks) {
    r->ended = true;
    return SLATE_E_READER_END;
  }
  ReaderSlot* cur = reader_holding(r, r->next);
  // read ahead: while a slot is free and blocks are left, ask for the next batch first -- unless the
  // current batch is known to end the iteration (a failing block: Go reads no further)
  if (r->fed_end < r->nblocks && r->w1 <= r->w0) {
    ReaderSlot* fr = reader_free_slot(r);
    bool stop = false;
    if (cur && cur->fast && !cur->synced) {
      if (hipEventQuery(cur->done) == hipSuccess) {
        int st = reader_sync(r, *cur);
        if (st) return st;
      } else {
        (void)hipGetLastError();  // (not ready is not an error: keep it out of the next launch's check)
      }
    }
    if (cur && cur->synced && cur->fail != UINT64_MAX) stop = true;
    if (fr && fr != cur && !stop) {
      reader_window(r);
      // a window whose byte range is inverted (a block Go's ReadRange fails on) is asked for only
      // when the caller reaches it: the failure must not surface before the blocks in front of it
      uint64_t s0, e0;
      block_range(r, r->w0, &s0, &e0);
      if (!cur || e0 >= s0) return SLATE_E_READER_NEED_DATA;
      r->w0 = r->w1 = 0;
    }
  }
  if (!cur) {
    if (r->w1 > r->w0) return SLATE_E_READER_NEED_DATA;  // the window asked for was not fed
    reader_window(r);
    return SLATE_E_READER_NEED_DATA;
  }
  SLATE_HIP(ctx_bind(r->ctx));
  int st = reader_sync(r, *cur);
  if (st) return st;
  const uint64_t i = r->next - cur->b0;
  view->block = r->next;
  view->meta = cur->meta_p[i];
  view->data = cur->out_p + cur->out_off[i];
  view->rows = cur->rows_p + cur->row_base[i];
  if (r->next == cur->fail) {  // the SST iterator's warning, and its end (iterator.go:59-68)
    r->ended = true;
    return view->meta.status ? view->meta.status : SLATE_E_HIP;
  }
  r->next++;
  return SLATE_OK;
}

int slate_block_reader_want(const slate_block_reader* r, uint64_t* range_start, uint64_t* range_end) {
  if (!r || !range_start || !range_end || r->w1 <= r->w0) return SLATE_E_INVALID_ARG;
  return slate_read_blocks_range(&r->info, r->index, r->w0, r->w1, range_start, range_end);
}

int slate_block_reader_feed(slate_block_reader* r, const uint8_t* data, size_t data_len) {
  if (!r || (data_len && !data) || r->w1 <= r->w0) return SLATE_E_INVALID_ARG;
  ReaderSlot* fr = reader_free_slot(r);
  if (!fr) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(r->ctx));
  uint64_t rs, re;
  int st = slate_read_blocks_range(&r->info, r->index, r->w0, r->w1, &rs, &re);
  if (st) return st;
  if (re < rs || data_len != re - rs) return SLATE_E_BLOB_RANGE;
  const uint64_t n = r->w1 - r->w0;
  std::vector<uint64_t> in_off(n + 1);
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t b = r->w0 + i;
    const uint64_t s0 = r->index->offsets[b] - rs;
    const uint64_t e0 = (b + 1 == r->nblocks) ? data_len : r->index->offsets[b + 1] - rs;
    if (s0 > data_len || e0 > data_len || s0 > e0) return SLATE_E_BLOB_RANGE;
    in_off[i] = s0;
    in_off[i + 1] = e0;
  }
  ReaderSlot& x = *fr;
  // the slot is free: its previous batch was served (and its decode finished before it was)
  if (x.fed && x.fast && !x.synced) SLATE_HIP(hipEventSynchronize(x.done));
  x.fed = false;
  x.fail = UINT64_MAX;
  bool taken = false;
  st = reader_feed_fast(r, x, data, in_off, &taken);
  if (st) return st;
  if (!taken) {
    // other codecs: one batch through slate_read_blocks, buffers sized by the first attempt's plan
    // and kept (a later batch decodes twice only when it needs more room than any before it)
    x.fast = false;
    x.out_off.resize(n + 1);
    x.row_base.resize(n + 1);
    x.meta.resize(n);
    if (x.out.size() < 16) x.out.resize(std::max<uint64_t>(16, 4 * data_len + 16 * n));
    if (x.rows.empty()) x.rows.resize(std::max<uint64_t>(1, x.out.size() / 15));
    uint64_t failed = UINT64_MAX;
    for (int pass = 0; pass < 2; pass++) {
      st = slate_read_blocks(r->ctx, &r->info, r->index, r->w0, r->w1, data, data_len, x.out.data(), x.out.size(),
                             x.out_off.data(), x.meta.data(), x.rows.data(), x.rows.size(), x.row_base.data(), &failed);
      if (st != SLATE_E_CAPACITY) break;
      x.out.resize(x.out_off[n] + 16);  // the sizes the plan reported
      x.rows.resize(x.row_base[n] + 1);
    }
    if (st) return st;
    x.fail = failed;
    x.synced = true;
    x.out_p = x.out.data();
    x.meta_p = x.meta.data();
    x.rows_p = x.rows.data();
  }
  x.b0 = r->w0;
  x.b1 = r->w1;
  x.fed = true;
  r->fed_end = r->w1;
  r->w0 = r->w1 = 0;
  return SLATE_OK;
}

// ---------------------------------------------------------------------- bloom
int slate_bloom_build(slate_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t bits_per_key,
                      uint8_t* bits, size_t bits_cap, size_t* bits_len, uint16_t* num_probes) {
  if (!ctx || (n && (!keys || !key_off))) return SLATE_E_INVALID_ARG;
  if (n == 0) {  // Build on an empty builder: Filter{}
    if (bits_len) *bits_len = 0;
    if (num_probes) *num_probes = 0;
    return SLATE_OK;
  }
  uint16_t np = bloom_num_probes(bits_per_key);
  uint64_t nb = bloom_filter_bytes(uint32_t(n), bits_per_key);
  if (bits_len) *bits_len = nb;
  if (num_probes) *num_probes = np;
  if (nb * 8 == 0 || nb * 8 > 0xFFFFFFFFull) return SLATE_E_INVALID_ARG;
  if (nb > bits_cap || !bits) return SLATE_E_CAPACITY;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  SLATE_HIP(ctx->e_a.ensure(key_off[n] - key_off[0] + 16));
  SLATE_HIP(ctx->e_c.ensure((n + 1) * 8 + n * 8 + 16));
  SLATE_HIP(ctx->e_f.ensure(((nb + 3) & ~uint64_t(3)) + 16));
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = key_off[i] - key_off[0];
  uint64_t* d_off = ctx->e_c.as<uint64_t>();
  uint64_t* d_hash = d_off + n + 1;
  SLATE_HIP(hipMemcpyAsync(ctx->e_a.p, keys + key_off[0], rel[n], hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(d_off, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  // FNV-1 hashes by the encode KV pass
  SLATE_HIP(ctx->e_d.ensure(n * 4 + 64));
  uint32_t* adj = ctx->e_d.as<uint32_t>();
  uint32_t* flags = adj + n;
  SLATE_HIP(hipMemsetAsync(flags, 0, 16, st));
  EncodeArgs a{ctx->e_a.as<uint8_t>(), d_off, ctx->e_a.as<uint8_t>(), d_off, nullptr, uint32_t(n), 0, 0};
  SLATE_HIP(launch_kv_hashes(st, a, d_hash, adj, flags));
  SLATE_HIP(hipMemsetAsync(ctx->e_f.p, 0, (nb + 3) & ~uint64_t(3), st));
  SLATE_HIP(launch_bloom_build(st, d_hash, n, np, uint32_t(nb * 8), ctx->e_f.as<uint32_t>()));
  SLATE_HIP(hipMemcpyAsync(bits, ctx->e_f.p, nb, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

int slate_bloom_encode(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len, int codec,
                       uint8_t* out, size_t out_cap, size_t* out_len) {
  if (!ctx || (bits_len && !bits)) return SLATE_E_INVALID_ARG;
  if (codec < SLATE_CODEC_NONE || codec > SLATE_CODEC_ZSTD) return SLATE_E_INVALID_CODEC;
  std::vector<uint8_t> raw(bits_len + 2), buf;
  raw[0] = uint8_t(num_probes >> 8);
  raw[1] = uint8_t(num_probes);
  if (bits_len) memcpy(raw.data() + 2, bits, bits_len);
  int est = codec_encode_host(ctx, codec, raw.data(), raw.size(), buf);
  if (est) return est;
  uint32_t crc = 0;
  int st = ctx_crc32_host_buffer(ctx, buf.data(), buf.size(), &crc);
  if (st) return st;
  put_be32(buf, crc);
  if (out_len) *out_len = buf.size();
  if (buf.size() > out_cap || !out) return SLATE_E_CAPACITY;
  memcpy(out, buf.data(), buf.size());
  return SLATE_OK;
}

int slate_bloom_decode(slate_ctx* ctx, const uint8_t* buf, size_t len, int codec, uint16_t* num_probes, uint8_t* bits,
                       size_t bits_cap, size_t* bits_len) {
  if (!ctx || (len && !buf)) return SLATE_E_INVALID_ARG;
  if (len < 2) return SLATE_E_FILTER_TOO_SMALL;
  if (len < 4) return SLATE_E_FILTER_PANIC;
  size_t ci = len - 4;
  std::vector<uint8_t> dec;
  const uint8_t* p = buf;
  size_t pn = ci;
  if (codec > SLATE_CODEC_NONE && codec <= SLATE_CODEC_ZSTD) {
    // the GPU payload path checks the CRC first (bloom.go:75-79), then decompresses: one upload
    int bst = 0;
    int st = ctx_payload_decode_buffer(ctx, codec, buf, len, dec, &bst);
    if (st) return st;
    if (bst) return bst == SLATE_E_BLOCK_CHECKSUM ? SLATE_E_FILTER_CHECKSUM : bst;
    p = dec.data();
    pn = dec.size();
  } else {
    uint32_t crc = 0;
    int st = ctx_crc32_host_buffer(ctx, buf, ci, &crc);
    if (st) return st;
    if (crc != ld_be32(buf + ci)) return SLATE_E_FILTER_CHECKSUM;
    if (codec != SLATE_CODEC_NONE) return SLATE_E_INVALID_CODEC;
  }
  if (pn < 2) return SLATE_E_FILTER_PANIC;
  if (num_probes) *num_probes = ld_be16(p);
  if (bits_len) *bits_len = pn - 2;
  if (pn - 2 > bits_cap || (!bits && pn > 2)) return SLATE_E_CAPACITY;  // the retry decodes again
  if (pn > 2) memcpy(bits, p + 2, pn - 2);
  return SLATE_OK;
}

int slate_bloom_has_keys(slate_ctx* ctx, uint16_t num_probes, const uint8_t* bits, size_t bits_len, const uint8_t* keys,
                         const uint64_t* key_off, uint64_t n, uint8_t* out) {
  if (!ctx || (n && (!keys || !key_off || !out)) || (bits_len && !bits)) return SLATE_E_INVALID_ARG;
  if (n == 0) return SLATE_OK;
  SLATE_HIP(ctx_bind(ctx));
  hipStream_t st = ctx->stream;
  uint64_t kb = key_off[n] - key_off[0];
  SLATE_HIP(ctx->e_a.ensure(kb + 16));
  SLATE_HIP(ctx->e_c.ensure((n + 1) * 8 + 16));
  SLATE_HIP(ctx->e_f.ensure(bits_len + 16));
  SLATE_HIP(ctx->e_b.ensure(n + 16));
  std::vector<uint64_t> rel(n + 1);
  for (uint64_t i = 0; i <= n; i++) rel[i] = key_off[i] - key_off[0];
  SLATE_HIP(hipMemcpyAsync(ctx->e_a.p, keys + key_off[0], kb, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(ctx->e_c.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  if (bits_len) SLATE_HIP(hipMemcpyAsync(ctx->e_f.p, bits, bits_len, hipMemcpyHostToDevice, st));
  SLATE_HIP(launch_bloom_check(st, ctx->e_a.as<uint8_t>(), ctx->e_c.as<uint64_t>(), n, ctx->e_f.as<uint8_t>(), bits_len,
                               num_probes, ctx->e_b.as<uint8_t>()));
  SLATE_HIP(hipMemcpyAsync(out, ctx->e_b.p, n, hipMemcpyDeviceToHost, st));
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

// block.Encode (block.go:54-75) for one block: buffer framing on the host, CRC on the GPU.
int slate_block_encode(slate_ctx* ctx, int codec, const uint8_t* data, size_t data_len, const uint16_t* offsets,
                       size_t n_offsets, uint8_t* out, size_t out_cap, size_t* out_len) {
  if (!ctx || (data_len && !data) || (n_offsets && !offsets)) return SLATE_E_INVALID_ARG;
  if (codec < SLATE_CODEC_NONE || codec > SLATE_CODEC_ZSTD) return SLATE_E_INVALID_CODEC;
  std::vector<uint8_t> raw(data_len + 2 * n_offsets + 2), buf;
  if (data_len) memcpy(raw.data(), data, data_len);
  for (size_t i = 0; i < n_offsets; i++) st_be16(raw.data() + data_len + 2 * i, offsets[i]);
  st_be16(raw.data() + data_len + 2 * n_offsets, uint16_t(n_offsets));
  int est = codec_encode_host(ctx, codec, raw.data(), raw.size(), buf);
  if (est) return est;
  uint32_t crc = 0;
  int st = ctx_crc32_host_buffer(ctx, buf.data(), buf.size(), &crc);
  if (st) return st;
  put_be32(buf, crc);
  if (out_len) *out_len = buf.size();
  if (buf.size() > out_cap || !out) return SLATE_E_CAPACITY;
  memcpy(out, buf.data(), buf.size());
  return SLATE_OK;
}

}  // extern "C"
