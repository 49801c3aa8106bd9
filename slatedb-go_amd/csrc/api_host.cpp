// C-ABI: host-buffer block decode (object-store GET buffers in, caller buffers out) and the
// round-robin sharding of one block set over several contexts / GPUs.
//
// Reference callers: sstable.ReadBlocks (internal/sstable/decode.go:107-149) and the
// compaction executor's per-SST block reads (slatedb/compaction/executor.go:92-151,
// internal/sstable/iterator.go:92-118).  Blocks are independent, so a batch is
// decoded in chunks through page-locked staging on two stream lanes per context, and a batch
// spread over G contexts sends block i to context i mod G with no collective.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "host_ctx.h"

using namespace slate;

thread_local CopyPool* t_pool = nullptr;
// at most this many copy tasks per copy on this thread (0: the pool's size): a sharded call's
// contexts share the host's cores unless their counts were set explicitly
thread_local size_t t_pool_cap = 0;

static size_t pool_threads() {
  const size_t n = t_pool ? t_pool->size() : 1;
  return t_pool_cap ? std::min(n, t_pool_cap) : n;
}

// memcpy split over the calling context's copy threads for large copies between caller memory
// and page-locked staging (one core copies ~10 GB/s, below what the PCIe link moves).
void par_memcpy(void* dst, const void* src, size_t n) {
  constexpr size_t kPiece = 4u << 20;
  const size_t threads = pool_threads();
  if (n < 2 * kPiece || threads == 1) {
    if (n) memcpy(dst, src, n);
    return;
  }
  const size_t t = std::max<size_t>(1, std::min<size_t>(threads, n / kPiece));
  const size_t step = (n + t - 1) / t;
  t_pool->run(t, [&](size_t i) {
    const size_t a = i * step;
    if (a < n) memcpy(static_cast<uint8_t*>(dst) + a, static_cast<const uint8_t*>(src) + a, std::min(n, a + step) - a);
  });
}

hipError_t lane_init(PipeLane& L) {
  if (L.stream) return hipSuccess;
  hipError_t e = hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  e = hipEventCreateWithFlags(&L.planned, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  return hipEventCreateWithFlags(&L.done, hipEventDisableTiming);
}

// ctx_h2d / ctx_d2h: 64 MiB pieces through the two lanes' page-locked input staging; the host
// copy of piece i overlaps the DMA of piece i-1.
constexpr size_t kXferPiece = 64u << 20;
constexpr size_t kXferDirect = 8u << 20;

int ctx_h2d(slate_ctx* ctx, void* dst, const void* src, size_t n, hipStream_t st) {
  if (n == 0) return SLATE_OK;
  PoolScope pool(ctx);
  if (n <= kXferDirect) {
    SLATE_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st));
    SLATE_HIP(hipStreamSynchronize(st));
    return SLATE_OK;
  }
  bool used[kPipeLanes] = {};
  size_t k = 0;
  for (size_t o = 0; o < n; o += kXferPiece, k++) {
    PipeLane& L = ctx->lanes[k % kPipeLanes];
    SLATE_HIP(lane_init(L));
    if (used[k % kPipeLanes]) SLATE_HIP(hipEventSynchronize(L.planned));  // its previous piece has left
    const size_t len = std::min(kXferPiece, n - o);
    SLATE_HIP(L.h_in.ensure(kXferPiece));
    par_memcpy(L.h_in.p, static_cast<const uint8_t*>(src) + o, len);
    SLATE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(dst) + o, L.h_in.p, len, hipMemcpyHostToDevice, st));
    SLATE_HIP(hipEventRecord(L.planned, st));
    used[k % kPipeLanes] = true;
  }
  SLATE_HIP(hipStreamSynchronize(st));
  return SLATE_OK;
}

static int d2h_pipe(PipeLane* lanes, void* dst, const void* src, size_t n, hipStream_t st) {
  if (n == 0) return SLATE_OK;
  if (n <= kXferDirect) {
    SLATE_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st));
    SLATE_HIP(hipStreamSynchronize(st));
    return SLATE_OK;
  }
  const size_t pieces = (n + kXferPiece - 1) / kXferPiece;
  auto issue = [&](size_t k) -> hipError_t {
    PipeLane& L = lanes[k % kPipeLanes];
    hipError_t e = lane_init(L);
    if (e == hipSuccess) e = L.h_in.ensure(kXferPiece);
    const size_t o = k * kXferPiece, len = std::min(kXferPiece, n - o);
    if (e == hipSuccess) e = hipMemcpyAsync(L.h_in.p, static_cast<const uint8_t*>(src) + o, len, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipEventRecord(L.planned, st);
    return e;
  };
  SLATE_HIP(issue(0));
  for (size_t k = 0; k < pieces; k++) {
    if (k + 1 < pieces) SLATE_HIP(issue(k + 1));  // the next piece moves while this one is copied out
    PipeLane& L = lanes[k % kPipeLanes];
    SLATE_HIP(hipEventSynchronize(L.planned));
    const size_t o = k * kXferPiece, len = std::min(kXferPiece, n - o);
    par_memcpy(static_cast<uint8_t*>(dst) + o, L.h_in.p, len);
  }
  return SLATE_OK;
}

int ctx_d2h(slate_ctx* ctx, void* dst, const void* src, size_t n, hipStream_t st) {
  PoolScope pool(ctx);
  return d2h_pipe(ctx->lanes, dst, src, n, st);
}

int ctx_d2h_side(slate_ctx* ctx, void* dst, const void* src, size_t n, hipEvent_t after) {
  SLATE_HIP(ctx_bind(ctx));
  PipeLane& L0 = ctx->d2h_lanes[0];
  SLATE_HIP(lane_init(L0));
  SLATE_HIP(lane_init(ctx->d2h_lanes[1]));
  SLATE_HIP(hipStreamWaitEvent(L0.stream, after, 0));
  // half the context's copy threads: the caller's thread keeps the pool for its uploads
  if (!ctx->d2h_pool) ctx->d2h_pool.reset(new CopyPool(std::max<size_t>(1, ctx->copy_threads / 2)));
  PoolScope pool(ctx->d2h_pool.get());
  return d2h_pipe(ctx->d2h_lanes, dst, src, n, L0.stream);
}

namespace {

constexpr uint32_t kChunkBlocks = 65536;
constexpr uint64_t kChunkBytes = 96ull << 20;


// Where decoded chunks go: the caller's arrays in chunk order, or (sharded decode, scatter
// mode) block by block to the positions the whole batch's layout gives local block j of shard
// g: global block i = g + j * G.
struct Sink {
  uint8_t* out = nullptr;
  uint64_t out_cap = 0;
  uint64_t* out_off = nullptr;
  slate_block_meta* meta = nullptr;
  slate_row* rows = nullptr;
  uint64_t rows_cap = 0;
  uint64_t* row_base = nullptr;
  // scatter mode (G > 0): out_off/row_base above are the shard's own plan, these the batch's
  uint32_t G = 0, g = 0;
  const uint64_t* g_out_off = nullptr;
  const uint64_t* g_row_base = nullptr;
  // device addresses of out / rows when both are page-locked (slate_hostbuf, hipHostMalloc or
  // hipHostRegister'ed) and 16-byte aligned: decoded chunks are then written there by the GPU
  // (blocks_to_host_kernel) instead of going through staging and a host copy
  uint8_t* out_dev = nullptr;
  slate_row* rows_dev = nullptr;
};

// Sets the sink's direct path when the caller's out and rows arrays are page-locked and aligned
// (SLATE_HOST_DIRECT=0 turns it off: A/B runs).
void sink_map(Sink& o) {
  static const bool off = [] {
    const char* e = getenv("SLATE_HOST_DIRECT");
    return e && *e == '0';
  }();
  // both arrays 16-byte aligned (blocks_to_host_kernel stores 16 bytes at a time into each) and
  // page-locked over their whole capacity, or the staging path
  if (off || !o.out || !o.rows || (reinterpret_cast<uintptr_t>(o.out) & 15) ||
      (reinterpret_cast<uintptr_t>(o.rows) & 15))
    return;
  void* od = mapped_range(o.out, o.out_cap);
  void* rd = od ? mapped_range(o.rows, o.rows_cap * sizeof(slate_row)) : nullptr;
  if (od && rd) {
    o.out_dev = static_cast<uint8_t*>(od);
    o.rows_dev = static_cast<slate_row*>(rd);
  }
}


}  // namespace

// plan_sizes_kernel's decoded length for CodecNone / CodecSnappy on the host (decode.hip
// decoded_len: the payload length, or golang/snappy decodedLen's varint header with the same
// rejections), so that a chunk's place in the outputs needs no GPU round trip.
bool host_plannable(int codec) { return codec == SLATE_CODEC_NONE || codec == SLATE_CODEC_SNAPPY; }
uint64_t host_decoded_len(int codec, const uint8_t* p, uint64_t len) {
  if (len < 6) return 0;
  const uint64_t clen = len - 4;
  if (codec == SLATE_CODEC_NONE) return clen;
  uint64_t x = 0;
  uint32_t sh = 0;
  for (uint64_t i = 0; i < clen; i++) {
    if (i == 10) return 0;
    const uint32_t b = p[i];
    if (b < 0x80) {
      if (i == 9 && b > 1) return 0;
      x |= uint64_t(b) << sh;
      if (x > 0xffffffffull || x > kSnappyMaxExpansion * clen) return 0;
      return x;
    }
    x |= uint64_t(b & 0x7f) << sh;
    sh += 7;
  }
  return 0;
}

namespace {

// SLATE_ONE_LAUNCH=0: slate_block_decode takes the generic plan + decode path for every codec
// (A/B and tests of both paths)
bool one_off() {
  static const bool off = [] {
    const char* e = getenv("SLATE_ONE_LAUNCH");
    return e && e[0] == '0';
  }();
  return off;
}

// slate_block_decode's outputs from the decoded block (m: its meta, dec: its decoded bytes)
int block_decode_finish(const slate_block_meta& m, const uint8_t* dec, uint8_t* out, size_t out_cap, size_t* out_len,
                        slate_block_meta* meta, uint16_t* offsets, size_t offsets_cap) {
  *meta = m;
  if (m.status != SLATE_OK) return m.status;
  // decoded length = data_len + 2 * n_rows + 2 for a successfully decoded block
  const size_t dl = size_t(m.data_len) + 2 * size_t(m.n_rows) + 2;
  if (out_len) *out_len = dl;
  if (dl > out_cap || (offsets && m.n_rows > offsets_cap)) return SLATE_E_CAPACITY;
  if (out && dl) memcpy(out, dec, dl);
  if (offsets)
    for (uint32_t i = 0; i < m.n_rows; i++) offsets[i] = ld_be16(dec + m.data_len + 2 * i);
  return SLATE_OK;
}

// Run fn(lo, hi) over [0, n) split across the calling context's copy threads (pieces of >= grain).
template <typename F>
void par_for(size_t n, size_t grain, F fn) {
  const size_t threads = pool_threads();
  const size_t t = std::max<size_t>(1, std::min<size_t>(threads, n / std::max<size_t>(grain, 1)));
  if (t == 1) {
    fn(size_t(0), n);
    return;
  }
  const size_t step = (n + t - 1) / t;
  t_pool->run(t, [&](size_t k) {
    const size_t a = k * step, b = std::min(n, a + step);
    if (a < b) fn(a, b);
  });
}

// The lane's chunk is decoded: copy its outputs into the sink.  Its rows arrive densely (the
// rows of decoded blocks only, rows_pack): block j's come from the running count of the meta's.
int lane_finish(PipeLane& L, Sink& o) {
  if (!L.busy) return SLATE_OK;
  L.busy = false;
  const double t0 = host_trace() ? now_ms() : 0.0;
  SLATE_HIP(hipEventSynchronize(L.done));
  if (host_trace()) fprintf(stderr, "[slate host]   wait decode+D2H %.2f ms\n", now_ms() - t0);
  if (!L.decoded) return SLATE_OK;
  if (L.direct) {  // bytes and rows are in place: the metas only
    const slate_block_meta* hm = L.h_meta.as<slate_block_meta>();
    if (o.G) {
      for (uint32_t k = 0; k < L.n; k++) o.meta[uint64_t(o.g) + uint64_t(L.b0 + k) * o.G] = hm[k];
    } else {
      memcpy(o.meta + L.b0, hm, size_t(L.n) * sizeof(slate_block_meta));
    }
    return SLATE_OK;
  }
  const uint8_t* hout = L.h_out.as<uint8_t>();
  const slate_row* hrows = L.h_rows.as<slate_row>();
  const slate_block_meta* hmeta = L.h_meta.as<slate_block_meta>();
  std::vector<uint64_t> doff(size_t(L.n) + 1, 0);
  for (uint32_t k = 0; k < L.n; k++) {
    const uint32_t j = L.b0 + k;
    const uint64_t cap = o.row_base[j + 1] - o.row_base[j];
    doff[k + 1] = doff[k] + (hmeta[k].status == SLATE_OK ? std::min<uint64_t>(hmeta[k].n_rows, cap) : 0);
  }
  if (o.G) {
    par_for(L.n, 2048, [&](size_t a, size_t b) {
      for (size_t k = a; k < b; k++) {
        const uint32_t j = L.b0 + uint32_t(k);
        const uint64_t i = uint64_t(o.g) + uint64_t(j) * o.G;
        const uint64_t ob = o.out_off[j + 1] - o.out_off[j], rb = doff[k + 1] - doff[k];
        if (ob) memcpy(o.out + o.g_out_off[i], hout + (o.out_off[j] - L.out_base), ob);
        if (rb) memcpy(o.rows + o.g_row_base[i], hrows + doff[k], rb * sizeof(slate_row));
        o.meta[i] = hmeta[k];
      }
    });
    return SLATE_OK;
  }
  par_memcpy(o.out + L.out_base, hout, L.out_total);
  memcpy(o.meta + L.b0, hmeta, size_t(L.n) * sizeof(slate_block_meta));
  par_for(L.n, 2048, [&](size_t a, size_t b) {
    for (size_t k = a; k < b; k++) {
      const uint64_t rb = doff[k + 1] - doff[k];
      if (rb) memcpy(o.rows + o.row_base[L.b0 + k], hrows + doff[k], rb * sizeof(slate_row));
    }
  });
  return SLATE_OK;
}

// Decode n host blocks: chunks of up to kChunkBlocks / kChunkBytes alternate between the two
// lanes.  Per chunk k: staging copy in, H2D and plan, chunk k's place in the outputs (computed
// on the host for None / Snappy, else the plan read back), decode and D2H enqueued, and only
// then chunk k-1 waited for and copied out of its staging -- so the copy engine always has the
// next chunk queued and the host thread spends its time copying.
// out_off/row_base are always filled; when the outputs do not fit (or are absent) the
// remaining chunks are only planned and SLATE_E_CAPACITY is returned.
// gsrc (sharded decode): local block j's bytes start at in + gsrc[j] (in_off then gives only
// the local layout, i.e. the sizes); null = block j at in + in_off[j].
// Abandons whatever a lane still has in flight (a previous call that returned early): waits for
// its stream and forgets the chunk, copying nothing into any caller's buffers.
void lanes_drain(slate_ctx* ctx) {
  for (PipeLane& L : ctx->lanes) {
    if (L.busy && L.stream) (void)hipStreamSynchronize(L.stream);
    L.busy = false;
    L.decoded = false;
  }
}

// Runs lanes_drain on every early return of host_decode (an error after a chunk was queued).
struct LaneGuard {
  slate_ctx* ctx;
  bool armed = true;
  ~LaneGuard() {
    if (armed) lanes_drain(ctx);
  }
};

int host_decode_body(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n, Sink& o,
                     const uint64_t* gsrc);

int host_decode(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n, Sink& o,
                const uint64_t* gsrc = nullptr) {
  lanes_drain(ctx);  // nothing of an earlier (failed) call may reach this call's sink
  PoolScope pool(ctx);
  LaneGuard guard{ctx};
  const int st = host_decode_body(ctx, codec, in, in_off, n, o, gsrc);
  guard.armed = st != SLATE_OK && st != SLATE_E_CAPACITY;
  return st;
}

int host_decode_body(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n, Sink& o,
                     const uint64_t* gsrc) {
  SLATE_HIP(ctx_bind(ctx));
  const bool trace = host_trace();
  const double t_start = trace ? now_ms() : 0.0;
  // chunk size in blocks; SLATE_PIPE_CHUNK_BLOCKS lowers it so tests cover many chunks cheaply
  static const uint32_t chunk_blocks = [] {
    const char* e = getenv("SLATE_PIPE_CHUNK_BLOCKS");
    const unsigned long v = e ? strtoul(e, nullptr, 0) : 0;
    return v ? uint32_t(std::min<unsigned long>(v, kChunkBlocks)) : kChunkBlocks;
  }();
  uint64_t out_acc = 0, rows_acc = 0;
  bool fits = o.meta != nullptr;
  uint64_t* out_off = o.out_off;
  uint64_t* row_base = o.row_base;
  out_off[0] = 0;
  row_base[0] = 0;
  int li = 0;
  for (uint32_t b = 0; b < n;) {
    uint32_t e = b + 1;
    while (e < n && e - b < chunk_blocks && in_off[e + 1] - in_off[b] <= kChunkBytes) e++;
    const uint32_t m = e - b;
    const uint64_t lo = in_off[b], bytes = in_off[e] - lo;
    if (in_off[e] < lo) return SLATE_E_INVALID_ARG;
    PipeLane& L = ctx->lanes[li];
    PipeLane& prev = ctx->lanes[(li + kPipeLanes - 1) % kPipeLanes];
    li = (li + 1) % kPipeLanes;
    SLATE_HIP(lane_init(L));
    int st = lane_finish(L, o);  // normally finished already (two chunks ago, below)
    if (st) return st;
    SLATE_HIP(L.h_in.ensure(bytes + 16));
    SLATE_HIP(L.h_in_off.ensure((size_t(m) + 1) * 8));
    SLATE_HIP(L.h_plan.ensure(2 * (size_t(m) + 1) * 8));
    SLATE_HIP(L.d_in.ensure(bytes + 32));
    SLATE_HIP(L.d_in_off.ensure((size_t(m) + 1) * 8));
    SLATE_HIP(L.d_out_off.ensure((size_t(m) + 1) * 8));
    SLATE_HIP(L.d_row_base.ensure((size_t(m) + 1) * 8));
    SLATE_HIP(L.d_scratch.ensure(decode_scratch_bytes_codec(m, codec) + 64));
    const double t0 = trace ? now_ms() : 0.0;
    if (gsrc) {
      uint8_t* h = L.h_in.as<uint8_t>();
      par_for(m, 2048, [&](size_t a, size_t e2) {
        for (size_t i = a; i < e2; i++) {
          const uint64_t len = in_off[b + i + 1] - in_off[b + i];
          if (len) memcpy(h + (in_off[b + i] - lo), in + gsrc[b + i], len);
        }
      });
    } else {
      par_memcpy(L.h_in.p, in + lo, bytes);
    }
    const double t1 = trace ? now_ms() : 0.0;
    uint64_t* ho = L.h_in_off.as<uint64_t>();
    for (uint32_t i = 0; i <= m; i++) ho[i] = in_off[b + i] - lo;
    hipStream_t s = L.stream;
    if (bytes) SLATE_HIP(hipMemcpyAsync(L.d_in.p, L.h_in.p, bytes, hipMemcpyHostToDevice, s));
    SLATE_HIP(hipMemcpyAsync(L.d_in_off.p, ho, (size_t(m) + 1) * 8, hipMemcpyHostToDevice, s));
    // CodecZlib: the plan is phase Z, staged for this chunk's decode (as slate_block_decode_plan_device)
    const bool zl_staged = codec == SLATE_CODEC_ZLIB && m >= 64 && !getenv("SLATE_ZL_NO_STAGE");
    ZlStage zg{};
    if (zl_staged) {
      SLATE_HIP(L.d_zlstage.ensure(zl_stage_bytes(m)));
      zg = zl_stage_carve(L.d_zlstage.p, m);
    }
    SLATE_HIP(launch_decode_plan(s, codec, L.d_in.as<uint8_t>(), L.d_in_off.as<uint64_t>(), m,
                                 L.d_out_off.as<uint64_t>(), L.d_row_base.as<uint64_t>(), L.d_scratch.p,
                                 zl_staged ? &zg : nullptr, ctx->num_cus));
    uint64_t* po = L.h_plan.as<uint64_t>();
    uint64_t* pr = po + m + 1;
    if (host_plannable(codec)) {
      // the same sizes as the plan kernels, computed here: no wait for the GPU
      po[0] = pr[0] = 0;
      par_for(m, 4096, [&](size_t a, size_t e2) {
        for (size_t i = a; i < e2; i++) {
          const uint64_t src = gsrc ? gsrc[b + i] : in_off[b + i];
          const uint64_t dl = host_decoded_len(codec, in + src, in_off[b + i + 1] - in_off[b + i]);
          po[i + 1] = align16(dl);
          pr[i + 1] = row_capacity(dl);
        }
      });
      for (uint32_t i = 0; i < m; i++) {
        po[i + 1] += po[i];
        pr[i + 1] += pr[i];
      }
    } else {
      SLATE_HIP(hipMemcpyAsync(po, L.d_out_off.p, (size_t(m) + 1) * 8, hipMemcpyDeviceToHost, s));
      SLATE_HIP(hipMemcpyAsync(pr, L.d_row_base.p, (size_t(m) + 1) * 8, hipMemcpyDeviceToHost, s));
      SLATE_HIP(hipEventRecord(L.planned, s));
      SLATE_HIP(hipEventSynchronize(L.planned));
    }
    const double t2 = trace ? now_ms() : 0.0;
    for (uint32_t i = 1; i <= m; i++) {
      out_off[b + i] = out_acc + po[i];
      row_base[b + i] = rows_acc + pr[i];
    }
    L.b0 = b;
    L.n = m;
    L.out_base = out_acc;
    L.row_base = rows_acc;
    L.out_total = po[m];
    L.rows_total = pr[m];
    out_acc += po[m];
    rows_acc += pr[m];
    if (!o.G)
      fits = fits && out_acc <= o.out_cap && rows_acc <= o.rows_cap && (out_acc == 0 || o.out) &&
             (rows_acc == 0 || o.rows);
    L.busy = true;
    L.decoded = false;
    if (fits) {
      SLATE_HIP(L.d_out.ensure(L.out_total + 16));
      SLATE_HIP(L.d_meta.ensure(size_t(m) * sizeof(slate_block_meta)));
      SLATE_HIP(L.d_rows.ensure((L.rows_total + 1) * sizeof(slate_row)));
      SLATE_HIP(L.h_out.ensure(L.out_total + 16));
      SLATE_HIP(L.h_meta.ensure(size_t(m) * sizeof(slate_block_meta)));
      SLATE_HIP(L.h_rows.ensure((L.rows_total + 1) * sizeof(slate_row)));
      DecodeArgs a{codec, L.d_in.as<uint8_t>(), L.d_in_off.as<uint64_t>(), m, L.d_out.as<uint8_t>(),
                   L.d_out_off.as<uint64_t>(), L.d_meta.as<slate_block_meta>(), L.d_rows.as<slate_row>(),
                   L.d_row_base.as<uint64_t>(), nullptr, nullptr, 0};
      a.side = &L.side;
      a.handbacks = ctx_handbacks(ctx);
      SLATE_HIP(launch_decode(s, a, L.d_scratch.p, ctx->num_cus, zl_staged ? &zg : nullptr));
      L.direct = o.out_dev != nullptr;
      if (L.direct) {
        // page-locked caller buffers: the GPU writes the chunk's bytes and rows in place
        const uint64_t* gout = nullptr;
        const uint64_t* grow = nullptr;
        if (o.G) {  // sharded: each block's place in the whole batch's layout
          SLATE_HIP(L.h_gmap.ensure(2 * size_t(m) * 8));
          SLATE_HIP(L.d_gmap.ensure(2 * size_t(m) * 8));
          uint64_t* hg = L.h_gmap.as<uint64_t>();
          for (uint32_t k = 0; k < m; k++) {
            const uint64_t i = uint64_t(o.g) + uint64_t(b + k) * o.G;
            hg[k] = o.g_out_off[i];
            hg[m + k] = o.g_row_base[i];
          }
          SLATE_HIP(hipMemcpyAsync(L.d_gmap.p, hg, 2 * size_t(m) * 8, hipMemcpyHostToDevice, s));
          gout = L.d_gmap.as<uint64_t>();
          grow = gout + m;
        }
        SLATE_HIP(launch_blocks_to_host(s, L.d_out.as<uint8_t>(), L.d_out_off.as<uint64_t>(),
                                        L.d_row_base.as<uint64_t>(), L.d_meta.as<slate_block_meta>(),
                                        L.d_rows.as<slate_row>(), m, o.out_dev, o.rows_dev, gout, grow, L.out_base,
                                        L.row_base));
        SLATE_HIP(hipMemcpyAsync(L.h_meta.p, L.d_meta.p, size_t(m) * sizeof(slate_block_meta), hipMemcpyDeviceToHost, s));
        L.decoded = true;
        SLATE_HIP(hipEventRecord(L.done, s));
        if (&prev != &L) {
          st = lane_finish(prev, o);
          if (st) return st;
        }
        b = e;
        continue;
      }
      // the rows, densely, written by the GPU straight into the page-locked staging
      SLATE_HIP(L.d_dense.ensure((size_t(m) + 1) * 8 + rows_pack_scratch_bytes(m)));
      void* hrows_dev = nullptr;
      SLATE_HIP(hipHostGetDevicePointer(&hrows_dev, L.h_rows.p, 0));
      SLATE_HIP(launch_rows_pack(s, L.d_meta.as<slate_block_meta>(), L.d_row_base.as<uint64_t>(), m,
                                 L.d_rows.as<slate_row>(), L.d_dense.as<uint64_t>(),
                                 L.d_dense.as<uint8_t>() + (size_t(m) + 1) * 8, static_cast<slate_row*>(hrows_dev)));
      if (L.out_total) SLATE_HIP(hipMemcpyAsync(L.h_out.p, L.d_out.p, L.out_total, hipMemcpyDeviceToHost, s));
      SLATE_HIP(hipMemcpyAsync(L.h_meta.p, L.d_meta.p, size_t(m) * sizeof(slate_block_meta), hipMemcpyDeviceToHost, s));
      L.decoded = true;
    }
    SLATE_HIP(hipEventRecord(L.done, s));
    // chunk k-1 out of its staging while chunk k decodes: the D2H engine has chunk k queued
    // behind chunk k-1, and the lane chunk k+1 takes is free by then
    if (&prev != &L) {
      st = lane_finish(prev, o);
      if (st) return st;
    }
    if (trace)
      fprintf(stderr, "[slate host] chunk %u blocks %u in %.1f MB: copy-in %.2f ms, plan %.2f ms, prev out %.2f ms\n",
              b, m, bytes / 1e6, t1 - t0, t2 - t1, now_ms() - t2);
    b = e;
  }
  for (PipeLane& L : ctx->lanes) {
    int st = lane_finish(L, o);
    if (st) return st;
  }
  if (trace) fprintf(stderr, "[slate host] %u blocks: %.2f ms\n", n, now_ms() - t_start);
  return fits ? SLATE_OK : SLATE_E_CAPACITY;
}

uint32_t shard_count(uint32_t n, uint32_t g, uint32_t s) { return s < n ? (n - s + g - 1) / g : 0u; }

}  // namespace

extern "C" {

int slate_block_decode_batch(slate_ctx* ctx, int codec, const uint8_t* in, const uint64_t* in_off, uint32_t n,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_off, slate_block_meta* meta,
                             slate_row* rows, uint64_t rows_cap, uint64_t* row_base) {
  if (!ctx || !in_off || !out_off || !row_base || (n && !in)) return SLATE_E_INVALID_ARG;
  if (n == 0) {
    out_off[0] = row_base[0] = 0;
    return SLATE_OK;
  }
  // offsets must not decrease (a decreasing offset inside a chunk would underflow its block
  // lengths): checked before any lane work starts, as slate_shard_pack does
  for (uint32_t i = 0; i < n; i++)
    if (in_off[i + 1] < in_off[i]) return SLATE_E_INVALID_ARG;
  Sink o;
  o.out = out;
  o.out_cap = out_cap;
  o.out_off = out_off;
  o.meta = meta;
  o.rows = rows;
  o.rows_cap = rows_cap;
  o.row_base = row_base;
  sink_map(o);
  return host_decode(ctx, codec, in, in_off, n, o);
}

// One block, lowest latency: pinned staging, plan, decode, two synchronisations.
int slate_block_decode(slate_ctx* ctx, int codec, const uint8_t* in, size_t in_len, uint8_t* out, size_t out_cap,
                       size_t* out_len, slate_block_meta* meta, uint16_t* offsets, size_t offsets_cap) {
  if (!ctx || !meta || (in_len && !in)) return SLATE_E_INVALID_ARG;
  if (in_len >= 0xFFFFFFF0ull) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  PipeLane& L = ctx->lanes[0];
  SLATE_HIP(lane_init(L));
  hipStream_t s = L.stream;
  SLATE_HIP(ctx->h_small.ensure(in_len + 256));
  uint8_t* h = ctx->h_small.as<uint8_t>();
  uint64_t* hv = reinterpret_cast<uint64_t*>(h);  // in_off[2] | out_off[2] | row_base[2] | meta (16 B)
  uint8_t* hin = h + 128;
  hv[0] = 0;
  hv[1] = in_len;
  if (in_len) memcpy(hin, in, in_len);
  // CodecNone / CodecSnappy within the large-block LDS budget: the plan here, one launch that
  // reads the staging and writes meta and decoded bytes through their device addresses, one wait
  uint64_t dl1 = host_plannable(codec) ? host_decoded_len(codec, in, in_len) : 0;
  if (host_plannable(codec) && in_len + 15 <= kLargeInCap && align16(dl1) <= kLargeOutCap && !one_off()) {
    const uint64_t osz = align16(dl1), rsz = row_capacity(dl1);
    SLATE_HIP(L.d_in.ensure(in_len + 32));
    SLATE_HIP(L.d_out.ensure(osz + 16));
    SLATE_HIP(L.d_rows.ensure((rsz + 1) * sizeof(slate_row)));
    SLATE_HIP(L.h_out.ensure(osz + 16));
    uint8_t* hin_dev = static_cast<uint8_t*>(mapped_ptr(hin));
    uint8_t* hout_dev = static_cast<uint8_t*>(mapped_ptr(L.h_out.p));
    slate_block_meta* hmeta = reinterpret_cast<slate_block_meta*>(hv + 6);
    slate_block_meta* hmeta_dev = static_cast<slate_block_meta*>(mapped_ptr(hmeta));
    if (hin_dev && hout_dev && hmeta_dev) {
      DecodeArgs a{codec, L.d_in.as<uint8_t>(), nullptr, 1, L.d_out.as<uint8_t>(), nullptr, hmeta_dev,
                   L.d_rows.as<slate_row>(), nullptr, nullptr, nullptr, 0};
      SLATE_HIP(launch_decode_one(s, a, hin_dev, in_len, osz, rsz, hout_dev));
      SLATE_HIP(hipStreamSynchronize(s));
      return block_decode_finish(*hmeta, L.h_out.as<uint8_t>(), out, out_cap, out_len, meta, offsets, offsets_cap);
    }
  }
  SLATE_HIP(L.d_in.ensure(in_len + 32));
  SLATE_HIP(L.d_in_off.ensure(64));
  SLATE_HIP(L.d_out_off.ensure(64));
  SLATE_HIP(L.d_row_base.ensure(64));
  SLATE_HIP(L.d_scratch.ensure(decode_scratch_bytes_codec(1, codec) + 64));
  SLATE_HIP(L.d_meta.ensure(64));
  if (in_len) SLATE_HIP(hipMemcpyAsync(L.d_in.p, hin, in_len, hipMemcpyHostToDevice, s));
  SLATE_HIP(hipMemcpyAsync(L.d_in_off.p, hv, 16, hipMemcpyHostToDevice, s));
  SLATE_HIP(launch_decode_plan(s, codec, L.d_in.as<uint8_t>(), L.d_in_off.as<uint64_t>(), 1,
                               L.d_out_off.as<uint64_t>(), L.d_row_base.as<uint64_t>(), L.d_scratch.p));
  SLATE_HIP(hipMemcpyAsync(hv + 2, L.d_out_off.p, 16, hipMemcpyDeviceToHost, s));
  SLATE_HIP(hipMemcpyAsync(hv + 4, L.d_row_base.p, 16, hipMemcpyDeviceToHost, s));
  SLATE_HIP(hipStreamSynchronize(s));
  const uint64_t cap = hv[3], slots = hv[5];
  SLATE_HIP(L.d_out.ensure(cap + 16));
  SLATE_HIP(L.d_rows.ensure((slots + 1) * sizeof(slate_row)));
  SLATE_HIP(L.h_out.ensure(cap + 16));
  DecodeArgs a{codec, L.d_in.as<uint8_t>(), L.d_in_off.as<uint64_t>(), 1, L.d_out.as<uint8_t>(),
               L.d_out_off.as<uint64_t>(), L.d_meta.as<slate_block_meta>(), L.d_rows.as<slate_row>(),
               L.d_row_base.as<uint64_t>(), nullptr, nullptr, 0};
  a.side = &L.side;
  a.handbacks = ctx_handbacks(ctx);
  SLATE_HIP(launch_decode(s, a, L.d_scratch.p, ctx->num_cus));
  SLATE_HIP(hipMemcpyAsync(hv + 6, L.d_meta.p, sizeof(slate_block_meta), hipMemcpyDeviceToHost, s));
  if (cap) SLATE_HIP(hipMemcpyAsync(L.h_out.p, L.d_out.p, cap, hipMemcpyDeviceToHost, s));
  SLATE_HIP(hipStreamSynchronize(s));
  return block_decode_finish(*reinterpret_cast<const slate_block_meta*>(hv + 6), L.h_out.as<uint8_t>(), out, out_cap,
                             out_len, meta, offsets, offsets_cap);
}

uint32_t slate_shard_blocks(uint32_t n_blocks, uint32_t n_shards, uint32_t shard) {
  if (n_shards == 0 || shard >= n_shards) return 0;
  return shard_count(n_blocks, n_shards, shard);
}

int slate_shard_pack(const uint8_t* in, const uint64_t* in_off, uint32_t n_blocks, uint32_t n_shards, uint32_t shard,
                     uint8_t* out, uint64_t out_cap, uint64_t* out_off) {
  if (!in_off || !out_off || n_shards == 0 || shard >= n_shards) return SLATE_E_INVALID_ARG;
  const uint32_t m = shard_count(n_blocks, n_shards, shard);
  uint64_t pos = 0;
  out_off[0] = 0;
  for (uint32_t j = 0; j < m; j++) {
    const uint64_t i = uint64_t(shard) + uint64_t(j) * n_shards;
    if (in_off[i + 1] < in_off[i]) return SLATE_E_INVALID_ARG;
    pos += in_off[i + 1] - in_off[i];
    out_off[j + 1] = pos;
  }
  if (pos > out_cap || (pos && (!out || !in))) return SLATE_E_CAPACITY;
  for (uint32_t j = 0; j < m; j++) {
    const uint64_t i = uint64_t(shard) + uint64_t(j) * n_shards;
    if (out_off[j + 1] > out_off[j]) memcpy(out + out_off[j], in + in_off[i], out_off[j + 1] - out_off[j]);
  }
  return SLATE_OK;
}

int slate_block_decode_sharded(slate_ctx* const* ctxs, uint32_t n_ctx, int codec, const uint8_t* in,
                               const uint64_t* in_off, uint32_t n, uint8_t* out, uint64_t out_cap, uint64_t* out_off,
                               slate_block_meta* meta, slate_row* rows, uint64_t rows_cap, uint64_t* row_base) {
  if (!ctxs || n_ctx == 0 || !in_off || !out_off || !row_base || (n && !in)) return SLATE_E_INVALID_ARG;
  for (uint32_t g = 0; g < n_ctx; g++) {
    if (!ctxs[g]) return SLATE_E_INVALID_ARG;
    // one host thread per context below: a context listed twice would share its lanes
    for (uint32_t h = 0; h < g; h++)
      if (ctxs[h] == ctxs[g]) return SLATE_E_INVALID_ARG;
  }
  // No re-pack: each context's staging gathers its blocks straight from the caller's buffer.
  struct Shard {
    std::vector<uint64_t> in_off, gsrc, out_off, row_base;
    uint32_t m = 0;
    int st = SLATE_OK;
  };
  std::vector<Shard> sh(n_ctx);
  // one host thread per context; each context's copies run on that context's own copy threads
  auto run = [&](auto&& fn) {
    std::vector<std::thread> th;
    for (uint32_t g = 1; g < n_ctx; g++) th.emplace_back(fn, g);
    fn(0);
    for (auto& t : th) t.join();
    for (uint32_t g = 0; g < n_ctx; g++)
      if (sh[g].st) return sh[g].st;
    return int(SLATE_OK);
  };
  // phase 1: each context's layout (block i -> context i mod n_ctx) and plan -- on the host for
  // None / Snappy (the varint header), else by a plan-only pass on the context's GPU
  int st = run([&](uint32_t g) {
    Shard& S = sh[g];
    S.m = shard_count(n, n_ctx, g);
    S.in_off.assign(size_t(S.m) + 1, 0);
    S.gsrc.assign(size_t(S.m) + 1, 0);
    S.out_off.assign(size_t(S.m) + 1, 0);
    S.row_base.assign(size_t(S.m) + 1, 0);
    for (uint32_t j = 0; j < S.m; j++) {
      const uint64_t i = uint64_t(g) + uint64_t(j) * n_ctx;
      if (in_off[i + 1] < in_off[i]) {
        S.st = SLATE_E_INVALID_ARG;
        return;
      }
      S.gsrc[j] = in_off[i];
      S.in_off[j + 1] = S.in_off[j] + (in_off[i + 1] - in_off[i]);
    }
    if (S.m == 0) return;
    if (host_plannable(codec)) {
      for (uint32_t j = 0; j < S.m; j++) {
        const uint64_t dl = host_decoded_len(codec, in + S.gsrc[j], S.in_off[j + 1] - S.in_off[j]);
        S.out_off[j + 1] = S.out_off[j] + align16(dl);
        S.row_base[j + 1] = S.row_base[j] + row_capacity(dl);
      }
      return;
    }
    Sink o;  // no meta: plan only
    o.out_off = S.out_off.data();
    o.row_base = S.row_base.data();
    const int r = host_decode(ctxs[g], codec, in, S.in_off.data(), S.m, o, S.gsrc.data());
    S.st = r == SLATE_E_CAPACITY ? SLATE_OK : r;
  });
  if (st) return st;
  // the batch's layout, in block order
  out_off[0] = row_base[0] = 0;
  for (uint32_t i = 0; i < n; i++) {
    const Shard& S = sh[i % n_ctx];
    const uint32_t j = i / n_ctx;
    out_off[i + 1] = out_off[i] + (S.out_off[j + 1] - S.out_off[j]);
    row_base[i + 1] = row_base[i] + (S.row_base[j + 1] - S.row_base[j]);
  }
  if (n == 0) return SLATE_OK;
  if (!meta || out_off[n] > out_cap || row_base[n] > rows_cap || (out_off[n] && !out) || (row_base[n] && !rows))
    return SLATE_E_CAPACITY;
  // phase 2: each context decodes its shard; chunks land block by block at their places
  return run([&](uint32_t g) {
    Shard& S = sh[g];
    if (S.m == 0) return;
    Sink o;
    o.out = out;
    o.out_cap = out_cap;
    o.meta = meta;
    o.rows = rows;
    o.rows_cap = rows_cap;
    o.out_off = S.out_off.data();
    o.row_base = S.row_base.data();
    o.G = n_ctx;
    o.g = g;
    o.g_out_off = out_off;
    o.g_row_base = row_base;
    // the device addresses are per device: each context maps the buffers for its own GPU
    if (ctx_bind(ctxs[g]) != hipSuccess) {
      S.st = SLATE_E_HIP;
      return;
    }
    sink_map(o);
    // G contexts on this host: kCopyThreads / G copy tasks each, unless the count was set
    t_pool_cap = ctxs[g]->copy_threads_set ? 0 : std::max<size_t>(1, kCopyThreads / n_ctx);
    S.st = host_decode(ctxs[g], codec, in, S.in_off.data(), S.m, o, S.gsrc.data());
    t_pool_cap = 0;
  });
}

}  // extern "C"
