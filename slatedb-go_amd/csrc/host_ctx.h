// Host-side context: one device + one HIP stream + reusable device/pinned
// buffers.  Each slate_ctx is used by one caller thread at a time; the library
// keeps no global mutable state (SURVEY 8b "Threading").
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "kernels.h"

// Device allocations keep kDevGuard readable bytes in front of p: the wave decoders' HBM mode
// (blocks beyond the LDS budget, index / filter payloads) reads the aligned dword or chunk around a
// block's first byte, which for a block at offset 0 lies before the buffer.
constexpr size_t kDevGuard = 256;
struct DevBuf {
  void* p = nullptr;
  void* base = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    size_t c = n < 4096 ? 4096 : n + n / 4;
    hipError_t e = hipMalloc(&base, c + kDevGuard);
    if (e != hipSuccess) {
      base = nullptr;
      return e;
    }
    p = static_cast<uint8_t*>(base) + kDevGuard;
    cap = c;
    return hipSuccess;
  }
  // grow preserving the first `keep` bytes (stream-ordered copy)
  hipError_t grow_keep(size_t n, size_t keep, hipStream_t st) {
    if (n <= cap) return hipSuccess;
    void* q = nullptr;
    size_t c = n + n / 2;
    hipError_t e = hipMalloc(&q, c + kDevGuard);
    if (e != hipSuccess) return e;
    void* qp = static_cast<uint8_t*>(q) + kDevGuard;
    if (p && keep) {
      e = hipMemcpyAsync(qp, p, keep, hipMemcpyDeviceToDevice, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) {
        (void)hipFree(q);
        return e;
      }
    }
    if (base) (void)hipFree(base);
    base = q;
    p = qp;
    cap = c;
    return hipSuccess;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
  void release() {
    if (base) (void)hipFree(base);
    p = base = nullptr;
    cap = 0;
  }
};

// Page-locked host staging (hipHostMalloc): DMA-able, so copies overlap kernels.
// The device address of page-locked host memory, null for pageable memory.
inline void* mapped_ptr(void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (at.type != hipMemoryTypeHost) return nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

// The context's hand-back counter (DecodeArgs::handbacks), zeroed when first made; nullptr if it
// cannot be allocated (decoding goes on uncounted).
struct slate_ctx;
uint64_t* ctx_handbacks(slate_ctx* ctx);

// The device address of host range [p, p + len) when the whole range is page-locked in one mapping
// (its last byte maps to d + len - 1); nullptr otherwise, e.g. when a caller registered only a prefix.
inline void* mapped_range(void* p, uint64_t len) {
  void* d = mapped_ptr(p);
  if (!d || len == 0) return d;
  void* e = mapped_ptr(static_cast<uint8_t*>(p) + (len - 1));
  return e == static_cast<uint8_t*>(d) + (len - 1) ? d : nullptr;
}

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t c = n < 65536 ? 65536 : n + n / 4;
    hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    cap = c;
    return hipSuccess;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// One lane of the host-buffer decode pipeline: its own stream, device buffers and pinned
// staging, so chunk c+1's upload and plan overlap chunk c's decode and download.
struct PipeLane {
  hipStream_t stream = nullptr;
  hipEvent_t planned = nullptr, done = nullptr;
  DevBuf d_in, d_in_off, d_out_off, d_row_base, d_scratch, d_out, d_meta, d_rows, d_dense, d_gmap;
  DevBuf d_zlstage;  // CodecZlib chunks: the staged plan (phase Z once, for the chunk's decode)
  PinBuf h_in, h_in_off, h_plan, h_out, h_meta, h_rows, h_gmap;  // h_rows: the chunk's rows, dense (rows_pack)
  bool direct = false;  // the chunk's bytes and rows went straight to the caller's page-locked buffers
  // the chunk in flight: blocks [b0, b0+n), its place in the caller's outputs
  uint32_t b0 = 0, n = 0;
  uint64_t out_base = 0, row_base = 0, out_total = 0, rows_total = 0;
  bool busy = false, decoded = false;
  slate::SideStream side;  // the lane's second stream (DecodeArgs::side)
  void release() {
    side.release();
    for (DevBuf* b : {&d_in, &d_in_off, &d_out_off, &d_row_base, &d_scratch, &d_out, &d_meta, &d_rows, &d_dense,
                      &d_gmap, &d_zlstage})
      b->release();
    for (PinBuf* b : {&h_in, &h_in_off, &h_plan, &h_out, &h_meta, &h_rows, &h_gmap}) b->release();
    if (planned) (void)hipEventDestroy(planned);
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
    planned = done = nullptr;
    stream = nullptr;
  }
};
constexpr int kPipeLanes = 2;

// Released encoded-SST host buffers (api_sst.cpp HostBytes mappings) kept for reuse by the
// context's next builds: a few, best fit.  Shared with the buffers, so it outlives whichever
// of them and the context goes last.
constexpr size_t kSegHuge = 2u << 20;
struct SegPool {
  struct Seg {
    void* p;
    size_t cap;
    bool pinned;  // registered with the runtime (hipHostRegister): the blocks' D2H lands in it directly
  };
  std::mutex mu;
  std::vector<Seg> free_list;
  bool open = true;
  static constexpr size_t kKeep = 8;  // (a build in pieces releases five: four block segments, the final chunk)
  bool take(size_t len, uint8_t** p, size_t* cap, bool* pinned) {
    std::lock_guard<std::mutex> g(mu);
    size_t best = free_list.size();
    for (size_t i = 0; i < free_list.size(); i++)
      if (free_list[i].cap >= len && free_list[i].cap <= 2 * len + kSegHuge &&
          (best == free_list.size() || free_list[i].cap < free_list[best].cap))
        best = i;
    if (best == free_list.size()) return false;
    *p = static_cast<uint8_t*>(free_list[best].p);
    *cap = free_list[best].cap;
    *pinned = free_list[best].pinned;
    free_list.erase(free_list.begin() + long(best));
    return true;
  }
  bool give(void* p, size_t cap, bool pinned) {  // false: the caller unmaps it
    std::lock_guard<std::mutex> g(mu);
    if (!open || free_list.size() >= kKeep) return false;
    free_list.push_back(Seg{p, cap, pinned});
    return true;
  }
  void close();  // unmaps the kept buffers (api_sst.cpp)
};

// A context's host copy threads: started on first use and kept, so the chunked host pipelines
// (api_host.cpp) do not create threads per chunk.  run(tasks, fn) calls fn(k) for every k in
// [0, tasks) on the workers and the calling thread and returns when all have run; one run at a
// time (a context serves one caller thread at a time).
class CopyPool {
 public:
  explicit CopyPool(size_t threads) : n_(threads ? threads : 1) {}
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  size_t size() const { return n_; }
  void run(size_t tasks, const std::function<void(size_t)>& fn) {
    if (tasks == 0) return;
    if (tasks == 1 || n_ == 1) {
      for (size_t k = 0; k < tasks; k++) fn(k);
      return;
    }
    std::lock_guard<std::mutex> one(run_mu_);
    std::unique_lock<std::mutex> g(mu_);
    while (th_.size() + 1 < std::min(n_, tasks)) th_.emplace_back([this] { worker(); });
    job_ = &fn;
    tasks_ = tasks;
    next_ = 0;
    pending_ = tasks;
    gen_++;
    cv_.notify_all();
    drain(g);
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  // takes tasks until none is left; called with mu_ held, returns with it held
  void drain(std::unique_lock<std::mutex>& g) {
    while (job_ && next_ < tasks_) {
      const size_t k = next_++;
      const std::function<void(size_t)>* f = job_;
      g.unlock();
      (*f)(k);
      g.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  void worker() {
    std::unique_lock<std::mutex> g(mu_);
    uint64_t seen = 0;
    for (;;) {
      cv_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      drain(g);
    }
  }
  const size_t n_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t tasks_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct slate_ctx {
  int device = 0;
  int num_cus = 256;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  PipeLane lanes[kPipeLanes];
  // a second download pipe (ctx_d2h_side): its own stream, page-locked pieces and copy threads, so
  // that a builder's finished blocks leave while the caller's thread uploads the next KVs
  PipeLane d2h_lanes[kPipeLanes];
  hipEvent_t d2h_after = nullptr;
  std::unique_ptr<CopyPool> d2h_pool;
  PinBuf h_small;  // single-block staging (slate_block_decode)
  PinBuf h_seek;   // slate_block_seek(_warn) inputs (one upload) and results (written by the kernel)
  // decode batch buffers
  DevBuf d_in, d_in_off, d_out, d_out_off, d_meta, d_rows, d_row_base, d_scratch;
  // encode / misc buffers
  DevBuf e_a, e_b, e_c, e_d, e_e, e_f, e_g, e_h, e_i, e_j, e_k;
  // Snappy encode: per-block slots, raw staging for oversized blocks, snappy LDS-free scratch
  DevBuf s_slots, s_raw, s_aux;
  // LZ4 / Zlib / Zstd encode (encode_codecs.hip): piece tables, tag and body slots, sequences, frames
  DevBuf c_meta, c_tags, c_bodies, c_seqs, c_out, c_in;
  // SST filter built beside the final flush (api_sst.cpp build_filter_aux): its own stream and buffers
  hipStream_t aux = nullptr;
  slate::SideStream side;  // the context stream's second stream (DecodeArgs::side)
  DevBuf d_handbacks;      // DecodeArgs::handbacks of every decode through this context (u64)
  // the staged CodecZlib plan (slate_block_decode_plan_device): phase Z's output, consumed by the
  // next slate_block_decode_device over the same inputs on the same stream (zl_armed)
  DevBuf zl_stage;
  struct {
    const uint8_t* in = nullptr;
    const uint64_t* in_off = nullptr;
    const uint64_t* out_off = nullptr;
    uint32_t n = 0;
    hipStream_t stream = nullptr;
  } zl_plan;
  bool zl_armed = false;
  DevBuf x_words, x_enc, x_slots, x_asm, x_crc, x_bkt;
  std::shared_ptr<SegPool> seg_pool = std::make_shared<SegPool>();
  // device time of the builder's GPU passes (slate_ctx_set_timing): nanoseconds, summed over the
  // kernel groups of every stream the context uses (GpuSpan)
  bool timing = false;
  std::atomic<uint64_t> gpu_ns{0};
  // the same spans as [start, end) in ms after t_ref (recorded on the context's stream when timing
  // is switched on), for their union: device time with the overlap of the side streams counted once
  hipEvent_t t_ref = nullptr;
  std::mutex span_mu;
  std::vector<std::pair<double, double>> spans;
  void add_span(hipEvent_t a, hipEvent_t b, double ms) {
    gpu_ns.fetch_add(uint64_t(ms * 1e6));
    float s0 = 0.f;
    if (!t_ref || hipEventElapsedTime(&s0, t_ref, a) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(span_mu);
    spans.emplace_back(double(s0), double(s0) + ms);
    (void)b;
  }
  double span_union_ms() {
    std::lock_guard<std::mutex> lk(span_mu);
    std::vector<std::pair<double, double>> v = spans;
    std::sort(v.begin(), v.end());
    double tot = 0, lo = 0, hi = 0;
    bool open = false;
    for (const auto& iv : v) {
      if (open && iv.first <= hi) {
        hi = std::max(hi, iv.second);
        continue;
      }
      if (open) tot += hi - lo;
      lo = iv.first;
      hi = iv.second;
      open = true;
    }
    if (open) tot += hi - lo;
    return tot;
  }
  // host copy threads of this context (slate_ctx_set_copy_threads; SLATE_COPY_THREADS or 16)
  size_t copy_threads = 16;
  bool copy_threads_set = false;  // set explicitly (API or SLATE_COPY_THREADS): sharded calls keep it
  std::unique_ptr<CopyPool> copy_pool;
  CopyPool* pool() {
    if (!copy_pool) copy_pool.reset(new CopyPool(copy_threads));
    return copy_pool.get();
  }
  void release_all() {
    if (seg_pool) seg_pool->close();
    for (DevBuf* b : {&d_in, &d_in_off, &d_out, &d_out_off, &d_meta, &d_rows, &d_row_base, &d_scratch, &e_a,
                      &e_b, &e_c, &e_d, &e_e, &e_f, &e_g, &e_h, &e_i, &e_j, &e_k, &s_slots, &s_raw, &s_aux, &c_meta,
                      &c_tags, &c_bodies, &c_seqs, &c_out, &c_in, &x_words, &x_enc, &x_slots, &x_asm, &x_crc, &x_bkt,
                      &d_handbacks, &zl_stage})
      b->release();
    if (aux) (void)hipStreamDestroy(aux);
    aux = nullptr;
    side.release();
    if (t_ref) (void)hipEventDestroy(t_ref);
    t_ref = nullptr;
    for (PipeLane& l : lanes) l.release();
    for (PipeLane& l : d2h_lanes) l.release();
    if (d2h_after) (void)hipEventDestroy(d2h_after);
    d2h_after = nullptr;
    h_small.release();
    h_seek.release();
  }
};

// A group of kernel launches on one stream, timed by two HIP events when the context's timing is
// on (slate_ctx_set_timing; a no-op otherwise): begin at construction, stop() after the group's
// last launch (before any copy the caller queues next), read at destruction -- callers synchronise
// the stream before they return anyway.
struct GpuSpan {
  slate_ctx* ctx;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  bool stopped = false;
  GpuSpan(slate_ctx* c, hipStream_t s) : ctx(c), st(s) {
    if (!c->timing) return;
    if (hipEventCreate(&a) != hipSuccess) {
      a = nullptr;
      return;
    }
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      a = b = nullptr;
      return;
    }
    (void)hipEventRecord(a, st);
  }
  void stop() {
    if (a && !stopped) (void)hipEventRecord(b, st);
    stopped = true;
  }
  ~GpuSpan() {
    if (!a) return;
    stop();
    float ms = 0.f;
    if (hipEventSynchronize(b) == hipSuccess && hipEventElapsedTime(&ms, a, b) == hipSuccess && ms > 0.f)
      ctx->add_span(a, b, double(ms));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
  GpuSpan(const GpuSpan&) = delete;
  GpuSpan& operator=(const GpuSpan&) = delete;
};

#define SLATE_HIP(expr)                                                                               \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "[slate hip] %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__);               \
      return hip_status(_e);                                                                          \
    }                                                                                                 \
  } while (0)

inline int hip_status(hipError_t e) {
  if (e == hipErrorOutOfMemory) return SLATE_E_OOM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
      e == hipErrorInvalidDeviceFunction)
    return SLATE_E_NO_DEVICE;
  return SLATE_E_HIP;
}

inline hipError_t ctx_bind(slate_ctx* ctx) { return hipSetDevice(ctx->device); }

// SLATE_HOST_TRACE=1: host phase times of the host pipelines on stderr (diagnostics for the
// numbers in DESIGN.md; read once per process).
inline bool host_trace() {
  static const bool on = [] {
    const char* e = getenv("SLATE_HOST_TRACE");
    return e && *e == '1';
  }();
  return on;
}
inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Host copies split over the context's copy threads (default 16: the CPU share one GPU's process
// gets on the MI355X boxes; one core copies ~10 GB/s, below the PCIe link) -- api_host.cpp.
constexpr size_t kCopyThreads = 16;
// The pool the calling thread's large copies use: set for the duration of a context's call by
// PoolScope (a sharded decode runs one host thread per context, each on its own pool); without
// one, par_memcpy copies on the calling thread alone.
extern thread_local CopyPool* t_pool;
struct PoolScope {
  CopyPool* keep;
  explicit PoolScope(slate_ctx* ctx) : keep(t_pool) { t_pool = ctx->pool(); }
  explicit PoolScope(CopyPool* p) : keep(t_pool) { t_pool = p; }
  ~PoolScope() { t_pool = keep; }
};
void par_memcpy(void* dst, const void* src, size_t n);
// A pipeline lane's stream and events, created on first use.
hipError_t lane_init(PipeLane& L);
// Large host <-> device copies through the context's page-locked lane staging (64 MiB pieces,
// two in flight; stream-ordered on st, synchronous on return); small ones go straight through.
// CodecNone / CodecSnappy block sizes known on the host (api_host.cpp): the decoded length from the
// payload length or golang/snappy's varint header (0 for a header the decoder rejects)
bool host_plannable(int codec);
uint64_t host_decoded_len(int codec, const uint8_t* p, uint64_t len);
int ctx_h2d(slate_ctx* ctx, void* dst, const void* src, size_t n, hipStream_t st);
int ctx_d2h(slate_ctx* ctx, void* dst, const void* src, size_t n, hipStream_t st);
// ctx_d2h through the context's second download pipe, after `after` (an event recorded on the
// stream that produced src); for a worker thread while the caller's thread runs ctx_h2d
int ctx_d2h_side(slate_ctx* ctx, void* dst, const void* src, size_t n, hipEvent_t after);

// compress.Decode of one `payload || BE32 CRC` buffer (an index or filter) on the GPU, CRC
// first: *bstatus = SLATE_OK, SLATE_E_BLOCK_CHECKSUM or the codec's status (api_sst.cpp).
int ctx_payload_decode_buffer(slate_ctx* ctx, int codec, const uint8_t* buf, size_t len, std::vector<uint8_t>& out,
                              int* bstatus);
// CRC32-IEEE of a host buffer computed on the context's GPU (stream-synchronous).
int ctx_crc32_host_buffer(slate_ctx* ctx, const uint8_t* data, size_t n, uint32_t* crc);
// CRC32-IEEE of a device buffer (stream-synchronous, result to host).
int ctx_crc32_device(slate_ctx* ctx, const uint8_t* d_data, size_t n, uint32_t* crc);
