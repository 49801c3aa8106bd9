// C-ABI: executeCompaction's SST-codec path in one call (slate_compact).
//
// slatedb/compaction/executor.go:92-151 builds an iter.MergeSort over the input SSTs' iterators
// (L0 SSTs, then sorted runs; executor.go:55-90), writes every entry it returns through an
// EncodedSSTableWriter (table_store.go:221-266: AddValue, so an empty value is a tombstone) and
// closes the writer once the running key + value size passes MaxSSTSize (executor.go:119-139).
// Here every byte of that runs on the GPU through the device-resident entry points, on device
// memory the library owns: the data blocks of each run of SSTs sharing a codec are decoded in one
// batch (block.Decode, as sstable.Iterator does per block, internal/sstable/iterator.go:92-118),
// their rows become (full key, value) entries (block.Iterator, block/iterator.go:84-107), the
// entries of all sources are merged (iter.MergeSort, internal/iter/merge.go:12-111), gathered in
// merged order, and fed to one SST builder per output SST.  The host reads only each SST's info
// and index (ReadInfo / ReadIndex, decode.go:25-103), block statuses and the offset arrays that
// decide where outputs split.  Scheduling, manifests and object storage stay with the caller.
#include <algorithm>
#include <cstring>
#include <memory>
#include <set>
#include <vector>

#include "../../include/slatecodec.h"
#include "host_ctx.h"

using namespace slate;

namespace {

// device memory scoped to one slate_compact call
struct Dev {
  DevBuf b;
  ~Dev() { b.release(); }
  template <typename T>
  T* as() const { return b.as<T>(); }
};

struct IndexFree {
  void operator()(slate_index* x) const { slate_index_free(x); }
};

// The KV view of some rows on the device: keys / values back to back, n + 1 offsets into them,
// a tombstone flag per entry.
struct View {
  std::shared_ptr<Dev> keys, key_off, vals, val_off, tomb;
  uint64_t n = 0, kb = 0, vb = 0;
};

int d2h_small(slate_ctx* ctx, void* dst, const void* src, size_t n) {
  SLATE_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->stream));
  SLATE_HIP(hipStreamSynchronize(ctx->stream));
  return SLATE_OK;
}

std::shared_ptr<Dev> dev(size_t bytes, hipError_t* e) {
  auto d = std::make_shared<Dev>();
  *e = d->b.ensure(std::max<size_t>(bytes, 16));
  return d;
}

#define DEV(var, bytes)                       \
  hipError_t var##_e;                         \
  auto var = dev((bytes), &var##_e);          \
  if (var##_e != hipSuccess) return hip_status(var##_e)

// A warning with the surviving rows its SST had produced before it (decides when MergeSort merges it).
struct Warn {
  slate_compact_warning w;
  uint64_t rows_before;  // rows of the warning's SST returned before it
};

// One device batch over the data blocks of SSTs that share a codec -> a KV view and the rows of
// each SST (in order), with Go's iterator semantics on corrupt input: a block that fails
// block.Decode ends its SST (sstable.Iterator.Next, iterator.go:59-68), a row that fails ends its
// block (block/iterator.go:92-96); each adds a warning.  blocks: the SSTs' data-block byte ranges,
// gathered on the host; sst0 / sst_src: the first SST's index and every SST's source.
// One host range of the group's data blocks (an SST's [offs[0], FilterOffset)), uploaded as it lies
// in the caller's buffer: no host-side gather of the blocks first.
struct Piece {
  const uint8_t* p;
  uint64_t len;
};

int decode_group(slate_ctx* ctx, int codec, const std::vector<Piece>& pieces, const std::vector<uint64_t>& in_off,
                 const std::vector<uint32_t>& sst_blocks, uint32_t sst0, const std::vector<uint32_t>& sst_src, View* v,
                 std::vector<uint64_t>* rows_per_sst, std::vector<Warn>* warns) {
  const uint32_t n = uint32_t(in_off.size() - 1);
  hipStream_t st = ctx->stream;
  const uint64_t total = in_off.back();
  DEV(d_in, total + 16);
  DEV(d_in_off, in_off.size() * 8);
  DEV(d_out_off, (size_t(n) + 1) * 8);
  DEV(d_row_base, (size_t(n) + 1) * 8);
  DEV(d_scr, decode_scratch_bytes_codec(n, codec) + 64);
  int s = SLATE_OK;
  uint64_t at = 0;
  for (const Piece& pc : pieces) {
    if ((s = ctx_h2d(ctx, d_in->as<uint8_t>() + at, pc.p, pc.len, st))) return s;
    at += pc.len;
  }
  SLATE_HIP(hipMemcpyAsync(d_in_off->b.p, in_off.data(), in_off.size() * 8, hipMemcpyHostToDevice, st));
  // CodecNone: block.Decode's Data aliases the input (block.go:122), so the decoded blocks are the
  // uploaded bytes themselves -- no plan, no decoded copy; the row slots from the payload lengths
  const bool alias = codec == SLATE_CODEC_NONE;
  uint64_t tot[2] = {0, 0};
  ZlStage zl_g{};
  const ZlStage* zg = (codec == SLATE_CODEC_ZLIB && n >= 64 && !getenv("SLATE_ZL_NO_STAGE")) ? &zl_g : nullptr;
  if (alias) {
    std::vector<uint64_t> rb(size_t(n) + 1, 0);
    for (uint32_t i = 0; i < n; i++) {
      const uint64_t len = in_off[i + 1] - in_off[i];
      rb[i + 1] = rb[i] + row_capacity(len >= 6 ? len - 4 : 0);  // plan_reduce_kernel's CodecNone sizes
    }
    tot[1] = rb[n];
    SLATE_HIP(hipMemcpyAsync(d_row_base->b.p, rb.data(), rb.size() * 8, hipMemcpyHostToDevice, st));
  } else {
    if (zg) {  // CodecZlib: the plan is phase Z, staged in the context for this decode
      SLATE_HIP(ctx->zl_stage.ensure(zl_stage_bytes(n)));
      ctx->zl_armed = false;  // (the device API's pending plan, if any, is overwritten)
      zl_g = zl_stage_carve(ctx->zl_stage.p, n);
    }
    {
      GpuSpan gs(ctx, st);  // device time (slate_ctx_set_timing): every kernel group of the compaction
      SLATE_HIP(launch_decode_plan(st, codec, d_in->as<uint8_t>(), d_in_off->as<uint64_t>(), n,
                                   d_out_off->as<uint64_t>(), d_row_base->as<uint64_t>(), d_scr->b.p, zg,
                                   ctx->num_cus));
    }
    if ((s = d2h_small(ctx, &tot[0], d_out_off->as<uint64_t>() + n, 8))) return s;
    if ((s = d2h_small(ctx, &tot[1], d_row_base->as<uint64_t>() + n, 8))) return s;
  }
  const uint64_t slots = tot[1];
  if (slots >= 0xFFFFFFFFull) return SLATE_E_LIMIT;
  DEV(d_out, alias ? 16 : tot[0] + 16);
  DEV(d_meta, size_t(n) * sizeof(slate_block_meta));
  DEV(d_rows, (slots + 1) * sizeof(slate_row));
  uint8_t* data = alias ? d_in->as<uint8_t>() : d_out->as<uint8_t>();
  const uint64_t* data_off = alias ? d_in_off->as<uint64_t>() : d_out_off->as<uint64_t>();
  DecodeArgs a{codec, d_in->as<uint8_t>(), d_in_off->as<uint64_t>(), n, data, data_off,
               d_meta->as<slate_block_meta>(), d_rows->as<slate_row>(), d_row_base->as<uint64_t>(), nullptr, nullptr, 0};
  a.no_data = alias ? 1u : 0u;
  if (st == ctx->stream) a.side = &ctx->side;
  a.handbacks = ctx_handbacks(ctx);
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_decode(st, a, d_scr->b.p, ctx->num_cus, zg));
  }
  // every block's status: the first failing block of an SST ends that SST's iterator with a
  // warning (iterator.go:62-68 wrapping decode.go:143-144); it and the SST's later blocks keep no
  // rows (their metas are patched to 0 rows for the rows phase)
  std::vector<slate_block_meta> meta(n);
  if ((s = ctx_d2h(ctx, meta.data(), d_meta->b.p, size_t(n) * sizeof(slate_block_meta), st))) return s;
  std::vector<int32_t> block_warn(n, 0);  // per block: status of its block.Decode failure (0 = none)
  bool patched = false;
  for (size_t j = 0; j + 1 < sst_blocks.size(); j++) {
    bool cut = false;
    for (uint32_t i = sst_blocks[j]; i < sst_blocks[j + 1]; i++) {
      if (!cut && meta[i].status == SLATE_OK && (meta[i].flags & SLATE_BLKF_ROWS_TRUNCATED)) return SLATE_E_LIMIT;
      if (!cut && meta[i].status != SLATE_OK) {
        cut = true;
        block_warn[i] = meta[i].status;
      }
      if (cut) {
        meta[i].status = SLATE_OK;
        meta[i].flags = 0;
        meta[i].n_rows = 0;
        patched = true;
      }
    }
  }
  if (patched) SLATE_HIP(hipMemcpyAsync(d_meta->b.p, meta.data(), size_t(n) * sizeof(slate_block_meta),
                                        hipMemcpyHostToDevice, st));
  // rows -> KV view
  DEV(key_off, (slots + 1) * 8);
  DEV(val_off, (slots + 1) * 8);
  DEV(tomb, slots + 1);
  DEV(d_nkv, 16);
  DEV(d_flags, 16);
  DEV(d_kvs, kv_scratch_bytes(slots) + 16);
  SLATE_HIP(hipMemsetAsync(d_nkv->b.p, 0, 16, st));
  SLATE_HIP(hipMemsetAsync(d_flags->b.p, 0, 16, st));
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_rows_lengths(st, d_row_base->as<uint64_t>(), n, d_meta->as<slate_block_meta>(),
                                  d_rows->as<slate_row>(), slots, key_off->as<uint64_t>(), val_off->as<uint64_t>(),
                                  tomb->as<uint8_t>(), d_nkv->as<uint64_t>(), d_flags->as<uint32_t>(), d_kvs->b.p));
  }
  uint32_t flags = 0;
  uint64_t n_kv = 0;
  if ((s = d2h_small(ctx, &flags, d_flags->b.p, 4))) return s;
  // rows each block returns: all of them, or those before its first failing row (the rows phase
  // dropped the rest, block/iterator.go:92-96); the failing rows' statuses are read only here
  std::vector<uint32_t> kept(n);
  std::vector<int32_t> row_warn(n, -1), row_status(n, 0);
  for (uint32_t i = 0; i < n; i++) kept[i] = meta[i].n_rows;
  if (flags & 2) {
    std::vector<int16_t> rst(slots + 1);
    SLATE_HIP(hipMemcpy2DAsync(rst.data(), 2, reinterpret_cast<const uint8_t*>(d_rows->b.p) + offsetof(slate_row, status),
                               sizeof(slate_row), 2, slots, hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> rb(size_t(n) + 1);
    if ((s = ctx_d2h(ctx, rb.data(), d_row_base->b.p, (size_t(n) + 1) * 8, st))) return s;
    for (uint32_t i = 0; i < n; i++) {
      for (uint32_t r = 0; r < meta[i].n_rows && rb[i] + r < rb[i + 1]; r++) {
        if (rst[rb[i] + r] != SLATE_OK) {
          kept[i] = r;
          row_warn[i] = int32_t(r);
          row_status[i] = rst[rb[i] + r];
          break;
        }
      }
    }
  }
  if ((s = d2h_small(ctx, &n_kv, d_nkv->b.p, 8))) return s;
  uint64_t kb = 0, vb = 0;
  if ((s = d2h_small(ctx, &kb, key_off->as<uint64_t>() + slots, 8))) return s;
  if ((s = d2h_small(ctx, &vb, val_off->as<uint64_t>() + slots, 8))) return s;
  DEV(keys, kb + 16);
  DEV(vals, vb + 16);
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_rows_copy(st, data, data_off, d_row_base->as<uint64_t>(), n,
                               d_rows->as<slate_row>(), slots, d_nkv->as<uint64_t>(), d_kvs->b.p,
                               key_off->as<uint64_t>(), keys->as<uint8_t>(), val_off->as<uint64_t>(),
                               vals->as<uint8_t>()));
  }
  SLATE_HIP(hipStreamSynchronize(st));
  // rows of each SST from its blocks' row counts; the warnings in the order its iterator adds them
  uint64_t acc = 0;
  size_t k = 0;
  for (size_t j = 0; j + 1 < sst_blocks.size(); j++) {
    uint64_t r = 0;
    const uint32_t sst = sst0 + uint32_t(j);
    for (; k < sst_blocks[j + 1]; k++) {
      const uint32_t blk = uint32_t(k - sst_blocks[j]), len = uint32_t(in_off[k + 1] - in_off[k]);
      if (block_warn[k]) warns->push_back({{sst_src[sst], sst, blk, -1, block_warn[k], len}, r});
      r += kept[k];
      if (row_warn[k] >= 0) warns->push_back({{sst_src[sst], sst, blk, row_warn[k], row_status[k], len}, r});
    }
    rows_per_sst->push_back(r);
    acc += r;
  }
  if (acc != n_kv) return SLATE_E_HIP;  // the row views disagree with the block metas: a defect
  v->keys = keys;
  v->key_off = key_off;
  v->vals = vals;
  v->val_off = val_off;
  v->tomb = tomb;
  v->n = n_kv;
  v->kb = kb;
  v->vb = vb;
  return SLATE_OK;
}

// Views of consecutive codec groups concatenated (offsets rebased on the device).
int concat_views(slate_ctx* ctx, const std::vector<View>& vs, View* out) {
  if (vs.size() == 1) {
    *out = vs[0];
    return SLATE_OK;
  }
  hipStream_t st = ctx->stream;
  uint64_t n = 0, kb = 0, vb = 0;
  for (const View& v : vs) {
    n += v.n;
    kb += v.kb;
    vb += v.vb;
  }
  DEV(keys, kb + 16);
  DEV(vals, vb + 16);
  DEV(key_off, (n + 1) * 8);
  DEV(val_off, (n + 1) * 8);
  DEV(tomb, n + 1);
  uint64_t i = 0, k = 0, b = 0;
  for (const View& v : vs) {
    if (v.kb) SLATE_HIP(hipMemcpyAsync(keys->as<uint8_t>() + k, v.keys->b.p, v.kb, hipMemcpyDeviceToDevice, st));
    if (v.vb) SLATE_HIP(hipMemcpyAsync(vals->as<uint8_t>() + b, v.vals->b.p, v.vb, hipMemcpyDeviceToDevice, st));
    if (v.n) SLATE_HIP(hipMemcpyAsync(tomb->as<uint8_t>() + i, v.tomb->b.p, v.n, hipMemcpyDeviceToDevice, st));
    SLATE_HIP(launch_u64_add(st, v.key_off->as<uint64_t>(), key_off->as<uint64_t>() + i, v.n, k));
    SLATE_HIP(launch_u64_add(st, v.val_off->as<uint64_t>(), val_off->as<uint64_t>() + i, v.n, b));
    i += v.n;
    k += v.kb;
    b += v.vb;
  }
  const uint64_t tail[2] = {kb, vb};
  SLATE_HIP(hipMemcpyAsync(key_off->as<uint64_t>() + n, &tail[0], 8, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipMemcpyAsync(val_off->as<uint64_t>() + n, &tail[1], 8, hipMemcpyHostToDevice, st));
  SLATE_HIP(hipStreamSynchronize(st));
  out->keys = keys;
  out->vals = vals;
  out->key_off = key_off;
  out->val_off = val_off;
  out->tomb = tomb;
  out->n = n;
  out->kb = kb;
  out->vb = vb;
  return SLATE_OK;
}

}  // namespace

extern "C" {

int slate_compact_ex(slate_ctx* ctx, const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst,
                     const uint32_t* src_sst, uint32_t n_src, const slate_sst_config* out_cfg, uint64_t max_sst_size,
                     slate_sst_table** out_tables, uint32_t out_cap, uint32_t* n_out, slate_compact_warning* warns,
                     uint32_t warn_cap, uint32_t* n_warn) {
  if (!ctx || !sst_off || !src_sst || !out_cfg || !n_out || n_src == 0 || (n_sst && !ssts) || (warn_cap && !warns))
    return SLATE_E_INVALID_ARG;
  *n_out = 0;
  if (n_warn) *n_warn = 0;
  if (src_sst[0] != 0 || src_sst[n_src] != n_sst) return SLATE_E_INVALID_ARG;
  for (uint32_t j = 0; j < n_src; j++)
    if (src_sst[j + 1] < src_sst[j]) return SLATE_E_INVALID_ARG;
  for (uint32_t i = 0; i < n_sst; i++)
    if (sst_off[i + 1] < sst_off[i]) return SLATE_E_INVALID_ARG;
  SLATE_HIP(ctx_bind(ctx));
  const bool trace = host_trace();  // SLATE_HOST_TRACE: the phases' host wall times on stderr
  double t_mark = trace ? now_ms() : 0.0;
  auto mark = [&](const char* what) {
    if (!trace) return;
    const double t = now_ms();
    fprintf(stderr, "[slate compact] %-22s %8.2f ms\n", what, t - t_mark);
    t_mark = t;
  };
  // ---- each SST's codec and data-block offsets (ReadInfo, ReadIndex, getBlockRange)
  std::vector<int> codec(n_sst);
  std::vector<std::vector<uint64_t>> offs(n_sst);
  for (uint32_t i = 0; i < n_sst; i++) {
    const uint8_t* sst = ssts + sst_off[i];
    const uint64_t len = sst_off[i + 1] - sst_off[i];
    slate_sst_info info{};
    // (the info is filled before the first key's capacity is checked; the key is not needed here)
    int s = slate_sst_read_info(sst, len, &info, nullptr, 0);
    if (s && s != SLATE_E_CAPACITY) return s;
    if (info.index_offset > len || info.index_len > len - info.index_offset || info.filter_offset > len)
      return SLATE_E_BLOB_RANGE;
    slate_index* ix = nullptr;
    s = slate_decode_index(ctx, sst + info.index_offset, info.index_len, info.codec, &ix);
    if (s) return s;
    std::unique_ptr<slate_index, IndexFree> hold(ix);
    const size_t nb = slate_index_num_blocks(ix);
    offs[i].resize(nb + 1);
    if (nb && (s = slate_index_block_offsets(ix, offs[i].data(), nb))) return s;
    offs[i][nb] = info.filter_offset;
    for (size_t b = 0; b < nb; b++)
      if (offs[i][b + 1] < offs[i][b] || offs[i][b + 1] > len) return SLATE_E_BLOB_RANGE;
    codec[i] = info.codec;
  }
  mark("info + index");
  std::vector<uint32_t> sst_src(n_sst);
  for (uint32_t j = 0; j < n_src; j++)
    for (uint32_t i = src_sst[j]; i < src_sst[j + 1]; i++) sst_src[i] = j;
  // ---- decode: one device batch per run of SSTs sharing a codec, views in source order
  std::vector<View> views;
  std::vector<uint64_t> rows_per_sst;
  std::vector<Warn> wl;
  for (uint32_t i = 0; i < n_sst;) {
    uint32_t e = i;
    while (e < n_sst && codec[e] == codec[i]) e++;
    std::vector<Piece> pieces;
    std::vector<uint64_t> in_off{0};
    std::vector<uint32_t> sst_blocks{0};
    uint64_t base = 0;
    for (uint32_t j = i; j < e; j++) {
      const std::vector<uint64_t>& o = offs[j];
      if (o.size() > 1) {  // the data blocks are contiguous: [offs[0], FilterOffset)
        pieces.push_back({ssts + sst_off[j] + o[0], o.back() - o[0]});
        for (size_t b = 1; b < o.size(); b++) in_off.push_back(base + (o[b] - o[0]));
        base += o.back() - o[0];
      }
      sst_blocks.push_back(uint32_t(in_off.size() - 1));
    }
    mark("gather blocks (host)");
    if (in_off.size() > 1) {
      View v;
      int s = decode_group(ctx, codec[i], pieces, in_off, sst_blocks, i, sst_src, &v, &rows_per_sst, &wl);
      mark("decode + row views");
      if (s) return s;
      views.push_back(v);
    } else {
      rows_per_sst.insert(rows_per_sst.end(), e - i, 0);
    }
    i = e;
  }
  // ---- iter.MergeSort: source j = the rows of its SSTs, in precedence order
  std::vector<uint64_t> src_start(size_t(n_src) + 1, 0), sst_rows_before(n_sst, 0);
  for (uint32_t j = 0; j < n_src; j++) {
    uint64_t r = 0;
    for (uint32_t i = src_sst[j]; i < src_sst[j + 1]; i++) {
      sst_rows_before[i] = r;
      r += rows_per_sst[i];
    }
    src_start[j + 1] = src_start[j] + r;
  }
  View all;
  int s = SLATE_OK;
  if (!views.empty() && (s = concat_views(ctx, views, &all))) return s;
  views.clear();
  // the warnings in the order types.ErrWarn gets them: NewMergeSort merges each source's warnings
  // up to its first row (merge.go:33-44), then a source's remaining ones when it ends (:55-63), and
  // sources end in the order their last entries (key, source) leave the heap
  {
    std::vector<std::pair<uint32_t, uint64_t>> order;  // (source, rank of its end) for sources with rows
    std::vector<std::pair<std::vector<uint8_t>, uint32_t>> last;
    for (uint32_t j = 0; j < n_src && !wl.empty(); j++) {
      if (src_start[j + 1] == src_start[j]) continue;
      uint64_t ko[2];
      if ((s = d2h_small(ctx, ko, all.key_off->as<uint64_t>() + src_start[j + 1] - 1, 16))) return s;
      std::vector<uint8_t> key(ko[1] - ko[0]);
      if (!key.empty() && (s = d2h_small(ctx, key.data(), all.keys->as<uint8_t>() + ko[0], key.size()))) return s;
      last.push_back({std::move(key), j});
    }
    std::sort(last.begin(), last.end());
    std::vector<uint32_t> end_rank(n_src, 0);
    for (size_t r = 0; r < last.size(); r++) end_rank[last[r].second] = uint32_t(r);
    std::vector<const Warn*> init, later;
    for (const Warn& w : wl) {
      const bool first = src_start[w.w.src + 1] == src_start[w.w.src] || sst_rows_before[w.w.sst] + w.rows_before == 0;
      (first ? init : later).push_back(&w);
    }
    std::stable_sort(later.begin(), later.end(),
                     [&](const Warn* a, const Warn* b) { return end_rank[a->w.src] < end_rank[b->w.src]; });
    // ErrWarn.Merge drops a text it already holds (types/errors.go:41-52).  A row warning's text
    // depends only on its row index and status ("while decoding block.Offset[%d]: %s" with a fixed
    // row.go message), a block warning's names its SST, so repeats are (row, status) pairs
    uint32_t k = 0;
    std::set<std::pair<int32_t, int32_t>> row_texts;
    for (const auto* part : {&init, &later})
      for (const Warn* w : *part) {
        if (w->w.row >= 0 && !row_texts.insert({w->w.row, w->w.status}).second) continue;
        if (k < warn_cap) warns[k] = w->w;
        k++;
      }
    if (n_warn) *n_warn = k;
  }
  const int done = wl.empty() ? SLATE_OK : SLATE_E_WARNINGS;
  if (all.n == 0) return done;  // no entries: no output SST (executor.go opens a writer on the first entry)
  if (all.n >= 0xFFFFFFFFull) return SLATE_E_LIMIT;
  hipStream_t st = ctx->stream;
  DEV(d_idx, all.n * 4 + 16);
  DEV(d_misc, 64);
  DEV(d_ms, slate_merge_scratch_bytes(all.n, n_src) + 16);
  SLATE_HIP(hipMemsetAsync(d_misc->b.p, 0, 64, st));
  uint64_t* d_n = d_misc->as<uint64_t>();
  uint32_t* d_flags = reinterpret_cast<uint32_t*>(d_n + 1);
  {
    GpuSpan gs(ctx, st);
    s = slate_merge_sorted_device(ctx, n_src, all.keys->as<uint8_t>(), all.key_off->as<uint64_t>(), src_start.data(),
                                  d_idx->as<uint32_t>(), d_n, d_flags, d_ms->b.p);
  }
  if (s) return s;
  uint64_t hm[2] = {0, 0};
  if ((s = d2h_small(ctx, hm, d_n, 16))) return s;
  mark("concat + merge");
  if (uint32_t(hm[1]) & 1) return SLATE_E_MERGE_UNSORTED;
  const uint64_t m = hm[0];
  // ---- the merged entries, gathered in order
  DEV(okey_off, (m + 1) * 8);
  DEV(oval_off, (m + 1) * 8);
  DEV(otomb, m + 1);
  DEV(d_gs, kv_scratch_bytes(m) + 16);
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_gather_lengths(st, d_idx->as<uint32_t>(), m, all.key_off->as<uint64_t>(),
                                    all.val_off->as<uint64_t>(), all.tomb->as<uint8_t>(), okey_off->as<uint64_t>(),
                                    oval_off->as<uint64_t>(), otomb->as<uint8_t>(), d_gs->b.p));
  }
  std::vector<uint64_t> hko(m + 1), hvo(m + 1);
  if ((s = ctx_d2h(ctx, hko.data(), okey_off->b.p, (m + 1) * 8, st))) return s;
  if ((s = ctx_d2h(ctx, hvo.data(), oval_off->b.p, (m + 1) * 8, st))) return s;
  mark("gather: offsets D2H");
  DEV(okeys, hko[m] + 16);
  DEV(ovals, hvo[m] + 16);
  mark("gather: allocations");
  {
    GpuSpan gs(ctx, st);
    SLATE_HIP(launch_gather_copy(st, d_idx->as<uint32_t>(), m, all.keys->as<uint8_t>(),
                                 all.key_off->as<uint64_t>(), all.vals->as<uint8_t>(), all.val_off->as<uint64_t>(),
                                 okeys->as<uint8_t>(), okey_off->as<uint64_t>(), ovals->as<uint8_t>(),
                                 oval_off->as<uint64_t>()));
  }
  SLATE_HIP(hipStreamSynchronize(st));
  all = View{};
  mark("gather");
  // ---- output SSTs: a writer closes right after the entry that takes currentSize past MaxSSTSize
  std::vector<uint64_t> ends;
  {
    uint64_t size = 0, start = 0;
    for (uint64_t e = 0; e < m; e++) {
      size += (hko[e + 1] - hko[e]) + (hvo[e + 1] - hvo[e]);
      if (size > max_sst_size) {
        ends.push_back(e + 1);
        size = 0;
        start = e + 1;
      }
    }
    if (start < m) ends.push_back(m);
  }
  if (ends.size() > out_cap || (!ends.empty() && !out_tables)) {
    *n_out = uint32_t(ends.size());
    return SLATE_E_CAPACITY;  // *n_out > out_cap: the number needed
  }
  uint64_t start = 0;
  uint32_t made = 0;
  auto fail = [&](int code) {
    for (uint32_t k = 0; k < made; k++) slate_sst_table_free(out_tables[k]);
    *n_out = 0;
    return code;
  };
  for (uint64_t end : ends) {
    int bs = 0;
    slate_sst_builder* b = slate_sst_builder_new(ctx, out_cfg, &bs);
    if (!b) return fail(bs);
    // AddValue semantics (table_store.go:221-223): an empty value is a tombstone
    s = slate_sst_builder_add_batch_device(b, okeys->as<uint8_t>(), okey_off->as<uint64_t>() + start,
                                           ovals->as<uint8_t>(), oval_off->as<uint64_t>() + start, nullptr, end - start);
    slate_sst_table* t = nullptr;
    if (!s) s = slate_sst_builder_build(b, &t);
    slate_sst_builder_free(b);
    if (s) return fail(s);
    out_tables[made++] = t;
    start = end;
    mark("output SST build");
  }
  *n_out = made;
  return done;
}

int slate_compact(slate_ctx* ctx, const uint8_t* ssts, const uint64_t* sst_off, uint32_t n_sst, const uint32_t* src_sst,
                  uint32_t n_src, const slate_sst_config* out_cfg, uint64_t max_sst_size, slate_sst_table** out_tables,
                  uint32_t out_cap, uint32_t* n_out) {
  slate_compact_warning w{};
  uint32_t nw = 0;
  const int s = slate_compact_ex(ctx, ssts, sst_off, n_sst, src_sst, n_src, out_cfg, max_sst_size, out_tables, out_cap,
                                 n_out, &w, 1, &nw);
  if (s != SLATE_E_WARNINGS) return s;
  // a compaction that returned an error has no sorted run (startCompaction, executor.go:166-173)
  for (uint32_t k = 0; k < *n_out; k++) slate_sst_table_free(out_tables[k]);
  *n_out = 0;
  return w.status;
}

}  // extern "C"
