"""executeCompaction (slatedb/compaction/executor.go:92-151) on the GPU, for the part of it that is
the SST codec path: the input SSTs' data blocks are decoded in one device batch
(block.Decode per block, as sstable.Iterator does it, internal/sstable/iterator.go:92-118), turned
into (full key, value | tombstone) rows (block.Iterator, block/iterator.go:84-107), merged with
first-iterator precedence (iter.MergeSort, internal/iter/merge.go:12-111), gathered in merged
order, and re-encoded by the SST builder (EncodedSSTableWriter.Add/Close, table_store.go:221-266),
cutting a new output SST whenever the running key+value size passes MaxSSTSize
(executor.go:124-139).  Scheduling, manifests and object storage stay with the caller.

Two drivers of the same chain, both over memory the library owns (slate_devbuf; no torch):
  compact()        one C-ABI call, slate_compact (csrc/api_compact.cpp) -- what a Go
                   executeCompaction calls through cgo;
  compact_steps()  the chain step by step through the device-resident entry points (plan ->
                   decode -> rows -> merge -> gather -> add_batch_device -> build), each on
                   slate_devbuf addresses, as a cgo caller composing its own pipeline would.

`sources` are the merge's iterators in precedence order (executor.go:55-90: L0 SSTs, then sorted
runs); each is a list of encoded SSTs read in order (a sorted run's SST list, or one L0 SST)."""
from __future__ import annotations

import time

import numpy as np

from . import (NONE, Context, DevBuf, SlateError, SstBuilder, _check, decode_scratch_bytes, devbuf_from, lib,
               read_info, E_MERGE_UNSORTED, META_DTYPE)
from . import compact as _compact_c


def compact(ctx: Context, sources: list[list[bytes]], max_sst_size: int, block_size: int = 4096,
            min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE) -> list[bytes]:
    """Returns the encoded output SSTs of the compaction, in order (slate_compact)."""
    return _compact_c(ctx, sources, max_sst_size, block_size, min_filter_keys, filter_bits_per_key, codec)


def _blocks_of(ctx: Context, sst: bytes):
    """Data-block offsets of one SST (ReadInfo + ReadIndex + getBlockRange, decode.go:25-103):
    block i = sst[offs[i]:offs[i+1]], the last one ending at FilterOffset."""
    st, info, _ = read_info(sst)
    _check(st, "read_info")
    st, index = ctx.decode_index(sst[info.index_offset:info.index_offset + info.index_len], info.codec)
    _check(st, "decode_index")
    offs = np.append(index.block_offsets(), np.uint64(info.filter_offset))
    return info.codec, offs


def _index_pool(ctx: Context, n: int) -> list[Context]:
    """Extra contexts (one HIP stream each) so the input SSTs' indexes decode concurrently.  The
    library is reentrant per context (one slate_ctx per goroutine in a Go port), and a context is
    never used by two threads at once: each worker owns one context for its whole slice."""
    pool = getattr(ctx, "_index_pool", None)
    if pool is None:
        pool = ctx._index_pool = []
    while len(pool) < n:
        pool.append(Context(ctx.device))
    return pool[:n]


def _all_blocks(ctx: Context, ssts: list[bytes]):
    if len(ssts) <= 1:
        return [_blocks_of(ctx, s) for s in ssts]
    from concurrent.futures import ThreadPoolExecutor
    w = min(8, len(ssts))
    pool = _index_pool(ctx, w)
    bounds = [len(ssts) * j // w for j in range(w + 1)]

    def run(j):
        return [_blocks_of(pool[j], ssts[i]) for i in range(bounds[j], bounds[j + 1])]

    with ThreadPoolExecutor(w) as ex:
        return [r for part in ex.map(run, range(w)) for r in part]


def _mark(ctx, prof, label):
    if prof is not None:
        ctx.synchronize()
        prof.append((label, time.perf_counter()))


class KvView:
    """Entries on the device: keys / values back to back (DevBufs), n + 1 u64 offsets into each,
    one tombstone byte per entry."""

    def __init__(self, keys: DevBuf, key_off: DevBuf, vals: DevBuf, val_off: DevBuf, tomb: DevBuf, n: int):
        self.keys, self.key_off, self.vals, self.val_off, self.tomb, self.n = keys, key_off, vals, val_off, tomb, n


def _empty_view(ctx) -> KvView:
    z = np.zeros(1, np.uint64)
    return KvView(DevBuf(ctx, 16), devbuf_from(ctx, z), DevBuf(ctx, 16), devbuf_from(ctx, z), DevBuf(ctx, 16), 0)


def decode_rows_kv(ctx: Context, sources: list[list[bytes]], prof: list | None = None):
    """Decode every data block of every input SST on the GPU -> (KvView, src_start), src_start =
    per-source row ranges.  Each SST carries its own codec (sstable.Info.CompressionCodec):
    consecutive SSTs that share one are decoded as one batch, and the views are concatenated."""
    _mark(ctx, prof, "start")
    flat = [sst for run in sources for sst in run]
    located = _all_blocks(ctx, flat)
    _mark(ctx, prof, "index")
    groups, i = [], 0
    while i < len(flat):
        j = i
        while j < len(flat) and located[j][0] == located[i][0]:
            j += 1
        groups.append((located[i][0], list(range(i, j))))
        i = j
    views, rows_per_sst = [], []
    for codec, idx in groups:
        v, per = _decode_group(ctx, codec, [(flat[k], located[k][1]) for k in idx], prof)
        views.append(v)
        rows_per_sst += per
    src_sst = np.cumsum([0] + [len(run) for run in sources])
    row_cum = np.concatenate([[0], np.cumsum(np.asarray(rows_per_sst, np.uint64))]).astype(np.uint64)
    src_start = row_cum[src_sst].astype(np.uint64) if len(flat) else np.zeros(len(sources) + 1, np.uint64)
    view = _concat(ctx, [v for v in views if v.n]) if views else _empty_view(ctx)
    assert int(src_start[-1]) == view.n
    _mark(ctx, prof, "rows_kv")
    return view, src_start


def _concat(ctx: Context, views: list[KvView]) -> KvView:
    """Views back to back: bytes copied device to device, offsets rebased (on the host: small)."""
    if not views:
        return _empty_view(ctx)
    if len(views) == 1:
        return views[0]
    kb = [v.key_off.u64(v.n) for v in views]
    vb = [v.val_off.u64(v.n) for v in views]
    n = sum(v.n for v in views)
    keys, vals, tomb = DevBuf(ctx, sum(kb) + 16), DevBuf(ctx, sum(vb) + 16), DevBuf(ctx, n + 16)
    ko, vo = [], []
    a = b = t = 0
    for v, k, w in zip(views, kb, vb):
        _check(lib().slate_devbuf_copy(ctx.handle, keys.handle, a, v.keys.handle, 0, k), "devbuf_copy")
        _check(lib().slate_devbuf_copy(ctx.handle, vals.handle, b, v.vals.handle, 0, w), "devbuf_copy")
        _check(lib().slate_devbuf_copy(ctx.handle, tomb.handle, t, v.tomb.handle, 0, v.n), "devbuf_copy")
        ko.append(v.key_off.download(8 * v.n, 0, np.uint64) + np.uint64(a))
        vo.append(v.val_off.download(8 * v.n, 0, np.uint64) + np.uint64(b))
        a, b, t = a + k, b + w, t + v.n
    ko.append(np.array([a], np.uint64))
    vo.append(np.array([b], np.uint64))
    return KvView(keys, devbuf_from(ctx, np.concatenate(ko)), vals, devbuf_from(ctx, np.concatenate(vo)), tomb, n)


def _decode_group(ctx: Context, codec: int, ssts: list, prof):
    """One device batch over the data blocks of SSTs that share a codec -> (KvView, rows per SST)."""
    pieces, offs_parts, sst_blocks = [], [np.zeros(1, np.uint64)], [0]
    base, nblk = 0, 0
    for sst, offs in ssts:
        if len(offs) > 1:  # the data blocks are contiguous: [offs[0], FilterOffset)
            lo, hi = int(offs[0]), int(offs[-1])
            pieces.append(np.frombuffer(sst, np.uint8, hi - lo, lo))
            offs_parts.append(offs[1:] - np.uint64(lo) + np.uint64(base))
            base += hi - lo
            nblk += len(offs) - 1
        sst_blocks.append(nblk)
    in_off = np.concatenate(offs_parts)
    n = len(in_off) - 1
    if n == 0:
        return _empty_view(ctx), [0] * len(ssts)
    d_in = devbuf_from(ctx, np.concatenate(pieces))
    d_in_off = devbuf_from(ctx, in_off)
    _mark(ctx, prof, "h2d")
    d_out_off, d_row_base = DevBuf(ctx, 8 * (n + 1)), DevBuf(ctx, 8 * (n + 1))
    d_scr = DevBuf(ctx, decode_scratch_bytes(n) + 64)
    ctx.decode_plan_device(codec, d_in.ptr, d_in_off.ptr, n, d_out_off.ptr, d_row_base.ptr, d_scr.ptr)
    total_out, slots = d_out_off.u64(n), d_row_base.u64(n)
    d_out, d_meta = DevBuf(ctx, total_out + 16), DevBuf(ctx, 16 * n)
    d_rows = DevBuf(ctx, 16 * max(slots, 1))
    ctx.decode_device(codec, d_in.ptr, d_in_off.ptr, n, d_out.ptr, d_out_off.ptr, d_meta.ptr, d_rows.ptr,
                      d_row_base.ptr)
    _mark(ctx, prof, "decode")
    # rows -> KV view
    d_key_off, d_val_off = DevBuf(ctx, 8 * (slots + 1)), DevBuf(ctx, 8 * (slots + 1))
    d_tomb = DevBuf(ctx, max(slots, 1))
    d_nkv, d_flags = DevBuf(ctx, 8).memset(0), DevBuf(ctx, 4).memset(0)
    d_kvs = DevBuf(ctx, lib().slate_kv_scratch_bytes(slots))
    _check(lib().slate_rows_kv_lengths_device(ctx.handle, n, d_row_base.ptr, d_meta.ptr, d_rows.ptr, slots,
                                              d_key_off.ptr, d_val_off.ptr, d_tomb.ptr, d_nkv.ptr, d_flags.ptr,
                                              d_kvs.ptr), "slate_rows_kv_lengths_device")
    # Every block's status is checked, whatever the row-slot flags say: a block that fails before
    # its decoded length is known owns no row slot (sstable.Iterator stops on the error and
    # executeCompaction returns it, iterator.go:62-68, executor.go:107-150).
    meta = d_meta.download(16 * n).view(META_DTYPE)
    bad = np.nonzero(meta["status"] != 0)[0]
    if len(bad):
        raise SlateError(int(meta["status"][bad[0]]), f"compaction input block {int(bad[0])} decode")
    if (meta["flags"] & 1).any():  # SLATE_BLKF_ROWS_TRUNCATED: more offsets than row slots
        raise SlateError(103, "compaction input block has more rows than row slots")
    if int(d_flags.download(4, 0, np.uint32)[0]) & 2:
        raise SlateError(102, "compaction input row decode")
    n_kv = d_nkv.u64(0)
    kb, vb = d_key_off.u64(slots), d_val_off.u64(slots)
    d_keys, d_vals = DevBuf(ctx, max(kb, 1)), DevBuf(ctx, max(vb, 1))
    _check(lib().slate_rows_kv_copy_device(ctx.handle, n, d_out.ptr, d_out_off.ptr, d_row_base.ptr, d_rows.ptr, slots,
                                           d_nkv.ptr, d_kvs.ptr, d_key_off.ptr, d_keys.ptr, d_val_off.ptr, d_vals.ptr),
           "slate_rows_kv_copy_device")
    rows_per_block = np.concatenate([[0], np.cumsum(meta["n_rows"].astype(np.uint64))])
    per_sst = np.diff(rows_per_block[np.array(sst_blocks)].astype(np.int64)).tolist()
    assert sum(per_sst) == n_kv
    ctx.synchronize()
    return KvView(d_keys, d_key_off, d_vals, d_val_off, d_tomb, n_kv), per_sst


def merge_kv(ctx: Context, view: KvView, src_start: np.ndarray, prof: list | None = None) -> KvView:
    """iter.MergeSort over the sources of a KV view, gathered in merged order (a device view)."""
    n_kv, k = view.n, len(src_start) - 1
    d_idx = DevBuf(ctx, 4 * max(n_kv, 1))
    d_n, d_flags = DevBuf(ctx, 8).memset(0), DevBuf(ctx, 4).memset(0)
    d_ms = DevBuf(ctx, lib().slate_merge_scratch_bytes(n_kv, k))
    ctx.merge_device(view.keys.ptr, view.key_off.ptr, src_start, d_idx.ptr, d_n.ptr, d_flags.ptr, d_ms.ptr)
    if int(d_flags.download(4, 0, np.uint32)[0]) & 1:
        raise SlateError(E_MERGE_UNSORTED, "compaction merge")
    _mark(ctx, prof, "merge")
    m = d_n.u64(0)
    d_okey_off, d_oval_off = DevBuf(ctx, 8 * (m + 1)), DevBuf(ctx, 8 * (m + 1))
    d_otomb = DevBuf(ctx, max(m, 1))
    d_gs = DevBuf(ctx, lib().slate_kv_scratch_bytes(m))
    _check(lib().slate_kv_gather_lengths_device(ctx.handle, d_idx.ptr, m, view.key_off.ptr, view.val_off.ptr,
                                                view.tomb.ptr, d_okey_off.ptr, d_oval_off.ptr, d_otomb.ptr, d_gs.ptr),
           "slate_kv_gather_lengths_device")
    kb, vb = d_okey_off.u64(m), d_oval_off.u64(m)
    d_okeys, d_ovals = DevBuf(ctx, max(kb, 1)), DevBuf(ctx, max(vb, 1))
    _check(lib().slate_kv_gather_copy_device(ctx.handle, d_idx.ptr, m, view.keys.ptr, view.key_off.ptr, view.vals.ptr,
                                             view.val_off.ptr, d_okeys.ptr, d_okey_off.ptr, d_ovals.ptr,
                                             d_oval_off.ptr), "slate_kv_gather_copy_device")
    ctx.synchronize()
    _mark(ctx, prof, "gather")
    return KvView(d_okeys, d_okey_off, d_ovals, d_oval_off, d_otomb, m)


def split_points(key_off: np.ndarray, val_off: np.ndarray, max_sst_size: int) -> list[int]:
    """executor.go:119-139: currentSize += len(key) + len(value); a writer closes right after the
    entry that takes currentSize past MaxSSTSize.  Returns the entry index where each output SST ends."""
    n = len(key_off) - 1
    size = np.cumsum((np.diff(key_off.astype(np.int64)) + np.diff(val_off.astype(np.int64))))
    ends, start, base = [], 0, 0
    while start < n:
        j = int(np.searchsorted(size, base + max_sst_size, side="right"))  # first entry with size > max
        end = min(j + 1, n)
        ends.append(end)
        base = int(size[end - 1])
        start = end
    return ends


def compact_steps(ctx: Context, sources: list[list[bytes]], max_sst_size: int, block_size: int = 4096,
                  min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE,
                  prof: list | None = None) -> list[bytes]:
    """The same compaction, step by step through the device-resident entry points on slate_devbufs."""
    view, src_start = decode_rows_kv(ctx, sources, prof)
    merged = merge_kv(ctx, view, src_start, prof)
    del view
    m = merged.n
    # the merged KVs stay on the device: only the offsets come back, for the output split
    h_key_off = merged.key_off.download(8 * (m + 1), 0, np.uint64)
    h_val_off = merged.val_off.download(8 * (m + 1), 0, np.uint64)
    out, start = [], 0
    for end in split_points(h_key_off, h_val_off, max_sst_size):
        b = SstBuilder(ctx, block_size, min_filter_keys, filter_bits_per_key, codec)
        # AddValue: empty value => tombstone (table_store.go:221-223)
        _check(b.add_batch_device(merged.keys.ptr, merged.key_off.at(8 * start), merged.vals.ptr,
                                  merged.val_off.at(8 * start), end - start), "add_batch_device")
        out.append(b.build().encode())
        start = end
    _mark(ctx, prof, "build")
    return out
