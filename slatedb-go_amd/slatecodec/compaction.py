"""executeCompaction (slatedb/compaction/executor.go:92-151) on the GPU, for the part of it that is
the SST codec path: the input SSTs' data blocks are decoded in one device batch
(block.Decode per block, as sstable.Iterator does it, internal/sstable/iterator.go:92-118), turned
into (full key, value | tombstone) rows (block.Iterator, block/iterator.go:84-107), merged with
first-iterator precedence (iter.MergeSort, internal/iter/merge.go:12-111), gathered in merged
order, and re-encoded by the SST builder (EncodedSSTableWriter.Add/Close, table_store.go:221-266),
cutting a new output SST whenever the running key+value size passes MaxSSTSize
(executor.go:124-139).  Device memory and streams come from torch (plumbing); every byte
operation runs in the HIP library through its C ABI.  Scheduling, manifests and object storage
stay with the caller.

`sources` are the merge's iterators in precedence order (executor.go:55-90: L0 SSTs, then sorted
runs); each is a list of encoded SSTs read in order (a sorted run's SST list, or one L0 SST)."""
from __future__ import annotations

import time

import numpy as np

from . import (NONE, Context, SlateError, SstBuilder, _check, decode_scratch_bytes, lib, read_info, E_MERGE_UNSORTED,
               META_DTYPE)


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
    """Extra contexts (one HIP stream each) so the input SSTs' indexes decode concurrently: each
    index is one serial Snappy stream that occupies a single wavefront (snappy_stream.hip).  The
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
    # w contiguous slices, one per worker and context (ctypes calls release the GIL)
    bounds = [len(ssts) * j // w for j in range(w + 1)]

    def run(j):
        return [_blocks_of(pool[j], ssts[i]) for i in range(bounds[j], bounds[j + 1])]

    with ThreadPoolExecutor(w) as ex:
        return [r for part in ex.map(run, range(w)) for r in part]


def _mark(prof, label):
    if prof is not None:
        import torch
        torch.cuda.synchronize()
        prof.append((label, time.perf_counter()))


def decode_rows_kv(ctx: Context, sources: list[list[bytes]], device, prof: list | None = None):
    """Decode every data block of every input SST on the GPU and return the rows as a device KV view:
    (keys, key_off, vals, val_off, tomb, n_kv, src_start) with src_start = per-source row ranges.
    Each SST carries its own codec (sstable.Info.CompressionCodec): consecutive SSTs that share one
    are decoded as one batch, and the batches' views are concatenated in source order."""
    import torch
    _mark(prof, "start")
    flat = [sst for run in sources for sst in run]
    located = _all_blocks(ctx, flat)
    _mark(prof, "index")
    groups, i = [], 0
    while i < len(flat):
        j = i
        while j < len(flat) and located[j][0] == located[i][0]:
            j += 1
        groups.append((located[i][0], list(range(i, j))))
        i = j
    views = [_decode_group(ctx, codec, [(flat[k], located[k][1]) for k in idx], device, prof)
             for codec, idx in groups]
    rows_per_sst = [r for v in views for r in v[6]]
    src_sst = np.cumsum([0] + [len(run) for run in sources])
    row_cum = np.concatenate([[0], np.cumsum(np.asarray(rows_per_sst, np.uint64))]).astype(np.uint64)
    src_start = row_cum[src_sst].astype(np.uint64) if len(flat) else np.zeros(len(sources) + 1, np.uint64)
    if len(views) == 1:
        v = views[0]
        out = v[:6] + (src_start,)
    elif not views:
        z = torch.zeros(1, dtype=torch.int64, device=device)
        u8 = torch.zeros(1, dtype=torch.uint8, device=device)
        out = (u8, z, u8, z, u8, 0, src_start)
    else:
        keys, vals, koffs, voffs, tombs, kb, vb, n_kv = [], [], [], [], [], 0, 0, 0
        for v in views:
            d_keys, d_key_off, d_vals, d_val_off, d_tomb, m = v[:6]
            k_end, v_end = int(d_key_off[m].item()), int(d_val_off[m].item())
            keys.append(d_keys[:k_end])
            vals.append(d_vals[:v_end])
            koffs.append(d_key_off[:m] + kb)
            voffs.append(d_val_off[:m] + vb)
            tombs.append(d_tomb[:m])
            kb, vb, n_kv = kb + k_end, vb + v_end, n_kv + m
        one = torch.ones(1, dtype=torch.int64, device=device)
        out = (torch.cat(keys + [torch.zeros(1, dtype=torch.uint8, device=device)]),
               torch.cat(koffs + [one * kb]), torch.cat(vals + [torch.zeros(1, dtype=torch.uint8, device=device)]),
               torch.cat(voffs + [one * vb]), torch.cat(tombs + [torch.zeros(1, dtype=torch.uint8, device=device)]),
               n_kv, src_start)
    assert int(src_start[-1]) == out[5]
    _mark(prof, "rows_kv")
    return out


def _decode_group(ctx: Context, codec: int, ssts: list, device, prof):
    """One device batch over the data blocks of SSTs that share a codec -> (keys, key_off, vals,
    val_off, tomb, n_kv, rows per SST)."""
    import torch
    pieces, offs_parts, sst_blocks = [], [np.zeros(1, np.uint64)], [0]
    base, nblk = 0, 0  # encoded bytes and blocks gathered so far
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
        z = torch.zeros(1, dtype=torch.int64, device=device)
        u8 = torch.zeros(1, dtype=torch.uint8, device=device)
        return u8, z, u8, z, u8, 0, [0] * len(ssts)
    blob = np.concatenate(pieces)
    _mark(prof, "gather_blocks")
    d_in = torch.from_numpy(blob).to(device)
    d_in_off = torch.from_numpy(in_off.view(np.int64)).to(device)
    _mark(prof, "h2d")
    d_out_off = torch.empty(n + 1, dtype=torch.int64, device=device)
    d_row_base = torch.empty(n + 1, dtype=torch.int64, device=device)
    d_scr = torch.empty(decode_scratch_bytes(n) + 64, dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    ctx.decode_plan_device(codec, d_in.data_ptr(), d_in_off.data_ptr(), n, d_out_off.data_ptr(),
                           d_row_base.data_ptr(), d_scr.data_ptr())
    ctx.synchronize()
    total_out = int(d_out_off[n].item())
    slots = int(d_row_base[n].item())
    d_out = torch.empty(total_out + 16, dtype=torch.uint8, device=device)
    d_meta = torch.empty(n * 16, dtype=torch.uint8, device=device)
    d_rows = torch.empty(max(slots, 1) * 16, dtype=torch.uint8, device=device)
    ctx.decode_device(codec, d_in.data_ptr(), d_in_off.data_ptr(), n, d_out.data_ptr(), d_out_off.data_ptr(),
                      d_meta.data_ptr(), d_rows.data_ptr(), d_row_base.data_ptr())
    _mark(prof, "decode")
    # rows -> KV view
    d_key_off = torch.empty(slots + 1, dtype=torch.int64, device=device)
    d_val_off = torch.empty(slots + 1, dtype=torch.int64, device=device)
    d_tomb = torch.empty(max(slots, 1), dtype=torch.uint8, device=device)
    d_nkv = torch.zeros(1, dtype=torch.int64, device=device)
    d_flags = torch.zeros(1, dtype=torch.int32, device=device)
    d_kvs = torch.empty(lib().slate_kv_scratch_bytes(slots), dtype=torch.uint8, device=device)
    _check(lib().slate_rows_kv_lengths_device(ctx.handle, n, d_row_base.data_ptr(), d_meta.data_ptr(),
                                              d_rows.data_ptr(), slots, d_key_off.data_ptr(), d_val_off.data_ptr(),
                                              d_tomb.data_ptr(), d_nkv.data_ptr(), d_flags.data_ptr(),
                                              d_kvs.data_ptr()), "slate_rows_kv_lengths_device")
    ctx.synchronize()
    # Every block's status is checked, whatever the row-slot flags say: a block that fails before
    # its decoded length is known owns no row slot (sstable.Iterator stops on the error and
    # executeCompaction returns it, iterator.go:62-68, executor.go:107-150).
    meta = np.frombuffer(d_meta.cpu().numpy().tobytes(), dtype=META_DTYPE)
    bad = np.nonzero(meta["status"] != 0)[0]
    if len(bad):
        raise SlateError(int(meta["status"][bad[0]]), f"compaction input block {int(bad[0])} decode")
    if (meta["flags"] & 1).any():  # SLATE_BLKF_ROWS_TRUNCATED: more offsets than row slots
        raise SlateError(103, "compaction input block has more rows than row slots")
    if int(d_flags.item()) & 2:
        raise SlateError(102, "compaction input row decode")
    n_kv = int(d_nkv.item())
    kb, vb = int(d_key_off[slots].item()), int(d_val_off[slots].item())
    d_keys = torch.empty(max(kb, 1), dtype=torch.uint8, device=device)
    d_vals = torch.empty(max(vb, 1), dtype=torch.uint8, device=device)
    _check(lib().slate_rows_kv_copy_device(ctx.handle, n, d_out.data_ptr(), d_out_off.data_ptr(),
                                           d_row_base.data_ptr(), d_rows.data_ptr(), slots, d_nkv.data_ptr(),
                                           d_kvs.data_ptr(), d_key_off.data_ptr(), d_keys.data_ptr(),
                                           d_val_off.data_ptr(), d_vals.data_ptr()), "slate_rows_kv_copy_device")
    # rows per SST from the blocks' row counts
    rows_per_block = np.concatenate([[0], np.cumsum(meta["n_rows"].astype(np.uint64))])
    per_sst = np.diff(rows_per_block[np.array(sst_blocks)].astype(np.int64)).tolist()
    assert sum(per_sst) == n_kv
    ctx.synchronize()
    return d_keys, d_key_off, d_vals, d_val_off, d_tomb, n_kv, per_sst


def merge_kv(ctx: Context, view, device, prof: list | None = None):
    """iter.MergeSort over the sources of a KV view, gathered in merged order (device arrays)."""
    import torch
    d_keys, d_key_off, d_vals, d_val_off, d_tomb, n_kv, src_start = view
    k = len(src_start) - 1
    d_idx = torch.empty(max(n_kv, 1), dtype=torch.int32, device=device)
    d_n = torch.zeros(1, dtype=torch.int64, device=device)
    d_flags = torch.zeros(1, dtype=torch.int32, device=device)
    d_ms = torch.empty(lib().slate_merge_scratch_bytes(n_kv, k), dtype=torch.uint8, device=device)
    ctx.merge_device(d_keys.data_ptr(), d_key_off.data_ptr(), src_start, d_idx.data_ptr(), d_n.data_ptr(),
                     d_flags.data_ptr(), d_ms.data_ptr())
    if int(d_flags.item()) & 1:
        raise SlateError(E_MERGE_UNSORTED, "compaction merge")
    _mark(prof, "merge")
    m = int(d_n.item())
    d_okey_off = torch.empty(m + 1, dtype=torch.int64, device=device)
    d_oval_off = torch.empty(m + 1, dtype=torch.int64, device=device)
    d_otomb = torch.empty(max(m, 1), dtype=torch.uint8, device=device)
    d_gs = torch.empty(lib().slate_kv_scratch_bytes(m), dtype=torch.uint8, device=device)
    _check(lib().slate_kv_gather_lengths_device(ctx.handle, d_idx.data_ptr(), m, d_key_off.data_ptr(),
                                                d_val_off.data_ptr(), d_tomb.data_ptr(), d_okey_off.data_ptr(),
                                                d_oval_off.data_ptr(), d_otomb.data_ptr(), d_gs.data_ptr()),
           "slate_kv_gather_lengths_device")
    ctx.synchronize()
    kb, vb = int(d_okey_off[m].item()), int(d_oval_off[m].item())
    d_okeys = torch.empty(max(kb, 1), dtype=torch.uint8, device=device)
    d_ovals = torch.empty(max(vb, 1), dtype=torch.uint8, device=device)
    _check(lib().slate_kv_gather_copy_device(ctx.handle, d_idx.data_ptr(), m, d_keys.data_ptr(), d_key_off.data_ptr(),
                                             d_vals.data_ptr(), d_val_off.data_ptr(), d_okeys.data_ptr(),
                                             d_okey_off.data_ptr(), d_ovals.data_ptr(), d_oval_off.data_ptr()),
           "slate_kv_gather_copy_device")
    ctx.synchronize()
    _mark(prof, "gather")
    return d_okeys, d_okey_off, d_ovals, d_oval_off, d_otomb, m


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


def compact(ctx: Context, sources: list[list[bytes]], max_sst_size: int, block_size: int = 4096,
            min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE, device=None) -> list[bytes]:
    """Returns the encoded output SSTs of the compaction, in order."""
    import torch
    device = device or torch.device("cuda", torch.cuda.current_device())
    view = decode_rows_kv(ctx, sources, device)
    keys, key_off, vals, val_off, tomb, m = merge_kv(ctx, view, device)
    # the merged KVs stay on the device: only the offsets come back, for the output split
    h_key_off = key_off.cpu().numpy().view(np.uint64)[: m + 1]
    h_val_off = val_off.cpu().numpy().view(np.uint64)[: m + 1]
    out, start = [], 0
    for end in split_points(h_key_off, h_val_off, max_sst_size):
        b = SstBuilder(ctx, block_size, min_filter_keys, filter_bits_per_key, codec)
        # AddValue: empty value => tombstone (table_store.go:221-223)
        _check(b.add_batch_device(keys.data_ptr(), key_off.data_ptr() + 8 * start, vals.data_ptr(),
                                  val_off.data_ptr() + 8 * start, end - start), "add_batch_device")
        out.append(b.build().encode())
        start = end
    return out
