"""Compaction fixtures and the oracle's executeCompaction (test infrastructure): input SSTs are
built with the oracle's sstable.Builder; the expected output SSTs come from the oracle restated
end to end -- ReadInfo/ReadIndex/block.Decode per block (decode.go:25-149), block.Iterator full
keys (block/iterator.go:84-107, row.go:72-79), iter.MergeSort (merge.go:12-111), and the
executeCompaction writer loop with its MaxSSTSize cut (slatedb/compaction/executor.go:92-151)
feeding EncodedSSTableWriter.Add = Builder.AddValue (store/table_store.go:221-223)."""
import random

from oracle import binding as ob


def build_sst(kvs: list[tuple[bytes, bytes | None]], codec: int = ob.NONE, block_size: int = 4096) -> bytes:
    b = ob.SstBuilder(block_size, 0, 10, codec)
    for k, v in kvs:
        assert b.add(k, v) == 0
    assert b.build() == 0
    return b.encode_table()


def sst_rows(sst: bytes) -> list[tuple[bytes, bytes | None]]:
    """sstable.Iterator over every row of one SST (oracle)."""
    st, info = ob.sst_read_info(sst)
    assert st == 0, st
    codec = info["codec"]
    st, metas = ob.decode_index(sst[info["index_offset"]:info["index_offset"] + info["index_len"]], codec)
    assert st == 0, st
    offs = [o for o, _ in metas] + [info["filter_offset"]]
    out = []
    for a, b in zip(offs, offs[1:]):
        m, data, rows = ob.block_decode(sst[a:b], codec)
        assert m["status"] == 0, m
        fk = b""
        for i, r in enumerate(rows):
            o, sl = int(r["row_off"]), int(r["key_suffix_len"])
            sfx = data[o + 4:o + 4 + sl]
            key = sfx if i == 0 else fk[:int(r["key_prefix_len"])] + sfx
            if i == 0:
                fk = key
            if r["flags"] & 1:
                out.append((key, None))
            else:
                vs = o + 4 + sl + int(r["meta_len"])
                out.append((key, data[vs:vs + int(r["value_len"])]))
    return out


def sst_rows_go(sst: bytes):
    """sstable.Iterator over one SST with Go's behaviour on corrupt input (oracle): a block that fails
    block.Decode ends the SST (iterator.go:59-68), a row that fails v0RowCodec.Decode ends its block
    (block/iterator.go:92-96).  -> (rows, warnings): warning = (block, row or -1, status, block_len,
    rows returned before it)."""
    st, info = ob.sst_read_info(sst)
    assert st == 0, st
    codec = info["codec"]
    st, metas = ob.decode_index(sst[info["index_offset"]:info["index_offset"] + info["index_len"]], codec)
    assert st == 0, st
    offs = [o for o, _ in metas] + [info["filter_offset"]]
    out, warns = [], []
    for bi, (a, b) in enumerate(zip(offs, offs[1:])):
        m, data, rows = ob.block_decode(sst[a:b], codec)
        if m["status"] != 0:
            warns.append((bi, -1, int(m["status"]), b - a, len(out)))
            break
        fk = b""
        for i, r in enumerate(rows):
            if int(r["status"]) != 0:
                warns.append((bi, i, int(r["status"]), b - a, len(out)))
                break
            o, sl = int(r["row_off"]), int(r["key_suffix_len"])
            sfx = data[o + 4:o + 4 + sl]
            key = sfx if i == 0 else fk[:int(r["key_prefix_len"])] + sfx
            if i == 0:
                fk = key
            if r["flags"] & 1:
                out.append((key, None))
            else:
                vs = o + 4 + sl + int(r["meta_len"])
                out.append((key, data[vs:vs + int(r["value_len"])]))
    return out, warns


def oracle_compact_go(sources: list[list[bytes]], max_sst_size: int, codec: int = ob.NONE, block_size: int = 4096):
    """executeCompaction with corrupt inputs (oracle): the rows Go's iterators still return, merged and
    written as oracle_compact does, and the warnings in the order types.ErrWarn receives them --
    NewMergeSort merges each source's warnings up to its first row, a source's remaining ones when
    it ends, sources ending in (last key, source) order (merge.go:33-63).
    -> (outputs, [(src, sst, block, row, status, block_len)])."""
    iters, early, late, last = [], [], {}, []
    k = 0
    for j, run in enumerate(sources):
        rows = []
        for sst in run:
            r, w = sst_rows_go(sst)
            for (blk, row, status, blen, before) in w:
                rec = (j, k, blk, row, status, blen)
                (early if len(rows) + before == 0 else late.setdefault(j, [])).append(rec)
            rows += r
            k += 1
        iters.append(rows)
        if rows:
            last.append((rows[-1][0], j))
    warns = list(early)
    for _, j in sorted(last):
        warns += late.get(j, [])
    # ErrWarn.Merge keeps a text once (types/errors.go:41-52): a row warning's text is its row index
    # and its status, a block warning's names its SST
    seen, kept = set(), []
    for w in warns:
        key = ("row", w[3], w[4]) if w[3] >= 0 else ("blk", w[1], w[2])
        if key not in seen:
            seen.add(key)
            kept.append(w)
    warns = kept
    flat = [kv for it in iters for kv in it]
    merged = [flat[i] for i in ob.merge_sort([[key for key, _ in it] for it in iters])]
    return _write_outputs(merged, max_sst_size, codec, block_size), warns


def _write_outputs(merged, max_sst_size, codec, block_size):
    out, size = [], 0
    w = ob.SstBuilder(block_size, 0, 10, codec)
    for k, v in merged:
        assert w.add_value(k, v or b"") == 0  # EncodedSSTableWriter.Add -> AddValue
        size += len(k) + (len(v) if v is not None else 0)
        if size > max_sst_size:
            size = 0
            assert w.build() == 0
            out.append(w.encode_table())
            w = ob.SstBuilder(block_size, 0, 10, codec)
    if size > 0:
        assert w.build() == 0
        out.append(w.encode_table())
    return out


def oracle_compact(sources: list[list[bytes]], max_sst_size: int, codec: int = ob.NONE,
                   block_size: int = 4096) -> list[bytes]:
    iters = [[kv for sst in run for kv in sst_rows(sst)] for run in sources]
    flat = [kv for it in iters for kv in it]
    merged = [flat[i] for i in ob.merge_sort([[k for k, _ in it] for it in iters])]
    return _write_outputs(merged, max_sst_size, codec, block_size)


def random_sources(rng: random.Random, n_sources: int, n_keys: int, space: int, codec: int = ob.NONE,
                   tomb: float = 0.05, run_ssts: int = 1, key_fmt="k%015d"):
    """n_sources sorted runs (each of run_ssts SSTs over consecutive key ranges) drawn from a
    shared key space, values of random length (0..120), some tombstones."""
    return [[build_sst(part, codec) for part in run]
            for run in random_kv_runs(rng, n_sources, n_keys, space, tomb, run_ssts, key_fmt)]


def random_kv_runs(rng: random.Random, n_sources: int, n_keys: int, space: int, tomb: float = 0.05,
                   run_ssts: int = 1, key_fmt="k%015d"):
    """random_sources' KVs before encoding: per source, its SSTs' sorted (key, value|None) lists."""
    srcs = []
    for _ in range(n_sources):
        ids = sorted(rng.sample(range(space), n_keys))
        kvs = []
        for i in ids:
            k = key_fmt(i) if callable(key_fmt) else (key_fmt % i).encode()
            if rng.random() < tomb:
                kvs.append((k, None))
            else:
                kvs.append((k, rng.randbytes(rng.randint(1, 120))))
        kvs.sort(key=lambda kv: kv[0])
        step = max(1, (len(kvs) + run_ssts - 1) // run_ssts)
        srcs.append([kvs[j:j + step] for j in range(0, len(kvs), step)])
    return srcs
