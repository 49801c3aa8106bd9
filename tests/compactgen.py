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


def oracle_compact(sources: list[list[bytes]], max_sst_size: int, codec: int = ob.NONE,
                   block_size: int = 4096) -> list[bytes]:
    iters = [[kv for sst in run for kv in sst_rows(sst)] for run in sources]
    flat = [kv for it in iters for kv in it]
    merged = [flat[i] for i in ob.merge_sort([[k for k, _ in it] for it in iters])]
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


def random_sources(rng: random.Random, n_sources: int, n_keys: int, space: int, codec: int = ob.NONE,
                   tomb: float = 0.05, run_ssts: int = 1, key_fmt="k%015d"):
    """n_sources sorted runs (each of run_ssts SSTs over consecutive key ranges) drawn from a
    shared key space, values of random length (0..120), some tombstones."""
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
        srcs.append([build_sst(kvs[j:j + step], codec) for j in range(0, len(kvs), step)])
    return srcs
