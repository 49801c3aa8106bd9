"""GPU parity of the point-read seeks: block.NewIteratorAtKey
(block/iterator.go:31-82, firstFullKey recovery :117-132) and
sstable.Iterator.firstBlockIncludingOrAfterKey (iterator.go:123-153) through the C-ABI, against
the oracle: the reference's seek cases (block_test.go:112-245), its corrupted-key cases
(:416-527), random blocks with random and corrupted row headers, and random SST indexes."""
import random

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _encode(kvs, block_size=4096, corrupt=(), partial=False):
    """Block of kvs (with partial=True, of the prefix of kvs that fits block_size)."""
    bb = ob.BlockBuilder(block_size)
    for k, v in kvs:
        ok = bb.add_value(k, v)
        if not ok and partial:
            break
        assert ok
    data, offs, _ = bb.build()
    data = bytearray(data)
    for r in corrupt:
        if r != "data0" and r >= len(offs):
            continue
        data[0 if r == "data0" else offs[r]] = 0xFF
    return ob.block_encode(bytes(data), offs, ob.NONE)[1], bytes(data), offs


def _layout(blocks):
    """Blocks in the decode layout (Data || BE16 offsets || BE16 count, 16-aligned, meta OK),
    built from the in-memory Block as the reference's iterator tests do (they corrupt rows of a
    built Block, so block.Decode never sees them)."""
    import slatecodec as sc
    parts, out_off, metas = [], [0], []
    for _, data, offs in blocks:
        raw = data + b"".join(o.to_bytes(2, "big") for o in offs) + len(offs).to_bytes(2, "big")
        raw += b"\0" * ((-len(raw)) % 16)
        parts.append(raw)
        out_off.append(out_off[-1] + len(raw))
        metas.append((0, 0, 0, len(data), len(offs), 0))
    out = np.frombuffer(b"".join(parts) + b"\0" * 16, np.uint8).copy()
    return out, np.array(out_off, np.uint64), np.array(metas, sc.META_DTYPE)


def _seek_both(ctx, blocks, queries):
    """queries: (block index, key).  GPU block_seek vs the oracle on each block's Data/Offsets."""
    out, out_off, meta = _layout(blocks)
    qb, qk = [q[0] for q in queries], [q[1] for q in queries]
    got = ctx.block_seek(out, out_off, meta, qb, qk)
    cap = 8
    got_w, warns = ctx.block_seek_warn(out, out_off, meta, qb, qk, warn_cap=cap)
    assert got_w.tobytes() == got.tobytes()
    for i, (b, key) in enumerate(queries):
        _, data, offs = blocks[b]
        (st, start, fi, fl, nw), ow = ob.block_seek_warnings(data, offs, key, cap)
        g = got[i]
        assert (int(g["status"]), int(g["n_warn"])) == (st, nw), (i, b, key, g, st, nw)
        if st == 0:
            assert (int(g["start"]), int(g["first_idx"]), int(g["first_len"])) == (start, fi, fl), (i, key)
        # ErrWarn's entries in order: what a shim needs to rebuild its text
        gw = [(int(w["kind"]), int(w["err"]), int(w["a"]), int(w["b"])) for w in warns[i][: min(nw, cap)]]
        assert gw == ow, (i, b, key, gw, ow)
    return got


def test_reference_seek_cases(ctx, ref_vectors):
    v = ref_vectors["iterator_seek"]
    blk = _encode([(k.encode(), val.encode()) for k, val in v["kvs"]], 1024)
    got = _seek_both(ctx, [blk], [(0, c["key"].encode()) for c in v["cases"]])
    assert [int(g["start"]) for g in got] == [c["start"] for c in v["cases"]]


def test_reference_corrupted_key_cases(ctx, ref_vectors):
    cases = ref_vectors["iterator_seek_corrupt"]
    blocks = [_encode([(k.encode(), val.encode()) for k, val in c["kvs"]], corrupt=c["corrupt"]) for c in cases]
    got = _seek_both(ctx, blocks, [(i, c["key"].encode()) for i, c in enumerate(cases)])
    for g, c in zip(got, cases):
        if "error" in c:
            import slatecodec as sc
            assert sc.status_string(int(g["status"])) == c["error"], c["name"]
        else:
            assert g["status"] == 0 and (g["n_warn"] > 0) == c["warnings"], c["name"]


@pytest.mark.parametrize("seed", range(3))
def test_random_blocks_and_keys(ctx, seed):
    rng = random.Random(seed)
    blocks = []
    for _ in range(60):
        kvs = bg.random_kvs(rng, rng.randint(1, 40), klen=(1, 12), vlen=(0, 30), alphabet=rng.choice([3, 256]))
        kvs = [(k, v) for k, v in kvs if k]
        if not kvs:
            continue
        corrupt = sorted(rng.sample(range(len(kvs)), rng.randint(0, min(3, len(kvs))))) if rng.random() < 0.4 else []
        blocks.append(_encode(kvs, rng.choice([256, 4096]), corrupt, partial=True))
    queries = []
    for b, (_, data, offs) in enumerate(blocks):
        for _ in range(12):
            queries.append((b, rng.randbytes(rng.randint(0, 12)) if rng.random() < 0.5 else
                            bytes(rng.choice(b"abc") for _ in range(rng.randint(0, 6)))))
    _seek_both(ctx, blocks, queries)


def test_block_seek_device(ctx):
    """The device-resident entries on library-owned memory (slate_devbuf, as a cgo caller holds it):
    plan -> decode -> seek with warnings, no torch allocation."""
    import slatecodec as sc
    rng = random.Random(7)
    kvs = bg.kv_synthetic(38 * 50)
    blocks = bg.sst_blocks(kvs, 4096, ob.SNAPPY)
    blob, off = bg.pack(blocks)
    n = len(blocks)
    ctx.set_stream(None)
    d_in, d_off = sc.devbuf_from(ctx, blob), sc.devbuf_from(ctx, off)
    d_oo, d_rb = sc.DevBuf(ctx, 8 * (n + 1)), sc.DevBuf(ctx, 8 * (n + 1))
    d_sc = sc.DevBuf(ctx, sc.decode_scratch_bytes(n) + 64)
    ctx.decode_plan_device(ob.SNAPPY, d_in.ptr, d_off.ptr, n, d_oo.ptr, d_rb.ptr, d_sc.ptr)
    d_out = sc.DevBuf(ctx, d_oo.u64(n) + 16)
    d_meta = sc.DevBuf(ctx, n * 16)
    d_rows = sc.DevBuf(ctx, d_rb.u64(n) * 16 + 16)
    ctx.decode_device(ob.SNAPPY, d_in.ptr, d_off.ptr, n, d_out.ptr, d_oo.ptr, d_meta.ptr, d_rows.ptr, d_rb.ptr)
    qb = [rng.randrange(n) for _ in range(500)]
    keys = [b"k%015d" % rng.randrange(38 * 50 + 40) for _ in qb]
    kd = np.frombuffer(b"".join(keys), np.uint8).copy()
    ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    d_q, d_k, d_ko = sc.devbuf_from(ctx, np.array(qb, np.uint32)), sc.devbuf_from(ctx, kd), sc.devbuf_from(ctx, ko)
    d_res = sc.DevBuf(ctx, len(qb) * 16)
    cap = 4
    d_warn = sc.DevBuf(ctx, len(qb) * cap * 16)
    sc._check(sc.lib().slate_block_seek_warn_device(ctx.handle, d_out.ptr, d_oo.ptr, d_meta.ptr, d_q.ptr, d_k.ptr,
                                                    d_ko.ptr, len(qb), d_res.ptr, d_warn.ptr, cap),
              "slate_block_seek_warn_device")
    got = d_res.download().view(sc.SEEK_DTYPE)
    assert (d_warn.download().view(sc.SEEK_WARN_DTYPE)["kind"][: (got["n_warn"] > 0).sum()] >= 0).all()
    # the plain device entry agrees with the warning variant
    d_res2 = sc.DevBuf(ctx, len(qb) * 16)
    ctx.block_seek_device(d_out.ptr, d_oo.ptr, d_meta.ptr, d_q.ptr, d_k.ptr, d_ko.ptr, len(qb), d_res2.ptr)
    assert d_res2.download().tobytes() == d_res.download().tobytes()
    o_out, o_off, o_meta, _, _ = ob.block_decode_batch(ob.SNAPPY, blob, off)
    for i, (b, k) in enumerate(zip(qb, keys)):
        a, dl, nr = int(o_off[b]), int(o_meta["data_len"][b]), int(o_meta["n_rows"][b])
        data = o_out[a:a + dl].tobytes()
        offs = [int.from_bytes(o_out[a + dl + 2 * r:a + dl + 2 * r + 2].tobytes(), "big") for r in range(nr)]
        st, start, fi, fl, nw = ob.block_seek(data, offs, k)
        assert (int(got[i]["status"]), int(got[i]["start"]), int(got[i]["n_warn"])) == (st, start, nw), i


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_index_seek(ctx, codec):
    import slatecodec as sc
    rng = random.Random(11 + codec)
    kvs = bg.random_kvs(rng, 3000, klen=(1, 20), vlen=(0, 60))
    b = ob.SstBuilder(256, 0, 10, codec)
    for k, v in kvs:
        assert b.add_value(k, v) == 0
    assert b.build() == 0
    sst = b.encode_table()
    st, info, _ = sc.read_info(sst)
    assert st == 0
    st, index = ctx.decode_index(sst[info.index_offset:info.index_offset + info.index_len], info.codec)
    assert st == 0
    first_keys = [fk for _, fk in index.block_metas()]
    keys = [rng.randbytes(rng.randint(0, 20)) for _ in range(400)] + [k for k, _ in rng.sample(kvs, 100)] + first_keys[:50]
    got = ctx.index_seek(index, keys)
    want = [ob.index_seek(first_keys, k) for k in keys]
    assert got.tolist() == want


@pytest.mark.parametrize("seed", range(2))
def test_point_reads_one_query_per_call(ctx, seed):
    """One query per call (the point read: slate_block_seek with n = 1 takes the staged,
    wave-cooperative form, seek.hip seek_one_wave), over blocks with corrupted rows: every result
    and every warning, in order, as the oracle's NewIteratorAtKey."""
    rng = random.Random(100 + seed)
    blocks = []
    for _ in range(30):
        kvs = bg.random_kvs(rng, rng.randint(1, 120), klen=(1, 12), vlen=(0, 30), alphabet=rng.choice([3, 256]))
        kvs = [(k, v) for k, v in kvs if k]
        if not kvs:
            continue
        corrupt = sorted(rng.sample(range(len(kvs)), rng.randint(0, min(5, len(kvs))))) if rng.random() < 0.5 else []
        blocks.append(_encode(kvs, rng.choice([256, 4096]), corrupt, partial=True))
    out, out_off, meta = _layout(blocks)
    cap = 8
    for b, (_, data, offs) in enumerate(blocks):
        for _ in range(8):
            key = (rng.randbytes(rng.randint(0, 12)) if rng.random() < 0.5 else
                   bytes(rng.choice(b"abc") for _ in range(rng.randint(0, 6))))
            a, e = int(out_off[b]), int(out_off[b + 1])
            one_off = np.array([0, e - a], np.uint64)  # the block alone: a point read's few KiB
            got_w, warns = ctx.block_seek_warn(out[a:e + 16].copy(), one_off, meta[b:b + 1].copy(), [0], [key],
                                               warn_cap=cap)
            (st, start, fi, fl, nw), ow = ob.block_seek_warnings(data, offs, key, cap)
            g = got_w[0]
            assert (int(g["status"]), int(g["n_warn"])) == (st, nw), (b, key, g, st, nw)
            if st == 0:
                assert (int(g["start"]), int(g["first_idx"]), int(g["first_len"])) == (start, fi, fl), (b, key)
            gw = [(int(w["kind"]), int(w["err"]), int(w["a"]), int(w["b"])) for w in warns[0][: min(nw, cap)]]
            assert gw == ow, (b, key, gw, ow)
