"""GPU parity: SST build (blocks, bloom, index, info), block encode, bloom and the
SST reader through the HIP C-ABI vs the CPU oracle — byte for byte (CodecNone)."""
import random
import struct

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    import slatecodec
    return slatecodec


@pytest.fixture(scope="module")
def ctx(sc):
    return sc.Context(0)


def _build_both(sc, ctx, kvs, block_size=4096, mfk=0, bpk=10, batch=False, next_every=0, codec=None):
    codec = ob.NONE if codec is None else codec
    g = sc.SstBuilder(ctx, block_size, mfk, bpk, codec)
    o = ob.SstBuilder(block_size, mfk, bpk, codec)
    g_blocks, o_blocks = [], []
    if batch:
        keys = [k for k, _ in kvs]
        vals = [v for _, v in kvs]
        kd, ko = sc._arena(keys)
        vd, vo = sc._arena(vals)
        assert g.add_batch(kd, ko, vd, vo) == 0
        for k, v in kvs:
            assert o.add_value(k, v) == 0
    else:
        for i, (k, v) in enumerate(kvs):
            assert g.add_value(k, v) == 0
            assert o.add_value(k, v) == 0
            if next_every and i % next_every == 0:
                while (b := g.next_block()) is not None:
                    g_blocks.append(b)
                while (b := o.next_block()) is not None:
                    o_blocks.append(b)
    assert g_blocks == o_blocks
    t = g.build()
    assert o.build() == 0
    return t, o, g_blocks


@pytest.mark.parametrize("seed", range(6))
def test_random_sst_bytes(sc, ctx, seed):
    rng = random.Random(seed)
    kvs = bg.random_kvs(rng, rng.randint(1, 1500), alphabet=rng.choice([3, 256]), tomb_p=0.15)
    bs = rng.choice([40, 128, 1024, 4096])
    mfk = rng.choice([0, 10, 100000])
    bpk = rng.choice([1, 10, 20])
    t, o, _ = _build_both(sc, ctx, kvs, bs, mfk, bpk, batch=seed % 2 == 0, next_every=rng.choice([0, 1, 7]))
    assert t.chunks() == o.chunks()
    assert t.encode() == o.encode_table()
    assert t.info() == o.info()
    assert t.bloom() == o.bloom()


@pytest.mark.parametrize("case", ["many_rows", "long_first_keys"])
def test_segmentation_windows_and_first_keys(sc, ctx, case):
    """enc_next_kernel's LDS window (1024 KVs from a workgroup's first) and kv_pick_copy_kernel's
    lane / wave split (first keys longer than 256 bytes): blocks of ~4000 tiny rows walk past the
    window into HBM; long first keys are copied by the wave, short ones by their lane."""
    rng = random.Random(7)
    if case == "many_rows":
        kvs = [(b"%08d" % i, b"" if i % 5 else b"v") for i in range(60000)]
        bs = 65536
    else:
        kvs = []
        for i in range(3000):
            k = b"%06d" % i
            if rng.random() < 0.3:
                k += bytes(rng.randrange(256) for _ in range(rng.choice([250, 257, 300, 1000, 5000])))
            kvs.append((k, bytes(rng.randrange(256) for _ in range(rng.randrange(1, 600)))))
        bs = 4096
    for batch in (True, False):
        t, o, _ = _build_both(sc, ctx, kvs, bs, batch=batch)
        assert t.encode() == o.encode_table()
        assert t.info() == o.info()


def test_kv_pass_key_lengths_and_prefixes(sc, ctx):
    """enc_kv_kernel's dword path (keys of <= 32 bytes: FNV-1 64, LCP with the previous key and the
    sortedness check from realigned aligned dwords) and its byte path (longer keys), with key lengths
    0-40 at every alignment and LCPs ending at every byte position."""
    rng = random.Random(11)
    keys = set()
    while len(keys) < 4000:
        base = bytes(rng.choice(b"ab\x00\xff") for _ in range(rng.randrange(1, 41)))
        keys.add(base)
        cut = rng.randrange(0, len(base) + 1)
        keys.add(base[:cut] + bytes([rng.randrange(256)]) + base[cut:][: rng.randrange(0, 8)])
    kvs = [(k, bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40)))) for k in sorted(keys) if k]
    for batch in (True, False):
        t, o, _ = _build_both(sc, ctx, kvs, 1024, batch=batch)
        assert t.encode() == o.encode_table()
        assert t.bloom() == o.bloom()
    # a descending pair inside the short path: the sortedness flag sends the segmentation to its
    # direct-LCP walk; bytes still equal the oracle's
    bad = kvs[:50] + [(kvs[60][0], b"x"), (kvs[55][0], b"y")] + kvs[70:120]
    t, o, _ = _build_both(sc, ctx, bad, 256, batch=True)
    assert t.encode() == o.encode_table()


@pytest.mark.parametrize("seed", range(4))
def test_next_block_after_each_add(sc, ctx, seed):
    """sstable.Builder.NextBlock timing (builder.go:160-190): after every AddValue, the blocks the
    library hands out are exactly the ones the reference's builder has finished by then (the block
    is finished by the Add whose row no longer fits), byte for byte."""
    rng = random.Random(100 + seed)
    kvs = bg.random_kvs(rng, rng.randint(200, 900), alphabet=rng.choice([3, 256]), tomb_p=0.1)
    bs = rng.choice([64, 200, 1024, 4096])
    g = sc.SstBuilder(ctx, bs, 0, 10, ob.NONE)
    o = ob.SstBuilder(bs, 0, 10, ob.NONE)
    for i, (k, v) in enumerate(kvs):
        assert g.add_value(k, v) == 0 and o.add_value(k, v) == 0
        gb, ob_ = [], []
        while (b := g.next_block()) is not None:
            gb.append(b)
        while (b := o.next_block()) is not None:
            ob_.append(b)
        assert gb == ob_, (i, len(gb), len(ob_))
    assert g.build().encode() == (o.build(), o.encode_table())[1]


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("seed", range(3))
def test_batch_in_pieces(sc, ctx, monkeypatch, codec, seed):
    """slate_sst_builder_add_batch in pieces (SLATE_ADD_PIECE KVs each, a flush after every piece but
    the last, its blocks downloaded on the context's second pipe while the next piece uploads): the
    SST, its chunks, info and bloom equal the oracle's, as do the blocks NextBlock hands out after
    the batch and after a second batch (tombstones by empty values and by flags)."""
    rng = random.Random(300 + seed)
    kvs = bg.random_kvs(rng, rng.randint(3000, 6000), alphabet=rng.choice([3, 256]), tomb_p=0.1)
    bs = rng.choice([256, 1024, 4096])
    monkeypatch.setenv("SLATE_ADD_PIECE", str(rng.choice([500, 900, 1500])))
    half = len(kvs) // 2
    g = sc.SstBuilder(ctx, bs, 0, 10, codec)
    o = ob.SstBuilder(bs, 0, 10, codec)
    for part, flags in ((kvs[:half], False), (kvs[half:], True)):
        kd, ko = sc._arena([k for k, _ in part])
        vd, vo = sc._arena([v for _, v in part])
        tomb = np.array([1 if not v else 0 for _, v in part], np.uint8) if flags else None
        assert g.add_batch(kd, ko, vd, vo, tomb) == 0
        for k, v in part:
            assert o.add_value(k, v) == 0
        gb, obl = [], []
        while (b := g.next_block()) is not None:
            gb.append(b)
        while (b := o.next_block()) is not None:
            obl.append(b)
        assert gb == obl
    t = g.build()
    assert o.build() == 0
    assert t.chunks() == o.chunks()
    assert t.encode() == o.encode_table()
    assert t.info() == o.info()
    assert t.bloom() == o.bloom()


def test_unsorted_and_duplicate_keys(sc, ctx):
    rng = random.Random(9)
    kvs = [(bytes(rng.randrange(3) for _ in range(rng.randint(1, 6))), b"v" * rng.randint(0, 40)) for _ in range(800)]
    kvs += [(b"dup", b"x")] * 20
    t, o, _ = _build_both(sc, ctx, kvs, 256, 0, 10)
    assert t.encode() == o.encode_table()


def test_make_blocks_available(sc, ctx, ref_vectors):
    v = ref_vectors["make_blocks_available"]
    g = sc.SstBuilder(ctx, v["block_size"], 0, 10, sc.NONE)
    for k, val in v["adds1"]:
        assert g.add_value(k.encode(), val.encode()) == 0
    for expect in v["blocks1"]:
        blk = g.next_block()
        meta, buf, rows = ob.block_decode(blk, ob.NONE)
        assert buf[4:4 + rows[0]["key_suffix_len"]] == expect[0].encode()
    assert g.next_block() is None
    for k, val in v["adds2"]:
        assert g.add_value(k.encode(), val.encode()) == 0
    blk = g.next_block()
    meta, buf, rows = ob.block_decode(blk, ob.NONE)
    assert buf[4:12] == v["blocks2"][0][0].encode()
    assert g.next_block() is None


@pytest.mark.parametrize("name", ["read_blocks_52", "read_all_blocks"])
def test_reference_layouts_and_reader(sc, ctx, ref_vectors, name):
    v = ref_vectors[name]
    bs = v.get("block_size") or ob.v0_estimate_block_size([(k.encode(), x.encode()) for k, x in v["estimate_kvs"]])
    kvs = [(k.encode(), x.encode()) for k, x in v["kvs"]]
    t, o, _ = _build_both(sc, ctx, kvs, bs, v["min_filter_keys"], 10)
    sst = t.encode()
    assert sst == o.encode_table()
    st, info, fk = sc.read_info(sst)
    assert st == 0 and fk == kvs[0][0]
    st, index = ctx.decode_index(sst[info.index_offset: info.index_offset + info.index_len], info.codec)
    assert st == 0
    metas = index.block_metas()
    assert [m[1] for m in metas] == [blk[0].encode() for blk in v["blocks"]]
    st, failed, (out, out_off, meta, rows, rb) = ctx.read_blocks(info, index, 0, len(metas), sst)
    assert st == 0 and failed == 2**64 - 1
    for i, blk in enumerate(v["blocks"]):
        assert meta[i]["n_rows"] == len(blk)
    # range errors (decode.go:108-114)
    assert ctx.read_blocks(info, index, 1, 1, sst)[0] == 46
    assert ctx.read_blocks(info, index, 0, len(metas) + 1, sst)[0] == 47


def test_dump_layout(sc, ctx, ref_vectors):
    v = ref_vectors["dump_layout_derived"]
    kvs = [(k.encode(), x.encode()) for k, x in v["kvs"]]
    t, o, _ = _build_both(sc, ctx, kvs, 35, 0, 10)
    info = t.info()
    assert info["filter_offset"] == v["filter_offset"] and info["filter_len"] == v["filter_len_now"]
    assert info["index_offset"] == v["index_offset_now"]
    assert info["index_len"] - 4 == v["dump_stale"]["index_len"]


def test_filter_encoded_len(sc, ctx, ref_vectors):
    for c in ref_vectors["filter_encoded_len"]:
        kvs = [(k.encode(), c["value"].encode()) for k in c["keys"]]
        t, o, _ = _build_both(sc, ctx, kvs, 4096, 0, c["bits_per_key"])
        assert t.info()["filter_len"] == c["expected_len"]


def test_bloom_api(sc, ctx, ref_vectors):
    v = ref_vectors["filter_has_key"]
    keys = [s.encode() for s in v["add"]]
    k, bits = ctx.bloom_build(keys, v["bits_per_key"])
    assert (k, bits) == ob.bloom_build(keys, v["bits_per_key"])
    probe = [s.encode() for s in v["present"] + v["absent"]]
    assert ctx.bloom_has_keys(k, bits, probe) == [True] * len(v["present"]) + [False] * len(v["absent"])
    st, enc = ctx.bloom_encode(k, bits, sc.NONE)
    assert st == 0 and enc == ob.bloom_encode(k, bits, ob.NONE)
    assert ctx.bloom_decode(enc, sc.NONE) == (0, k, bits)
    assert ctx.bloom_decode(enc[:-1] + bytes([enc[-1] ^ 1]), sc.NONE)[0] == 31
    assert ctx.bloom_decode(b"\x00", sc.NONE)[0] == 30
    # TestFilterEffective scale
    many = [struct.pack(">I", i) for i in range(100000)]
    k2, bits2 = ctx.bloom_build(many, 10)
    assert bits2 == ob.bloom_build(many, 10)[1]
    res = ctx.bloom_has_keys(k2, bits2, [struct.pack(">I", i) for i in range(100000, 200000)])
    assert sum(res) / 100000 < 0.01
    assert ctx.bloom_has_keys(0, b"", [b"x"]) == [False]


def test_block_encode_single(sc, ctx, ref_vectors):
    for c in ref_vectors["block_roundtrips"]:
        bb = ob.BlockBuilder(c["block_size"])
        for k, val in c["kvs"]:
            bb.add_value(k.encode(), (val or "").encode())
        data, offs, _ = bb.build()
        st, enc = ctx.block_encode(data, offs, sc.NONE)
        assert st == 0 and enc == ob.block_encode(data, offs, ob.NONE)[1]


def test_large_rows(sc, ctx):
    """Single rows larger than the pack kernel's per-wave LDS budget."""
    kvs = [(b"a%03d" % i, bytes([i % 251]) * n) for i, n in enumerate([10, 9000, 30000, 5, 20000, 100])]
    t, o, _ = _build_both(sc, ctx, kvs, 4096, 0, 10)
    assert t.encode() == o.encode_table()


def test_vhalf_workload_batch(sc, ctx):
    kvs = bg.kv_synthetic(38 * 500, half=True, tomb_every=20)
    t, o, _ = _build_both(sc, ctx, kvs, 4096, 0, 10, batch=True)
    assert t.encode() == o.encode_table()


def test_empty_builder(sc, ctx):
    t, o, _ = _build_both(sc, ctx, [], 4096, 0, 10)
    assert t.encode() == o.encode_table()


# ------------------------------------------------------------------ Snappy
# golang/snappy v0.0.4 encoded bytes: the oracle restates encode_other.go; it is
# byte-identical to libsnappy on the probes in test_oracle (parity vs Go itself
# unpinned).

@pytest.mark.parametrize("seed", range(6))
def test_snappy_sst_bytes(sc, ctx, seed):
    rng = random.Random(100 + seed)
    kvs = bg.random_kvs(rng, rng.randint(1, 1500), alphabet=rng.choice([3, 256]), tomb_p=0.15)
    bs = rng.choice([40, 128, 1024, 4096, 16384])
    t, o, _ = _build_both(sc, ctx, kvs, bs, rng.choice([0, 10]), rng.choice([1, 10]), batch=seed % 2 == 0,
                          next_every=rng.choice([0, 7]), codec=ob.SNAPPY)
    assert t.chunks() == o.chunks()
    assert t.encode() == o.encode_table()
    assert t.info() == o.info()


def test_snappy_vhalf_and_read_back(sc, ctx):
    kvs = bg.kv_synthetic(38 * 300, half=True, tomb_every=20)
    t, o, _ = _build_both(sc, ctx, kvs, 4096, 0, 10, batch=True, codec=ob.SNAPPY)
    sst = t.encode()
    assert sst == o.encode_table()
    st, info, fk = sc.read_info(sst)
    assert st == 0 and info.codec == ob.SNAPPY
    st, index = ctx.decode_index(sst[info.index_offset: info.index_offset + info.index_len], info.codec)
    assert st == 0
    n = len(index.block_metas())
    st, failed, (out, out_off, meta, rows, rb) = ctx.read_blocks(info, index, 0, n, sst)
    assert st == 0 and failed == 2**64 - 1
    assert int(meta["n_rows"].astype(np.int64).sum()) == len(kvs)
    # bloom filter read back through the Snappy path
    filt = sst[info.filter_offset: info.filter_offset + info.filter_len]
    st, k, bits = ctx.bloom_decode(filt, sc.SNAPPY)
    assert st == 0 and (k, bits) == (t.bloom()[0], t.bloom()[1])


def test_snappy_large_rows_and_blocks(sc, ctx):
    rng = random.Random(5)
    vals = [bytes(rng.randrange(256) for _ in range(n)) for n in (10, 9000, 30000, 5)]
    vals += [b"ab" * 20000, bytes(70000), b"xyz" * 30000]
    kvs = [(b"a%03d" % i, v) for i, v in enumerate(vals)]
    t, o, _ = _build_both(sc, ctx, kvs, 4096, 0, 10, codec=ob.SNAPPY)
    assert t.encode() == o.encode_table()


def test_snappy_block_encode_and_bloom(sc, ctx, ref_vectors):
    for c in ref_vectors["block_roundtrips"]:
        bb = ob.BlockBuilder(c["block_size"])
        for k, val in c["kvs"]:
            bb.add_value(k.encode(), (val or "").encode())
        data, offs, _ = bb.build()
        st, enc = ctx.block_encode(data, offs, sc.SNAPPY)
        assert st == 0 and enc == ob.block_encode(data, offs, ob.SNAPPY)[1]
    rng = np.random.default_rng(3)
    for nbytes in (0, 1, 15, 16, 17, 100, 65534, 65535, 65536, 65537, 200_000, 1_000_003):
        bits = rng.integers(0, 4, nbytes, dtype=np.uint8).tobytes()  # compressible
        st, enc = ctx.bloom_encode(6, bits, sc.SNAPPY)
        assert st == 0 and enc == ob.bloom_encode(6, bits, ob.SNAPPY), nbytes
        assert ctx.bloom_decode(enc, sc.SNAPPY) == (0, 6, bits)
    bad = bytearray(ctx.bloom_encode(6, b"abc" * 100, sc.SNAPPY)[1])
    bad[3] ^= 0x40
    assert ctx.bloom_decode(bytes(bad), sc.SNAPPY)[0] == 31


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_builder_gpu_time(sc, codec):
    """slate_ctx_set_timing / slate_ctx_gpu_time (the bench's configs[2] kernel time): nothing is
    summed while timing is off, a build sums its GPU passes when it is on, and the bytes do not
    change either way."""
    c = sc.Context(0)
    kvs = bg.kv_synthetic(38 * 300, half=True)
    t0, o, _ = _build_both(sc, c, kvs, codec=codec)
    assert c.gpu_time_ms() == 0.0
    c.set_timing(True)
    t1, _, _ = _build_both(sc, c, kvs, codec=codec)
    ms = c.gpu_time_ms(reset=True)
    assert 0.0 < ms < 10_000.0
    assert c.gpu_time_ms() == 0.0
    c.set_timing(False)
    assert t0.encode() == t1.encode() == o.encode_table()
    c.close()
