"""GPU parity: block decode through the HIP C-ABI vs the CPU oracle.

Bit-exact on every field: plan layout (out_off / row_base), per-block meta
(status, detail, aux, data_len, n_rows, flags), decoded bytes, row descriptors.
"""
import random
import struct

import numpy as np
import pytest

from tests import blockgen as bg
from oracle import binding as ob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _compare(ctx, codec, blocks, misalign=0):
    blob, off = bg.pack(blocks, misalign)
    g_out, g_off, g_meta, g_rows, g_rb = ctx.decode_batch(codec, blob, off)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, off)
    n = len(blocks)
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i in range(n):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om, blocks[i][:32].hex())
        st = int(om["status"])
        if st == 0 or 3 <= st <= 7:
            dl = bg.decoded_len(blocks[i], codec)
            a, b = int(o_off[i]), int(o_off[i]) + dl
            assert g_out[a:b].tobytes() == o_out[a:b].tobytes(), i
        if st == 0:
            r0 = int(o_rb[i])
            nr = min(int(om["n_rows"]), int(o_rb[i + 1]) - r0)
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i
    return g_meta


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_reference_fixture_blocks(ctx, ref_vectors, codec):
    blocks = []
    for c in ref_vectors["block_roundtrips"]:
        bb = ob.BlockBuilder(c["block_size"])
        for k, v in c["kvs"]:
            bb.add_value(k.encode(), (v or "").encode())
        data, offs, _ = bb.build()
        blocks.append(ob.block_encode(data, offs, codec)[1])
    meta = _compare(ctx, codec, blocks)
    assert (meta["status"] == 0).all()


def test_reference_corrupt_blocks(ctx, ref_vectors):
    from tests.test_oracle import _corrupt
    v = ref_vectors["corrupt_block"]
    bb = ob.BlockBuilder(v["block_size"])
    for k, val in v["kvs"]:
        bb.add_value(k.encode(), val.encode())
    data, offs, _ = bb.build()
    enc = ob.block_encode(data, offs, ob.NONE)[1]
    blocks = [_corrupt(enc, c["mutation"]) for c in v["cases"]]
    meta = _compare(ctx, ob.NONE, blocks)
    import slatecodec as sc
    for c, m in zip(v["cases"], meta):
        assert c["error"] in sc.status_string(int(m["status"])), c["name"]


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("seed", range(4))
def test_random_ssts(ctx, codec, seed):
    rng = random.Random(seed)
    kvs = bg.random_kvs(rng, rng.randint(200, 2000), alphabet=rng.choice([4, 256]))
    blocks = bg.sst_blocks(kvs, rng.choice([64, 512, 4096]), codec)
    meta = _compare(ctx, codec, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("fix_crc", [False, True])
def test_random_corruption(ctx, codec, fix_crc):
    rng = random.Random(1000 + codec * 2 + fix_crc)
    kvs = bg.random_kvs(rng, 3000, alphabet=8)
    blocks = bg.sst_blocks(kvs, 1024, codec)
    bad = [bg.mutate(rng, b, fix_crc) for b in blocks]
    meta = _compare(ctx, codec, bad + blocks[:5])
    assert len(set(meta["status"].tolist())) > 1


def test_edge_lengths(ctx):
    blocks = [b"", b"\x00", b"\x00" * 5, bg.recrc(b"\x00\x00"), bg.recrc(b"\x00\x01"), bg.recrc(b"\x00\x00\x00"),
              bg.recrc(b"\xff\xff\x00\x00"), bg.recrc(b"\x00\x00\x00\x00\x00\x01")]
    _compare(ctx, ob.NONE, blocks)
    sn = [bg.recrc(b"\x00"), bg.recrc(b"\x02\x04ab"), bg.recrc(b"\xff" * 11), bg.recrc(b"\x80"),
          bg.recrc(b"\x05\x00a\x01\x01"), bg.recrc(b"\x7f\x00a")]
    _compare(ctx, ob.SNAPPY, sn)


def test_empty_batch(ctx):
    out, off, meta, rows, rb = ctx.decode_batch(ob.NONE, np.zeros(16, np.uint8), np.zeros(1, np.uint64))
    assert len(meta) == 0 and off[0] == 0


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_large_blocks(ctx, codec):
    """Blocks beyond the fast kernel's LDS budget go through decode_large_kernel."""
    rng = random.Random(5)
    kvs = [(b"big%05d" % i, bytes(rng.randrange(4) for _ in range(rng.choice([100, 6000, 20000]))))
           for i in range(40)]
    blocks = bg.sst_blocks(kvs, 32768, codec)
    assert max(len(b) for b in blocks) > 4608 or codec == ob.SNAPPY
    meta = _compare(ctx, codec, blocks)
    assert (meta["status"] == 0).all()


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_vhalf_workload(ctx, codec):
    """The bench workload shape (38 rows x 100 B KV per 4 KiB block) at 2000 blocks."""
    kvs = bg.kv_synthetic(38 * 2000, half=True, tomb_every=20)
    blocks = bg.sst_blocks(kvs, 4096, codec)
    meta = _compare(ctx, codec, blocks)
    assert (meta["status"] == 0).all()


def test_single_block_api(ctx, ref_vectors):
    bb = ob.BlockBuilder(4096)
    for k, v in (("key1", "value1"), ("key2", "value2")):
        bb.add_value(k.encode(), v.encode())
    data, offs, _ = bb.build()
    for codec in (ob.NONE, ob.SNAPPY):
        enc = ob.block_encode(data, offs, codec)[1]
        st, m, d, o = ctx.block_decode(enc, codec)
        assert st == 0 and d == data and o == offs
        st, m, d, o = ctx.block_decode(enc[:-1] + bytes([enc[-1] ^ 1]), codec)
        assert st == 2


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
def test_single_block_api_matrix(ctx, codec):
    """slate_block_decode: the one-launch path (CodecNone / CodecSnappy blocks within the large-block
    LDS budget, plan on the host) and the generic plan + decode path beyond it, meta bit-exact
    against the oracle's batch decode of the same block, decoded bytes and offsets on success.
    Valid blocks of several block sizes, mutated blocks (stale and fixed CRC), the edge lengths,
    and a block whose decoded length is past the budget (90112 B)."""
    rng = random.Random(31 + codec)
    blocks = []
    for bs in (64, 512, 4096, 32768):
        kvs = bg.random_kvs(rng, 300, alphabet=rng.choice([4, 256]))
        blocks += bg.sst_blocks(kvs, bs, codec)[:6]
    blocks += [bg.mutate(rng, b, fix) for b in blocks[:16] for fix in (False, True)]
    blocks += [b"", b"\x00", b"\x00" * 5, bg.recrc(b"\x00\x00"), bg.recrc(b"\x00\x00\x00\x00\x00\x01"),
               bg.recrc(b"\x00"), bg.recrc(b"\x02\x04ab"), bg.recrc(b"\xff" * 11), bg.recrc(b"\x80"),
               bg.recrc(b"\x05\x00a\x01\x01")]
    big = [(b"big%05d" % i, bytes(rng.randrange(3) for _ in range(30000))) for i in range(4)]
    blocks += bg.sst_blocks([(b"one", bytes(rng.randrange(3) for _ in range(70000)))], 4096, codec)
    blocks += bg.sst_blocks(big, 1 << 17, codec)[:1]
    assert max(len(b) for b in blocks[-1:]) > 90112 or codec == ob.SNAPPY
    for i, blk in enumerate(blocks):
        st, m, data, offs = ctx.block_decode(blk, codec)
        blob, off = bg.pack([blk])
        o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, off)
        assert m.tobytes() == o_meta[0].tobytes(), (i, m, o_meta[0], blk[:16].hex())
        assert st == int(o_meta[0]["status"])
        if st == 0:
            assert data == o_out[: int(m["data_len"])].tobytes(), i
            assert offs == [int(r["row_off"]) for r in o_rows[: int(m["n_rows"])]], i


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY, ob.LZ4, ob.ZLIB, ob.ZSTD])
def test_blocks_beyond_lds_budget(ctx, codec):
    """Blocks holding one large value (encoded > 64 KiB or decoded > 88 KiB: beyond the large-block
    kernel's LDS budget) decode with input and output in HBM, like the oracle -- block.Decode has no
    size limit (block.go:78-101) and a Builder puts a value larger than BlockSize in a block of its
    own.  Batch and single-block calls, with smaller blocks around them, under flipped CRCs too."""
    from tests import sstgen
    rng = random.Random(11 + codec)
    nrng = np.random.default_rng(11 + codec)
    blocks = []
    for vl in (70000, 100000, 200000):
        kv = [(b"one%06d" % vl, nrng.integers(0, 4, vl, dtype=np.uint8).tobytes())]
        raw = bg.sst_blocks(kv, 4096, ob.NONE)[0][:-4]
        blocks.append(sstgen.crc(sstgen.compress(codec, raw, rng)))
    small = [sstgen.crc(sstgen.compress(codec, b[:-4], rng))
             for b in bg.sst_blocks(bg.random_kvs(rng, 200), 4096, ob.NONE)[:4]]
    flipped = [b[:-1] + bytes([b[-1] ^ 1]) for b in blocks[:2]]
    meta = _compare(ctx, codec, small[:2] + blocks + small[2:] + flipped)
    assert (meta["status"][:7] == 0).all() and (meta["status"][7:] == 2).all(), meta["status"]
    for blk in blocks:
        st, m, data, offs = ctx.block_decode(blk, codec)
        om, odata, orows = ob.block_decode(blk, codec)
        assert st == 0 == int(om["status"]) and data == odata[:int(om["data_len"])]
        assert offs == [int(r["row_off"]) for r in orows]


@pytest.mark.parametrize("misalign", [0, 1, 7, 12, 13, 15])
def test_none_size_window(ctx, misalign):
    """CodecNone blocks around the streaming kernel's window (decode_none.hip: 4..5104 data bytes in
    five register rows of 64 chunks; outside it the exact wave path): valid one- and many-row blocks
    of exact data lengths, random bytes under a valid CRC (the block checks' error paths) and a
    flipped CRC, at every chunk phase."""
    rng = random.Random(77 + misalign)
    blocks = []
    for t in [4, 5, 6, 15, 16, 17, 31, 33, 63, 64, 65, 1023, 1024, 1025, 2047, 4095, 4096, 4097, 5087, 5088, 5089,
              5103, 5104, 5105, 5120, 5200, 6000]:
        if t >= 26:  # one KV: 4 + key + 8 + 1 + 4 + value bytes, then one offset and the count
            bb = ob.BlockBuilder(1 << 16)
            bb.add_value(b"k" * 5, bytes(rng.randrange(256) for _ in range(t - 26)))
            data, offs, _ = bb.build()
            assert len(data) + 2 * len(offs) + 2 == t
            blocks.append(ob.block_encode(data, offs, ob.NONE)[1])
        body = bytes(rng.randrange(256) for _ in range(t))
        blocks.append(bg.recrc(body))
        blocks.append(body + bytes([rng.randrange(256) for _ in range(4)]))
        if t >= 8:  # random rows under a plausible offset array: the bounds / FirstKey / row error paths
            cnt = rng.randint(1, min(80, (t - 4) // 2))
            osi = t - 2 - 2 * cnt
            offs = [rng.randrange(osi + 2) if rng.random() < 0.1 else rng.randrange(max(osi - 12, 1))
                    for _ in range(cnt)]
            data = bytearray(body[:osi])
            if rng.random() < 0.7 and offs[0] + 2 <= osi:  # a FirstKey that fits: rows decode (or fail) one by one
                data[offs[0]:offs[0] + 2] = struct.pack(">H", rng.randrange(max(1, min(9, osi - offs[0] - 1))))
            body2 = bytes(data) + b"".join(struct.pack(">H", o) for o in offs) + struct.pack(">H", cnt)
            blocks.append(bg.recrc(body2))
    kvs = bg.random_kvs(rng, 400, alphabet=16)
    for bs in (300, 4096, 5000, 5100):
        blocks += bg.sst_blocks(kvs, bs, ob.NONE)
    meta = _compare(ctx, ob.NONE, blocks, misalign=misalign)
    assert (meta["status"] == 0).sum() > 20 and len(set(meta["status"].tolist())) > 3


def test_single_block_parallel_snappy(ctx):
    """slate_block_decode of CodecSnappy blocks within the workgroup-parallel decoder's window
    (decode.hip decode_one_par_kernel: tag chain by pointer doubling, bytes by pointer jumping):
    V-half and random blocks, and the same blocks with one byte flipped and the CRC re-sealed (a
    tag, a length, an offset, the varint header), so that every refusal of the parallel passes and
    every serial fallback is exercised -- meta, bytes and offsets against the oracle."""
    rng = random.Random(77)
    blocks = bg.sst_blocks(bg.kv_synthetic(38 * 40), 4096, ob.SNAPPY)[:40]
    blocks += bg.sst_blocks(bg.random_kvs(rng, 2000, alphabet=4), 4096, ob.SNAPPY)[:20]
    blocks += bg.sst_blocks(bg.kv_synthetic(38 * 20, half=False), 4096, ob.SNAPPY)[:10]
    muts = []
    for b in blocks:
        for _ in range(3):
            body = bytearray(b[:-4])
            pos = rng.choice([0, 1, rng.randrange(len(body)), rng.randrange(min(len(body), 40))])
            body[pos] ^= 1 << rng.randrange(8)
            muts.append(bg.recrc(bytes(body)))
    for i, blk in enumerate(blocks + muts):
        st, m, data, offs = ctx.block_decode(blk, ob.SNAPPY)
        blob, off = bg.pack([blk])
        o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.SNAPPY, blob, off)
        assert m.tobytes() == o_meta[0].tobytes(), (i, m, o_meta[0])
        assert st == int(o_meta[0]["status"])
        if st == 0:
            assert data == o_out[: int(m["data_len"])].tobytes(), i
            assert offs == [int(r["row_off"]) for r in o_rows[: int(m["n_rows"])]], i
