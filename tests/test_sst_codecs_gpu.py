"""GPU parity for opening SSTs of every codec: ReadInfo -> DecodeIndex (flatbuf.go:83-100) ->
ReadBlocks (decode.go:107-149) -> ReadFilter / bloom.Decode (bloom.go:70-91) through the C-ABI,
for CodecLz4 / CodecZlib / CodecZstd SSTs whose blocks, filter and index are frames of the codec's
reference library (tests/sstgen.py), against the oracle: index metas, every block's meta /
bytes / rows, the filter, and the statuses of damaged index and filter payloads.  Index and
filter payloads above the LDS budget (decoded > 88 KiB) take the HBM-resident payload kernel
like small ones."""
import random

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tests import sstgen, zstdgen

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not zstdgen.available(), reason="libzstd not in this image")]
CODECS = [ob.LZ4, ob.ZLIB, ob.ZSTD]


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _open_and_compare(ctx, sst: bytes, codec: int):
    import slatecodec as sc
    st, info, fk = sc.read_info(sst)
    ost, oinfo = ob.sst_read_info(sst)
    assert st == ost == 0 and info.codec == codec == oinfo["codec"] and fk == oinfo["first_key"]
    ib = sst[info.index_offset:info.index_offset + info.index_len]
    st, index = ctx.decode_index(ib, codec)
    ost, ometas = ob.decode_index(ib, codec, cap=1 << 21)
    assert st == ost == 0
    metas = index.block_metas()
    assert metas == ometas
    n = len(metas)
    st, failed, (out, out_off, meta, rows, rb) = ctx.read_blocks(info, index, 0, n, sst)
    assert st == 0 and failed == 2**64 - 1
    blob = np.frombuffer(sst[metas[0][0]:info.filter_offset if info.filter_len else info.index_offset], np.uint8)
    in_off = np.array([m[0] - metas[0][0] for m in metas] + [len(blob)], np.uint64)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, in_off)
    assert meta.tobytes() == o_meta.tobytes()
    for i in range(n):
        a, dl = int(o_off[i]), int(o_meta["data_len"][i]) + 2 * int(o_meta["n_rows"][i]) + 2
        assert out[int(out_off[i]):int(out_off[i]) + dl].tobytes() == o_out[a:a + dl].tobytes(), i
        nr = int(o_meta["n_rows"][i])
        assert rows[int(rb[i]):int(rb[i]) + nr].tobytes() == o_rows[int(o_rb[i]):int(o_rb[i]) + nr].tobytes(), i
    if info.filter_len:
        fb = sst[info.filter_offset:info.filter_offset + info.filter_len]
        g = ctx.bloom_decode(fb, codec)
        o = ob.bloom_decode(fb, codec, cap=1 << 22)
        assert g[0] == o[0] == 0 and g[1:] == o[1:]
    return index, metas


@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("seed", range(2))
def test_open_random_sst(ctx, codec, seed):
    rng = random.Random(100 * codec + seed)
    kvs = bg.random_kvs(rng, rng.randint(50, 1500), alphabet=rng.choice([4, 256]))
    sst = sstgen.recode(sstgen.none_sst(kvs, rng.choice([256, 1024, 4096])), codec, rng)
    index, metas = _open_and_compare(ctx, sst, codec)
    # the point-read seek over the decoded index
    keys = [k for k, _ in rng.sample(kvs, min(50, len(kvs)))] + [rng.randbytes(rng.randint(0, 10)) for _ in range(50)]
    assert ctx.index_seek(index, keys).tolist() == [ob.index_seek([m[1] for m in metas], k) for k in keys]


@pytest.mark.parametrize("codec", CODECS)
def test_open_sst_large_index_and_filter(ctx, codec):
    """~6 k blocks of 256 bytes with 40-byte keys (index > 300 KiB decoded) and a ~50 KiB
    filter, so index, filter and blocks all go through payloads larger than any LDS stage."""
    rng = random.Random(7 + codec)
    n = 40_000
    kvs = [(b"key-%036d" % (i * 7), rng.randbytes(rng.randint(0, 24))) for i in range(n)]
    sst = sstgen.recode(sstgen.none_sst(kvs, 256), codec, rng)
    _, metas = _open_and_compare(ctx, sst, codec)
    assert len(metas) > 5000


@pytest.mark.parametrize("codec", CODECS)
def test_damaged_index_and_filter(ctx, codec):
    """Bytes of the compressed index / filter flipped (CRC recomputed so that decompression runs):
    DecodeIndex / bloom.Decode statuses equal the oracle's."""
    rng = random.Random(31 + codec)
    kvs = bg.random_kvs(rng, 800)
    sst = sstgen.recode(sstgen.none_sst(kvs, 512), codec, rng)
    _, oinfo = ob.sst_read_info(sst)
    ib = sst[oinfo["index_offset"]:oinfo["index_offset"] + oinfo["index_len"]]
    fb = sst[oinfo["filter_offset"]:oinfo["filter_offset"] + oinfo["filter_len"]]
    seen = set()
    for trial in range(60):
        src = ib if trial % 2 == 0 else fb
        body = bytearray(src[:-4])
        if trial % 5 == 4:
            body = body[:rng.randrange(1, len(body))]  # truncated payload
        else:
            for _ in range(rng.randint(1, 3)):
                body[rng.randrange(len(body))] ^= 1 << rng.randrange(8)
        buf = sstgen.crc(bytes(body))
        if trial % 2 == 0:
            st, _ = ctx.decode_index(buf, codec)
            ost, _ = ob.decode_index(buf, codec, cap=1 << 21)
        else:
            st = ctx.bloom_decode(buf, codec)[0]
            ost = ob.bloom_decode(buf, codec, cap=1 << 22)[0]
        assert st == ost, (trial, st, ost)
        seen.add(st)
    assert len(seen) >= 2
    # a damaged CRC is reported before any decompression
    bad = ib[:-1] + bytes([ib[-1] ^ 1])
    assert ctx.decode_index(bad, codec)[0] == ob.decode_index(bad, codec)[0] != 0


@pytest.mark.parametrize("codec", [ob.LZ4, ob.ZSTD, ob.ZLIB])
def test_split_payloads(ctx, codec):
    """Index and filter payloads of this builder's LZ4 / Zstd frames and Zlib streams (independent
    64 KiB pieces, more than 32 KiB: api_sst.cpp lz4_ / zstd_ / zlib_payload_split, one wave per piece)
    decoded like the oracle; damaged ones (flipped bytes under a valid CRC, a wrong content
    checksum, a wrong CRC) reach the serial path or the CRC check with the oracle's statuses."""
    import slatecodec as sc
    from tools.bench_encode import kv_arrays
    keys, key_off, vals, val_off = kv_arrays(1_200_000)
    b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
    assert b.add_batch(keys, key_off, vals, val_off) == 0
    sst = b.build().encode()
    st, info, _ = sc.read_info(sst)
    ib = sst[info.index_offset:info.index_offset + info.index_len]
    fb = sst[info.filter_offset:info.filter_offset + info.filter_len]
    assert len(ib) > 256 * 1024 and len(fb) > 512 * 1024  # many 64 KiB pieces each
    st, index = ctx.decode_index(ib, codec)
    ost, ometas = ob.decode_index(ib, codec, cap=1 << 24)
    assert st == ost == 0 and index.block_metas() == ometas
    g = ctx.bloom_decode(fb, codec)
    o = ob.bloom_decode(fb, codec, cap=1 << 24)
    assert g[0] == o[0] == 0 and g[1:] == o[1:]
    rng = random.Random(5)
    for trial in range(12):
        src = ib if trial % 2 == 0 else fb
        body = bytearray(src[:-4])
        if trial % 4 == 3:
            body[-1] ^= 0x10  # the content checksum
        else:
            for _ in range(rng.randint(1, 3)):
                body[rng.randrange(11, len(body) - 8)] ^= 1 << rng.randrange(8)
        buf = sstgen.crc(bytes(body))
        if trial % 2 == 0:
            st, _ = ctx.decode_index(buf, codec)
            ost, _ = ob.decode_index(buf, codec, cap=1 << 24)
        else:
            st = ctx.bloom_decode(buf, codec)[0]
            ost = ob.bloom_decode(buf, codec, cap=1 << 24)[0]
        assert st == ost, (trial, st, ost)
    bad = fb[:-1] + bytes([fb[-1] ^ 1])
    assert ctx.bloom_decode(bad, codec)[0] == ob.bloom_decode(bad, codec, cap=1 << 24)[0] != 0
