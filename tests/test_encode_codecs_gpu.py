"""GPU encode for CodecLz4 / CodecZlib / CodecZstd (compress.Encode, compression.go:80-116) through
the C-ABI: block.Encode (block.go:54-75), bloom.Encode (bloom.go:52-67) and whole SSTs from the
builder (builder.go:92-268).  The reference's encoders (pierrec/lz4 v4, compress/zlib,
klauspost/compress/zstd) are absent, so their bytes are parity unpinned; what is checked is what
the readers need: every frame decodes -- with the oracle's restatements of the reference readers,
with the GPU decoders, and with the codec's own library (zlib, libzstd, liblz4) -- to the input,
payload sizes around the 64 KiB pieces included, and an SST built with the codec holds the same
blocks, first keys and filter as the CodecNone SST of the same KVs."""
import ctypes as C
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tests import zstdgen

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not zstdgen.available(), reason="libzstd not in this image")]
CODECS = [ob.LZ4, ob.ZLIB, ob.ZSTD]


@pytest.fixture(scope="module")
def sc():
    import slatecodec
    return slatecodec


@pytest.fixture(scope="module")
def ctx(sc):
    return sc.Context(0)


def _lz4_lib_decode(frame: bytes, n: int) -> bytes:
    """liblz4's frame decoder (LZ4F_decompress), an independent reader."""
    L = C.CDLL("liblz4.so.1")
    L.LZ4F_createDecompressionContext.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    L.LZ4F_decompress.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p, C.POINTER(C.c_size_t),
                                  C.c_void_p]
    L.LZ4F_decompress.restype = C.c_size_t
    L.LZ4F_isError.argtypes = [C.c_size_t]
    L.LZ4F_freeDecompressionContext.argtypes = [C.c_void_p]
    dctx = C.c_void_p()
    assert L.LZ4F_createDecompressionContext(C.byref(dctx), 100) == 0
    out = C.create_string_buffer(n + 64)
    src = C.create_string_buffer(frame, len(frame))
    got, pos = b"", 0
    while pos < len(frame):
        dst_n = C.c_size_t(len(out))
        src_n = C.c_size_t(len(frame) - pos)
        r = L.LZ4F_decompress(dctx, out, C.byref(dst_n), C.byref(src, pos), C.byref(src_n), None)
        assert not L.LZ4F_isError(r), "liblz4 rejected the frame"
        got += out.raw[:dst_n.value]
        pos += src_n.value
        if r == 0:
            break
    L.LZ4F_freeDecompressionContext(dctx)
    assert pos == len(frame)
    return got


def _lib_decode(codec: int, frame: bytes, n: int) -> bytes:
    if codec == ob.ZLIB:
        return zlib.decompress(frame)
    if codec == ob.ZSTD:
        L = zstdgen.lib()
        out = C.create_string_buffer(n + 64)
        r = L.ZSTD_decompress(out, len(out), frame, len(frame))
        assert not L.ZSTD_isError(r), L.ZSTD_getErrorName(r)
        return out.raw[:r]
    return _lz4_lib_decode(frame, n)


def _payloads(rng):
    out = [b"", b"\x00", bytes(range(12)), bytes(13), rng.randbytes(100)]
    for n in (4096, 65535, 65536, 65537, 200_000):
        out.append(rng.randbytes(n))  # incompressible: raw / stored forms
        half = rng.randbytes(n // 2)
        out.append((half + half + b"x")[:n])  # one long match
        out.append(bytes(rng.choice(b"ab") for _ in range(min(n, 9000))) * (n // min(n, 9000) + 1))
    out.append(b"".join(b"k%015d" % i + struct.pack(">Q", i * 4096) for i in range(20_000)))  # index-like
    return out


@pytest.mark.parametrize("codec", CODECS)
def test_filter_payloads_round_trip(sc, ctx, codec):
    """bloom.Encode framing around arbitrary payloads (the BE16 probe count + bits): decoded by
    the oracle, the GPU and the codec's library."""
    rng = random.Random(codec)
    for i, pl in enumerate(_payloads(rng)):
        npr, bits = 7, pl
        st, enc = ctx.bloom_encode(npr, bits, codec)
        assert st == 0, (i, st)
        frame = enc[:-4]
        assert struct.unpack(">I", enc[-4:])[0] == zlib.crc32(frame)
        raw = struct.pack(">H", npr) + bits
        assert _lib_decode(codec, frame, len(raw)) == raw, i
        ost, onp, obits = ob.bloom_decode(enc, codec, cap=len(raw) + 64)
        assert (ost, onp, obits) == (0, npr, bits), i
        g = ctx.bloom_decode(enc, codec)
        assert g == (0, npr, bits), i


@pytest.mark.parametrize("codec", CODECS)
def test_block_encode_round_trip(sc, ctx, codec):
    """block.Encode of random blocks: decoded by the oracle's block.Decode and the GPU batch."""
    rng = random.Random(10 + codec)
    blocks = []
    for _ in range(40):
        kvs = bg.random_kvs(rng, rng.randint(1, 60), alphabet=rng.choice([4, 256]))
        bb = ob.BlockBuilder(rng.choice([512, 4096, 65536]))
        for k, v in kvs:
            if not bb.add_value(k, v):
                break
        data, offs, _ = bb.build()
        st, enc = ctx.block_encode(data, offs, codec)
        assert st == 0
        m, dec, rows = ob.block_decode(enc, codec)
        assert int(m["status"]) == 0
        assert dec[:int(m["data_len"])] == data
        blocks.append(enc)
    blob, off = bg.pack(blocks, misalign=3)
    g_out, g_off, g_meta, _, _ = ctx.decode_batch(codec, blob, off)
    o_out, o_off, o_meta, _, _ = ob.block_decode_batch(codec, blob, off)
    assert g_meta.tobytes() == o_meta.tobytes() and (o_meta["status"] == 0).all()


@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("seed", range(2))
def test_sst_with_codec(sc, ctx, codec, seed):
    """An SST built with the codec: the same blocks (decoded), first keys and filter bits as the
    CodecNone SST of the same KVs, its index and filter decoded by the oracle and the GPU."""
    rng = random.Random(100 * codec + seed)
    kvs = bg.random_kvs(rng, rng.randint(200, 3000), alphabet=rng.choice([4, 256]))
    bs = rng.choice([256, 4096])
    ssts = {}
    for c in (ob.NONE, codec):
        b = sc.SstBuilder(ctx, bs, 0, 10, c)
        for k, v in kvs:
            assert b.add_value(k, v) == 0
        ssts[c] = b.build().encode()
    st, info_n = ob.sst_read_info(ssts[ob.NONE])
    st2, info_c = ob.sst_read_info(ssts[codec])
    assert st == st2 == 0 and info_c["codec"] == codec and info_c["first_key"] == info_n["first_key"]
    sn, sx = ssts[ob.NONE], ssts[codec]
    st, metas_n = ob.decode_index(sn[info_n["index_offset"]:info_n["index_offset"] + info_n["index_len"]], ob.NONE)
    st2, metas_c = ob.decode_index(sx[info_c["index_offset"]:info_c["index_offset"] + info_c["index_len"]], codec,
                                   cap=1 << 22)
    assert st == st2 == 0 and [k for _, k in metas_n] == [k for _, k in metas_c]
    # every block decodes to the CodecNone block's bytes
    def blocks(sst, info, metas):
        end = info["filter_offset"] if info["filter_len"] else info["index_offset"]
        return [sst[o:(metas[i + 1][0] if i + 1 < len(metas) else end)] for i, (o, _) in enumerate(metas)]
    for bn, bc in zip(blocks(sn, info_n, metas_n), blocks(sx, info_c, metas_c)):
        mn, dn, _ = ob.block_decode(bn, ob.NONE)
        mc, dc, _ = ob.block_decode(bc, codec)
        assert int(mc["status"]) == 0 and dc[:int(mc["data_len"])] == dn[:int(mn["data_len"])]
    fn = sn[info_n["filter_offset"]:info_n["filter_offset"] + info_n["filter_len"]]
    fc = sx[info_c["filter_offset"]:info_c["filter_offset"] + info_c["filter_len"]]
    assert ob.bloom_decode(fc, codec, cap=1 << 22) == ob.bloom_decode(fn, ob.NONE)
    # and the GPU reader opens it
    gst, ginfo, gfk = sc.read_info(sx)
    assert gst == 0
    gst, gindex = ctx.decode_index(sx[ginfo.index_offset:ginfo.index_offset + ginfo.index_len], codec)
    assert gst == 0 and gindex.block_metas() == metas_c
    gst, failed, _ = ctx.read_blocks(ginfo, gindex, 0, len(metas_c), sx)
    assert gst == 0 and failed == 2**64 - 1


@pytest.mark.parametrize("codec", CODECS)
def test_vhalf_blocks_compress(sc, ctx, codec):
    """V-half blocks come out smaller than CodecNone's, and large SSTs (index and
    filter above 64 KiB: several pieces) round-trip."""
    kvs = bg.kv_synthetic(60_000)
    sizes = {}
    for c in (ob.NONE, codec):
        b = sc.SstBuilder(ctx, 4096, 0, 10, c)
        for k, v in kvs:
            assert b.add_value(k, v) == 0
        sizes[c] = b.build().encode()
    assert len(sizes[codec]) < 0.8 * len(sizes[ob.NONE])
    st, info = ob.sst_read_info(sizes[codec])
    ib = sizes[codec][info["index_offset"]:info["index_offset"] + info["index_len"]]
    st, metas = ob.decode_index(ib, codec, cap=1 << 23)
    assert st == 0 and len(metas) > 1000
    fb = sizes[codec][info["filter_offset"]:info["filter_offset"] + info["filter_len"]]
    assert ob.bloom_decode(fb, codec, cap=1 << 23)[0] == 0


@pytest.mark.parametrize("codec", [ob.ZLIB, ob.ZSTD])
def test_vhalf_block_ratio(sc, ctx, codec):
    """configs[1]-shaped blocks (100-byte V-half KVs, 4 KiB): block.Encode's Zlib bodies (a hash-chain
    parse with dynamic Huffman codes) and Zstd bodies (repeat offsets, FSE_Compressed tables) come
    within 2 % of the library each Go writer stands for (zlib level 6 + Go's 5-byte final block;
    libzstd level 3), and every one decodes to its block (oracle and the library)."""
    kvs = bg.kv_synthetic(38 * 120)
    ours = lib = 0
    bb = None
    blocks = []
    for k, v in kvs:
        if bb is None:
            bb = ob.BlockBuilder(4096)
        if not bb.add_value(k, v):
            blocks.append(bb.build()[:2])
            bb = ob.BlockBuilder(4096)
            assert bb.add_value(k, v)
    for data, offs in blocks:
        st, enc = ctx.block_encode(data, offs, codec)
        assert st == 0
        m, dec, _ = ob.block_decode(enc, codec)
        assert int(m["status"]) == 0 and dec[:int(m["data_len"])] == data
        frame = enc[:-4]
        raw = bytes(dec[:len(dec)])
        raw = raw[:int(m["data_len"]) + 2 * len(offs) + 2]
        assert _lib_decode(codec, frame, len(raw)) == raw
        ours += len(frame)
        lib += len(zlib.compress(raw, 6)) + 5 if codec == ob.ZLIB else len(zstdgen.frame(raw, 3, True, True))
    assert ours <= 1.02 * lib, (ours, lib, ours / lib)
