"""SSTs of every codec for the reader tests (test infrastructure).

The oracle's builder writes None and Snappy SSTs (compress.Encode's other codecs are not on the
GPU write path); an LZ4 / Zlib / Zstd SST is made by re-encoding a CodecNone SST piece by piece
the way sstable.Builder would have (builder.go:92-268): each block payload, the filter and the
index flatbuffer compressed by the codec's reference library (liblz4-format frames from
tests/lz4gen, zlib 1.2.11, libzstd 1.4.8), then `|| BE32 CRC32`, the info re-encoded with the
new offsets and codec (flatbuf.go:62-81), and the info offset last."""
import random
import struct
import zlib

from oracle import binding as ob
from tests import lz4gen, zstdgen


def compress(codec: int, data: bytes, rng: random.Random) -> bytes:
    if codec == ob.NONE:
        return data
    if codec == ob.SNAPPY:
        return ob.snappy_encode(data)
    if codec == ob.ZSTD:
        return zstdgen.frame(data, level=rng.choice([-1, 1, 3, 9, 19]), checksum=rng.random() < 0.5,
                             content_size=rng.random() < 0.7)
    if codec == ob.LZ4:
        return lz4gen.frame(data, bsid=rng.choice([4, 5, 6, 7]), indep=rng.random() < 0.5,
                            block_checksum=rng.random() < 0.3, content_checksum=rng.random() < 0.5,
                            content_size=rng.random() < 0.3, rng=rng)
    if codec == ob.ZLIB:
        return zlib.compress(data, rng.choice([1, 6, 9]))
    raise ValueError(codec)


def crc(body: bytes) -> bytes:
    return body + struct.pack(">I", zlib.crc32(body))


def go_zlib(raw: bytes, level: int = 6) -> bytes:
    """A zlib stream in the shape Go's compress/zlib writer closes with: the data's (non-final)
    deflate blocks, then an empty FINAL stored block (compress/flate deflate.go close ->
    huffmanBitWriter.writeStoredHeader(0, true): bytes ..01 00 00 FF FF), then the Adler-32.
    Built from zlib's sync flush, whose empty non-final stored block is made final by setting its
    BFINAL bit (the one bit flip after which a raw inflater ends there with the same bytes).  Go's
    own block splitting is not reproduced (parity for it is unpinned)."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(raw) + c.flush(zlib.Z_SYNC_FLUSH)
    assert body.endswith(b"\x00\x00\xff\xff")
    for pos in (len(body) - 5, len(body) - 6):
        for bit in range(8):
            t = bytearray(body)
            t[pos] ^= 1 << bit
            d = zlib.decompressobj(-15)
            try:
                out = d.decompress(bytes(t))
            except zlib.error:
                continue
            if d.eof and out == raw and not d.unused_data:
                return b"\x78\x9c" + bytes(t) + struct.pack(">I", zlib.adler32(raw))
    raise AssertionError("no BFINAL bit found")


def recode(sst_none: bytes, codec: int, rng: random.Random) -> bytes:
    """The CodecNone SST `sst_none` re-encoded with `codec` (same keys, blocks and filter bits)."""
    st, info = ob.sst_read_info(sst_none)
    assert st == 0 and info["codec"] == ob.NONE
    io, il, fo, fl = info["index_offset"], info["index_len"], info["filter_offset"], info["filter_len"]
    st, metas = ob.decode_index(sst_none[io:io + il], ob.NONE)
    assert st == 0
    blocks_end = fo if fl else io
    out = bytearray()
    new_metas = []
    for i, (off, fk) in enumerate(metas):
        end = metas[i + 1][0] if i + 1 < len(metas) else blocks_end
        payload = sst_none[off:end][:-4]
        new_metas.append((len(out), fk))
        out += crc(compress(codec, payload, rng))
    f_off, f_len = 0, 0
    if fl:
        assert fo == blocks_end and io == fo + fl
        filt = crc(compress(codec, sst_none[fo:fo + fl][:-4], rng))
        f_off, f_len = len(out), len(filt)
        out += filt
    index = crc(compress(codec, ob.encode_index(new_metas, ob.NONE)[:-4], rng))
    i_off = len(out)
    out += index
    info_b = ob.encode_info(info["first_key"] if info["first_key_len"] else None, i_off, len(index), f_off, f_len,
                            codec)
    info_off = len(out)
    out += info_b + struct.pack(">I", info_off)
    return bytes(out)


def none_sst(kvs, block_size=4096, min_filter_keys=0, bits_per_key=10) -> bytes:
    b = ob.SstBuilder(block_size, min_filter_keys, bits_per_key, ob.NONE)
    for k, v in kvs:
        assert b.add(k, v) == 0
    assert b.build() == 0
    return b.encode_table()
