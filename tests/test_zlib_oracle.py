"""The oracle's zlib/inflate restatement (compress.Decode CodecZlib, compression.go:134-140)
checked against the zlib library (Python's zlib module) on streams of every deflate
strategy and level, plus the status codes of damaged streams.  CPU only."""
import random
import struct
import zlib

import pytest

from oracle import binding as ob

E_HEADER, E_DICT, E_CHECKSUM, E_CORRUPT, E_UNEXPECTED_EOF = 50, 51, 52, 53, 54
STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FILTERED]


def zstream(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, wbits=15, memlevel=8) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, wbits, memlevel, strategy)
    return co.compress(data) + co.flush()


@pytest.mark.parametrize("seed", range(6))
def test_zlib_library_streams(seed):
    rng = random.Random(seed)
    for _ in range(60):
        n = rng.choice([0, 1, 2, 50, 700, 4000, 40000, 70000])
        alpha = rng.choice([2, 4, 16, 256])
        data = bytes(rng.randrange(alpha) for _ in range(n))
        if rng.random() < 0.5:
            data = data[: n // 3] * 3
        c = zstream(data, rng.choice([0, 1, 6, 9]), rng.choice(STRATEGIES), rng.choice([9, 12, 15]),
                    rng.choice([1, 8, 9]))
        assert ob.zlib_decode(c) == (0, data)


def test_damaged_streams():
    data = b"".join(b"row-%05d:%s|" % (i, b"x" * (i % 13)) for i in range(600))
    c = zstream(data)
    assert ob.zlib_decode(c) == (0, data)
    assert ob.zlib_decode(bytes([0x79]) + c[1:])[0] == E_HEADER  # CINFO 7 kept, FCHECK broken
    assert ob.zlib_decode(bytes([0x89, 0x9c]) + c[2:])[0] == E_HEADER  # CINFO 8
    assert ob.zlib_decode(c[:-1] + bytes([c[-1] ^ 1]))[0] == E_CHECKSUM
    assert ob.zlib_decode(c[:-4])[0] == E_UNEXPECTED_EOF
    assert ob.zlib_decode(c[: len(c) // 2])[0] == E_UNEXPECTED_EOF
    assert ob.zlib_decode(c + b"trailing bytes are not read")[0] == 0
    # FDICT: dictionary id 1 (Adler-32 of no dictionary) passes, any other fails
    flg = 0x20 | 0x00
    cmf = 0x78
    flg += (31 - ((cmf << 8) | flg) % 31) % 31
    raw = c[2:]
    assert ob.zlib_decode(bytes([cmf, flg]) + struct.pack(">I", 1) + raw) == (0, data)
    assert ob.zlib_decode(bytes([cmf, flg]) + struct.pack(">I", 7) + raw)[0] == E_DICT
    # block type 3 and a stored block with a bad NLEN
    assert ob.zlib_decode(bytes([0x78, 0x9c, 0x07]))[0] == E_CORRUPT
    assert ob.zlib_decode(bytes([0x78, 0x9c, 0x01, 0x05, 0x00, 0x00, 0x00]) + b"abcde" + b"\0" * 4)[0] == E_CORRUPT
    rng = random.Random(3)
    seen = set()
    for _ in range(300):
        b = bytearray(c)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(2, len(b))] ^= 1 << rng.randrange(8)
        seen.add(ob.zlib_decode(bytes(b))[0])
    assert {E_CORRUPT, E_CHECKSUM} <= seen, seen
