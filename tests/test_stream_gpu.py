"""GPU parity for large single-stream Snappy payloads (an SST's bloom filter or index,
bloom.go:70-91, decode.go:83-100), which take the one-wave streaming decoder
(csrc/snappy_stream.hip) above 16 KiB decoded: filters and indexes from real builders, payloads
from the golang/snappy restatement, hand-made streams with literals longer than the input window
and copies reaching past the 64 KiB output ring, and damaged streams -- status and bytes
against the oracle."""
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import binding as ob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _lit(b: bytes) -> bytes:
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    nb = (n.bit_length() + 7) // 8
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + b


def _copy4(off: int, ln: int) -> bytes:  # tag type 3: 4-byte offset, len 1..64
    return bytes([((ln - 1) << 2) | 3]) + struct.pack("<I", off)


def _filter_buf(payload: bytes) -> bytes:
    """bloom.Encode layout around an arbitrary Snappy payload: payload || BE32 CRC."""
    return payload + struct.pack(">I", zlib.crc32(payload))


def _check(ctx, buf):
    g = ctx.bloom_decode(buf, ob.SNAPPY)
    o = ob.bloom_decode(buf, ob.SNAPPY)
    assert g[0] == o[0], (g[0], o[0])
    if o[0] == 0:
        assert g[1] == o[1] and g[2] == o[2]


@pytest.mark.parametrize("n_keys", [20_000, 300_000])
def test_real_filters(ctx, n_keys):
    keys = [b"k%015d" % i for i in range(n_keys)]
    npr, bits = ob.bloom_build(keys, 10)
    _check(ctx, ob.bloom_encode(npr, bits, ob.SNAPPY))


@pytest.mark.parametrize("seed", range(6))
def test_snappy_payloads(ctx, seed):
    rng = random.Random(seed)
    parts = []
    for _ in range(rng.randint(5, 40)):
        kind = rng.random()
        if kind < 0.4:
            parts.append(rng.randbytes(rng.randint(1, 9000)))
        elif kind < 0.8 and parts:
            parts.append(parts[rng.randrange(len(parts))][: rng.randint(1, 5000)])
        else:
            parts.append(bytes([rng.randrange(256)]) * rng.randint(1, 20000))
    raw = b"\x00\x06" + b"".join(parts)
    _check(ctx, _filter_buf(ob.snappy_encode(raw)))


def test_long_literal_and_far_copies(ctx):
    rng = random.Random(7)
    a = rng.randbytes(70_000)  # literal longer than the 32 KiB input window
    stream = _lit(b"\x00\x06" + a)
    d = 2 + len(a)
    stream += _copy4(69_000, 64) + _copy4(65_600, 33) + _copy4(3, 64) + _lit(rng.randbytes(100))
    d += 64 + 33 + 64 + 100
    _check(ctx, _filter_buf(_varint(d) + stream))


def test_damaged(ctx):
    rng = random.Random(3)
    keys = [b"k%015d" % i for i in range(40_000)]
    npr, bits = ob.bloom_build(keys, 10)
    good = ob.bloom_encode(npr, bits, ob.SNAPPY)
    payload = good[:-4]
    _check(ctx, good[:-1] + bytes([good[-1] ^ 1]))  # checksum
    for _ in range(25):
        p = bytearray(payload)
        for _ in range(rng.randint(1, 4)):
            i = rng.randrange(len(_varint(0)) + 2, len(p))
            p[i] = rng.randrange(256)
        _check(ctx, _filter_buf(bytes(p)))
    _check(ctx, _filter_buf(payload[: len(payload) // 2]))  # truncated
    _check(ctx, _filter_buf(_varint(40_000) + _lit(rng.randbytes(30_000)) + _copy4(40_000, 10)))  # offset > d


def test_large_index(ctx):
    import slatecodec as sc
    n = 150_000
    keys = np.zeros((n, 16), np.uint8)
    keys[:, 0] = ord("k")
    v = np.arange(n)
    for c in range(15, 0, -1):
        keys[:, c] = 48 + v % 10
        v //= 10
    vals = np.tile(np.frombuffer(b"v" * 84, np.uint8), n)
    b = sc.SstBuilder(ctx, 4096, 0, 10, sc.SNAPPY)
    assert b.add_batch(keys.reshape(-1), np.arange(n + 1, dtype=np.uint64) * 16, vals,
                       np.arange(n + 1, dtype=np.uint64) * 84) == 0
    sst = b.build().encode()
    st, info = ob.sst_read_info(sst)
    assert st == 0
    ib = sst[info["index_offset"]:info["index_offset"] + info["index_len"]]
    st, idx = ctx.decode_index(ib, sc.SNAPPY)
    assert st == 0
    ost, ometas = ob.decode_index(ib, ob.SNAPPY)
    assert ost == 0 and idx.block_metas() == ometas
    bad = bytearray(ib)
    bad[len(bad) // 3] ^= 0x40
    assert ctx.decode_index(bytes(bad), sc.SNAPPY)[0] == ob.decode_index(bytes(bad), ob.SNAPPY)[0]


@pytest.mark.parametrize("n", [65_536 * 2, 65_536 * 3 + 1, 65_536 * 5 - 7, 3_000_000])
def test_golang_framed_sizes(ctx, n):
    """golang/snappy-framed payloads (the tag-parallel path)
    at and around fragment multiples, mixing literals, near copies and runs."""
    rng = random.Random(n)
    parts, size = [], 0
    while size < n:
        k = rng.random()
        part = rng.randbytes(rng.randint(1, 3000)) if k < 0.4 else (
            bytes([rng.randrange(256)]) * rng.randint(1, 5000) if k < 0.6 else
            (parts[rng.randrange(len(parts))][:rng.randint(1, 2000)] if parts else b"x"))
        parts.append(part)
        size += len(part)
    raw = (b"\x00\x06" + b"".join(parts))[:n]
    _check(ctx, _filter_buf(ob.snappy_encode(raw)))


def test_fragment_boundary_streams(ctx):
    """Valid streams not split golang's way (copies across 64 KiB pieces, a literal across one): a copy
    at a 64 KiB boundary reaching into the previous fragment, and a literal across a boundary."""
    rng = random.Random(11)
    a = b"\x00\x06" + rng.randbytes(65_534)
    s1 = _lit(a[:60_000]) + _lit(a[60_000:]) + _copy4(1000, 64) + _lit(rng.randbytes(5000))
    _check(ctx, _filter_buf(_varint(65_536 + 64 + 5000) + s1))
    s2 = _lit(a[:30_000]) + _lit(a[30_000:] + rng.randbytes(40_000)) + _copy4(7, 20)
    _check(ctx, _filter_buf(_varint(65_536 + 40_000 + 20) + s2))
    # damage inside the third fragment of a golang-framed stream
    raw = b"\x00\x06" + b"".join(rng.randbytes(300) * 3 for _ in range(300))
    enc = bytearray(ob.snappy_encode(raw))
    for pos in (len(enc) * 2 // 3, len(enc) - 10):
        bad = bytearray(enc)
        bad[pos] ^= 0x3C
        _check(ctx, _filter_buf(bytes(bad)))
