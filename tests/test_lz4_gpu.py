"""GPU parity for CodecLz4 blocks (compress.Decode, compression.go:143-144) through the C ABI:
block.Decode with LZ4 frames - every frame option, liblz4-written frames, and damaged frames
with their status codes - bit-exact against the oracle (plan, meta, decoded bytes, rows)."""
import json
import os
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tests import lz4gen

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _crc(frame: bytes) -> bytes:
    return frame + struct.pack(">I", zlib.crc32(frame))


def _compare(ctx, blocks, misalign=0):
    blob, off = bg.pack(blocks, misalign)
    g_out, g_off, g_meta, g_rows, g_rb = ctx.decode_batch(ob.LZ4, blob, off)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.LZ4, blob, off)
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i, blk in enumerate(blocks):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om)
        st = int(om["status"])
        if st == 0 or 3 <= st <= 7:
            dec = ob.lz4_decode(blk[:-4])[1]
            a = int(o_off[i])
            assert g_out[a:a + len(dec)].tobytes() == dec == o_out[a:a + len(dec)].tobytes(), i
        if st == 0:
            r0 = int(o_rb[i])
            nr = min(int(om["n_rows"]), int(o_rb[i + 1]) - r0)
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i
    return o_meta


def _sst_plain(rng, n_kv, block_size):
    kvs = bg.random_kvs(rng, n_kv, alphabet=rng.choice([4, 256]))
    return [b[:-4] for b in bg.sst_blocks(kvs, block_size, ob.NONE)]  # decoded blocks


@pytest.mark.parametrize("seed", range(4))
def test_random_lz4_ssts(ctx, seed):
    rng = random.Random(seed)
    blocks = []
    for dec in _sst_plain(rng, rng.randint(300, 1500), rng.choice([512, 4096])):
        blocks.append(_crc(lz4gen.frame(dec, bsid=rng.choice([4, 7]), indep=rng.random() < 0.7,
                                        block_checksum=rng.random() < 0.3, content_checksum=rng.random() < 0.8,
                                        content_size=rng.random() < 0.3, stored_p=0.1, rng=rng,
                                        block_split=rng.choice([None, None, 700]))))
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


def test_vhalf_lz4_blocks(ctx):
    kvs = bg.kv_synthetic(38 * 200, half=True, tomb_every=25)
    rng = random.Random(5)
    blocks = [_crc(lz4gen.frame(b[:-4], rng=rng)) for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    meta = _compare(ctx, blocks, misalign=7)
    assert (meta["status"] == 0).all()


def test_liblz4_frames(ctx):
    cases = json.load(open(os.path.join(GOLDEN, "lz4_frames.json")))["cases"]
    blocks = [_crc(bytes.fromhex(c["frame"])) for c in cases]
    _compare(ctx, blocks, misalign=3)


def test_damaged_lz4_blocks(ctx):
    rng = random.Random(9)
    decs = _sst_plain(rng, 800, 1024)
    blocks = []
    for dec in decs:
        f = bytearray(lz4gen.frame(dec, bsid=4, block_checksum=rng.random() < 0.5,
                                   content_checksum=rng.random() < 0.7, rng=rng, block_split=300))
        kind = rng.randrange(6)
        if kind == 0:
            f[rng.randrange(len(f))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            f = f[: rng.randrange(len(f))]
        elif kind == 2:
            f += bytes(rng.randrange(256) for _ in range(rng.randint(1, 5)))
        elif kind == 3:
            i = rng.randrange(7, len(f))
            f[i:i + 2] = bytes([rng.randrange(256), rng.randrange(256)])
        elif kind == 4:
            f[4] ^= rng.choice([1, 2, 8, 0x80])
        blocks.append(_crc(bytes(f)))
    meta = _compare(ctx, blocks, misalign=1)
    st = set(int(x) for x in meta["status"])
    assert {0, 18} <= st, st


def _recrc(block: bytes) -> bytes:
    return _crc(block[:-4])


def test_lz4_fast_path_shapes(ctx):
    """The lane-per-block path (one-block frames: decode_lpb2.hip lz4_parse) and its hand-backs to
    the exact path: every alignment, content size / checksum options, literal and match length
    extensions inside and beyond the 8-byte window, far and overlapping matches, damaged content
    checksums under a valid CRC, multi-block frames and trailing bytes."""
    rng = random.Random(11)
    kvs = bg.kv_synthetic(38 * 64, half=True, tomb_every=9)
    plain = [b[:-4] for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    blocks = []
    for i, dec in enumerate(plain):
        blocks.append(_crc(lz4gen.frame(dec, content_size=i % 3 == 0, content_checksum=i % 4 != 1, rng=rng)))
    # long literal runs (1, 2 and 7+ extension bytes) and long matches (several extension bytes)
    for n_lit in (20, 300, 700, 1600, 2200):
        kv = [(b"key%06d" % j, bytes(rng.randrange(256) for _ in range(n_lit)) + b"x" * 600) for j in range(3)]
        for dec in (b[:-4] for b in bg.sst_blocks(kv, 1 << 16, ob.NONE)):
            blocks.append(_crc(lz4gen.frame(dec, rng=rng)))
    # damaged content checksums and flipped literal bytes under a valid CRC -> LZ4_FRAME_CHECKSUM
    for dec in plain[:6]:
        f = bytearray(lz4gen.frame(dec, rng=rng))
        f[-1] ^= 0x40
        blocks.append(_crc(bytes(f)))
        g = bytearray(lz4gen.frame(dec, rng=rng))
        g[40] ^= 0x01  # inside the first literal run (the header is 7 + 4 bytes)
        blocks.append(_crc(bytes(g)))
    # shapes the lane path hands back: two data blocks, trailing bytes, stored, block checksums
    for dec in plain[6:10]:
        blocks.append(_crc(lz4gen.frame(dec, block_split=1500, rng=rng)))
        blocks.append(_crc(lz4gen.frame(dec, rng=rng) + b"\x00\x01"))
        blocks.append(_crc(lz4gen.frame(dec, stored_p=1.0, rng=rng)))
        blocks.append(_crc(lz4gen.frame(dec, block_checksum=True, rng=rng)))
    # structural damage under a valid CRC in one-block frames: the lane plan's and the lane
    # decoder's checks (truncation, flipped bytes in tokens / offsets / lengths, trailing bytes)
    for dec in plain[10:50]:
        f = bytearray(lz4gen.frame(dec, content_checksum=rng.random() < 0.5, rng=rng))
        kind = rng.randrange(4)
        if kind == 0:
            f = f[: rng.randrange(7, len(f))]
        elif kind == 1:
            i = rng.randrange(11, len(f) - 8)
            f[i] ^= 1 << rng.randrange(8)
        elif kind == 2:
            i = rng.randrange(11, len(f) - 10)
            f[i:i + 2] = bytes([rng.randrange(256), rng.randrange(256)])
        else:
            f[7:11] = struct.pack("<I", struct.unpack("<I", bytes(f[7:11]))[0] + rng.choice([-3, -1, 1, 2]))
        blocks.append(_crc(bytes(f)))
    for mis in (0, 5, 13):
        meta = _compare(ctx, blocks, misalign=mis)
        st = [int(x) for x in meta["status"]]
        assert st.count(0) >= len(plain) + 5, st
        assert 18 in st or 17 in st, st  # the damaged content checksums
