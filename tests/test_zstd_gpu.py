"""GPU parity for CodecZstd blocks (compress.Decode, compression.go:146-153) through the C ABI:
block.Decode with Zstandard frames written by libzstd 1.4.9 (every level band and strategy,
raw/RLE/compressed blocks, 1- and 4-stream Huffman literals, FSE/RLE/predefined/repeat tables,
with and without content size and checksum, multi-block and concatenated frames), plus damaged
frames with their status codes, bit-exact against the oracle (plan, meta, decoded bytes,
rows).  tests/test_zstd_oracle.py pins the oracle to libzstd."""
import random
import struct
import zlib

import numpy as np
import pytest

from tests import zstdgen

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not zstdgen.available(), reason="libzstd not in this image")]
LEVELS = [-5, -1, 1, 3, 6, 12, 19]


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _crc(stream: bytes) -> bytes:
    return stream + struct.pack(">I", zlib.crc32(stream))


def _z(data: bytes, level=3, checksum=True, content_size=True, window_log=0, strategy=0) -> bytes:
    return zstdgen.frame(data, level, checksum, content_size, window_log, strategy)


def _compare(ctx, blocks, misalign=0):
    blob, off = bg.pack(blocks, misalign)
    g_out, g_off, g_meta, g_rows, g_rb = ctx.decode_batch(ob.ZSTD, blob, off)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.ZSTD, blob, off)
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i, blk in enumerate(blocks):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om)
        st = int(om["status"])
        if st == 0 or 3 <= st <= 7:
            dec = ob.zstd_decode(blk[:-4])[1]
            a = int(o_off[i])
            assert g_out[a:a + len(dec)].tobytes() == dec == o_out[a:a + len(dec)].tobytes(), i
        if st == 0:
            r0 = int(o_rb[i])
            nr = min(int(om["n_rows"]), int(o_rb[i + 1]) - r0)
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i
    return o_meta


def _sst_plain(rng, n_kv, block_size):
    kvs = bg.random_kvs(rng, n_kv, alphabet=rng.choice([4, 256]))
    return [b[:-4] for b in bg.sst_blocks(kvs, block_size, ob.NONE)]


@pytest.mark.parametrize("seed", range(4))
def test_random_zstd_ssts(ctx, seed):
    rng = random.Random(seed)
    blocks = [_crc(_z(dec, rng.choice(LEVELS), rng.random() < 0.7, rng.random() < 0.7, rng.choice([0, 0, 10]),
                      rng.choice([0, 0, 1, 5, 9])))
              for dec in _sst_plain(rng, rng.randint(300, 1500), rng.choice([512, 4096]))]
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


def test_mixed_config_blocks(ctx):
    """BASELINE configs[4]: 4 KiB blocks of 1 KiB V-half values and Zipf-prefixed 8-256 B keys, level 3 + checksum."""
    kvs = bg.kv_mixed(2000)
    blocks = [_crc(_z(b[:-4], 3, True)) for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    meta = _compare(ctx, blocks, misalign=7)
    assert (meta["status"] == 0).all()


def test_large_and_concatenated_zstd_blocks(ctx):
    """Blocks beyond the fast kernel's LDS budget (large-block kernel), multi-block frames
    (small windows), concatenated and skippable frames."""
    rng = random.Random(11)
    blocks = [_crc(_z(dec, rng.choice([1, 3, 19]), True, rng.random() < 0.5, rng.choice([0, 10])))
              for dec in _sst_plain(rng, 2500, 40000)]
    decs = _sst_plain(rng, 400, 1024)
    cat = b"".join(_z(d, rng.choice([1, 3]), rng.random() < 0.5, rng.random() < 0.5) for d in decs[:3])
    blocks.append(_crc(cat[:0] + struct.pack("<II", 0x184D2A53, 3) + b"xyz" + cat))
    _compare(ctx, blocks, misalign=5)


def test_fast_path_shapes_and_checksums(ctx):
    """Blocks of the fast path's shape (one frame, one compressed block, raw literals, predefined
    tables: zstd_fast.hip) mixed with ones it hands to the exact path, with: a wrong SST CRC32
    (phase C's first check), a flipped literal byte with the CRC32 recomputed (the frame's
    XXH64 no longer matches), frames without checksum or content size, RLE literals, and
    blocks at every input alignment."""
    rng = random.Random(5)
    kvs = bg.kv_mixed(600)
    decs = [b[:-4] for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    blocks = []
    for i, dec in enumerate(decs * 3):
        f = bytearray(_z(dec, 3, checksum=i % 5 != 1, content_size=i % 7 != 2))
        kind = i % 6
        if kind == 3:  # literal byte flipped (raw literals start right after the headers)
            f[len(f) // 3] ^= 0x10
        blk = bytearray(_crc(bytes(f)))
        if kind == 4:
            blk[-1] ^= 0x01  # stored CRC32 wrong
        blocks.append(bytes(blk))
    blocks.append(_crc(_z(bytes(4000), 3)))  # RLE-heavy
    blocks.append(_crc(_z(b"k" * 10 + bytes(range(256)) * 12, 3)))
    meta = _compare(ctx, blocks, misalign=3)
    st = set(int(x) for x in meta["status"])
    assert 0 in st and 2 in st, st


def test_damaged_zstd_blocks(ctx):
    rng = random.Random(9)
    decs = _sst_plain(rng, 800, 1024)
    blocks = []
    for dec in decs:
        f = bytearray(_z(dec, rng.choice([1, 3, 9]), rng.random() < 0.8, rng.random() < 0.8))
        kind = rng.randrange(6)
        if kind == 0:
            f[rng.randrange(len(f))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            f = f[: rng.randrange(len(f))]
        elif kind == 2:
            f += bytes(rng.randrange(256) for _ in range(rng.randint(1, 5)))
        elif kind == 3:
            i = rng.randrange(4, len(f))
            f[i:i + 2] = bytes([rng.randrange(256), rng.randrange(256)])
        elif kind == 4:
            f[4] ^= rng.choice([1, 2, 8, 0x20, 0x80])
        blocks.append(_crc(bytes(f)))
    blocks += [_crc(b""), _crc(b"\x28\xb5"), _crc(b"\x28\xb5\x2f\xfd"), _crc(b"\x28\xb5\x2f\xfd\x00\x00\x07\x00\x00")]
    meta = _compare(ctx, blocks, misalign=1)
    st = set(int(x) for x in meta["status"])
    assert {0, 58} <= st, st


@pytest.mark.parametrize("misalign", [0, 1, 4, 7, 13, 15])
def test_fast_path_crc_every_length(ctx, misalign):
    """The fast path's SST CRC32 (one wave per block, zs_crc_wave_kernel): frames of every
    compressed length mod 16 from 1 to ~4.6 KiB at this input alignment; a third keep a stale
    stored CRC after one byte is flipped near the start, middle or end of the frame, and some
    have the stored CRC itself wrong."""
    rng = random.Random(100 + misalign)
    kvs = bg.kv_mixed(700)
    decs = [b[:-4] for b in bg.sst_blocks(kvs, rng.choice([1024, 4096]), ob.NONE)]
    blocks = []
    for i in range(96):
        dec = decs[i % len(decs)]
        dec = dec if i % 6 == 0 else dec[: rng.randint(16, len(dec))]  # prefixes: row checks fail, CRC still counts
        f = _z(dec, rng.choice([1, 3]), checksum=rng.random() < 0.8)
        blk = bytearray(_crc(f))
        kind = i % 6
        if kind in (1, 2, 3):
            pos = {1: rng.randrange(min(16, len(f))), 2: len(f) // 2, 3: len(f) - 1 - rng.randrange(min(16, len(f)))}[kind]
            blk[pos] ^= 1 << rng.randrange(8)
        elif kind == 4:
            blk[-1 - rng.randrange(4)] ^= 0x40
        blocks.append(bytes(blk))
    meta = _compare(ctx, blocks, misalign=misalign)
    st = [int(x) for x in meta["status"]]
    assert [i for i, x in enumerate(st) if x == 2] == [i for i in range(96) if i % 6 in (1, 2, 3, 4)], st
    assert st.count(0) >= 10, st


def _kv100_blocks(n_kv, seed=20250307):
    """configs[1]'s block shape: 16-byte keys, 84-byte V-half values, 4 KiB blocks, CodecNone bodies."""
    kvs = bg.kv_synthetic(n_kv, seed=seed, half=True)
    return [b[:-4] for b in bg.sst_blocks(kvs, 4096, ob.NONE)]


@pytest.mark.parametrize("level", [1, 3, 6, 9, 19])
def test_kv100_fse_table_blocks(ctx, level):
    """4 KiB blocks of 100-byte KVs through libzstd: ~112 sequences and FSE_Compressed LL / OF / ML
    tables per block (zstd_fast.hip phase A', the lane-per-block FSE parse), at every input alignment,
    with and without checksum and content size; bit-exact against the oracle, and (level 3, the
    reference writer's default class) no block handed to the exact path."""
    bodies = _kv100_blocks(38 * 96)
    for misalign in range(16):
        chk, fcs = misalign % 3 != 1, misalign % 4 != 2
        blocks = [_crc(_z(d, level, chk, fcs)) for d in bodies[misalign * 6:misalign * 6 + 12]]
        ctx.handbacks(reset=True)
        meta = _compare(ctx, blocks, misalign=misalign)
        assert (meta["status"] == 0).all()
        if level == 3:
            assert ctx.handbacks() == 0, misalign


def test_kv100_fse_damaged(ctx):
    """The same frames with one byte of the sequences section (table descriptions or bitstream) or
    of the literals flipped under a re-sealed CRC, or a stale CRC: every status and byte is the
    exact path's (the FSE parse hands back whatever fails a check)."""
    rng = random.Random(5)
    bodies = _kv100_blocks(38 * 40)
    blocks = []
    for d in bodies:
        f = bytearray(_z(d, 3, True, True))
        kind = rng.randrange(4)
        if kind == 0:  # the sequences section (the frame's last ~150 bytes before the checksum)
            f[len(f) - 4 - rng.randrange(1, 150)] ^= 1 << rng.randrange(8)
        elif kind == 1:  # a literal byte (XXH64 mismatch -> exact path)
            f[rng.randrange(20, 200)] ^= 0x40
        elif kind == 2:  # the checksum itself
            f[-1] ^= 1
        blk = _crc(bytes(f))
        if kind == 3:  # stale CRC
            blk = blk[:-1] + bytes([blk[-1] ^ 0xFF])
        blocks.append(blk)
    _compare(ctx, blocks, misalign=3)


def test_kv100_fse_large_batch(ctx):
    """A few thousand configs[1]-shaped Zstd blocks in one batch: phase A' over many rounds."""
    bodies = _kv100_blocks(38 * 3000, seed=7)
    blocks = [_crc(_z(d, 3, True, True)) for d in bodies]
    ctx.handbacks(reset=True)
    meta = _compare(ctx, blocks, misalign=9)
    assert (meta["status"] == 0).all()
    assert ctx.handbacks() == 0


def _short_sequences(rng, n):
    """Bytes of many short literal runs and matches of every length 3..140 (long FSE table
    descriptions and long sequence bitstreams)."""
    out = bytearray(rng.randbytes(64))
    while len(out) < n:
        out += rng.randbytes(rng.choice([0, 1, 2, 3, 5, 8, 13, 21, 34]))
        m, o = rng.randint(3, 140), rng.randint(1, min(len(out), 2000))
        s = len(out) - o
        for i in range(m):
            out.append(out[s + i])
    return bytes(out[:n])


@pytest.mark.parametrize("misalign", [0, 6, 11, 15])
def test_fse_window_limits(ctx, misalign):
    """Phase A''s LDS window (zstd_fast.hip zs_fse_parse_kernel: the table descriptions within the 4
    chunks from the sequences section's first, the bitstream within the 10 from its own first):
    frames of many short sequences, raw and as SST blocks, at this alignment.  tests/zsection.py
    measures each frame's section; the set holds frames A' would take that run past each limit and
    frames within both.  Every status and decoded byte is the oracle's, and the frames past a limit
    are handed to the exact path."""
    from tests import zsection
    rng = random.Random(40 + misalign)
    blocks = [_crc(_z(_short_sequences(rng, 4000), rng.choice([3, 19]))) for _ in range(96)]
    stream = _short_sequences(rng, 120000)
    kvs, p = [], 0
    for i in range(700):
        m = rng.randint(30, 300)
        kvs.append((b"key%08d" % i, stream[p:p + m]))
        p += m
    blocks += [_crc(_z(b[:-4], rng.choice([3, 9, 19]))) for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    _, off = bg.pack(blocks, misalign)
    past_hdr = past_bits = fits = 0
    for i, blk in enumerate(blocks):
        z = zsection.section_shape(blk[:-4], int(off[i]) & 15)
        if z is None or z["nseq"] > 128 or max(z["logs"]) > 7 or z["logs"][0] > 6 or z["logs"][1] > 5:
            continue
        if z["hdr_end_in_chunk"] > 64:
            past_hdr += 1
        elif z["chunks_from_bitstream"] > 10:
            past_bits += 1
        else:
            fits += 1
    assert past_hdr and past_bits and fits, (past_hdr, past_bits, fits)
    ctx.handbacks(reset=True)
    meta = _compare(ctx, blocks, misalign=misalign)
    assert all(x == 0 or 3 <= x <= 7 for x in meta["status"].tolist()), meta["status"]  # (decoded: bytes compared)
    assert ctx.handbacks() >= past_hdr + past_bits


def _huf_blocks(rng, n_kv, vlen, block_size, alpha=256, zipf=0.8):
    """SST blocks whose level-3 frames have Huffman-coded literals (a new tree; 4 streams, and 1
    stream for small sections) and few sequences with predefined tables: the fast path's phases
    H1 / H2 (zstd_fast.hip)."""
    w = [1.0 / ((i + 1) ** zipf) for i in range(alpha)]
    keys = sorted({bytes(rng.randrange(256) for _ in range(rng.randint(4, 20))) for _ in range(n_kv)})
    kvs = [(k, bytes(rng.choices(range(alpha), w, k=rng.randint(*vlen)))) for k in keys]
    return [b[:-4] for b in bg.sst_blocks(kvs, block_size, ob.NONE)]


def _lit_type(frame: bytes) -> int:
    """The first block's literals section type (2: Huffman with a new tree) and stream count."""
    fhd = frame[4]
    fcsf, ss, dif = fhd >> 6, (fhd >> 5) & 1, fhd & 3
    p = 5 + (0 if ss else 1) + (0, 1, 2, 4)[dif] + ((0, 2, 4, 8)[fcsf] if fcsf else ss)
    b0 = frame[p + 3]
    return (b0 & 3, 1 if ((b0 >> 2) & 3) == 0 else 4)


@pytest.mark.parametrize("misalign", [0, 5, 11])
def test_huffman_literal_blocks(ctx, misalign):
    """Huffman-literal frames (4- and 1-stream) through phases H1 / H2, none handed back, and the
    same frames with a flipped byte in the literal streams under a recomputed block CRC (the stream
    no longer ends at its first bit, or the frame checksum fails: the exact path reports it); every
    status, byte and row identical to the oracle."""
    rng = random.Random(70 + misalign)
    decs = _huf_blocks(rng, 500, (800, 1100), 4096) + _huf_blocks(rng, 400, (20, 40), 256, 200, 1.1)
    frames = [_z(d, 3) for d in decs]
    kinds = [_lit_type(f) for f in frames]
    assert sum(1 for t in kinds if t == (2, 4)) >= 100 and sum(1 for t in kinds if t == (2, 1)) >= 20, kinds
    ctx.handbacks(reset=True)
    meta = _compare(ctx, [_crc(f) for f in frames], misalign=misalign)
    assert (meta["status"] == 0).all()
    assert ctx.handbacks() == 0
    damaged = []
    for f in frames:
        g = bytearray(f)
        g[rng.randrange(len(g) // 3, len(g) - 16)] ^= 1 << rng.randrange(8)
        damaged.append(_crc(bytes(g)))
    meta = _compare(ctx, damaged + [_crc(f) for f in frames[:50]], misalign=misalign)
    assert (meta["status"][-50:] == 0).all() and (meta["status"][:-50] != 0).any()


def test_huffman_literal_blocks_beyond_slots(ctx):
    """More Huffman-literal blocks in one batch than H1 / H2 have slots for (zf_huf_cap: n / 16 + 64
    past 1024 blocks): the rest take phase B'; every block identical to the oracle."""
    rng = random.Random(77)
    decs = []
    while len(decs) < 1500:
        decs += _huf_blocks(rng, 600, (800, 1100), 4096)
    blocks = [_crc(_z(d, 3)) for d in decs[:1500]]
    ctx.handbacks(reset=True)
    meta = _compare(ctx, blocks, misalign=9)
    assert (meta["status"] == 0).all()
    assert ctx.handbacks() == 0
