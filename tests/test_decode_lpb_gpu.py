"""GPU parity for the Snappy decoder's separate tag paths (hand-built streams).

The oracle's encoder never emits some tag shapes the lane-per-block decoder
(csrc/decode_lpb2.hip) treats specially, so these streams are built tag by tag
(tests/snappygen.py) and decoded by both sides:
  * far copies (offset > 112, past the output ring): short ones become "holes"
    filled four steps later, long ones go through the far-copy path;
  * far copies back to back, and near copies that read bytes of a pending hole;
  * short-period overlapping copies (offsets 1..16) and ring-boundary offsets;
  * literal lengths with 1- and 2-byte extensions;
  * rows with expire/create timestamps, tombstones, blocks with hundreds of rows;
  * corrupt streams (offset before the start, length mismatch, truncated tags).
Every field is compared bit-exactly with the oracle (plan, meta, bytes, rows).
"""
import random
import struct

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tests import snappygen as sg

pytestmark = pytest.mark.gpu

DECODED_OK = {0, 3, 4, 5, 6, 7} | set(range(20, 30))


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _stream_len(blk: bytes):
    x = s = 0
    for c in blk[:5]:
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x
    return None


def _compare(ctx, blocks, misalign=0):
    blob, off = bg.pack(blocks, misalign)
    g_out, g_off, g_meta, g_rows, g_rb = ctx.decode_batch(ob.SNAPPY, blob, off)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.SNAPPY, blob, off)
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i in range(len(blocks)):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om)
        st = int(om["status"])
        if st in DECODED_OK:
            a = int(o_off[i])
            b = a + _stream_len(blocks[i])
            assert g_out[a:b].tobytes() == o_out[a:b].tobytes(), (i, st)
        if st == 0:
            r0 = int(o_rb[i])
            nr = min(int(om["n_rows"]), int(o_rb[i + 1]) - r0)
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i
    return o_meta


BOUNDARY_OFFS = [1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 32, 63, 64, 65, 111, 112, 113, 114, 127, 128, 129, 200]


def _value_ops(rng: random.Random, avail: int, n_ops: int):
    """A list of (kind, off, len) ops for one value; copies stay within `avail` + emitted."""
    ops, total = [], 0
    for _ in range(n_ops):
        pos = avail + total
        r = rng.random()
        if r < 0.15 or pos < 8:
            n = rng.choice([1, 2, 3, 5, 15, 16, 17, 59, 60, 61, 64, 65, 200, 255, 256, 257, 300])
            ops.append(("lit", 0, n))
        elif r < 0.40:  # short far copy -> hole
            ops.append(("copy", rng.randint(113, min(pos, 2000)), rng.randint(1, 16)))
        elif r < 0.50:  # long far copy
            ops.append(("copy", rng.randint(113, min(pos, 4000)), rng.randint(17, 64)))
        elif r < 0.65:  # near copy right after (may read a pending hole)
            ops.append(("copy", rng.randint(1, min(pos, 40)), rng.randint(1, 64)))
        elif r < 0.85:
            offs = [o for o in BOUNDARY_OFFS if o <= pos]
            ops.append(("copy", rng.choice(offs), rng.randint(1, 64)))
        else:  # periodic run
            ops.append(("copy", rng.randint(1, min(pos, 16)), rng.randint(30, 64)))
        total += ops[-1][2]
    return ops, total


def crafted_block(rng: random.Random, n_pre=None, n_ops=None, ts_p=0.4):
    """A valid block whose middle row's value is written with chosen tags."""
    s = sg.Stream()
    pre = sg.rows_for(rng, n_pre if n_pre is not None else rng.randint(1, 30), ts_p=ts_p)
    # a long random value so far offsets have a source
    pre.append(sg.v0_row(0, b"zz", bytes(rng.randrange(256) for _ in range(rng.randint(100, 2200)))))
    rows = list(pre)
    head = b"".join(pre)
    s.emit(head, rng)
    ops, vlen = _value_ops(rng, len(head), n_ops if n_ops is not None else rng.randint(5, 60))
    hdr = struct.pack(">HH", 0, 3) + b"mid" + struct.pack(">QB", 7, 6) + struct.pack(">qq", 11, -5)
    hdr += struct.pack(">I", vlen)
    s.lit(hdr)
    v0 = len(s.out)
    for kind, off, n in ops:
        if kind == "lit":
            s.lit(bytes(rng.randrange(256) for _ in range(n)))
        else:
            s.copy(off, n, rng.choice([None, 2, 4]))
    rows.append(bytes(s.out[len(head):]))
    assert len(s.out) - v0 == vlen
    post = sg.rows_for(rng, rng.randint(0, 20), ts_p=ts_p)[1:]
    rows += post
    full = sg.block_bytes(rows)
    s.emit(full[len(s.out):], rng)
    assert bytes(s.out) == full
    return s.block()


@pytest.mark.parametrize("seed", range(6))
def test_crafted_tags(ctx, seed):
    rng = random.Random(1000 + seed)
    blocks = [crafted_block(rng) for _ in range(rng.randint(70, 200))]
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


def test_hole_then_near_copy(ctx):
    """Short far copies immediately followed by copies that overlap them."""
    rng = random.Random(7)
    blocks = []
    for i in range(128):
        s = sg.Stream()
        s.lit(bytes(rng.randrange(256) for _ in range(300)))
        for _ in range(rng.randint(4, 30)):
            s.copy(rng.randint(113, len(s.out)), rng.randint(1, 16), rng.choice([2, 4]))
            if rng.random() < 0.5:
                s.copy(rng.randint(113, len(s.out)), rng.randint(1, 16), 2)
            s.copy(rng.randint(1, 24), rng.randint(1, 64), rng.choice([None, 2]))
        s.lit(struct.pack(">H", 0) + struct.pack(">H", 1))  # offsets [0], count 1 -> row error, bytes compared
        blocks.append(s.block())
    _compare(ctx, blocks, misalign=3)


def test_periodic_short_offsets(ctx):
    rng = random.Random(8)
    blocks = []
    for off in range(1, 33):
        for length in (1, 4, 11, 16, 17, 33, 64):
            s = sg.Stream()
            s.lit(bytes(rng.randrange(256) for _ in range(off + rng.randint(0, 5))))
            for _ in range(rng.randint(1, 40)):
                s.copy(off, length, rng.choice([None, 2, 4]))
            s.lit(b"\x00\x00\x00\x01")
            blocks.append(s.block())
    _compare(ctx, blocks)


def test_literal_extensions(ctx):
    rng = random.Random(9)
    blocks = []
    for n in [1, 59, 60, 61, 62, 255, 256, 257, 258, 1000, 65535, 65536 - 4]:
        s = sg.Stream()
        data = bytes(rng.randrange(256) for _ in range(n))
        s.tags += sg.tag_literal(data)
        s.out += data
        s.lit(b"\x00\x00\x00\x01")
        blocks.append(s.block())
    _compare(ctx, blocks, misalign=5)


@pytest.mark.parametrize("n_rows", [1, 2, 55, 56, 57, 120, 400])
def test_many_rows_with_timestamps(ctx, n_rows):
    rng = random.Random(n_rows)
    blocks = []
    for _ in range(80):
        rows = sg.rows_for(rng, n_rows, ts_p=0.6, tomb_p=0.3, period=rng.choice([None, b"ab", b"xyz0123"]))
        if rng.random() < 0.5:  # tiny rows: short suffix, no value
            rows = [rows[0]] + [sg.v0_row(rng.randint(0, 4), b"%d" % i, None) for i in range(1, n_rows)]
        full = sg.block_bytes(rows)
        if len(full) > 65000:
            continue
        s = sg.Stream()
        s.emit(full, rng)
        blocks.append(s.block())
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


def test_ragged_mixture(ctx):
    """Tiny, crafted and oracle-encoded blocks interleaved in one batch."""
    rng = random.Random(10)
    blocks = []
    kvs = bg.random_kvs(rng, 600)
    enc = bg.sst_blocks(kvs, 512, ob.SNAPPY)
    for i in range(300):
        r = rng.random()
        if r < 0.3:
            blocks.append(crafted_block(rng, n_pre=rng.randint(0, 3), n_ops=rng.randint(1, 8)))
        elif r < 0.6:
            blocks.append(rng.choice(enc))
        else:
            s = sg.Stream()
            s.emit(sg.block_bytes(sg.rows_for(rng, rng.randint(1, 3))), rng)
            blocks.append(s.block())
    meta = _compare(ctx, blocks, misalign=11)
    assert (meta["status"] == 0).all()


def _corrupt_cases(rng: random.Random):
    good = sg.Stream()
    good.emit(sg.block_bytes(sg.rows_for(rng, 20)), rng)
    body = sg.varint(len(good.out)) + bytes(good.tags)
    out = []
    # copy offset before the start of the output
    s = sg.Stream()
    s.lit(b"abcdefgh")
    s.tags += sg.tag_copy(9, 4, 2)
    s.tags += sg.tag_copy(200, 8, 4)
    out.append(bg.recrc(sg.varint(20) + bytes(s.tags)))
    # offset 0
    out.append(bg.recrc(sg.varint(12) + sg.tag_literal(b"abcdefgh") + bytes([2 | (3 << 2), 0, 0])))
    # header longer / shorter than the stream
    out.append(bg.recrc(sg.varint(len(good.out) + 1) + bytes(good.tags)))
    out.append(bg.recrc(sg.varint(len(good.out) - 1) + bytes(good.tags)))
    # copy running past the declared length
    out.append(bg.recrc(sg.varint(10) + sg.tag_literal(b"abcdefgh") + sg.tag_copy(8, 8, 2)))
    # literal running past the input; truncated copy tags; huge header
    out.append(bg.recrc(sg.varint(100) + bytes([(50 << 2)]) + b"x" * 10))
    out.append(bg.recrc(sg.varint(100) + sg.tag_literal(b"abcdefgh") + bytes([3 | (7 << 2), 1, 0])))
    out.append(bg.recrc(sg.varint(100) + sg.tag_literal(b"abcdefgh") + bytes([2])))
    out.append(bg.recrc(sg.varint(1 << 31) + sg.tag_literal(b"abcdefgh")))
    out.append(bg.recrc(sg.varint(1 << 20) + sg.tag_literal(b"abcdefgh")))
    out.append(bg.recrc(bytes([0x80] * 6) + sg.tag_literal(b"abcdefgh")))
    # literal length extension bytes missing
    out.append(bg.recrc(sg.varint(300) + bytes([61 << 2, 0x2B])))
    # random tag-level damage to a good stream with the CRC recomputed
    for _ in range(40):
        b = bytearray(body)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(1, len(b))] = rng.randrange(256)
        out.append(bg.recrc(bytes(b)))
    return out


def test_corrupt_streams(ctx):
    rng = random.Random(11)
    blocks = []
    for _ in range(3):
        blocks += _corrupt_cases(rng)
    rng.shuffle(blocks)
    _compare(ctx, blocks, misalign=1)
