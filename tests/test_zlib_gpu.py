"""GPU parity for CodecZlib blocks (compress.Decode, compression.go:134-140) through the C ABI:
block.Decode with zlib streams of every deflate strategy/level (stored, fixed and dynamic
Huffman blocks), plus damaged streams with their status codes, bit-exact against the oracle
(plan, meta, decoded bytes, rows).  The streams come from the zlib library (Python's zlib
module), which the oracle's inflater is pinned to in tests/test_zlib_oracle.py."""
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu
STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FILTERED]


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _crc(stream: bytes) -> bytes:
    return stream + struct.pack(">I", zlib.crc32(stream))


def _z(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, wbits=15) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, wbits, 8, strategy)
    return co.compress(data) + co.flush()


class _Device:
    """One device-resident batch (slate_block_decode_plan_device + _device, bench.py's entries): with
    CodecZlib and >= 64 blocks the plan is phase Z itself, staged in the context for the decode."""

    def __init__(self, ctx, blob, off):
        import slatecodec as sc
        self.ctx, self.n = ctx, len(off) - 1
        self.d_in, self.d_off = sc.devbuf_from(ctx, blob), sc.devbuf_from(ctx, off)
        self.d_oo, self.d_rb = sc.DevBuf(ctx, 8 * (self.n + 1)), sc.DevBuf(ctx, 8 * (self.n + 1))
        self.d_sc = sc.DevBuf(ctx, sc.decode_scratch_bytes(self.n) + 64)
        self.plan()
        self.d_out, self.d_meta = sc.DevBuf(ctx, self.d_oo.u64(self.n) + 16), sc.DevBuf(ctx, 16 * max(self.n, 1))
        self.d_rows = sc.DevBuf(ctx, 16 * self.d_rb.u64(self.n) + 16)

    def plan(self):
        self.ctx.decode_plan_device(ob.ZLIB, self.d_in.ptr, self.d_off.ptr, self.n, self.d_oo.ptr, self.d_rb.ptr,
                                    self.d_sc.ptr)

    def decode(self):
        import slatecodec as sc
        self.d_out.memset(0xEE)
        self.d_meta.memset(0xEE)
        self.ctx.decode_device(ob.ZLIB, self.d_in.ptr, self.d_off.ptr, self.n, self.d_out.ptr, self.d_oo.ptr,
                               self.d_meta.ptr, self.d_rows.ptr, self.d_rb.ptr)
        return (self.d_out.download(), self.d_oo.download(dtype=np.uint64),
                self.d_meta.download().view(sc.META_DTYPE)[:self.n], self.d_rows.download().view(sc.ROW_DTYPE),
                self.d_rb.download(dtype=np.uint64))


def _check_same(blocks, got, want):
    g_out, g_off, g_meta, g_rows, g_rb = got
    o_out, o_off, o_meta, o_rows, o_rb = want
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i, blk in enumerate(blocks):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om)
        st = int(om["status"])
        if st == 0 or 3 <= st <= 7:
            dec = ob.zlib_decode(blk[:-4])[1]
            a = int(o_off[i])
            assert g_out[a:a + len(dec)].tobytes() == dec == o_out[a:a + len(dec)].tobytes(), i
        if st == 0:
            r0 = int(o_rb[i])
            nr = min(int(om["n_rows"]), int(o_rb[i + 1]) - r0)
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i


def _compare(ctx, blocks, misalign=0):
    """The host batch (slate_block_decode_batch) and the device-resident plan + decode, each against
    the oracle."""
    blob, off = bg.pack(blocks, misalign)
    want = ob.block_decode_batch(ob.ZLIB, blob, off)
    _check_same(blocks, _Device(ctx, blob, off).decode(), want)
    g_out, g_off, g_meta, g_rows, g_rb = ctx.decode_batch(ob.ZLIB, blob, off)
    o_out, o_off, o_meta, o_rows, o_rb = want
    assert np.array_equal(g_off, o_off), "plan: out_off"
    assert np.array_equal(g_rb, o_rb), "plan: row_base"
    for i, blk in enumerate(blocks):
        gm, om = g_meta[i], o_meta[i]
        assert gm.tobytes() == om.tobytes(), (i, gm, om)
        st = int(om["status"])
        if st == 0 or 3 <= st <= 7:
            dec = ob.zlib_decode(blk[:-4])[1]
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
def test_random_zlib_ssts(ctx, seed):
    rng = random.Random(seed)
    blocks = [_crc(_z(dec, rng.choice([0, 1, 6, 9]), rng.choice(STRATEGIES), rng.choice([9, 15])))
              for dec in _sst_plain(rng, rng.randint(300, 1500), rng.choice([512, 4096]))]
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert (meta["status"] == 0).all()


def test_vhalf_zlib_blocks(ctx):
    kvs = bg.kv_synthetic(38 * 200, half=True, tomb_every=25)
    blocks = [_crc(_z(b[:-4])) for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    meta = _compare(ctx, blocks, misalign=7)
    assert (meta["status"] == 0).all()


def test_large_zlib_blocks(ctx):
    """Blocks beyond the fast kernel's LDS budget go through the large-block kernel."""
    rng = random.Random(11)
    blocks = [_crc(_z(dec, rng.choice([1, 6]), rng.choice(STRATEGIES)))
              for dec in _sst_plain(rng, 2500, 40000)]
    blocks.append(_crc(_z(_sst_plain(rng, 600, 60000)[0], 0)))  # stored blocks, > 64 KiB cap? plan decides
    _compare(ctx, blocks, misalign=5)


def test_damaged_zlib_blocks(ctx):
    rng = random.Random(9)
    decs = _sst_plain(rng, 800, 1024)
    blocks = []
    for dec in decs:
        f = bytearray(_z(dec, rng.choice([1, 6, 9]), rng.choice(STRATEGIES)))
        kind = rng.randrange(6)
        if kind == 0:
            f[rng.randrange(len(f))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            f = f[: rng.randrange(len(f))]
        elif kind == 2:
            f += bytes(rng.randrange(256) for _ in range(rng.randint(1, 5)))
        elif kind == 3:
            i = rng.randrange(2, len(f))
            f[i:i + 2] = bytes([rng.randrange(256), rng.randrange(256)])
        elif kind == 4:
            f[rng.choice([0, 1])] ^= rng.choice([1, 2, 0x20, 0x80])
        blocks.append(_crc(bytes(f)))
    blocks += [_crc(b""), _crc(b"\x78"), _crc(b"\x78\x9c"), _crc(b"\x78\x9c\x07"),
               _crc(bytes([0x78, 0x9c, 0x01, 0x05, 0x00, 0x00, 0x00]) + b"abcde" + b"\0" * 4)]
    meta = _compare(ctx, blocks, misalign=1)
    st = set(int(x) for x in meta["status"])
    assert {0, 53, 54} <= st, st


@pytest.mark.parametrize("misalign", [0, 3, 9, 15])
def test_kv100_go_zlib_fast_path(ctx, misalign):
    """configs[1]'s block shape (4 KiB blocks of 100-byte V-half KVs) as Go's compress/zlib writes
    it (level 6, then the empty final stored block; tools/benchgen.c go_zlib6): every block takes
    the lane-per-block fast path (zlib_fast.hip + the build phase; none handed back), the plan's
    lane-per-block sizes included, bit-exact against the oracle at every input alignment."""
    import slatecodec as sc
    from tools import workload as wl
    dec, doff = wl.decoded_blocks(300, seed=misalign + 1, half=True)
    blob, off = wl.encode_blocks(ob.ZLIB, dec, doff, threads=4)
    blocks = [blob[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
    ctx.handbacks(reset=True)
    meta = _compare(ctx, blocks, misalign=misalign)
    assert (meta["status"] == 0).all()
    assert ctx.handbacks() == 0
    del sc


def test_zlib_fast_path_shapes(ctx):
    """Streams the fast path takes (dynamic and fixed Huffman blocks, several deflate blocks per
    stream, an empty stored block) and ones it hands back (stored blocks with data, a single
    distance code, corrupted Adler-32 under a valid block CRC): every block identical to the
    oracle, statuses included."""
    rng = random.Random(21)
    blocks = []
    for dec in _sst_plain(rng, 2400, 4096):
        kind = rng.randrange(6)
        if kind == 0:
            f = _z(dec, 6, zlib.Z_FIXED)
        elif kind == 1:  # several deflate blocks: a full flush in the middle
            co = zlib.compressobj(6)
            h = len(dec) // 2
            f = co.compress(dec[:h]) + co.flush(zlib.Z_FULL_FLUSH) + co.compress(dec[h:]) + co.flush()
        elif kind == 2:
            f = _z(dec, 0)  # stored blocks with data: handed back
        elif kind == 3:  # a wrong Adler-32 (valid block CRC): the exact path reports it
            f = bytearray(_z(dec, 6))
            f[-1] ^= 0x40
            f = bytes(f)
        else:
            f = _z(dec, rng.choice([1, 6, 9]))
        blocks.append(_crc(f))
    meta = _compare(ctx, blocks, misalign=rng.randrange(16))
    assert set(int(x) for x in meta["status"]) <= {0, 52}, set(int(x) for x in meta["status"])


def test_staged_plan_pairing(ctx):
    """The staged CodecZlib plan is used by the one decode that follows it over the same inputs and
    plan outputs; a second decode, a decode of other inputs in between, or a later plan of other
    inputs each decode on their own (phase Z again) -- every result identical to the oracle."""
    from tools import workload as wl
    batches = []
    for seed in (3, 4):
        dec, doff = wl.decoded_blocks(200, seed=seed, half=True)
        blob, off = wl.encode_blocks(ob.ZLIB, dec, doff, threads=4)
        blob, off = np.ascontiguousarray(blob), np.ascontiguousarray(off, np.uint64)
        blocks = [blob[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
        batches.append((blocks, _Device(ctx, blob, off), ob.block_decode_batch(ob.ZLIB, blob, off)))
    (ba, da, wa), (bb, db, wb) = batches
    ctx.handbacks(reset=True)
    da.plan()
    _check_same(ba, da.decode(), wa)   # staged
    _check_same(ba, da.decode(), wa)   # the stage was consumed: phase Z again
    da.plan()
    db.plan()                          # a later plan of other inputs replaces the stage
    _check_same(ba, da.decode(), wa)
    _check_same(bb, db.decode(), wb)   # (not armed: a's decode disarmed it)
    db.plan()
    _check_same(bb, db.decode(), wb)
    assert ctx.handbacks() == 0
