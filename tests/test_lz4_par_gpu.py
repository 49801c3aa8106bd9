"""CodecLz4 index / filter payloads whose data blocks exceed 64 KiB -- pierrec/lz4 v4's writer defaults
(4 MiB independent blocks, a content checksum), the shape an SST written by the reference carries --
decoded through the tag-parallel block passes (api_sst.cpp lz4_payload_par_run, snappy_stream.hip
launch_lz4_par_chain / _bytes), against the oracle's restatement of the reference reader
(compression.go:143-144 under bloom.Decode bloom.go:70-91 and DecodeIndex flatbuf.go:83-100):
decoded bytes and statuses.  liblz4's frames here have linked blocks (LZ4F's default mode), so
matches that reach into the block before are covered too.  Damaged payloads (flipped bytes under a valid CRC, a wrong content
checksum) fail a check of the parallel passes and reach the exact decoder, which reports them."""
import random
import time

import numpy as np
import pytest

from oracle import binding as ob
from tests import lz4gen, sstgen, zstdgen

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not zstdgen.available(), reason="liblz4 not in this image")]


@pytest.fixture(scope="module")
def sc():
    import slatecodec
    return slatecodec


@pytest.fixture(scope="module")
def ctx(sc):
    return sc.Context(0)


def _liblz4_frame(raw: bytes) -> bytes:
    """liblz4 LZ4F_compressFrame with pierrec's defaults (tools/benchgen.c: 4 MiB blocks, content
    checksum) || BE32 CRC32."""
    from tools import workload as wl
    dec = np.frombuffer(raw, np.uint8).copy()
    blob, off = wl.encode_blocks(ob.LZ4, dec, np.array([0, len(raw)], np.uint64), threads=1)
    return bytes(blob[: int(off[1])])


def _check_filter(ctx, frame: bytes):
    g = ctx.bloom_decode(frame, ob.LZ4)
    o = ob.bloom_decode(frame, ob.LZ4, cap=1 << 25)
    assert g[0] == o[0] and g[1:] == o[1:], (g[0], o[0])
    return g[0]


def _block_sizes(frame: bytes):
    """(bmax, [data block size words]) of a frame (structure only)."""
    flg, bd = frame[4], frame[5]
    pos = 4 + 2 + (8 if flg & 8 else 0) + 1
    words = []
    while True:
        w = int.from_bytes(frame[pos:pos + 4], "little")
        pos += 4
        if w == 0:
            break
        words.append(w)
        pos += w & 0x7FFFFFFF
    return 1 << (8 + 2 * ((bd >> 4) & 7)), words


def test_lz4_large_blocks_sst_payloads(sc, ctx):
    """A CodecNone SST's index and filter (4 M KV: a 5 MB filter in two 4 MiB blocks, an index of
    compressed 4 MiB blocks) re-framed with liblz4 at pierrec's defaults decode like the oracle, in
    far less time than the exact path's ~2 MB/s would take."""
    from tools.bench_encode import kv_arrays
    keys, key_off, vals, val_off = kv_arrays(4_000_000)
    b = sc.SstBuilder(ctx, 4096, 0, 10, ob.NONE)
    assert b.add_batch(keys, key_off, vals, val_off) == 0
    sst = b.build().encode()
    st, info, _ = sc.read_info(sst)
    ib = sst[info.index_offset:info.index_offset + info.index_len][:-4]
    fb = sst[info.filter_offset:info.filter_offset + info.filter_len][:-4]
    fz = _liblz4_frame(fb)
    bmax, words = _block_sizes(fz)
    assert bmax == 4 << 20 and len(words) == 2  # filter bits barely compress: stored blocks, likely
    t0 = time.perf_counter()
    assert _check_filter(ctx, fz) == 0
    dt_f = time.perf_counter() - t0
    assert dt_f < 1.5, dt_f  # the exact one-wave path: > 2.5 s for 5 MB
    iz = _liblz4_frame(ib)
    bmax, words = _block_sizes(iz)
    assert bmax == 4 << 20 and len(words) >= 1 and not any(w >> 31 for w in words)
    t0 = time.perf_counter()
    st, index = ctx.decode_index(iz, ob.LZ4)
    dt = time.perf_counter() - t0
    ost, ometas = ob.decode_index(iz, ob.LZ4, cap=1 << 25)
    assert st == ost == 0 and index.block_metas() == ometas
    assert dt < 1.5, dt
    print(f"\n4 M KV: filter {len(fb)} B in {dt_f * 1e3:.1f} ms, index {len(ib)} B ({len(words)} compressed "
          f"blocks) in {dt * 1e3:.1f} ms, from 4 MiB LZ4 blocks")


@pytest.mark.parametrize("kind", ["zeros", "random", "pattern"])
def test_lz4_large_blocks_shapes(ctx, kind):
    """Stream shapes: one long overlapping match (offset 1, a 16 k-byte length extension), stored
    (incompressible) blocks, and short matches with mixed offsets and literal runs."""
    rng = np.random.default_rng(11)
    if kind == "zeros":
        raw = bytes(5_000_000)
    elif kind == "random":
        raw = rng.integers(0, 256, 6_000_000, dtype=np.uint8).tobytes()
    else:
        unit = rng.integers(0, 256, 700, dtype=np.uint8)
        parts = []
        for i in range(9000):
            u = unit.copy()
            u[rng.integers(0, 700, 12)] = rng.integers(0, 256, 12, dtype=np.uint8)
            parts.append(u[: 300 + (i * 37) % 400].tobytes())
        raw = b"".join(parts)
    fz = _liblz4_frame(raw)
    assert _check_filter(ctx, fz) == 0


def test_lz4_large_blocks_generated_and_damaged(ctx):
    """lz4gen frames (256 KiB / 1 MiB independent blocks, 64 KiB linked blocks whose matches reach
    into the block before; content size and checksum, stored blocks mixed in) decode like the
    oracle, then damaged copies give the oracle's statuses."""
    rng = random.Random(3)
    nrng = np.random.default_rng(3)
    unit = nrng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    raw = b"".join(unit[rng.randrange(0, 4000):][: rng.randrange(50, 1000)] +
                   nrng.integers(0, 256, rng.randrange(0, 300), dtype=np.uint8).tobytes()
                   + bytes(rng.randrange(0, 600)) for _ in range(1400))
    frames = [lz4gen.frame(raw, bsid=5, indep=True, content_checksum=True, content_size=True, rng=rng),
              lz4gen.frame(raw, bsid=6, indep=True, content_checksum=False, stored_p=0.3, rng=rng,
                           block_split=200_000),
              lz4gen.frame(raw, bsid=4, indep=False, content_checksum=True, rng=rng)]  # linked 64 KiB
    for f in frames:
        assert _block_sizes(f)[0] > 65536 or not (f[4] & 0x20)
        assert _check_filter(ctx, sstgen.crc(f)) == 0
    for trial in range(10):
        body = bytearray(frames[trial % 3])
        if trial % 5 == 4:
            body[-1] ^= 0x20  # the content checksum (or, without one, the EndMark)
        else:
            for _ in range(rng.randint(1, 3)):
                body[rng.randrange(11, len(body) - 8)] ^= 1 << rng.randrange(8)
        _check_filter(ctx, sstgen.crc(bytes(body)))


def test_lz4_large_blocks_cross_block_matches(ctx):
    """Linked blocks whose matches reach into the block before decode like the oracle; the same
    frame declared independent (FLG bit 5 set, header checksum redone) has matches reaching before
    their block, which the parallel passes must reject so the exact path reports the corruption."""
    rng = random.Random(9)
    unit = np.random.default_rng(9).integers(0, 256, 30_000, dtype=np.uint8).tobytes()
    raw = b"".join(unit[i * 7:] + unit[: i * 7] for i in range(12))
    f = lz4gen.frame(raw, bsid=5, indep=False, block_split=100_000, content_checksum=True, rng=rng)
    assert not (f[4] & 0x20) and len(_block_sizes(f)[1]) >= 3
    assert _check_filter(ctx, sstgen.crc(f)) == 0
    g = bytearray(f)
    g[4] |= 0x20
    g[6] = (lz4gen.xxh32(bytes(g[4:6])) >> 8) & 0xFF
    assert _check_filter(ctx, sstgen.crc(bytes(g))) != 0


def test_bloom_decode_capacity_retry(sc, ctx):
    """slate_bloom_decode with a buffer too small reports the filter's length (SLATE_E_CAPACITY); the
    retry with that length returns the oracle's bytes, and calls in between (another payload of the
    same length, another codec) do not disturb it."""
    import ctypes as C
    rng = np.random.default_rng(5)
    raw1 = b"\x00\x06" + rng.integers(0, 4, 300_000, dtype=np.uint8).tobytes()
    raw2 = b"\x00\x07" + rng.integers(0, 4, 300_000, dtype=np.uint8).tobytes()
    f1, f2 = _liblz4_frame(raw1), _liblz4_frame(raw2)
    if len(f2) != len(f1):  # same length, different bytes: pad the shorter frame's source
        f2 = f1[:-5] + bytes([f1[-5] ^ 1]) + f1[-4:]  # a damaged copy (CRC now wrong)
    L = sc.lib()

    def call(buf: bytes, cap: int, codec: int = ob.LZ4):
        b = np.frombuffer(buf, np.uint8)
        out = np.zeros(max(cap, 1), np.uint8)
        k, n = C.c_uint16(), C.c_size_t()
        st = L.slate_bloom_decode(ctx._h, sc._ptr(b), len(buf), codec, C.byref(k), sc._ptr(out), cap, C.byref(n))
        return st, k.value, n.value, out[: n.value].tobytes()

    st, k, n, _ = call(f1, 16)
    assert st == sc.E_CAPACITY and n == len(raw1) - 2
    o2 = ob.bloom_decode(f2, ob.LZ4, cap=1 << 22)
    st2, k2, n2, bits2 = call(f2, n + 64)  # not the kept filter
    assert st2 == o2[0] and (st2 != 0 or (k2, bits2) == (o2[1], o2[2]))
    st, k, n, _ = call(f1, 16)
    assert st == sc.E_CAPACITY
    assert call(f1, n + 64, ob.ZSTD)[0] != 0  # same bytes, another codec: decoded (and rejected) afresh
    st, k, n, _ = call(f1, 16)
    st, k, n1, bits = call(f1, n)  # the retry
    o1 = ob.bloom_decode(f1, ob.LZ4, cap=1 << 22)
    assert st == o1[0] == 0 and (k, bits) == (o1[1], o1[2])
