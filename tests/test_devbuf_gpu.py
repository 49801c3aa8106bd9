"""Library-owned memory for the device-resident entry points (SURVEY 8b "Ownership": device-resident
mode uses opaque handles owned by the C side): slate_devbuf / slate_hostbuf through the C-ABI --
synchronous and stream-ordered copies, bounds checks, and the headline decode path run entirely on
them (plan -> decode, the bench's entry points), bit-exact vs the oracle."""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def test_devbuf_copies_and_bounds(ctx):
    import slatecodec as sc
    L = sc.lib()
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, 50_000_000, dtype=np.uint8)  # > the 8 MiB direct-copy threshold
    d = sc.devbuf_from(ctx, a)
    assert L.slate_devbuf_size(d.handle) == a.size and d.ptr % 16 == 0
    assert np.array_equal(d.download(), a)
    assert np.array_equal(d.download(1000, 12345), a[12345:13345])
    e = sc.DevBuf(ctx, 4096).memset(0x5A)
    sc._check(L.slate_devbuf_copy(ctx.handle, e.handle, 100, d.handle, 7, 300), "copy")
    ctx.synchronize()
    got = e.download()
    assert (got[:100] == 0x5A).all() and np.array_equal(got[100:400], a[7:307]) and (got[400:] == 0x5A).all()
    # out of range: rejected, nothing written
    big = np.zeros(5000, np.uint8)
    assert L.slate_devbuf_upload(ctx.handle, e.handle, 0, big.ctypes.data, big.size) == sc.E_INVALID_ARG
    assert L.slate_devbuf_download(ctx.handle, big.ctypes.data, e.handle, 4000, 97) == sc.E_INVALID_ARG
    assert L.slate_devbuf_copy(ctx.handle, e.handle, 4095, d.handle, 0, 2) == sc.E_INVALID_ARG
    assert L.slate_devbuf_memset(ctx.handle, e.handle, 2 ** 63, 0, 2 ** 63) == sc.E_INVALID_ARG
    assert np.array_equal(e.download(), got)
    # zero-byte buffers have a valid address
    z = sc.DevBuf(ctx, 0)
    assert z.ptr and L.slate_devbuf_size(z.handle) == 0


def test_hostbuf_async_copies(ctx):
    import slatecodec as sc
    L = sc.lib()
    h = sc.HostBuf(ctx, 1 << 20)
    h.view[:] = np.arange(1 << 20, dtype=np.uint32).astype(np.uint8)
    d = sc.DevBuf(ctx, 1 << 20)
    sc._check(L.slate_devbuf_upload_async(ctx.handle, d.handle, 0, h.handle, 0, 1 << 20), "upload_async")
    h2 = sc.HostBuf(ctx, 1 << 20)
    sc._check(L.slate_devbuf_download_async(ctx.handle, h2.handle, 0, d.handle, 0, 1 << 20), "download_async")
    ctx.synchronize()
    assert np.array_equal(h2.view, h.view)
    assert L.slate_devbuf_upload_async(ctx.handle, d.handle, 1, h.handle, 0, 1 << 20) == sc.E_INVALID_ARG


def test_headline_decode_on_devbufs(ctx):
    """plan + decode (slate_block_decode_plan_device / _device, the entries bench.py times) with every
    buffer a slate_devbuf, against the oracle: Snappy V-half and CodecNone blocks, misaligned input."""
    import slatecodec as sc
    for codec in (ob.SNAPPY, ob.NONE):
        blocks = bg.sst_blocks(bg.kv_synthetic(38 * 200, half=True, tomb_every=13), 4096, codec)
        blob, off = bg.pack(blocks, misalign=7)
        n = len(blocks)
        d_in, d_off = sc.devbuf_from(ctx, blob), sc.devbuf_from(ctx, off)
        d_oo, d_rb = sc.DevBuf(ctx, 8 * (n + 1)), sc.DevBuf(ctx, 8 * (n + 1))
        d_sc = sc.DevBuf(ctx, sc.decode_scratch_bytes(n) + 64)
        ctx.decode_plan_device(codec, d_in.ptr, d_off.ptr, n, d_oo.ptr, d_rb.ptr, d_sc.ptr)
        d_out, d_meta = sc.DevBuf(ctx, d_oo.u64(n) + 16), sc.DevBuf(ctx, 16 * n)
        d_rows = sc.DevBuf(ctx, 16 * d_rb.u64(n) + 16)
        ctx.decode_device(codec, d_in.ptr, d_off.ptr, n, d_out.ptr, d_oo.ptr, d_meta.ptr, d_rows.ptr, d_rb.ptr)
        o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, off)
        assert np.array_equal(d_oo.download(dtype=np.uint64), o_off) and np.array_equal(d_rb.download(dtype=np.uint64),
                                                                                       o_rb)
        meta = d_meta.download().view(sc.META_DTYPE)
        assert meta.tobytes() == o_meta.tobytes() and (meta["status"] == 0).all()
        out = d_out.download()
        rows = d_rows.download().view(sc.ROW_DTYPE)
        for i in range(n):
            a, dl = int(o_off[i]), int(o_meta["data_len"][i]) + 2 * int(o_meta["n_rows"][i]) + 2
            assert out[a:a + dl].tobytes() == o_out[a:a + dl].tobytes(), i
            r0, nr = int(o_rb[i]), int(o_meta["n_rows"][i])
            assert rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i


def test_codec_none_aliased_decode(ctx):
    """CodecNone with d_out = NULL decodes as Go's block.Decode does, without a copy (block.go:122
    aliases the input): metas and rows identical to the oracle's, every row descriptor read against
    the input bytes themselves (a block's data starts at its input offset); blocks beyond the
    one-wave kernel's window (large values) take the large-block path in the same mode; a damaged
    CRC reports as in the copying mode."""
    import random
    import slatecodec as sc
    rng = random.Random(5)
    kvs = bg.kv_synthetic(38 * 120, half=True, tomb_every=11)
    blocks = bg.sst_blocks(kvs, 4096, ob.NONE)
    blocks += bg.sst_blocks([(b"big%03d" % i, bytes(rng.randrange(256) for _ in range(7000))) for i in range(3)],
                            4096, ob.NONE)
    bad = bytearray(blocks[5])
    bad[-1] ^= 1
    blocks[5] = bytes(bad)
    blob, off = bg.pack(blocks, misalign=3)
    n = len(blocks)
    d_in, d_off = sc.devbuf_from(ctx, blob), sc.devbuf_from(ctx, off)
    d_oo, d_rb = sc.DevBuf(ctx, 8 * (n + 1)), sc.DevBuf(ctx, 8 * (n + 1))
    d_sc = sc.DevBuf(ctx, sc.decode_scratch_bytes(n) + 64)
    ctx.decode_plan_device(ob.NONE, d_in.ptr, d_off.ptr, n, d_oo.ptr, d_rb.ptr, d_sc.ptr)
    d_meta, d_rows = sc.DevBuf(ctx, 16 * n), sc.DevBuf(ctx, 16 * d_rb.u64(n) + 16)
    ctx.decode_device(ob.NONE, d_in.ptr, d_off.ptr, n, 0, 0, d_meta.ptr, d_rows.ptr, d_rb.ptr)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.NONE, blob, off)
    meta = d_meta.download().view(sc.META_DTYPE)
    assert meta.tobytes() == o_meta.tobytes()
    assert int(meta["status"][5]) != 0 and (np.delete(meta["status"], 5) == 0).all()
    rows = d_rows.download().view(sc.ROW_DTYPE)
    for i in range(n):
        if int(o_meta["status"][i]):
            continue
        r0, nr = int(o_rb[i]), int(o_meta["n_rows"][i])
        assert rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i
        a, dl = int(o_off[i]), int(o_meta["data_len"][i])
        assert blob[int(off[i]):int(off[i]) + dl].tobytes() == o_out[a:a + dl].tobytes(), i
    # other codecs still need an output buffer
    assert sc.lib().slate_block_decode_device(ctx.handle, ob.SNAPPY, d_in.ptr, d_off.ptr, n, None, d_oo.ptr,
                                              d_meta.ptr, d_rows.ptr, d_rb.ptr) == sc.E_INVALID_ARG
