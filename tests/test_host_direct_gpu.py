"""Host decode into page-locked caller buffers (slate_hostbuf): the GPU writes each chunk's bytes
and rows straight into the caller's memory (csrc/api_host.cpp sink_map + decode.hip
blocks_to_host_kernel) instead of staging + a host copy.  Checked against the same call with
pageable buffers and against the oracle: slate_block_decode_batch (chunked) and
slate_block_decode_sharded (blocks scattered to their places in the batch), outputs at an offset
inside the page-locked buffer, one corrupt block among them."""
import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    import slatecodec as sc
    cs = [sc.Context(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


def _workload(codec, corrupt):
    kvs = bg.kv_synthetic(38 * 300, half=True)
    blocks = bg.sst_blocks(kvs, 4096, codec)
    if corrupt:
        b = bytearray(blocks[17])
        b[9] ^= 0x55
        blocks[17] = bytes(b)
    return bg.pack(blocks, misalign=5)


def _plan(ctx, sc, codec, blob, off):
    n = len(off) - 1
    out_off, row_base = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    meta = np.zeros(n, sc.META_DTYPE)
    st = ctx.decode_batch_into(codec, blob, off, np.zeros(1, np.uint8), np.zeros(1, sc.ROW_DTYPE), meta, out_off,
                               row_base)
    assert st == sc.E_CAPACITY
    return out_off, row_base


def _pinned(ctx, sc, nbytes, shift, dtype):
    hb = sc.HostBuf(ctx, nbytes + shift + 64)
    hb.view[:] = 0xEE
    item = np.dtype(dtype).itemsize
    n = nbytes // item
    return hb, hb.view[shift:shift + n * item].view(dtype)


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("sharded", [False, True])
def test_pinned_outputs_match_pageable(ctxs, monkeypatch, codec, sharded):
    import slatecodec as sc
    monkeypatch.setenv("SLATE_PIPE_CHUNK_BLOCKS", "64")  # (read once per process: may not apply)
    blob, off = _workload(codec, corrupt=True)
    n = len(off) - 1
    out_off, row_base = _plan(ctxs[0], sc, codec, blob, off)
    out_p, rows_p, meta_p = np.zeros(int(out_off[n]) + 16, np.uint8), np.zeros(int(row_base[n]) + 1, sc.ROW_DTYPE), \
        np.zeros(n, sc.META_DTYPE)
    oo_p, rb_p = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    hb_o, out_h = _pinned(ctxs[0], sc, int(out_off[n]) + 16, 48, np.uint8)
    hb_r, rows_h = _pinned(ctxs[0], sc, 16 * (int(row_base[n]) + 1), 32, sc.ROW_DTYPE)
    meta_h = np.zeros(n, sc.META_DTYPE)
    oo_h, rb_h = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    if sharded:
        st_p = sc.decode_sharded_into(ctxs, codec, blob, off, out_p, rows_p, meta_p, oo_p, rb_p)
        st_h = sc.decode_sharded_into(ctxs, codec, blob, off, out_h, rows_h, meta_h, oo_h, rb_h)
    else:
        st_p = ctxs[0].decode_batch_into(codec, blob, off, out_p, rows_p, meta_p, oo_p, rb_p)
        st_h = ctxs[0].decode_batch_into(codec, blob, off, out_h, rows_h, meta_h, oo_h, rb_h)
    assert st_p == st_h == sc.OK
    assert np.array_equal(oo_p, oo_h) and np.array_equal(rb_p, rb_h)
    assert meta_p.tobytes() == meta_h.tobytes()
    assert meta_h["status"][17] != 0 and (np.delete(meta_h["status"], 17) == 0).all()
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, off)
    assert o_meta.tobytes() == meta_h.tobytes()
    for i in range(n):
        if meta_h["status"][i]:
            continue
        dl = int(meta_h["data_len"][i]) + 2 * int(meta_h["n_rows"][i]) + 2
        a = int(oo_h[i])
        assert out_h[a:a + dl].tobytes() == out_p[a:a + dl].tobytes() == o_out[int(o_off[i]):int(o_off[i]) + dl].tobytes()
        r, k = int(rb_h[i]), int(meta_h["n_rows"][i])
        assert rows_h[r:r + k].tobytes() == rows_p[r:r + k].tobytes() == o_rows[int(o_rb[i]):int(o_rb[i]) + k].tobytes()
    del hb_o, hb_r


def test_partly_registered_outputs_use_staging(ctxs):
    """Outputs whose first pages only are page-locked (hipHostRegister over a prefix): the library
    must not write them through device addresses (the rest is not mapped) and decodes through
    staging instead -- same bytes as the oracle, no fault (api_host.cpp sink_map / mapped_range)."""
    import ctypes
    import slatecodec as sc
    sc.lib()
    # the HIP runtime already in the process, by its soname (a second copy by path would bind to
    # whatever HSA runtime torch loaded and may not resolve)
    hip = ctypes.CDLL("libamdhip64.so.7")
    codec = ob.SNAPPY
    blob, off = _workload(codec, corrupt=False)
    n = len(off) - 1
    out_off, row_base = _plan(ctxs[0], sc, codec, blob, off)
    page = 4096

    def aligned(nbytes):
        raw = np.zeros(nbytes + 2 * page, np.uint8)
        a = (-raw.ctypes.data) % page
        return raw, raw[a:a + nbytes]

    out_raw, out_h = aligned(int(out_off[n]) + 16 + page)
    rows_raw, rows_b = aligned(16 * (int(row_base[n]) + 1) + page)
    rows_h = rows_b[:16 * (int(row_base[n]) + 1)].view(sc.ROW_DTYPE)
    regs = []
    for arr in (out_h, rows_b):
        ptr, size = ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(page)  # the first page only
        assert hip.hipHostRegister(ptr, size, ctypes.c_uint(0)) == 0
        regs.append(ptr)
    try:
        meta_h = np.zeros(n, sc.META_DTYPE)
        oo_h, rb_h = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
        st = ctxs[0].decode_batch_into(codec, blob, off, out_h, rows_h, meta_h, oo_h, rb_h)
        assert st == sc.OK
        o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blob, off)
        assert o_meta.tobytes() == meta_h.tobytes()
        for i in range(n):
            dl = int(meta_h["data_len"][i]) + 2 * int(meta_h["n_rows"][i]) + 2
            a = int(oo_h[i])
            assert out_h[a:a + dl].tobytes() == o_out[int(o_off[i]):int(o_off[i]) + dl].tobytes()
            r, k = int(rb_h[i]), int(meta_h["n_rows"][i])
            assert rows_h[r:r + k].tobytes() == o_rows[int(o_rb[i]):int(o_rb[i]) + k].tobytes()
    finally:
        for ptr in regs:
            hip.hipHostUnregister(ptr)
    del out_raw, rows_raw
