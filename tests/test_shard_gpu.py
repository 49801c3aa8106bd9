"""GPU parity of the host-buffer paths and the round-robin sharding (BASELINE configs[3],
SURVEY 8e): slate_block_decode_batch through page-locked staging over many chunks, and
slate_block_decode_sharded with G = 2..4 and 8 contexts on device 0 over one batch, against the
oracle block by block, in the original order (plan layout, meta, decoded bytes, rows)."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tools import workload as wl

pytestmark = pytest.mark.gpu


def _check_against_oracle(codec, blocks_blob, off, got):
    g_out, g_off, g_meta, g_rows, g_rb = got
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(codec, blocks_blob, off)
    assert np.array_equal(g_off, o_off) and np.array_equal(g_rb, o_rb)
    assert g_meta.tobytes() == o_meta.tobytes()
    n = len(off) - 1
    for i in range(n):
        st = int(o_meta["status"][i])
        if st == 0:
            a = int(o_off[i])
            dl = int(o_meta["data_len"][i]) + 2 * int(o_meta["n_rows"][i]) + 2
            assert g_out[a:a + dl].tobytes() == o_out[a:a + dl].tobytes(), i
            r0 = int(o_rb[i])
            nr = int(o_meta["n_rows"][i])
            assert g_rows[r0:r0 + nr].tobytes() == o_rows[r0:r0 + nr].tobytes(), i


def _mixed_batch(seed, n_good):
    """Set blocks plus random, ragged and corrupt blocks, shuffled (statuses differ per shard)."""
    rng = random.Random(seed)
    blob, off = wl.block_set(ob.SNAPPY, seed, 3, n_good, threads=4)
    blocks = [bytes(blob[int(off[i]):int(off[i + 1])]) for i in range(n_good)]
    kvs = bg.random_kvs(rng, 300, klen=(1, 40), vlen=(0, 300))
    blocks += bg.sst_blocks(kvs, 512, ob.SNAPPY)
    blocks += [bg.mutate(rng, blocks[rng.randrange(n_good)], fix_crc=rng.random() < 0.5) for _ in range(40)]
    blocks += [b"", b"\x01\x02\x03", bg.recrc(b"\x00")]
    rng.shuffle(blocks)
    return blocks


@pytest.mark.parametrize("g", [2, 3, 4, 8])
def test_sharded_decode_matches_oracle(g):
    import slatecodec as sc
    ctxs = [sc.Context(0) for _ in range(g)]
    for c in ctxs:  # every context has its own copy threads: 8 x 2 on the box's 16-core share
        c.set_copy_threads(16 // g if g > 4 else 4)
    blocks = _mixed_batch(g, 3000)
    blob, off = bg.pack(blocks, misalign=5)
    got = sc.decode_sharded(ctxs, sc.SNAPPY, blob, off)
    _check_against_oracle(sc.SNAPPY, blob, off, got)
    for c in ctxs:
        c.close()


def test_sharded_more_contexts_than_blocks():
    import slatecodec as sc
    ctxs = [sc.Context(0) for _ in range(4)]
    blocks = _mixed_batch(7, 2)[:3]
    blob, off = bg.pack(blocks)
    got = sc.decode_sharded(ctxs, sc.SNAPPY, blob, off)
    _check_against_oracle(sc.SNAPPY, blob, off, got)


def test_host_pipeline_many_chunks():
    """slate_block_decode_batch with 512-block chunks (two lanes alternate) in a child process
    (the chunk size is read once per process), against the oracle."""
    code = r"""
import sys, numpy as np
sys.path[:0] = [%r, %r]
import torch; torch.cuda.init()
import slatecodec as sc
from tests.test_shard_gpu import _mixed_batch, _check_against_oracle
from tests import blockgen as bg
blocks = _mixed_batch(11, 5000)
blob, off = bg.pack(blocks, misalign=3)
ctx = sc.Context(0)
got = ctx.decode_batch(sc.SNAPPY, blob, off)
_check_against_oracle(sc.SNAPPY, blob, off, got)
# 8 contexts, several chunks each, chunks in flight on all of them at once
ctxs = [sc.Context(0) for _ in range(8)]
for c in ctxs:
    c.set_copy_threads(2)
_check_against_oracle(sc.SNAPPY, blob, off, sc.decode_sharded(ctxs, sc.SNAPPY, blob, off))
# one pass into caller-sized buffers, twice (reused staging)
n = len(off) - 1
out = np.zeros(int(got[1][n]) + 16, np.uint8); rows = np.zeros(int(got[4][n]) + 1, sc.ROW_DTYPE)
meta = np.zeros(n, sc.META_DTYPE); oo = np.zeros(n + 1, np.uint64); rb = np.zeros(n + 1, np.uint64)
for _ in range(2):
    assert ctx.decode_batch_into(sc.SNAPPY, blob, off, out, rows, meta, oo, rb) == sc.OK
    _check_against_oracle(sc.SNAPPY, blob, off, (out, oo, meta, rows, rb))
print("ok")
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
       os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slatedb-go_amd"))
    env = dict(os.environ, SLATE_PIPE_CHUNK_BLOCKS="512")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]


def test_single_block_decode_matches_oracle():
    import slatecodec as sc
    ctx = sc.Context(0)
    for blk in _mixed_batch(13, 50)[:80]:
        st, m, data, offs = ctx.block_decode(blk, sc.SNAPPY)
        om, odata, orows = ob.block_decode(blk, sc.SNAPPY)
        assert int(m["status"]) == int(om["status"])
        if st == 0:
            assert data == odata[:int(om["data_len"])]
            assert offs == [int(r["row_off"]) for r in orows][:len(offs)]


@pytest.mark.parametrize("codec", ["lz4", "zstd", "none"])
def test_sharded_decode_other_codecs(codec):
    """slate_block_decode_sharded for codecs the host cannot plan (LZ4 / Zstd: a plan-only GPU
    pass per context over its gathered shard) and for CodecNone, against the oracle."""
    import slatecodec as sc
    c = {"lz4": sc.LZ4, "zstd": sc.ZSTD, "none": sc.NONE}[codec]
    rng = random.Random(17)
    kvs = bg.kv_synthetic(38 * 300, half=True, tomb_every=11)
    plain = [b[:-4] for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    dec = np.frombuffer(b"".join(plain), np.uint8)
    doff = np.cumsum([0] + [len(b) for b in plain]).astype(np.uint64)
    eblob, eoff = wl.encode_blocks(c, dec, doff, threads=4)  # liblz4 / libzstd frames + CRC
    blocks = [bytes(eblob[int(eoff[i]):int(eoff[i + 1])]) for i in range(len(plain))]
    blocks += [bg.mutate(rng, blocks[rng.randrange(len(blocks))], fix_crc=rng.random() < 0.5) for _ in range(20)]
    blocks += [b"", bg.recrc(b"\x00\x01")]
    rng.shuffle(blocks)
    blob, off = bg.pack(blocks, misalign=3)
    ctxs = [sc.Context(0) for _ in range(3)]
    got = sc.decode_sharded(ctxs, c, blob, off)
    _check_against_oracle(c, blob, off, got)
    for x in ctxs:
        x.close()


def test_failed_batches_then_valid_batch_same_context():
    """A batch that fails (decreasing offsets: SLATE_E_INVALID_ARG before any lane work; outputs too
    small: SLATE_E_CAPACITY after planning every chunk) leaves nothing in flight on the context: the
    next, smaller batch on it decodes exactly and writes nothing past its own outputs."""
    import slatecodec as sc
    ctx = sc.Context(0)
    big = _mixed_batch(21, 3000)
    blob, off = bg.pack(big, misalign=5)
    n = len(off) - 1
    bad = off.copy()
    bad[n // 2] = bad[n // 2 + 1] + 7  # offset i > offset i+1
    z = lambda k, dt: np.zeros(k, dt)  # noqa: E731
    st = ctx.decode_batch_into(sc.SNAPPY, blob, bad, z(1 << 20, np.uint8), z(1 << 16, sc.ROW_DTYPE),
                               z(n, sc.META_DTYPE), z(n + 1, np.uint64), z(n + 1, np.uint64))
    assert st == sc.E_INVALID_ARG
    st = ctx.decode_batch_into(sc.SNAPPY, blob, off, z(64, np.uint8), z(4, sc.ROW_DTYPE), z(n, sc.META_DTYPE),
                               z(n + 1, np.uint64), z(n + 1, np.uint64))
    assert st == sc.E_CAPACITY
    small = big[:37]
    sblob, soff = bg.pack(small, misalign=1)
    m = len(soff) - 1
    ref = ob.block_decode_batch(sc.SNAPPY, sblob, soff)
    pad = 4096
    out = np.full(int(ref[1][m]) + pad, 0xA5, np.uint8)
    rows = np.zeros(int(ref[4][m]) + 64, sc.ROW_DTYPE)
    rows["row_off"] = 0xDEADBEEF
    meta = np.zeros(m, sc.META_DTYPE)
    oo, rb = np.zeros(m + 1, np.uint64), np.zeros(m + 1, np.uint64)
    assert ctx.decode_batch_into(sc.SNAPPY, sblob, soff, out, rows, meta, oo, rb) == sc.OK
    _check_against_oracle(sc.SNAPPY, sblob, soff, (out, oo, meta, rows, rb))
    assert (out[int(oo[m]) + 16:] == 0xA5).all(), "bytes written past the batch's outputs"
    used = int(np.sum(np.where(meta["status"] == 0, meta["n_rows"].astype(np.int64), 0)))
    assert (rows["row_off"][int(rb[m]):] == 0xDEADBEEF).all() and used <= int(rb[m])


def test_copy_threads_setting():
    """slate_ctx_set_copy_threads: 1..256 accepted (a batch decodes the same with 1 or 64 threads),
    0 and > 256 rejected."""
    import slatecodec as sc
    ctx = sc.Context(0)
    blocks = _mixed_batch(5, 600)
    blob, off = bg.pack(blocks, misalign=2)
    for t in (1, 64, 16):
        ctx.set_copy_threads(t)
        _check_against_oracle(sc.SNAPPY, blob, off, ctx.decode_batch(sc.SNAPPY, blob, off))
    for bad in (0, 257):
        with pytest.raises(sc.SlateError):
            ctx.set_copy_threads(bad)


def test_sharded_rejects_duplicate_context():
    import slatecodec as sc
    ctx = sc.Context(0)
    blocks = _mixed_batch(3, 100)
    blob, off = bg.pack(blocks)
    n = len(off) - 1
    st = sc.decode_sharded_into([ctx, ctx], sc.SNAPPY, blob, off, np.zeros(1 << 20, np.uint8),
                                np.zeros(1 << 15, sc.ROW_DTYPE), np.zeros(n, sc.META_DTYPE), np.zeros(n + 1, np.uint64),
                                np.zeros(n + 1, np.uint64))
    assert st == sc.E_INVALID_ARG
