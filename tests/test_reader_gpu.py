"""The read-ahead block reader (slate_block_reader_*): sstable.Iterator.nextBlockIter's contract
(internal/sstable/iterator.go:92-118, one block per step, in order, the iteration ending at the
first block that fails block.Decode with that block's status) with read_ahead blocks fetched and
decoded per GPU call.  Every block against the oracle's block.Decode of its bytes."""
import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _sst(sc, ctx, codec, n_kv=38 * 200):
    b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
    for k, v in bg.kv_synthetic(n_kv):
        assert b.add_value(k, v) == 0
    return b.build().encode()


def _open(sc, ctx, sst, codec):
    st, info, _ = sc.read_info(sst)
    assert st == 0
    st, index = ctx.decode_index(sst[info.index_offset:info.index_offset + info.index_len], codec)
    assert st == 0
    return info, index


def _meta_eq(meta, m):
    return all(int(meta[f]) == int(m[f]) for f in meta.dtype.names)


def _oracle_block(sst, info, metas, i):
    end = metas[i + 1][0] if i + 1 < len(metas) else info.filter_offset if info.filter_len else info.index_offset
    return ob.block_decode(sst[metas[i][0]:end], info.codec)


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("ahead", [1, 5, 64, 100000])
def test_reader_walks_every_block(ctx, codec, ahead):
    import slatecodec as sc
    sst = _sst(sc, ctx, codec)
    info, index = _open(sc, ctx, sst, codec)
    metas = index.block_metas()
    nb = len(metas)
    got, fetches = sc.reader_walk(ctx, info, index, sst, 0, ahead)
    assert [g[0] for g in got] == list(range(nb)) and all(g[1] == 0 for g in got)
    assert len(fetches) == -(-nb // ahead)
    assert fetches[0][0] == metas[0][0] and all(a[1] == b[0] for a, b in zip(fetches, fetches[1:]))
    for blk, st, meta, data, rows in got:
        om, odata, orows = _oracle_block(sst, info, metas, blk)
        assert _meta_eq(meta, om), blk
        assert data == odata[:len(data)], blk
        assert rows.tobytes() == orows[:len(rows)].tobytes(), blk


def test_reader_from_a_block_and_ending_on_a_corrupt_one(ctx):
    import slatecodec as sc
    sst = bytearray(_sst(sc, ctx, ob.SNAPPY))
    info, index = _open(sc, ctx, bytes(sst), ob.SNAPPY)
    metas = index.block_metas()
    bad = 77
    sst[metas[bad][0] + 9] ^= 0x5A  # stale CRC: block.Decode's checksum mismatch
    sst = bytes(sst)
    got, fetches = sc.reader_walk(ctx, info, index, sst, 40, 16)
    assert [g[0] for g in got] == list(range(40, bad + 1))
    assert all(g[1] == 0 for g in got[:-1]) and got[-1][1] == 2  # SLATE_E_BLOCK_CHECKSUM
    om, _, _ = _oracle_block(sst, info, metas, bad)
    assert int(om["status"]) == 2 and _meta_eq(got[-1][2], om)
    # read-ahead: the two batches after the failing block's may already have been asked for (the
    # reader learns of the failure only when that batch's decode completes); none beyond them
    k = -(-(bad + 1 - 40) // 16)
    assert fetches[0][0] == metas[40][0] and k <= len(fetches) <= k + 2


def _kvs_mixed(n, big):
    """n ascending keys; every value 100 B except those at the indices in `big` (index -> length)."""
    rng = np.random.default_rng(7)
    out = []
    for i in range(n):
        ln = big.get(i, 100)
        r = rng.integers(0, 256, size=(ln + 1) // 2, dtype=np.uint8).tobytes()
        out.append((b"k%015d" % i, (r + r)[:ln]))
    return out


@pytest.mark.parametrize("codec", [ob.SNAPPY, ob.NONE, ob.ZSTD, ob.LZ4])
def test_reader_block_shapes_and_codecs(ctx, codec):
    """Blocks of every size class the reader routes: 4 KiB blocks (the workgroup-per-block Snappy
    decoder), 10-40 KiB blocks (the one-wave decoder), a 100 KiB block (the batch path), and codecs
    the host cannot plan (the batch path through slate_read_blocks)."""
    import slatecodec as sc
    kvs = _kvs_mixed(3000, {500: 10000, 501: 40000, 1700: 100000, 2999: 7000})
    b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
    for k, v in kvs:
        assert b.add_value(k, v) == 0
    sst = b.build().encode()
    info, index = _open(sc, ctx, sst, codec)
    metas = index.block_metas()
    for ahead in (7, 64):
        got, fetches = sc.reader_walk(ctx, info, index, sst, 0, ahead)
        assert [g[0] for g in got] == list(range(len(metas))) and all(g[1] == 0 for g in got)
        assert len(fetches) == -(-len(metas) // ahead)
        for blk, st, meta, data, rows in got:
            om, odata, orows = _oracle_block(sst, info, metas, blk)
            assert _meta_eq(meta, om), (codec, ahead, blk)
            assert data == odata[:len(data)], (codec, ahead, blk)
            assert rows.tobytes() == orows[:len(rows)].tobytes(), (codec, ahead, blk)


def test_reader_serves_blocks_before_an_inverted_range(ctx):
    """An index whose block j has an inverted byte range (BlockMeta offsets not increasing): Go's
    nextBlockIter reads one block per call, so it serves blocks 0..j-1 and fails at j's ReadRange.
    The reader cuts its batch before j (a batch-level range error used to fail all of them)."""
    import ctypes as C

    import slatecodec as sc
    sst = _sst(sc, ctx, ob.SNAPPY)
    info, index = _open(sc, ctx, sst, ob.SNAPPY)
    metas = [(o, bytes(k)) for o, k in index.block_metas()]
    j = 30
    metas[j + 1] = (metas[j][0] - 10, metas[j + 1][1])  # block j: [off_j, off_j - 10)
    st, index2 = ctx.decode_index(ob.encode_index(metas, ob.NONE), ob.NONE)
    assert st == 0
    h = C.c_void_p()
    assert sc.lib().slate_block_reader_create(ctx._h, C.byref(info), index2.handle, 0, 64, C.byref(h)) == 0
    served, windows, failed = [], [], None
    try:
        v = sc.BlockView()
        while True:
            st = sc.lib().slate_block_reader_next(h, C.byref(v))
            if st == sc.E_READER_END:
                break
            if st == sc.E_READER_NEED_DATA:
                rs, re_ = C.c_uint64(), C.c_uint64()
                assert sc.lib().slate_block_reader_want(h, C.byref(rs), C.byref(re_)) == 0
                windows.append((rs.value, re_.value))
                if re_.value < rs.value:  # the object store's GetRange fails here, as Go's ReadRange
                    failed = len(served)
                    break
                buf = np.frombuffer(sst[rs.value:re_.value] or b"\0", dtype=np.uint8)
                assert sc.lib().slate_block_reader_feed(h, buf.ctypes.data, re_.value - rs.value) == 0
                continue
            assert st == 0
            served.append(int(v.block))
    finally:
        sc.lib().slate_block_reader_free(h)
    assert failed == j and served == list(range(j))
    assert windows[-1] == (metas[j][0], metas[j + 1][0])
