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
    assert fetches[0][0] == metas[40][0] and len(fetches) == -(-(bad + 1 - 40) // 16)
