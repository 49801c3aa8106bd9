"""GPU parity of the device-input SST builder (slate_sst_builder_add_batch_device; compaction's
re-encode, slatedb/compaction/executor.go:100-146 through table_store.go:221-266): SSTs built from
device-resident KVs -- in one batch, in many batches, mixed with host batches and single adds,
with NextBlock between them, with explicit tombstone flags and with empty values as tombstones
-- are byte-identical to the oracle's Go builder restatement fed the same KVs one by one."""
import random

import numpy as np
import pytest

from oracle import binding as ob
from tests import blockgen as bg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    import slatecodec
    return slatecodec


@pytest.fixture(scope="module")
def ctx(sc):
    return sc.Context(0)


def _dev(a: np.ndarray):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).to("cuda")


def _arrays(kvs, tomb_flags=False):
    keys = np.frombuffer(b"".join(k for k, _ in kvs) or b"\0", np.uint8)
    vals = np.frombuffer(b"".join(v or b"" for _, v in kvs) or b"\0", np.uint8)
    ko = np.concatenate([[0], np.cumsum([len(k) for k, _ in kvs])]).astype(np.int64)
    vo = np.concatenate([[0], np.cumsum([len(v or b"") for _, v in kvs])]).astype(np.int64)
    tomb = np.array([v is None for _, v in kvs], np.uint8) if tomb_flags else None
    return keys, ko, vals, vo, tomb


def _oracle(kvs, block_size, codec, next_at=()):
    o = ob.SstBuilder(block_size, 0, 10, codec)
    blocks = []
    for i, (k, v) in enumerate(kvs):
        assert o.add(k, v) == 0
        if i + 1 in next_at:
            while (b := o.next_block()) is not None:
                blocks.append(b)
    assert o.build() == 0
    return o.encode_table(), blocks


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("seed", range(3))
def test_device_batches_match_oracle(sc, ctx, codec, seed):
    rng = random.Random(seed)
    kvs = [(k, v or None) for k, v in bg.random_kvs(rng, rng.randint(1, 3000), klen=(1, 30), vlen=(1, 200), tomb_p=0.1)]
    block_size = rng.choice([256, 1024, 4096])
    # batch boundaries; a NextBlock drain after each batch
    cuts = sorted({0, len(kvs)} | {rng.randrange(len(kvs)) for _ in range(rng.randint(0, 6))})
    g = sc.SstBuilder(ctx, block_size, 0, 10, codec)
    g_blocks = []
    for a, b in zip(cuts, cuts[1:]):
        part = kvs[a:b]
        mode = rng.choice(["device", "device_tomb", "host", "single"])
        keys, ko, vals, vo, tomb = _arrays(part, tomb_flags=mode == "device_tomb")
        if mode.startswith("device"):
            dk, dko, dv, dvo = _dev(keys), _dev(ko), _dev(vals), _dev(vo)
            dt = _dev(tomb) if tomb is not None else None
            assert g.add_batch_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), len(part),
                                      dt.data_ptr() if dt is not None else None) == 0
        elif mode == "host":
            assert g.add_batch(keys, ko.view(np.uint64), vals, vo.view(np.uint64)) == 0
        else:
            for k, v in part:
                assert g.add(k, v) == 0
        while (blk := g.next_block()) is not None:
            g_blocks.append(blk)
    sst = g.build().encode()
    want, o_blocks = _oracle(kvs, block_size, codec, next_at=set(cuts[1:]))
    assert g_blocks == o_blocks
    assert sst == want


def test_device_batch_offsets_not_from_zero(sc, ctx):
    """A slice of a larger device array (key_off[0] > 0), as compaction passes its output splits."""
    rng = random.Random(9)
    kvs = [(k, v or None) for k, v in bg.random_kvs(rng, 2000, vlen=(1, 120), tomb_p=0.2)]
    keys, ko, vals, vo, _ = _arrays(kvs)
    dk, dko, dv, dvo = _dev(keys), _dev(ko), _dev(vals), _dev(vo)
    a, b = 700, 1900
    g = sc.SstBuilder(ctx, 1024, 0, 10, sc.SNAPPY)
    assert g.add_batch_device(dk.data_ptr(), dko.data_ptr() + 8 * a, dv.data_ptr(), dvo.data_ptr() + 8 * a,
                              b - a) == 0
    assert g.build().encode() == _oracle(kvs[a:b], 1024, ob.SNAPPY)[0]


def test_device_batch_empty_key_stops(sc, ctx):
    """block.go:163: an empty key fails the add; the KVs before it are in."""
    kvs = [(b"a", b"1"), (b"b", b"2"), (b"", b"3"), (b"d", b"4")]
    keys, ko, vals, vo, _ = _arrays(kvs)
    dk, dko, dv, dvo = _dev(keys), _dev(ko), _dev(vals), _dev(vo)
    g = sc.SstBuilder(ctx, 4096, 0, 10, sc.NONE)
    assert g.add_batch_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), 4) == sc.E_INVALID_ARG
    assert g.build().encode() == _oracle(kvs[:2], 4096, ob.NONE)[0]


def test_large_device_batch(sc, ctx):
    """200 k V-half KVs in one device batch (several 64 MiB transfer pieces on the way out)."""
    n = 200_000
    kvs = [(k, v or None) for k, v in bg.kv_synthetic(n)]
    keys, ko, vals, vo, _ = _arrays(kvs)
    dk, dko, dv, dvo = _dev(keys), _dev(ko), _dev(vals), _dev(vo)
    g = sc.SstBuilder(ctx, 4096, 0, 10, sc.NONE)
    assert g.add_batch_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), n) == 0
    o = ob.SstBuilder(4096, 0, 10, ob.NONE)
    assert o.add_batch(keys, ko.view(np.uint64), vals, vo.view(np.uint64)) == 0
    assert o.build() == 0
    assert g.build().encode() == o.encode_table()


@pytest.mark.parametrize("bpk", [1, 7, 23])
def test_bucketed_bloom_filter_shapes(sc, ctx, bpk):
    """Filters of >= 64 k keys take the bucketed build (probes per 64 KiB slice OR-ed in LDS):
    1, 5 and 16 probes, 1-33 slices with a partial last one, bits equal to the oracle's."""
    n = 90_001
    kvs = [(k, v or None) for k, v in bg.kv_synthetic(n)]
    keys, ko, vals, vo, _ = _arrays(kvs)
    dk, dko, dv, dvo = _dev(keys), _dev(ko), _dev(vals), _dev(vo)
    g = sc.SstBuilder(ctx, 4096, 0, bpk, sc.NONE)
    assert g.add_batch_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), n) == 0
    o = ob.SstBuilder(4096, 0, bpk, ob.NONE)
    assert o.add_batch(keys, ko.view(np.uint64), vals, vo.view(np.uint64)) == 0
    assert o.build() == 0
    t = g.build()
    assert t.bloom() == o.bloom()
    assert t.encode() == o.encode_table()
