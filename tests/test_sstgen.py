"""CPU checks of the SST recoder the every-codec reader tests use (tests/sstgen.py): re-encoding a
CodecNone SST with CodecNone gives back the same bytes, and with CodecSnappy the bytes the oracle's
own Snappy builder writes (builder.go order: blocks, filter, index, info, info offset); LZ4 /
Zlib / Zstd SSTs open in the oracle."""
import random

import pytest

from oracle import binding as ob
from tests import blockgen as bg
from tests import sstgen, zstdgen


@pytest.mark.parametrize("seed", range(3))
def test_recode_none_and_snappy_match_builder(seed):
    rng = random.Random(seed)
    kvs = bg.random_kvs(rng, rng.randint(1, 600))
    bs = rng.choice([128, 512, 4096])
    s = sstgen.none_sst(kvs, bs)
    assert sstgen.recode(s, ob.NONE, rng) == s
    b = ob.SstBuilder(bs, 0, 10, ob.SNAPPY)
    for k, v in kvs:
        assert b.add(k, v) == 0
    assert b.build() == 0
    assert sstgen.recode(s, ob.SNAPPY, rng) == b.encode_table()


@pytest.mark.skipif(not zstdgen.available(), reason="libzstd not in this image")
@pytest.mark.parametrize("codec", [ob.LZ4, ob.ZLIB, ob.ZSTD])
def test_recoded_ssts_open_in_oracle(codec):
    rng = random.Random(codec)
    kvs = bg.random_kvs(rng, 400)
    s = sstgen.recode(sstgen.none_sst(kvs, 512), codec, rng)
    st, info = ob.sst_read_info(s)
    assert st == 0 and info["codec"] == codec
    st, metas = ob.decode_index(s[info["index_offset"]:info["index_offset"] + info["index_len"]], codec)
    assert st == 0 and metas[0][1] == kvs[0][0]
    st, npr, bits = ob.bloom_decode(s[info["filter_offset"]:info["filter_offset"] + info["filter_len"]], codec)
    assert st == 0 and all(ob.bloom_has_key(npr, bits, k) for k, _ in kvs)
