"""GPU executeCompaction for the SST codec path (slatecodec.compaction.compact: device decode of
every input block -> full-key rows -> MergeSort -> gather -> SST builder, cut at MaxSSTSize) against
the oracle's restatement of the same loop (tests/compactgen.py): output SST bytes bit-exact.
Cases: L0 SSTs with overlapping keys and tombstones, sorted runs of several SSTs, Snappy inputs
and outputs, an output split into many SSTs, keys with skewed shared prefixes."""
import random

import pytest

from oracle import binding as ob
from tests import compactgen as cg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    torch.cuda.init()
    torch.cuda.set_device(0)
    import slatecodec as sc
    return sc.Context(0)


@pytest.mark.parametrize("seed,n_src,n_keys,space,codec,run_ssts,max_size,out_codec", [
    (1, 3, 400, 900, ob.NONE, 1, 1 << 30, ob.NONE),
    (2, 4, 1500, 3000, ob.SNAPPY, 1, 1 << 30, ob.SNAPPY),
    (3, 2, 3000, 5000, ob.NONE, 3, 40_000, ob.NONE),
    (4, 5, 800, 1200, ob.SNAPPY, 2, 9_000, ob.NONE),
    (5, 1, 2000, 2000, ob.NONE, 4, 1 << 30, ob.SNAPPY),
])
def test_compaction_bit_exact(ctx, seed, n_src, n_keys, space, codec, run_ssts, max_size, out_codec):
    from slatecodec import compaction
    rng = random.Random(seed)
    srcs = cg.random_sources(rng, n_src, n_keys, space, codec=codec, run_ssts=run_ssts)
    got = compaction.compact(ctx, srcs, max_size, codec=out_codec)
    want = cg.oracle_compact(srcs, max_size, codec=out_codec)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"output SST {i}"


def test_compaction_skewed_prefixes(ctx):
    from slatecodec import compaction
    rng = random.Random(9)
    # shared-prefix lengths from a few bytes to ~70 (past the merge's 16-byte key head)
    def key(i):
        return b"t" + b"/" * (i % 7) * (i % 11) + b"%08d" % i
    srcs = cg.random_sources(rng, 3, 600, 1500, key_fmt=key)
    got = compaction.compact(ctx, srcs, 20_000)
    assert got == cg.oracle_compact(srcs, 20_000)
