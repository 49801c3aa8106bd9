"""The C restatement of executeCompaction (oracle/compact_oracle.c, or_compact: bench.py's compaction
CPU baseline) against the Python-driven oracle loop of tests/compactgen.py (oracle_compact:
sstable.Iterator per SST, iter.MergeSort, the MaxSSTSize writer loop of
slatedb/compaction/executor.go:92-151): the same output SST bytes, on one thread and on several."""
import random

import pytest

from oracle import binding as ob
from tests import compactgen as cg


@pytest.mark.parametrize("codec", [ob.NONE, ob.SNAPPY])
@pytest.mark.parametrize("shape", [(4, 2000, 6000, 1, 1 << 16), (3, 500, 800, 3, 5000), (1, 100, 200, 1, 1 << 30),
                                   (5, 300, 301, 2, 1)])
def test_or_compact_equals_compactgen(codec, shape):
    k, n, space, run_ssts, max_sst = shape
    srcs = cg.random_sources(random.Random(hash(shape) & 0xFFFF), k, n, space, codec=codec, run_ssts=run_ssts)
    want = cg.oracle_compact(srcs, max_sst, codec=codec)
    for nthreads in (1, 4):
        assert ob.compact(srcs, max_sst, codec, nthreads) == want


def test_or_compact_mixed_codecs_and_outputs():
    """Sources written with different codecs; outputs in a third."""
    rng = random.Random(11)
    srcs = cg.random_sources(rng, 2, 800, 2000, codec=ob.NONE) + cg.random_sources(rng, 2, 800, 2000, codec=ob.SNAPPY)
    for out_codec in (ob.NONE, ob.SNAPPY):
        want = cg.oracle_compact(srcs, 20000, codec=out_codec)
        assert ob.compact(srcs, 20000, out_codec, 3) == want
