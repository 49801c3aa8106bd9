"""The oracle's executeCompaction restatement (tests/compactgen.py) against a direct statement of
what compaction must produce: for every key the entry of the first source holding it (merge.go
precedence), in key order, tombstones kept, and output SSTs cut after the entry whose running
key+value size passes MaxSSTSize (executor.go:119-139)."""
import random

from tests import compactgen as cg


def _expected(srcs):
    seen = {}
    for run in srcs:
        for sst in run:
            for k, v in cg.sst_rows(sst):
                seen.setdefault(k, v)
    return sorted(seen.items())


def test_oracle_compaction_semantics():
    rng = random.Random(5)
    srcs = cg.random_sources(rng, 4, 300, 700, run_ssts=2)
    out = cg.oracle_compact(srcs, 6000)
    rows = [kv for sst in out for kv in cg.sst_rows(sst)]
    assert rows == _expected(srcs)
    # every output SST but the last passed MaxSSTSize exactly at its last entry
    for sst in out[:-1]:
        sizes = [len(k) + (len(v) if v is not None else 0) for k, v in cg.sst_rows(sst)]
        assert sum(sizes) > 6000 and sum(sizes[:-1]) <= 6000


def test_oracle_compaction_single_output():
    rng = random.Random(6)
    srcs = cg.random_sources(rng, 2, 200, 300)
    out = cg.oracle_compact(srcs, 1 << 40)
    assert len(out) == 1
    assert [kv for kv in cg.sst_rows(out[0])] == _expected(srcs)
